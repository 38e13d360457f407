// r06: one radix-8 stage of the C3 FFT kernel's forward transforms, three ways, as a
// measured prototype - not the product.
//   valu : the product's form (fir_fft.hip dft8 + twiddles): one 8-point vector per lane, packed fp32 VALU.
//   mf32 : exact fp32 on the matrix cores, v_mfma_f32_16x16x4_f32 - the 8-point DFT as a 16 x 16 real
//          matrix (complex F / sqrt 8, interleaved re / im) times 16 vectors (K = 16 as four K = 4 steps),
//          then the per-element twiddles in VALU, then a 4 x 4 (lane group, register) transpose
//          (v_permlane32_swap + v_permlane16_swap) that turns the output layout back into the B layout.
//   mf16 : split f16 on the matrix cores, v_mfma_f32_16x16x16_f16, x = xh + xl and F = Fh + Fl as f16 limbs,
//          D = Fh xh + Fl xh + Fh xl (three products; the 16x16x16 B layout is the output layout: no shuffle).
// Every variant runs R stages on data held in registers (the stage's arithmetic alone: C3's question is the
// energy of its transforms under the power cap), over 2 048 x 4 waves x 64 vectors, launched back to back
// for ~1.5 s per variant in interleaved rounds. Reported: us per launch, stage-vectors per ns, and the
// in-kernel clock (s_memtime cycles over s_memrealtime ticks at 100 MHz, mean over waves). Accuracy: each
// variant's output against a float64 run of the same stages on the host (max |err| / max |x|).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++20 tools/exp/fft_radix_mfma.hip -o <dir>/fft_radix_mfma
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <complex>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef _Float16 h4 __attribute__((ext_vector_type(4)));

constexpr int kWaves = 4, kThreads = 64 * kWaves, kBlocks = 2048;
constexpr int kVec = kBlocks * kWaves * 64;  // 8-point vectors
constexpr float kS = 0.70710678118654752440f;
constexpr float kNorm = 0.35355339059327376220f;  // 1 / sqrt 8: the stages keep the data's magnitude

#define HIPCHK(x)                                                                   \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                      \
    }                                                                               \
  } while (0)

// twiddle of vector v, point j (unit modulus; the same values in every variant and on the host)
__host__ __device__ inline void twiddle(int v, int j, float& c, float& s) {
  const int e = (j * (v & 63)) & 511;
  const float a = -6.283185307179586f * (float)e / 512.0f;
  c = cosf(a);
  s = sinf(a);
}

__device__ inline f2 cmul(f2 a, f2 b) { return f2{a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x}; }
__device__ inline f2 mulMi(f2 v) { return f2{v.y, -v.x}; }  // -i v

// the product's 8-point DFT (fir_fft.hip dft8<false>), scaled by 1 / sqrt 8
__device__ inline void dft8(f2 (&z)[8]) {
  const f2 a0 = z[0] + z[4], a1 = z[0] - z[4], a2 = z[2] + z[6], a3 = z[2] - z[6];
  const f2 a4 = z[1] + z[5], a5 = z[1] - z[5], a6 = z[3] + z[7], a7 = z[3] - z[7];
  const f2 b0 = a0 + a2, b2 = a0 - a2, b4 = a4 + a6, b6 = a4 - a6;
  const f2 b1 = a1 + mulMi(a3), b3 = a1 - mulMi(a3), b5 = a5 + mulMi(a7), b7 = a5 - mulMi(a7);
  const f2 t5 = f2{b5.x + b5.y, b5.y - b5.x};  // (1 - i) b5
  const f2 t7 = f2{b7.x - b7.y, b7.x + b7.y};  // (1 + i) b7
  const f2 sv = {kS, kS}, nv = {kNorm, kNorm};
  z[0] = (b0 + b4) * nv;
  z[4] = (b0 - b4) * nv;
  z[2] = (b2 + mulMi(b6)) * nv;
  z[6] = (b2 - mulMi(b6)) * nv;
  z[1] = (b1 + t5 * sv) * nv;
  z[5] = (b1 - t5 * sv) * nv;
  z[3] = (b3 - t7 * sv) * nv;
  z[7] = (b3 + t7 * sv) * nv;
}

__device__ inline void clockBegin(unsigned long long& t, unsigned long long& r) {
  t = __builtin_amdgcn_s_memtime();
  r = __builtin_amdgcn_s_memrealtime();
}
__device__ inline void clockEnd(unsigned long long t, unsigned long long r, unsigned long long* clk) {
  const unsigned long long dt = __builtin_amdgcn_s_memtime() - t, dr = __builtin_amdgcn_s_memrealtime() - r;
  if ((threadIdx.x & 63) == 0) {
    const int w = blockIdx.x * kWaves + (threadIdx.x >> 6);
    clk[2 * w] = dt;  // plain stores, one per wave (no scalar-cache writes)
    clk[2 * w + 1] = dr;
  }
}

// ---- valu: vector v = global lane, z[j] = x[v][j] ----------------------------------------------------
__global__ __launch_bounds__(kThreads) void stageValu(const f2* x, f2* y, int R, unsigned long long* clk) {
  const int v = blockIdx.x * kThreads + threadIdx.x;
  f2 z[8], tw[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    z[j] = x[8 * v + j];
    float c, sn;
    twiddle(v, j, c, sn);
    tw[j] = f2{c, sn};
  }
  unsigned long long t0, r0;
  clockBegin(t0, r0);
  for (int r = 0; r < R; ++r) {
    dft8(z);
#pragma unroll
    for (int j = 1; j < 8; ++j) z[j] = cmul(z[j], tw[j]);
  }
  clockEnd(t0, r0, clk);
#pragma unroll
  for (int j = 0; j < 8; ++j) y[8 * v + j] = z[j];
}

// Real 16 x 16 form of F / sqrt 8 with interleaved (re, im): R[2j + p][2n + q].
__host__ __device__ inline float fReal(int row, int col) {
  const int j = row >> 1, p = row & 1, n = col >> 1, q = col & 1;
  const int e = (j * n) & 7;
  const float a = -6.283185307179586f * (float)e / 8.0f;
  const float c = cosf(a) * kNorm, s = sinf(a) * kNorm;
  // (re, im) out = [[c, -s], [s, c]] (re, im) in
  return p == 0 ? (q == 0 ? c : -s) : (q == 0 ? s : c);
}

// MFMA layouts (wave of 64 lanes, l = 16 g + n): 16 x 16 blocks of 16 vectors (columns n); the real
// index k = 4 g + i of column n sits in lane l register i (the D layout of 16x16xK, and the B layout of
// 16x16x16 f16). Vector of block b, column n: 16 b + n of the wave.
__device__ inline void loadMf(const f2* x, int waveVec0, int l, f4 (&d)[4]) {
  const int g = l >> 4, n = l & 15;
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    const int v = waveVec0 + 16 * b + n;
    // k = 4 g + i -> point j = 2 g + (i >> 1), component i & 1
    const f2 p0 = x[8 * v + 2 * g], p1 = x[8 * v + 2 * g + 1];
    d[b] = f4{p0.x, p0.y, p1.x, p1.y};
  }
}
__device__ inline void storeMf(f2* y, int waveVec0, int l, const f4 (&d)[4]) {
  const int g = l >> 4, n = l & 15;
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    const int v = waveVec0 + 16 * b + n;
    y[8 * v + 2 * g] = f2{d[b].x, d[b].y};
    y[8 * v + 2 * g + 1] = f2{d[b].z, d[b].w};
  }
}
// twiddles of the lane's two points (j = 2 g, 2 g + 1) in each block
__device__ inline void twMf(int waveVec0, int l, f2 (&tw)[4][2]) {
  const int g = l >> 4, n = l & 15;
#pragma unroll
  for (int b = 0; b < 4; ++b)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      float c, sn;
      twiddle(waveVec0 + 16 * b + n, 2 * g + h, c, sn);
      tw[b][h] = f2{c, sn};
    }
}
__device__ inline void twApply(f4& d, const f2 (&t)[2], int g) {
  // point 0 (g = 0, h = 0) has twiddle 1 like the VALU form's z[0]; applied uniformly anyway (t = 1 there)
  const f2 a = cmul(f2{d.x, d.y}, t[0]), b = cmul(f2{d.z, d.w}, t[1]);
  d = f4{a.x, a.y, b.x, b.y};
}

__device__ inline void swap32(float& a, float& b) { asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(a), "+v"(b)); }
__device__ inline void swap16(float& a, float& b) { asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(a), "+v"(b)); }

// D layout (lane group g holds rows 4 g + i) -> the 16x16x4 f32 B layout of K step c (lane group g holds
// row 4 c + g): element (group g, register i) <- (group i, register g), a 4 x 4 transpose.
__device__ inline void transpose44(f4& d) {
  float e0 = d.x, e1 = d.y, e2 = d.z, e3 = d.w;
  swap32(e0, e2);  // group bit 1 <-> register bit 1
  swap32(e1, e3);
  swap16(e0, e1);  // group bit 0 <-> register bit 0
  swap16(e2, e3);
  d = f4{e0, e1, e2, e3};
}

// ---- mf32: exact fp32 MFMA --------------------------------------------------------------------------
__global__ __launch_bounds__(kThreads) void stageMf32(const f2* x, f2* y, int R, unsigned long long* clk) {
  const int l = threadIdx.x & 63, g = l >> 4, n = l & 15;
  const int waveVec0 = (blockIdx.x * kWaves + (threadIdx.x >> 6)) * 64;
  float a[4];  // A of K step c: lane l holds R[n][4 c + g]
#pragma unroll
  for (int c = 0; c < 4; ++c) a[c] = fReal(n, 4 * c + g);
  f4 d[4];
  f2 tw[4][2];
  loadMf(x, waveVec0, l, d);
  twMf(waveVec0, l, tw);
  unsigned long long t0, r0;
  clockBegin(t0, r0);
  for (int r = 0; r < R; ++r) {
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      f4 bt = d[b];
      transpose44(bt);  // bt register c = B of K step c: row 4 c + g, column n
      f4 acc = f4{0.0f, 0.0f, 0.0f, 0.0f};
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[0], bt.x, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[1], bt.y, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[2], bt.z, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[3], bt.w, acc, 0, 0, 0);
      twApply(acc, tw[b], g);
      d[b] = acc;
    }
  }
  clockEnd(t0, r0, clk);
  storeMf(y, waveVec0, l, d);
}

// ---- mf16: split f16 MFMA ---------------------------------------------------------------------------
__global__ __launch_bounds__(kThreads) void stageMf16(const f2* x, f2* y, int R, unsigned long long* clk) {
  const int l = threadIdx.x & 63, g = l >> 4, n = l & 15;
  const int waveVec0 = (blockIdx.x * kWaves + (threadIdx.x >> 6)) * 64;
  h4 ah, al;  // A: lane l holds R[n][4 g + i], i < 4, as hi + lo
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float v = fReal(n, 4 * g + i);
    ah[i] = (_Float16)v;
    al[i] = (_Float16)(v - (float)ah[i]);
  }
  f4 d[4];
  f2 tw[4][2];
  loadMf(x, waveVec0, l, d);
  twMf(waveVec0, l, tw);
  unsigned long long t0, r0;
  clockBegin(t0, r0);
  for (int r = 0; r < R; ++r) {
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      h4 xh, xl;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        xh[i] = (_Float16)d[b][i];
        xl[i] = (_Float16)(d[b][i] - (float)xh[i]);
      }
      f4 acc = f4{0.0f, 0.0f, 0.0f, 0.0f};
      acc = __builtin_amdgcn_mfma_f32_16x16x16f16(ah, xh, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x16f16(al, xh, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x16f16(ah, xl, acc, 0, 0, 0);
      twApply(acc, tw[b], g);
      d[b] = acc;
    }
  }
  clockEnd(t0, r0, clk);
  storeMf(y, waveVec0, l, d);
}

typedef void (*Kern)(const f2*, f2*, int, unsigned long long*);

int main(int argc, char** argv) {
  const int R = argc > 1 ? atoi(argv[1]) : 64;
  const double seconds = argc > 2 ? atof(argv[2]) : 1.5;
  std::vector<f2> hx(8 * (size_t)kVec);
  uint64_t s = 0x9E3779B97F4A7C15ull;
  for (auto& v : hx) {
    s = s * 6364136223846793005ull + 1442695040888963407ull;
    const float a = (float)((s >> 40) & 0xffffff) / 16777216.0f - 0.5f;
    s = s * 6364136223846793005ull + 1442695040888963407ull;
    const float b = (float)((s >> 40) & 0xffffff) / 16777216.0f - 0.5f;
    v = f2{a, b};
  }
  f2 *dx, *dy;
  unsigned long long* dclk;
  HIPCHK(hipMalloc(&dx, sizeof(f2) * hx.size()));
  HIPCHK(hipMalloc(&dy, sizeof(f2) * hx.size()));
  HIPCHK(hipMalloc(&dclk, sizeof(unsigned long long) * 2 * kBlocks * kWaves));
  HIPCHK(hipMemcpy(dx, hx.data(), sizeof(f2) * hx.size(), hipMemcpyHostToDevice));

  // float64 reference of R stages for the first 256 vectors
  const int nRef = 256;
  std::vector<std::complex<double>> ref(8 * nRef);
  for (int v = 0; v < nRef; ++v) {
    std::complex<double> z[8];
    for (int j = 0; j < 8; ++j) z[j] = {hx[8 * v + j].x, hx[8 * v + j].y};
    for (int r = 0; r < R; ++r) {
      std::complex<double> o[8];
      for (int k = 0; k < 8; ++k) {
        o[k] = 0;
        for (int j = 0; j < 8; ++j) o[k] += z[j] * std::polar(1.0 / std::sqrt(8.0), -2 * M_PI * ((j * k) % 8) / 8.0);
      }
      for (int k = 0; k < 8; ++k) {
        float c, sn;
        twiddle(v, k, c, sn);
        z[k] = k == 0 ? o[k] : o[k] * std::complex<double>(c, sn);
      }
    }
    for (int j = 0; j < 8; ++j) ref[8 * v + j] = z[j];
  }

  struct V {
    const char* name;
    Kern k;
    std::vector<double> us, mhz;
    double err = 0;
  } vars[] = {{"valu (product form)", stageValu, {}, {}}, {"mf32 16x16x4 f32", stageMf32, {}, {}},
              {"mf16 16x16x16 f16 x3", stageMf16, {}, {}}};
  hipEvent_t e0, e1;
  HIPCHK(hipEventCreate(&e0));
  HIPCHK(hipEventCreate(&e1));
  for (auto& v : vars) {  // accuracy (one launch) and warm-up
    hipLaunchKernelGGL(v.k, dim3(kBlocks), dim3(kThreads), 0, 0, dx, dy, R, dclk);
    HIPCHK(hipDeviceSynchronize());
    std::vector<f2> hy(8 * nRef);
    HIPCHK(hipMemcpy(hy.data(), dy, sizeof(f2) * hy.size(), hipMemcpyDeviceToHost));
    double m = 0, mx = 0;
    for (int i = 0; i < 8 * nRef; ++i) {
      m = std::max(m, std::abs(std::complex<double>(hy[i].x, hy[i].y) - ref[i]));
      mx = std::max(mx, std::abs(ref[i]));
    }
    v.err = m / mx;
  }
  for (int round = 0; round < 3; ++round)
    for (auto& v : vars) {
      // back to back for `seconds` (the clock settles under the power controller), timing the last 20
      const auto t0 = std::chrono::steady_clock::now();
      int launches = 0;
      while (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < seconds) {
        for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(v.k, dim3(kBlocks), dim3(kThreads), 0, 0, dx, dy, R, dclk);
        HIPCHK(hipDeviceSynchronize());
        launches += 20;
      }
      HIPCHK(hipEventRecord(e0));
      for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(v.k, dim3(kBlocks), dim3(kThreads), 0, 0, dx, dy, R, dclk);
      HIPCHK(hipEventRecord(e1));
      HIPCHK(hipEventSynchronize(e1));
      float ms = 0;
      HIPCHK(hipEventElapsedTime(&ms, e0, e1));
      std::vector<unsigned long long> c(2 * kBlocks * kWaves);
      HIPCHK(hipMemcpy(c.data(), dclk, sizeof(unsigned long long) * c.size(), hipMemcpyDeviceToHost));
      double cyc = 0, ticks = 0;
      for (int w = 0; w < kBlocks * kWaves; ++w) {
        cyc += (double)c[2 * w];
        ticks += (double)c[2 * w + 1];
      }
      v.us.push_back(1000.0 * ms / 20);
      v.mhz.push_back(ticks > 0 ? 100.0 * cyc / ticks : 0.0);
      (void)launches;
    }
  printf("R = %d stages over %d 8-point vectors per launch (%.1f M stage-vectors)\n", R, kVec, R * (double)kVec / 1e6);
  for (auto& v : vars) {
    std::vector<double> u = v.us, m = v.mhz;
    std::sort(u.begin(), u.end());
    std::sort(m.begin(), m.end());
    printf("%-24s median %9.1f us/launch  %7.2f stage-vectors/ns  in-kernel clock %6.0f MHz (rounds %.1f %.1f %.1f us)"
           "  max|err|/max|x| %.2e\n",
           v.name, u[1], R * (double)kVec / (u[1] * 1e3), m[1], v.us[0], v.us[1], v.us[2], v.err);
  }
  return 0;
}
