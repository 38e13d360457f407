// MFMA FIR for cf32 input and real taps (gsdrFirFC / gsdrFirFCAmDemod: the C3 / C4 chains, up to
// K = 15 D + T <= 1536), split-precision bf16 on v_mfma_f32_16x16x32_bf16.
//
// Arithmetic. Every fp32 value v (sample component or tap) is split EXACTLY into three bf16
// limbs by round-to-nearest: v0 = bf16(v), v1 = bf16(v - v0), v2 = v - v0 - v1 (<= 8 significant
// bits, exact in bf16), |v1| <= 2^-9 |v|, |v2| <= 2^-18 |v|. The kernel sums the six products
// x_i h_j with i + j <= 2; the dropped ones are below 2^-26 |x h|. The MFMA forms each bf16
// product exactly and accumulates in fp32, so the result carries the rounding of an fp32
// accumulation - the class of the reference's fp32 direct form (tests: 1e-6 of sum |h||x|).
//
// GEMM shape (decimating Toeplitz). Output k = 16 m + n of a row block (m < 8 output rows,
// n < 16 columns):
//     C[m][n] = sum_kappa A[m][kappa] B[kappa][n],  A[m][kappa] = x[16 D m + kappa],
//     B[kappa][n] = h[kappa - n D] (0 <= kappa - n D < T, else 0),  kappa < K = 15 D + T.
// A rows 0-7 take the re parts, rows 8-15 the im parts of the same 8 output rows. A tile is two
// row blocks (256 outputs).
//
// Work split. One 512-thread block per CU walks a contiguous range of tiles. The K range is split
// over the 8 waves (KS K-steps of 32 each): a wave's B fragments (3 limbs x KS K-steps of the
// Toeplitz tap matrix) stay in VGPRs for the whole launch. The tile's input window (W = 240 D +
// 256 KS samples) is loaded into registers two tiles ahead and split into six bf16 planes (3
// limbs x re/im) in one of two LDS buffers one tile ahead, so a tile's split and its MFMAs use
// different buffers: waves 0-3 split before their MFMAs, waves 4-7 after, and the two waves that
// share a SIMD overlap the vector work of one with the matrix work of the other. One barrier per
// tile; partial accumulators meet in (double-buffered) LDS and 256 threads reduce one output each.
// The plane layout (padding, re/im plane offset) is picked per D against bank conflicts.
//
// Non-finite samples: the Toeplitz product multiplies a sample by the zero taps of outputs whose
// windows do not contain it (0 * inf = NaN). A tile whose reduced outputs are not all finite is
// recomputed in the direct fp32 form by the same threads (reference semantics).
#include <mutex>

#include "kcommon.h"
#include "fir_launch.h"

#ifndef GSDR_CF_EXPERIMENT
#define GSDR_CF_EXPERIMENT 0  // attribution builds only (tools/exp): 1 = skip split, 2 = skip MFMA,
                              // 4 = skip loads
#endif

namespace gsdr_amd {

typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf2 __attribute__((ext_vector_type(2)));

constexpr int kCfWaves = 8;
constexpr int kCfThreads = kCfWaves * kWave;
constexpr int kCfRB = 2;                       // row blocks per tile
constexpr int kCfTileOut = 128 * kCfRB;        // 256 outputs: 16 output rows x 16 columns
constexpr int kCfMaxKS = 6;                    // K-steps of 32 per wave: K <= 8 x 6 x 32 = 1536
constexpr int kCfPartBytes = kCfWaves * 4 * kCfRB * kWave * 4;  // one partial buffer (16 KB)
constexpr int kCfDynLdsMax = 160 * 1024 - 256;                  // the rest: static flags

struct CfFirArgs {
  const float* x;       // interleaved re, im (16-byte aligned)
  const float* taps;
  void* out;
  int64_t nOut;
  int64_t nIn;          // complex samples readable: (nOut - 1) D + T
  int32_t T;
  int32_t D;
  int32_t KS;           // K-steps per wave
  int32_t tiles;
  int32_t Wu;           // window units (8 samples) per tile = 30 D + 32 KS
  int32_t padShift;     // plane unit u at u + (u >> padShift) (31: no padding)
  int32_t planeStride;  // bytes between planes (limb l, component c at 2 l + c)
};

// fp32 pair -> three bf16 limb pairs (exact).
__device__ __forceinline__ void split3(float a, float b, uint32_t& l0, uint32_t& l1, uint32_t& l2) {
  typedef float f2v __attribute__((ext_vector_type(2)));
  const f2v v = {a, b};
  const bf2 h0 = __builtin_convertvector(v, bf2);
  const f2v r1 = v - __builtin_convertvector(h0, f2v);
  const bf2 h1 = __builtin_convertvector(r1, bf2);
  const f2v r2 = r1 - __builtin_convertvector(h1, f2v);
  const bf2 h2 = __builtin_convertvector(r2, bf2);
  l0 = __builtin_bit_cast(uint32_t, h0);
  l1 = __builtin_bit_cast(uint32_t, h1);
  l2 = __builtin_bit_cast(uint32_t, h2);
}

// Window registers: G groups of 8 samples (64 B) per thread, group g = tid + 512 j.
template <int G>
struct CfWindow {
  f4 v[G][4];  // native vector type: HIP's float4 union defeats register promotion
};

// Branch-free, so the loads stay in flight until the split that consumes them; f4 index
// arithmetic on the kernel-argument pointer keeps them global_load (a flat load would also count
// on lgkmcnt and stall the LDS waits of the MFMA loop). Blocks past the input end re-read the last
// one (their samples feed only outputs >= nOut or meet zero taps); surplus groups repeat the last.
template <int G>
__device__ __forceinline__ void loadWindow(const CfFirArgs& a, int tile, int tid, CfWindow<G>& w) {
  const f4* x4 = reinterpret_cast<const f4*>(a.x);
  const int64_t base = (int64_t)tile * kCfTileOut * a.D / 2;
  const int64_t last = (a.nIn - 1) >> 1;
#pragma unroll
  for (int j = 0; j < G; ++j) {
    const int g = min(tid + kCfThreads * j, a.Wu - 1);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int64_t i = base + 4 * (int64_t)g + q;
      w.v[j][q] = x4[i < last ? i : last];
    }
  }
}

__device__ __forceinline__ int cfUnit(int u, int p) { return u + (u >> p); }

template <int G>
__device__ __forceinline__ void splitWindow(const CfFirArgs& a, const CfWindow<G>& w, int8_t* buf, int tid) {
#pragma unroll
  for (int j = 0; j < G; ++j) {
    const int g = min(tid + kCfThreads * j, a.Wu - 1);
    uint32_t iL[3][4], qL[3][4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {  // samples 2q, 2q + 1: (re, im, re, im)
      split3(w.v[j][q].x, w.v[j][q].z, iL[0][q], iL[1][q], iL[2][q]);
      split3(w.v[j][q].y, w.v[j][q].w, qL[0][q], qL[1][q], qL[2][q]);
    }
    const int off = 16 * cfUnit(g, a.padShift);
#pragma unroll
    for (int l = 0; l < 3; ++l) {
      *reinterpret_cast<uint4*>(buf + (2 * l) * a.planeStride + off) = uint4{iL[l][0], iL[l][1], iL[l][2], iL[l][3]};
      *reinterpret_cast<uint4*>(buf + (2 * l + 1) * a.planeStride + off) = uint4{qL[l][0], qL[l][1], qL[l][2], qL[l][3]};
    }
  }
}

// This wave's share of one tile: both row blocks over its KS K-steps, 6 MFMAs per K-step and
// row block, into the partial-sum buffer `part` ([wave][register][lane]).
__device__ __forceinline__ void tileMfma(const CfFirArgs& a, const int8_t* buf, const bf8 (&bf)[kCfMaxKS][3],
                                         float* part, int wave, int lane) {
  typedef float v4f __attribute__((ext_vector_type(4)));
  const int r = lane & 15;
  const int8_t* plane = buf + (r >> 3) * a.planeStride;  // re rows 0-7, im rows 8-15
  const int uRow = 2 * a.D * (r & 7) + (lane >> 4) + 4 * wave * a.KS;
  v4f acc[kCfRB];
#pragma unroll
  for (int rb = 0; rb < kCfRB; ++rb) acc[rb] = v4f{};
#pragma unroll
  for (int s = 0; s < kCfMaxKS; ++s) {
    if (s < a.KS && !(GSDR_CF_EXPERIMENT & 2)) {
#pragma unroll
      for (int rb = 0; rb < kCfRB; ++rb) {
        const int off = 16 * cfUnit(uRow + 16 * a.D * rb + 4 * s, a.padShift);
        const bf8 x0 = *reinterpret_cast<const bf8*>(plane + off);
        const bf8 x1 = *reinterpret_cast<const bf8*>(plane + 2 * a.planeStride + off);
        const bf8 x2 = *reinterpret_cast<const bf8*>(plane + 4 * a.planeStride + off);
        acc[rb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x0, bf[s][0], acc[rb], 0, 0, 0);
        acc[rb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x0, bf[s][1], acc[rb], 0, 0, 0);
        acc[rb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x1, bf[s][0], acc[rb], 0, 0, 0);
        acc[rb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x0, bf[s][2], acc[rb], 0, 0, 0);
        acc[rb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x1, bf[s][1], acc[rb], 0, 0, 0);
        acc[rb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x2, bf[s][0], acc[rb], 0, 0, 0);
      }
    }
  }
#pragma unroll
  for (int rb = 0; rb < kCfRB; ++rb)
#pragma unroll
    for (int i = 0; i < 4; ++i) part[(wave * 4 * kCfRB + 4 * rb + i) * kWave + lane] = acc[rb][i];
}

// Direct fp32 form of output k (tiles holding a non-finite value).
template <int EPI>
__device__ __forceinline__ void cfDirectOutput(const CfFirArgs& a, int64_t k) {
  if (k >= a.nOut) return;
  const f2* x = reinterpret_cast<const f2*>(a.x) + k * a.D;
  f2 y = f2{0.0f, 0.0f};
  for (int j = 0; j < a.T; ++j) y += a.taps[j] * x[j];
  if (EPI == kEpiAm) reinterpret_cast<float*>(a.out)[k] = amEnvelope(y);
  else reinterpret_cast<f2*>(a.out)[k] = y;
}

template <int G, int EPI>
__global__ __launch_bounds__(kCfThreads, 1) void firCfMfmaKernel(CfFirArgs a) {
  extern __shared__ __attribute__((aligned(16))) int8_t smem[];
  const int bufBytes = 6 * a.planeStride;
  float* parts = reinterpret_cast<float*>(smem + 2 * bufBytes);  // two partial buffers
  __shared__ int nonFinite[3];  // per tile mod 3: a reduced output was inf / NaN

  const int tid = threadIdx.x;
  const int lane = tid & (kWave - 1);
  const int wave = waveUniform(tid >> 6);
  const int D = a.D, T = a.T, KS = a.KS;

  // contiguous tile range of this block
  const int q = a.tiles / (int)gridDim.x, r = a.tiles % (int)gridDim.x;
  const int t0 = (int)blockIdx.x * q + min((int)blockIdx.x, r);
  const int n = q + ((int)blockIdx.x < r ? 1 : 0);
  if (n <= 0) return;

  CfWindow<G> win;
  loadWindow<G>(a, t0, tid, win);

  // ---- taps -> LDS (zero-padded to [-15 D, 256 KS)), then this wave's B fragments -------------
  if (tid < 3) nonFinite[tid] = 0;
  const int off0 = 15 * D;
  const int span = off0 + 256 * KS;
  for (int i = tid; i < span; i += kCfThreads) {
    const int j = i - off0;
    parts[i] = (j >= 0 && j < T) ? a.taps[j] : 0.0f;
  }
  __syncthreads();
  const int col = lane & 15;
  bf8 bf[kCfMaxKS][3];
#pragma unroll
  for (int s = 0; s < kCfMaxKS; ++s) {
    if (s < KS) {
      const int kap = 32 * (wave * KS + s) + 8 * (lane >> 4);  // first kappa of this lane's 8
      uint32_t l[3][4];
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const float h0 = parts[off0 + kap + 2 * p - col * D];
        const float h1 = parts[off0 + kap + 2 * p + 1 - col * D];
        split3(h0, h1, l[0][p], l[1][p], l[2][p]);
      }
#pragma unroll
      for (int i = 0; i < 3; ++i) bf[s][i] = __builtin_bit_cast(bf8, uint4{l[i][0], l[i][1], l[i][2], l[i][3]});
    } else {
#pragma unroll
      for (int i = 0; i < 3; ++i) bf[s][i] = bf8{};
    }
  }
  __syncthreads();  // the tap staging area becomes the partial buffers

  // ---- prologue: tile t0 into buffer 0, tile t0 + 1's loads in flight ------------------------
  if (!(GSDR_CF_EXPERIMENT & 1)) splitWindow<G>(a, win, smem, tid);
  if (n > 1 && !(GSDR_CF_EXPERIMENT & 4)) loadWindow<G>(a, t0 + 1, tid, win);
  __syncthreads();

  for (int i = 0; i < n; ++i) {
    const int tile = t0 + i;
    const int8_t* cur = smem + (i & 1) * bufBytes;
    int8_t* nxt = smem + ((i + 1) & 1) * bufBytes;
    float* part = parts + (i & 1) * (kCfPartBytes / 4);
    const bool splitNext = i + 1 < n && !(GSDR_CF_EXPERIMENT & 1);
    // waves 0-3 split tile + 1 first, waves 4-7 run their MFMAs first (wave-uniform)
    if (wave < 4) {
      if (splitNext) splitWindow<G>(a, win, nxt, tid);
      tileMfma(a, cur, bf, part, wave, lane);
    } else {
      tileMfma(a, cur, bf, part, wave, lane);
      if (splitNext) splitWindow<G>(a, win, nxt, tid);
    }
    if (i + 2 < n && !(GSDR_CF_EXPERIMENT & 4)) loadWindow<G>(a, tile + 2, tid, win);
    __syncthreads();  // partials of tile, planes of tile + 1 complete
    if (tid == 0) nonFinite[(i + 1) % 3] = 0;  // tile i - 2's flag, read before this barrier

    if (tid < kCfTileOut) {
      // tile - 1 left a non-finite output: redo it in the direct form (same thread, same output)
      if (i > 0 && nonFinite[(i + 2) % 3]) cfDirectOutput<EPI>(a, (int64_t)(tile - 1) * kCfTileOut + tid);
      // reduction + epilogue: output o = tid of this tile
      const int o = tid, rb = o >> 7, orow = (o >> 4) & 7;
      const int laneI = 16 * (orow >> 2) + (o & 15);
      const int reg = 4 * rb + (orow & 3);
      float yi = 0.0f, yq = 0.0f;
#pragma unroll
      for (int v = 0; v < kCfWaves; ++v) {
        yi += part[(v * 4 * kCfRB + reg) * kWave + laneI];
        yq += part[(v * 4 * kCfRB + reg) * kWave + laneI + 32];
      }
      const int64_t k = (int64_t)tile * kCfTileOut + o;
      if (k < a.nOut) {
        if (EPI == kEpiAm) reinterpret_cast<float*>(a.out)[k] = amEnvelope(f2{yi, yq});
        else reinterpret_cast<f2*>(a.out)[k] = f2{yi, yq};
        if (!(__builtin_isfinite(yi) && __builtin_isfinite(yq))) nonFinite[i % 3] = 1;
      }
    }
  }
  __syncthreads();
  if (tid < kCfTileOut && nonFinite[(n - 1) % 3]) cfDirectOutput<EPI>(a, (int64_t)(t0 + n - 1) * kCfTileOut + tid);
}

// ---- host side ------------------------------------------------------------------------------

namespace {

// Lane groups of ds_read_b128 (MI355X_MICROARCH.md, LDS): 4 x 16 lanes, one LDS cycle each.
constexpr int kB128Groups[4][16] = {
    {0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27},
    {4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31},
    {32, 33, 34, 35, 44, 45, 46, 47, 52, 53, 54, 55, 56, 57, 58, 59},
    {36, 37, 38, 39, 40, 41, 42, 43, 48, 49, 50, 51, 60, 61, 62, 63}};

struct CfLayout {
  int padShift;
  int planeStride;
};

// Pick the plane padding and the re/im plane offset that minimise the A-fragment bank conflicts
// for this (D, KS) within the LDS budget (2 plane buffers + 2 partial buffers).
CfLayout cfLayout(int D, int KS, int Wu) {
  CfLayout best{31, 0};
  double bestCost = 1e30;
  const int shifts[] = {31, 6, 5, 4, 3, 2, 1};
  for (int p : shifts) {
    const int units = Wu + (p < 31 ? (Wu >> p) : 0) + 1;
    const int base = (16 * units + 255) / 256 * 256;
    for (int qoff = 0; qoff < 16; ++qoff) {
      const int stride = base + 16 * qoff;
      if (2 * 6 * stride + 2 * kCfPartBytes > kCfDynLdsMax) continue;
      double cost = 0;
      for (int rb = 0; rb < kCfRB; ++rb) {
        for (int s = 0; s < kCfWaves * KS; ++s) {
          for (const auto& grp : kB128Groups) {
            int units16[16][4];
            int cnt[16] = {};
            int worst = 1;
            for (int li = 0; li < 16; ++li) {
              const int l = grp[li];
              const int rr = l & 15;
              const int u = 2 * D * ((rr & 7) + 8 * rb) + (l >> 4) + 4 * s;
              const int unit = u + (p < 31 ? (u >> p) : 0) + ((rr >> 3) ? stride / 16 : 0);
              const int slot = unit & 15;
              bool dup = false;
              for (int c = 0; c < cnt[slot]; ++c) dup |= units16[slot][c] == unit;
              if (!dup && cnt[slot] < 4) units16[slot][cnt[slot]++] = unit;
              worst = cnt[slot] > worst ? cnt[slot] : worst;
            }
            cost += worst;
          }
        }
      }
      cost += 1e-3 * (12.0 * stride) / 1024.0;  // tie-break: less LDS
      if (cost < bestCost) {
        bestCost = cost;
        best = CfLayout{p, stride};
      }
    }
  }
  return best;
}

template <int G, int EPI>
hipError_t launchCf(const CfFirArgs& a, size_t lds, int grid, hipStream_t stream) {
  static std::once_flag once;
  static hipError_t attrErr = hipSuccess;
  std::call_once(once, [] {
    attrErr = hipFuncSetAttribute(reinterpret_cast<const void*>(&firCfMfmaKernel<G, EPI>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, kCfDynLdsMax);
  });
  if (attrErr != hipSuccess) return attrErr;
  hipLaunchKernelGGL((firCfMfmaKernel<G, EPI>), dim3(grid), dim3(kCfThreads), lds, stream, a);
  return hipGetLastError();
}

}  // namespace

bool firCfMfmaEligible(size_t tapCount, size_t decimation, const void* in) {
  const size_t d = decimation < 1 ? 1 : decimation;
  if (tapCount < 64 || d > 32 || 15 * d + tapCount > (size_t)(kCfWaves * kCfMaxKS * 32) ||
      (reinterpret_cast<uintptr_t>(in) & 15u) != 0)
    return false;
  const size_t ksteps = (15 * d + tapCount + 31) / 32;
  const size_t ks = (ksteps + kCfWaves - 1) / kCfWaves;
  const size_t wu = 30 * d + 32 * ks;
  if (wu > 2 * (size_t)kCfThreads) return false;  // window registers: at most 2 groups per thread
  const size_t stride = (16 * (wu + 1) + 255) / 256 * 256 + 16 * 15;  // unpadded, worst offset
  return 12 * stride + 2 * kCfPartBytes <= (size_t)kCfDynLdsMax;
}

hipError_t launchFirCfMfma(const float* x, const float* taps, size_t tapCount, size_t decimation, void* out,
                           size_t nOut, int epi, hipStream_t stream) {
  CfFirArgs a{};
  a.x = x;
  a.taps = taps;
  a.out = out;
  a.D = (int32_t)(decimation < 1 ? 1 : decimation);
  a.T = (int32_t)tapCount;
  a.nOut = (int64_t)nOut;
  a.nIn = (int64_t)(nOut - 1) * a.D + (int64_t)tapCount;
  const int ksteps = (15 * a.D + a.T + 31) / 32;
  a.KS = (ksteps + kCfWaves - 1) / kCfWaves;
  const int64_t tiles = ((int64_t)nOut + kCfTileOut - 1) / kCfTileOut;
  if (tiles > 0x7fffffff) return hipErrorInvalidValue;
  a.tiles = (int32_t)tiles;
  a.Wu = 30 * a.D + 32 * a.KS;
  static std::mutex mu;
  static int cachedD = -1, cachedKS = -1;
  static CfLayout cached{};
  {
    std::lock_guard<std::mutex> lock(mu);
    if (cachedD != a.D || cachedKS != a.KS) {
      cached = cfLayout(a.D, a.KS, a.Wu);
      cachedD = a.D;
      cachedKS = a.KS;
    }
    a.padShift = cached.padShift;
    a.planeStride = cached.planeStride;
  }
  if (a.planeStride == 0) return hipErrorInvalidValue;
  const size_t lds = 12 * (size_t)a.planeStride + 2 * kCfPartBytes;
  const int grid = (int)(tiles < 256 ? tiles : 256);
  if (a.Wu <= kCfThreads)
    return epi == kEpiAm ? launchCf<1, kEpiAm>(a, lds, grid, stream) : launchCf<1, kEpiComplex>(a, lds, grid, stream);
  return epi == kEpiAm ? launchCf<2, kEpiAm>(a, lds, grid, stream) : launchCf<2, kEpiComplex>(a, lds, grid, stream);
}

}  // namespace gsdr_amd
