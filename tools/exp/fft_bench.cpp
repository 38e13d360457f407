// Microbenchmark of attribution builds of the FFT FIR (tools/exp/run_fft_variants.sh): C3 shape
// (2^28 - 6 cf32 samples, 1023 taps, D = 10, AM epilogue) and the C5 RF shape (125 M int8 IQ
// samples, 1023 taps, D = 10), HIP-event timed, every variant's output compared with the first.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define DECL(N)                                                                                        \
  namespace f##N {                                                                                     \
  struct FftMix {                                                                                      \
    bool on = false;                                                                                   \
    uint64_t phase0 = 0, step = 0;                                                                     \
  };                                                                                                   \
  hipError_t launchFirFft(const void*, bool, const float*, size_t, size_t, void*, size_t, int, hipStream_t, FftMix, bool); \
  inline hipError_t launchPlain(const void* i, bool b, const float* t, size_t T, size_t D, void* o, size_t n, int e, \
                                hipStream_t s) { return launchFirFft(i, b, t, T, D, o, n, e, s, FftMix{}, false); } \
  uint32_t kernelPolicy() { return 0; }                                                              \
  bool firI8MfmaEligible(size_t, size_t, const void*) { return false; }                              \
  bool firI8DecMfmaEligible(size_t, size_t, const void*) { return false; }                           \
  hipError_t fftStampsRead(unsigned long long*, size_t) __attribute__((weak));                         \
  }
VARIANT_DECLS

typedef hipError_t (*LaunchFn)(const void*, bool, const float*, size_t, size_t, void*, size_t, int, hipStream_t);
typedef hipError_t (*StampFn)(unsigned long long*, size_t);

// two tones like bench.py's synthetic C3 input (gsdrSynthWidebandCf32: exp(j 2 pi f1 n) +
// 0.5 exp(j 2 pi f2 n) + noise), selected with FFT_BENCH_DATA=twotone
__global__ void fillTwoTone(float* x, size_t n, uint64_t seed, float noise) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const double s = (double)(i / 2);
    const double p1 = 2.0 * M_PI * fmod(0.013 * s, 1.0), p2 = 2.0 * M_PI * fmod(0.31 * s, 1.0);
    uint64_t z = (i + seed) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z ^= z >> 31;
    const double t = (i & 1) ? sin(p1) + 0.5 * sin(p2) : cos(p1) + 0.5 * cos(p2);
    x[i] = (float)t + noise * ((float)(int32_t)(z >> 32) * (1.0f / 2147483648.0f));
  }
}

__global__ void fillKernel(float* x, size_t n, uint64_t seed, float noise) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const double ph = 2.0 * M_PI * fmod(0.013 * (double)(i / 2), 1.0);
    uint64_t z = (i + seed) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z ^= z >> 31;
    x[i] = (float)((i & 1) ? sin(ph) : cos(ph)) + noise * ((float)(int32_t)(z >> 32) * (1.0f / 2147483648.0f));
  }
}

// reference read bandwidth: grid-stride float4 loads (optionally non-temporal), one sum per thread
typedef float f4v __attribute__((ext_vector_type(4)));
template <int NT>
__global__ void streamRead(const f4v* x, size_t n4, float* sink) {
  float acc = 0.0f;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
    f4v v;
    if (NT) v = __builtin_nontemporal_load(x + i);
    else v = x[i];
    acc += v.x + v.y + v.z + v.w;
  }
  if (acc == 12345.678f) sink[0] = acc;
}

// per-wave chunked loads like the FFT kernel: each wave reads 40 KB blocks (40 x 1 KB coalesced
// dwordx4 instructions) then consumes them; W waves per workgroup, one workgroup per CU
template <int W, int AUX>
__global__ void chunkRead(const char* x, size_t nBlocks, float* sink) {
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), l = threadIdx.x & 63;
  float acc = 0.0f;
  for (size_t b = blockIdx.x * (size_t)W + w; b < nBlocks; b += (size_t)gridDim.x * W) {
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)(x + b * 40960), (short)0, 40960, 0x00020000);
    float4 v[40];
#pragma unroll
    for (int i = 0; i < 40; ++i) v[i] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, (i * 64 + l) * 16, 0, AUX));
#pragma unroll
    for (int i = 0; i < 40; ++i) acc += v[i].x + v[i].w;
  }
  if (acc == 12345.678f) sink[0] = acc;
}

// chunk reads with the FFT kernel's geometry: block stride STRIDE bytes (32800 = 410 rows x 80 B),
// 40 KB per block; ROT: wave-dependent rotation of the 40 instructions' issue order
template <int W, int STRIDE, int ROT>
__global__ void chunkReadV(const char* x, size_t nBlocks, float* sink) {
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), l = threadIdx.x & 63;
  float acc = 0.0f;
  for (size_t b = blockIdx.x * (size_t)W + w; b < nBlocks; b += (size_t)gridDim.x * W) {
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)(x + b * STRIDE), (short)0, 40960, 0x00020000);
    float4 v[40];
    const int rot = ROT ? (int)(b % 8) * 5 : 0;
#pragma unroll
    for (int i = 0; i < 40; ++i) {
      int ii = i + rot;
      ii = ii >= 40 ? ii - 40 : ii;
      v[i] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, (ii * 64 + l) * 16, 0, 0));
    }
#pragma unroll
    for (int i = 0; i < 40; ++i) acc += v[i].x + v[i].w;
  }
  if (acc == 12345.678f) sink[0] = acc;
}

// the same 8 blocks per workgroup, but read as one interleaved sweep: instruction i of wave w
// loads 1 KB piece 8 i + w of the workgroup's contiguous 8-block region
__global__ void chunkReadSweep(const char* x, size_t nGroups, float* sink) {
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), l = threadIdx.x & 63;
  float acc = 0.0f;
  for (size_t g = blockIdx.x; g < nGroups; g += gridDim.x) {
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)(x + g * 8 * 40960), (short)0, 8 * 40960, 0x00020000);
    float4 v[40];
#pragma unroll
    for (int i = 0; i < 40; ++i)
      v[i] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, ((i * 8 + w) * 64 + l) * 16, 0, 0));
#pragma unroll
    for (int i = 0; i < 40; ++i) acc += v[i].x + v[i].w;
  }
  if (acc == 12345.678f) sink[0] = acc;
}

// per-wave chunks with the 40 loads issued at raised wave priority (PRIO = 1: s_setprio 3 around
// the issue, so a wave tends to issue its whole block before its SIMD partner interleaves)
template <int W, int PRIO>
__global__ void chunkReadPrio(const char* x, size_t nBlocks, float* sink) {
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), l = threadIdx.x & 63;
  float acc = 0.0f;
  for (size_t b = blockIdx.x * (size_t)W + w; b < nBlocks; b += (size_t)gridDim.x * W) {
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)(x + b * 40960), (short)0, 40960, 0x00020000);
    float4 v[40];
    if (PRIO) __builtin_amdgcn_s_setprio(3);
#pragma unroll
    for (int i = 0; i < 40; ++i) v[i] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, (i * 64 + l) * 16, 0, 0));
    if (PRIO) __builtin_amdgcn_s_setprio(0);
#pragma unroll
    for (int i = 0; i < 40; ++i) acc += v[i].x + v[i].w;
  }
  if (acc == 12345.678f) sink[0] = acc;
}

// sweeps shared by groups of G waves: the G waves of a group read their G-block region
// interleaved (instruction i of member m loads piece G i + m), 8 / G groups per workgroup
template <int G>
__global__ void chunkReadSweepG(const char* x, size_t nRegions, float* sink) {
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), l = threadIdx.x & 63, grp = w / G, m = w % G;
  float acc = 0.0f;
  for (size_t r = blockIdx.x * (size_t)(8 / G) + grp; r < nRegions; r += (size_t)gridDim.x * (8 / G)) {
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)(x + r * G * 40960), (short)0, G * 40960, 0x00020000);
    float4 v[40];
#pragma unroll
    for (int i = 0; i < 40; ++i)
      v[i] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, ((i * G + m) * 64 + l) * 16, 0, 0));
#pragma unroll
    for (int i = 0; i < 40; ++i) acc += v[i].x + v[i].w;
  }
  if (acc == 12345.678f) sink[0] = acc;
}

void readBw(void* x, size_t bytes) {
  float* sink;
  hipMalloc(&sink, 64);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto timeit = [&](const char* name, auto launch) {
    for (int w = 0; w < 2; ++w) launch();
    hipEventRecord(e0);
    for (int r = 0; r < 10; ++r) launch();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    printf("read   %-28s %9.1f us  %7.3f TB/s\n", name, ms * 100.0, bytes / (ms * 1e-4) / 1e12);
    fflush(stdout);
  };
  const size_t n4 = bytes / 16;
  for (int bpc : {2, 4, 8}) {
    char nm[64];
    snprintf(nm, sizeof nm, "grid-stride f4 x%d/CU", bpc);
    timeit(nm, [&] { streamRead<0><<<256 * bpc, 256>>>((const f4v*)x, n4, sink); });
    snprintf(nm, sizeof nm, "grid-stride f4 nt x%d/CU", bpc);
    timeit(nm, [&] { streamRead<1><<<256 * bpc, 256>>>((const f4v*)x, n4, sink); });
  }
  const size_t nb = bytes / 40960;
  timeit("chunk 8 waves", [&] { chunkRead<8, 0><<<256, 512>>>((const char*)x, nb, sink); });
  timeit("chunk 8 waves nt", [&] { chunkRead<8, 2><<<256, 512>>>((const char*)x, nb, sink); });
  timeit("chunk 4 waves", [&] { chunkRead<4, 0><<<256, 256>>>((const char*)x, nb, sink); });
  timeit("chunk 16 waves", [&] { chunkRead<16, 0><<<256, 1024>>>((const char*)x, nb, sink); });
  timeit("sweep 8 waves (8 blocks/WG)", [&] { chunkReadSweep<<<256, 512>>>((const char*)x, bytes / (8 * 40960), sink); });
  timeit("chunk 8 waves setprio", [&] { chunkReadPrio<8, 1><<<256, 512>>>((const char*)x, nb, sink); });
  timeit("chunk 8 waves 2 WG/CU", [&] { chunkRead<8, 0><<<512, 512>>>((const char*)x, nb, sink); });
  timeit("sweep groups of 2 waves", [&] { chunkReadSweepG<2><<<256, 512>>>((const char*)x, bytes / (2 * 40960), sink); });
  timeit("sweep groups of 4 waves", [&] { chunkReadSweepG<4><<<256, 512>>>((const char*)x, bytes / (4 * 40960), sink); });
  timeit("sweep groups of 8 waves", [&] { chunkReadSweepG<8><<<256, 512>>>((const char*)x, bytes / (8 * 40960), sink); });
  timeit("sweep 8 waves x2 WG/CU", [&] { chunkReadSweepG<8><<<512, 512>>>((const char*)x, bytes / (8 * 40960), sink); });
  const size_t nb2 = (bytes - 40960) / 32800;
  timeit("chunkV 8w stride32800", [&] { chunkReadV<8, 32800, 0><<<256, 512>>>((const char*)x, nb2, sink); });
  timeit("chunkV 8w stride32800 rot", [&] { chunkReadV<8, 32800, 1><<<256, 512>>>((const char*)x, nb2, sink); });
  timeit("chunkV 8w stride40960 rot", [&] { chunkReadV<8, 40960, 1><<<256, 512>>>((const char*)x, nb, sink); });
  timeit("chunkV 8w stride41216", [&] { chunkReadV<8, 41216, 0><<<256, 512>>>((const char*)x, (bytes - 40960) / 41216, sink); });
  hipFree(sink);
}

int main() {
  struct Shape { const char* name; size_t n, T, D; bool i8; } shapes[] = {{"c3", (1u << 28) - 6, 1023, 10, false},
                                                                          {"c5rf", 125000000, 1023, 10, true},
                                                                          {"c4", (1u << 27), 1023, 1, false}};
  struct V { const char* name; LaunchFn fn; StampFn stamps; } vars[] = {VARIANT_TABLE};
  const int nv = sizeof(vars) / sizeof(vars[0]);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (auto& sh : shapes) {
    const size_t nOut = (sh.n - sh.T) / sh.D + 1, nIn = (nOut - 1) * sh.D + sh.T;
    void *x, *out, *ref;
    float* taps;
    const size_t inBytes = nIn * (sh.i8 ? 2 : 8);
    hipMalloc(&x, inBytes + 64);
    hipMalloc(&taps, sh.T * 4);
    hipMalloc(&out, nOut * 4);
    hipMalloc(&ref, nOut * 4);
    if (sh.i8) {
      std::vector<int8_t> h(inBytes);
      for (size_t i = 0; i < inBytes; ++i) h[i] = (int8_t)(100.0 * cos(0.37 * (double)i) + (double)((i * 7919) % 7) - 3);
      hipMemcpy(x, h.data(), inBytes, hipMemcpyHostToDevice);
    } else {
      // FFT_BENCH_NOISE: amplitude of the uniform noise on the tone (default 0.01; ~1 is wideband)
      const float noise = getenv("FFT_BENCH_NOISE") ? (float)atof(getenv("FFT_BENCH_NOISE")) : 0.01f;
      if (getenv("FFT_BENCH_DATA") && strcmp(getenv("FFT_BENCH_DATA"), "twotone") == 0)
        fillTwoTone<<<1024, 256>>>((float*)x, 2 * nIn, 12345, noise);
      else
        fillKernel<<<1024, 256>>>((float*)x, 2 * nIn, 12345, noise);
    }
    std::vector<float> ht(sh.T);
    for (size_t j = 0; j < sh.T; ++j) {
      const double n = (double)j - (sh.T - 1) / 2.0;
      ht[j] = (float)(0.08 * (n == 0 ? 1.0 : sin(M_PI * 0.08 * n) / (M_PI * 0.08 * n)) *
                      (0.42 - 0.5 * cos(2 * M_PI * j / (sh.T - 1)) + 0.08 * cos(4 * M_PI * j / (sh.T - 1))));
    }
    hipMemcpy(taps, ht.data(), sh.T * 4, hipMemcpyHostToDevice);
    if (!sh.i8 && getenv("FFT_BENCH_READBW")) readBw(x, inBytes);
    // FFT_BENCH_STAMPS=1 (variants built with STAMPS=1): per variant, FFT_BENCH_STAMP_S seconds of
    // back-to-back launches (default 2.5), then the in-kernel clock of the last launch from its wave
    // stamps: (shader-clock delta) / (100 MHz real-time delta) per wave, median over waves
    // (MI355X_MICROARCH.md DVFS give-back item 6). Two interleaved rounds.
    if (getenv("FFT_BENCH_STAMPS")) {
      if (sh.i8 || sh.D == 1) { hipFree(x); hipFree(taps); hipFree(out); hipFree(ref); continue; }
      const double secs = getenv("FFT_BENCH_STAMP_S") ? atof(getenv("FFT_BENCH_STAMP_S")) : 2.5;
      std::vector<unsigned long long> st(256 * 8 * 4);
      for (int rd = 0; rd < 2; ++rd)
        for (int v = 0; v < nv; ++v) {
          if (!vars[v].stamps) { printf("%s: no stamps in this build (STAMPS=1)\n", vars[v].name); continue; }
          double el = 0.0, lastUs = 0.0;
          int launches = 0;
          while (el < secs * 1e3) {
            hipEventRecord(e0);
            for (int r = 0; r < 200; ++r) vars[v].fn(x, sh.i8, taps, sh.T, sh.D, out, nOut, 2, 0);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            el += ms;
            launches += 200;
            lastUs = ms * 1e3 / 200;
          }
          hipDeviceSynchronize();
          std::fill(st.begin(), st.end(), 0ull);
          vars[v].stamps(st.data(), st.size());
          if (const char* dump = getenv("FFT_BENCH_STAMP_DUMP")) {  // raw stamps: <dump>_<variant>_<round>.bin
            char path[512];
            snprintf(path, sizeof path, "%s_%s_%d.bin", dump, vars[v].name, rd);
            if (FILE* f = fopen(path, "wb")) {
              fwrite(st.data(), sizeof(unsigned long long), st.size(), f);
              fclose(f);
            }
          }
          std::vector<double> clk, dur, start;
          unsigned long long rtMin = ~0ull;
          for (int wv = 0; wv < 256 * 8; ++wv)
            if (st[4 * wv + 3] > st[4 * wv + 1]) rtMin = std::min(rtMin, st[4 * wv + 1]);
          for (int wv = 0; wv < 256 * 8; ++wv) {
            const unsigned long long* q = &st[4 * wv];
            if (q[3] <= q[1] || q[2] <= q[0]) continue;
            clk.push_back((double)(q[2] - q[0]) / (double)(q[3] - q[1]) * 100.0);  // MHz
            dur.push_back((double)(q[3] - q[1]) * 0.01);                           // us
            start.push_back((double)(q[1] - rtMin) * 0.01);
          }
          if (clk.empty()) { printf("%s: no stamps read\n", vars[v].name); continue; }
          std::sort(clk.begin(), clk.end());
          std::sort(dur.begin(), dur.end());
          std::sort(start.begin(), start.end());
          printf("stamps %-10s round %d: %d launches in %.2f s, last 200 at %.1f us/launch | clock MHz median %.0f "
                 "[p10 %.0f, p90 %.0f] over %zu waves | wave span us median %.1f [min %.1f, max %.1f] | start skew "
                 "max %.1f us\n",
                 vars[v].name, rd, launches, el * 1e-3, lastUs, clk[clk.size() / 2], clk[clk.size() / 10],
                 clk[clk.size() * 9 / 10], clk.size(), dur[dur.size() / 2], dur[0], dur.back(), start.back());
          fflush(stdout);
        }
      hipFree(x); hipFree(taps); hipFree(out); hipFree(ref);
      continue;
    }
    // FFT_BENCH_LOOP=<variant name>: loop that variant for FFT_BENCH_REPS launches (power / clock
    // probes sample amd-smi meanwhile), printing the mean launch time every 2000 launches
    if (const char* lv = getenv("FFT_BENCH_LOOP")) {
      if (sh.i8 || sh.D == 1) { hipFree(x); hipFree(taps); hipFree(out); hipFree(ref); continue; }
      const int reps = getenv("FFT_BENCH_REPS") ? atoi(getenv("FFT_BENCH_REPS")) : 20000;
      for (int v = 0; v < nv; ++v) {
        if (strcmp(vars[v].name, lv) != 0) continue;
        for (int r0 = 0; r0 < reps; r0 += 2000) {
          hipEventRecord(e0);
          for (int r = 0; r < 2000; ++r) vars[v].fn(x, sh.i8, taps, sh.T, sh.D, out, nOut, 2, 0);
          hipEventRecord(e1);
          hipEventSynchronize(e1);
          float ms = 0;
          hipEventElapsedTime(&ms, e0, e1);
          printf("loop %-10s %6d launches  %8.1f us/launch\n", lv, r0 + 2000, ms * 1e3 / 2000);
          fflush(stdout);
        }
      }
      hipFree(x); hipFree(taps); hipFree(out); hipFree(ref);
      continue;
    }
    std::vector<float> a(nOut), b(nOut);
    // correctness: every variant's output against the first
    std::vector<double> md(nv, 0.0);
    for (int v = 0; v < nv; ++v) {
      void* o = v == 0 ? ref : out;
      vars[v].fn(x, sh.i8, taps, sh.T, sh.D, o, nOut, 2, 0);
      hipDeviceSynchronize();
      if (v > 0) {
        hipMemcpy(a.data(), ref, nOut * 4, hipMemcpyDeviceToHost);
        hipMemcpy(b.data(), out, nOut * 4, hipMemcpyDeviceToHost);
        for (size_t i = 0; i < nOut; ++i) md[v] = fmax(md[v], fabs((double)a[i] - (double)b[i]));
      }
    }
    // timing: rounds interleave the variants (clock / thermal drift hits all alike); per variant
    // the minimum and median over rounds of the per-launch average of 10 launches
    const int rounds = 7, reps = 10;
    std::vector<std::vector<double>> t(nv);
    for (int rd = 0; rd < rounds; ++rd) {
      for (int v = 0; v < nv; ++v) {
        for (int w = 0; w < 2; ++w) vars[v].fn(x, sh.i8, taps, sh.T, sh.D, out, nOut, 2, 0);
        hipEventRecord(e0);
        for (int r = 0; r < reps; ++r) vars[v].fn(x, sh.i8, taps, sh.T, sh.D, out, nOut, 2, 0);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        t[v].push_back(ms * 1e3 / reps);
      }
    }
    for (int v = 0; v < nv; ++v) {
      std::vector<double> s2 = t[v];
      std::sort(s2.begin(), s2.end());
      const double us = s2[s2.size() / 2];
      printf("%-6s %-16s median %8.1f  min %8.1f us/launch  %7.3f TB/s algorithmic (median)  max|diff| vs first %.3g\n",
             sh.name, vars[v].name, us, s2[0], (double)(inBytes + nOut * 4) / (us * 1e-6) / 1e12, md[v]);
      fflush(stdout);
    }
    hipFree(x);
    hipFree(taps);
    hipFree(out);
    hipFree(ref);
  }
  return 0;
}
