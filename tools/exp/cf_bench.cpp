// Microbenchmark of build variants of the cf32 split-precision MFMA FIR
// (tools/exp/run_cf_variants.sh): C3 shape (2^28 - 6 samples, 1023 taps, D = 10, AM epilogue)
// and C4 shape (2^26 samples, 1023 taps, D = 1), HIP-event timed. The input is pseudo-random with
// a quiet stretch (direct-path tiles); every variant's output is compared with the first one's
// (max |diff| and the count of differing words; variants that only re-schedule the same
// arithmetic must be bit-identical).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <cstring>
#include <cmath>
#include <cstdlib>

#include <cstdint>
#define DECL(N)                                                                                    \
  namespace c##N {                                                                                 \
  hipError_t launchFirCfMfma(const float*, const float*, size_t, size_t, void*, size_t, int, hipStream_t); \
  uint32_t kernelPolicy() { return POLICY_FOR_VARIANTS; }                                          \
  hipError_t wsReadStamps(unsigned long long*);                                                    \
  }
#ifndef POLICY_FOR_VARIANTS
#define POLICY_FOR_VARIANTS 0u
#endif
VARIANT_DECLS

typedef hipError_t (*LaunchFn)(const float*, const float*, size_t, size_t, void*, size_t, int, hipStream_t);
typedef hipError_t (*StampFn)(unsigned long long*);

__global__ void fillKernel(float* x, size_t n, uint64_t seed, int quiet) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint64_t z = (i + seed) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    float v = (float)(int32_t)(z >> 32) * (1.0f / 2147483648.0f);
    const size_t s = i / 2;
    if (quiet && s % 4000000 < 3000) v *= 1e-6f;  // quiet stretches: direct-path tiles
    x[i] = v;
  }
}

int main() {
  struct Shape { const char* name; size_t n, T, D; } shapes[] = {{"c3", (1u << 28) - 6, 1023, 10},
                                                                 {"c4", 1u << 26, 1023, 1}};
  struct V { const char* name; LaunchFn fn; StampFn st; } vars[] = {VARIANT_TABLE};
  static unsigned long long stamps[256 * 16][2];
  const int nv = sizeof(vars) / sizeof(vars[0]);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (auto& sh : shapes) {
    const size_t nOut = sh.n / sh.D, nIn = (nOut - 1) * sh.D + sh.T;
    float *x, *taps, *out;
    hipMalloc(&x, nIn * 8);
    hipMalloc(&taps, sh.T * 4);
    hipMalloc(&out, nOut * 8);
    if (getenv("CF_FILL_CONST")) hipMemset(x, 0x3c, nIn * 8);  // the r01 pattern: every sample equal
    else fillKernel<<<1024, 256>>>(x, 2 * nIn, 12345, getenv("CF_NO_QUIET") ? 0 : 1);
    std::vector<float> ht(sh.T);
    for (size_t j = 0; j < sh.T; ++j) ht[j] = 0.001f * (float)((j * 7) % 13) - 0.005f;
    hipMemcpy(taps, ht.data(), sh.T * 4, hipMemcpyHostToDevice);
    std::vector<uint32_t> ref, cur(nOut);
    for (int vi = 0; vi < nv; ++vi) {
      auto& v = vars[vi];
      hipMemset(out, 0xff, nOut * 4);
      for (int w = 0; w < 2; ++w) v.fn(x, taps, sh.T, sh.D, out, nOut, 2, 0);
      hipDeviceSynchronize();
      const int reps = 5;
      hipEventRecord(e0, 0);
      for (int r = 0; r < reps; ++r) v.fn(x, taps, sh.T, sh.D, out, nOut, 2, 0);
      hipEventRecord(e1, 0);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      if (v.st(&stamps[0][0]) == hipSuccess) v.st(&stamps[0][0]);  // clear, then one stamped launch
      v.fn(x, taps, sh.T, sh.D, out, nOut, 2, 0);
      hipDeviceSynchronize();
      if (v.st(&stamps[0][0]) == hipSuccess) {
        // per role: mean over blocks of (wait cycles, total cycles) of waves 0-7 (consumers) and
        // 8-15 (producers)
        double w[2] = {0, 0}, t[2] = {0, 0}, cnt[2] = {0, 0};
        for (int b = 0; b < 256; ++b)
          for (int wv = 0; wv < 16; ++wv) {
            w[wv >= 8] += stamps[b * 16 + wv][0];
            t[wv >= 8] += stamps[b * 16 + wv][1];
            cnt[wv >= 8] += stamps[b * 16 + wv][1] != 0;
          }
        printf("   stamps: consumers wait %.0f of %.0f cycles/wave; producers wait %.0f of %.0f\n", w[0] / cnt[0],
               t[0] / cnt[0], w[1] / cnt[1], t[1] / cnt[1]);
      }
      hipMemcpy(cur.data(), out, nOut * 4, hipMemcpyDeviceToHost);
      size_t ndiff = 0;
      double maxd = 0;
      if (vi == 0) {
        ref = cur;
      } else {
        for (size_t k = 0; k < nOut; ++k) {
          if (cur[k] != ref[k]) {
            ++ndiff;
            float a, b;
            memcpy(&a, &cur[k], 4);
            memcpy(&b, &ref[k], 4);
            const double d = std::isfinite(a) && std::isfinite(b) ? fabs((double)a - b) : INFINITY;
            maxd = d > maxd ? d : maxd;
          }
        }
      }
      printf("%s %-32s %9.1f us/launch  %s  diff vs first: %zu words, max %.3g\n", sh.name, v.name,
             1000.0f * ms / reps, hipGetErrorString(hipGetLastError()), ndiff, maxd);
      fflush(stdout);
    }
    hipFree(x);
    hipFree(taps);
    hipFree(out);
  }
  return 0;
}
