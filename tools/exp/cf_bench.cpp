// Microbenchmark of build variants of the cf32 split-precision MFMA FIR
// (tools/exp/run_cf_variants.sh): C3 shape (2^28 - 6 samples, 1023 taps, D = 10, AM epilogue)
// and C4 shape (2^26 samples, 1023 taps, D = 1), HIP-event timed. Results are not checked here.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <cstring>

#include <cstdint>
#define DECL(N)                                                                                    \
  namespace c##N {                                                                                 \
  hipError_t launchFirCfMfma(const float*, const float*, size_t, size_t, void*, size_t, int, hipStream_t); \
  uint32_t kernelPolicy() { return POLICY_FOR_VARIANTS; }                                          \
  }
#ifndef POLICY_FOR_VARIANTS
#define POLICY_FOR_VARIANTS 0u
#endif
VARIANT_DECLS

typedef hipError_t (*LaunchFn)(const float*, const float*, size_t, size_t, void*, size_t, int, hipStream_t);

int main() {
  struct Shape { const char* name; size_t n, T, D; } shapes[] = {{"c3", (1u << 28) - 6, 1023, 10},
                                                                 {"c4", 1u << 26, 1023, 1}};
  struct V { const char* name; LaunchFn fn; } vars[] = {VARIANT_TABLE};
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (auto& sh : shapes) {
    const size_t nOut = sh.n / sh.D, nIn = (nOut - 1) * sh.D + sh.T;
    float *x, *taps, *out;
    hipMalloc(&x, nIn * 8);
    hipMalloc(&taps, sh.T * 4);
    hipMalloc(&out, nOut * 8);
    hipMemset(x, 0x3c, nIn * 8);  // finite pattern
    std::vector<float> ht(sh.T);
    for (size_t j = 0; j < sh.T; ++j) ht[j] = 0.001f * (float)((j * 7) % 13) - 0.005f;
    hipMemcpy(taps, ht.data(), sh.T * 4, hipMemcpyHostToDevice);
    for (auto& v : vars) {
      for (int w = 0; w < 2; ++w) v.fn(x, taps, sh.T, sh.D, out, nOut, 2, 0);
      hipDeviceSynchronize();
      const int reps = 5;
      hipEventRecord(e0, 0);
      for (int r = 0; r < reps; ++r) v.fn(x, taps, sh.T, sh.D, out, nOut, 2, 0);
      hipEventRecord(e1, 0);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      printf("%s %-32s %9.1f us/launch  %s\n", sh.name, v.name, 1000.0f * ms / reps, hipGetErrorString(hipGetLastError()));
      if (strstr(v.name, "stamp")) {  // block 0: per wave [work, barrier, reduce] cycles, tiles
        uint32_t st[32];
        hipMemcpy(st, out, sizeof(st), hipMemcpyDeviceToHost);
        for (int w = 0; w < 8; ++w)
          printf("   wave %d: vec %u mfma %u barrier %u cycles over %u tiles (%.0f / %.0f / %.0f per tile)\n", w,
                 st[4 * w], st[4 * w + 1], st[4 * w + 2], st[4 * w + 3], (double)st[4 * w] / st[4 * w + 3],
                 (double)st[4 * w + 1] / st[4 * w + 3], (double)st[4 * w + 2] / st[4 * w + 3]);
      }
    }
    hipFree(x);
    hipFree(taps);
    hipFree(out);
  }
  return 0;
}
