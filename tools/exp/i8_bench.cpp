// Microbenchmark of build variants of the int8 IQ MFMA FIR (tools/exp/run_i8_variants.sh):
// times each variant's launch over the C2 workload (20 M outputs, 127 taps, AM epilogue) with
// HIP events. Variant results are NOT checked here (attribution builds skip work on purpose);
// parity is tests/test_gpu_parity.py's job on the product build.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include <cstring>

#define DECL(N)                                                                                            \
  namespace v##N {                                                                                         \
  hipError_t launchFirI8Mfma(const int8_t*, const float*, size_t, void*, size_t, int, hipStream_t, int8_t*); \
  }
VARIANT_DECLS

typedef hipError_t (*LaunchFn)(const int8_t*, const float*, size_t, void*, size_t, int, hipStream_t, int8_t*);

int main() {
  const size_t nOut = 20000000, T = 127, nIn = nOut + T - 1;
  int8_t* iq;
  float *taps, *out;
  hipMalloc(&iq, 2 * nIn + 256);
  hipMalloc(&taps, T * sizeof(float));
  hipMalloc(&out, nOut * sizeof(float));
  std::vector<int8_t> h(2 * nIn + 256);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (int8_t)((i * 2654435761u) >> 13);
  hipMemcpy(iq, h.data(), h.size(), hipMemcpyHostToDevice);
  std::vector<float> ht(T);
  for (size_t j = 0; j < T; ++j) ht[j] = 0.01f * (float)((j * 7) % 13) - 0.05f;
  hipMemcpy(taps, ht.data(), T * sizeof(float), hipMemcpyHostToDevice);
  struct V { const char* name; LaunchFn fn; } vars[] = {VARIANT_TABLE};
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int8_t* src = iq + 252;  // the bench's [126-sample history | segment] offset
  for (auto& v : vars) {
    for (int w = 0; w < (getenv("WARM") ? atoi(getenv("WARM")) : 3); ++w) v.fn(src, taps, T, out, nOut, 2, 0, nullptr);
    hipDeviceSynchronize();
    const int reps = getenv("REPS") ? atoi(getenv("REPS")) : 20;
    hipEventRecord(e0, 0);
    for (int r = 0; r < reps; ++r) v.fn(src, taps, T, out, nOut, 2, 0, nullptr);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    const hipError_t err = hipGetLastError();
    printf("%-40s %8.2f us/launch  %s", v.name, 1000.0f * ms / reps, hipGetErrorString(err));
    if (strstr(v.name, "clk")) {  // per block: cycles, loop ticks, start tick, loop-start tick; end ticks
      std::vector<uint32_t> st(5 * 768);
      hipMemcpy(st.data(), out, st.size() * 4, hipMemcpyDeviceToHost);
      std::vector<double> f, setup, loop;
      uint32_t s0 = 0xffffffffu, s1 = 0, e1 = 0;
      for (int b = 0; b < 768; ++b) {
        const uint32_t* r = &st[4 * b];
        if (!r[1]) continue;
        f.push_back(100.0 * r[0] / r[1]);
        setup.push_back(0.01 * (r[3] - r[2]));
        loop.push_back(0.01 * r[1]);
        s0 = std::min(s0, r[2]); s1 = std::max(s1, r[2]);
        e1 = std::max(e1, st[4 * 768 + b]);
      }
      auto med = [](std::vector<double> x) { std::sort(x.begin(), x.end()); return x[x.size() / 2]; };
      auto mx = [](std::vector<double> x) { return *std::max_element(x.begin(), x.end()); };
      if (!f.empty())
        printf("  clk %.0f MHz | setup med %.2f max %.2f us | loop med %.2f max %.2f us | start spread %.2f us | first start->last end %.2f us",
               med(f), med(setup), mx(setup), med(loop), mx(loop), 0.01 * (s1 - s0), 0.01 * (e1 - s0));
    }
    printf("\n");
  }
  return 0;
}
