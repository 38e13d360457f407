// Microbenchmark of build variants of the 4-way int8 kernel (csrc/kernels/fir_i8_ws4.hip) at the fused C5
// shape (tools/exp/run_w4_variants.sh): every variant's launch over the bench's N = 1 C5 step (125 M + 3 600
// int8 IQ samples, 1023 taps D = 10 -> AM -> 255 taps D = 20, AM not stored) timed with HIP events in
// interleaved rounds (median us per launch), and each variant's audio compared with variant 0's (max |diff|
// relative to max |audio|; the product's float64 parity lives in tests/, not here).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "ws_common.h"

#define DECL(N)                                                                        \
  extern "C" hipError_t w4v##N(const void*, int, hipStream_t);                         \
  namespace v##N {                                                                     \
  hipError_t wsPrepareLaunch(hipStream_t, int32_t& spin, uint32_t*& abortOut) {         \
    spin = 1 << 22;                                                                    \
    abortOut = nullptr;                                                                \
    return hipSuccess;                                                                 \
  }                                                                                    \
  }
#define DECLW(N) extern "C" hipError_t w4w##N(unsigned long long*, size_t, int);
#define DECLS(N) extern "C" hipError_t w4s##N(unsigned long long*, size_t, int);
VARIANT_DECLS

typedef hipError_t (*Fn)(const void*, int, hipStream_t);
typedef hipError_t (*WaitsFn)(unsigned long long*, size_t, int);

__global__ void fillIq(int8_t* p, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const uint64_t h = (i + 0x9E3779B97F4A7C15ull) * 0xBF58476D1CE4E5B9ull;
    p[i] = (int8_t)(100.0f * __sinf(0.0471f * (float)(i >> 1)) + (float)((h >> 58) & 7) - 3.5f);
  }
}

int main() {
  const int T = 1023, D = 10, Ta = 255, Da = 20;
  const size_t nIn = 125000000 + 3600;
  const size_t nOut = (nIn - T) / D + 1;
  const size_t aN = (nOut - Ta) / Da + 1;
  int8_t* iq;
  float *taps, *aTaps, *aOut, *hist;
  hipMalloc(&iq, 2 * nIn + 64);
  hipMalloc(&taps, T * sizeof(float));
  hipMalloc(&aTaps, Ta * sizeof(float));
  hipMalloc(&aOut, aN * sizeof(float));
  hipMalloc(&hist, 64);
  hipLaunchKernelGGL(fillIq, dim3(4096), dim3(256), 0, 0, iq, 2 * nIn);
  std::vector<float> h(T), ha(Ta);
  for (int j = 0; j < T; ++j) {  // Blackman-windowed sinc, cutoff 0.04
    const double n = j - (T - 1) / 2.0, w = 0.42 - 0.5 * cos(2 * M_PI * j / (T - 1)) + 0.08 * cos(4 * M_PI * j / (T - 1));
    h[j] = (float)(0.08 * (n == 0 ? 1.0 : sin(M_PI * 0.08 * n) / (M_PI * 0.08 * n)) * w);
  }
  for (int j = 0; j < Ta; ++j) ha[j] = 1.0f / Ta;
  hipMemcpy(taps, h.data(), T * sizeof(float), hipMemcpyHostToDevice);
  hipMemcpy(aTaps, ha.data(), Ta * sizeof(float), hipMemcpyHostToDevice);
  gsdr_amd::I8DecArgs a{};
  a.iq4 = iq;
  a.sub = 0;
  a.taps = taps;
  a.out = nullptr;
  a.nOut = (int64_t)nOut;
  a.nIn = (int64_t)nIn;
  a.T = T;
  a.D = D;
  a.tiles = (int32_t)((nOut + 511) / 512);
  a.aTaps = aTaps;
  a.aOut = aOut;
  a.amHist = hist;
  a.aN = (int64_t)aN;
  a.aT = Ta;
  a.aD = Da;
  a.amH = 0;
  const int ksteps = (31 * D + T + 15) / 16;
  struct V { const char* name; Fn fn; WaitsFn waits; WaitsFn stamps; } vars[] = {VARIANT_TABLE};
  const int nv = sizeof(vars) / sizeof(vars[0]);
  std::vector<std::vector<float>> outs(nv, std::vector<float>(aN));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int reps = getenv("REPS") ? atoi(getenv("REPS")) : 20;
  const int rounds = getenv("ROUNDS") ? atoi(getenv("ROUNDS")) : 5;
  std::vector<std::vector<float>> us(nv);
  // ~1 s of warm-up launches (the clock leaves its idle state), then interleaved rounds
  for (int w = 0; w < 200; ++w) vars[w % nv].fn(&a, ksteps, 0);
  hipDeviceSynchronize();
  for (int r = 0; r < rounds; ++r)
    for (int v = 0; v < nv; ++v) {
      hipEventRecord(e0, 0);
      for (int k = 0; k < reps; ++k) vars[v].fn(&a, ksteps, 0);
      hipEventRecord(e1, 0);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      us[v].push_back(1000.0f * ms / reps);
    }
  for (int v = 0; v < nv; ++v) {
    hipMemset(aOut, 0, aN * sizeof(float));
    const hipError_t e = vars[v].fn(&a, ksteps, 0);
    hipDeviceSynchronize();
    hipMemcpy(outs[v].data(), aOut, aN * sizeof(float), hipMemcpyDeviceToHost);
    std::vector<float> s = us[v];
    std::sort(s.begin(), s.end());
    double diff = 0, mx = 0;
    for (size_t j = 0; j < aN; ++j) {
      diff = std::max(diff, (double)fabsf(outs[v][j] - outs[0][j]));
      mx = std::max(mx, (double)fabsf(outs[0][j]));
    }
    printf("%-28s median %8.2f us/launch (min %8.2f, max %8.2f)  rel diff vs %s %.3g  %s\n", vars[v].name, s[s.size() / 2],
           s.front(), s.back(), vars[0].name, diff / mx, hipGetErrorString(e));
    if (vars[v].stamps) {  // GSDR_W4_STAMPS build: one more launch, phase cycles per wave
      const size_t ns = 256 * 8 * 9 + 2 * 128 * 4;
      std::vector<unsigned long long> w(ns, 0);
      vars[v].stamps(w.data(), ns, 1);
      vars[v].fn(&a, ksteps, 0);
      vars[v].stamps(w.data(), ns, 1);
      const char* cn[8] = {"planesFull wait", "partsFull wait", "MFMA loop", "signals", "partsFree wait",
                           "partials write", "epilogue", "last reduce"};
      const char* pn[5] = {"audio", "window wait", "planesFree wait", "convert+writes+loads", "(of audio: ring-slot wait)"};
      for (int role = 0; role < 2; ++role) {
        double tot[9] = {};
        for (int g = 0; g < 256; ++g)
          for (int wv = 4 * role; wv < 4 * role + 4; ++wv)
            for (int k = 0; k < 9; ++k) tot[k] += (double)w[(g * 8 + wv) * 9 + k];
        printf("   %s: span %.0f cycles/wave;", role ? "producers" : "consumers", tot[8] / 1024.0);
        for (int k = 0; k < (role ? 5 : 8); ++k) printf(" %s %.1f%%", role ? pn[k] : cn[k], 100.0 * tot[k] / tot[8]);
        printf("\n");
      }
      // per-tile trace of block 128: consumer wave 0 e0 loop start, e1 loop end (+ limb combine), e2 tile end;
      // producer wave 4 f0 tile start, f1 audio done, f2 planesFree seen, f3 planesFull signalled
      const unsigned long long* tr = w.data() + 256 * 8 * 9;
      auto C = [&](int i, int e) { return (double)tr[i * 4 + e]; };
      auto P = [&](int i, int e) { return (double)tr[(128 + i) * 4 + e]; };
      double s[10] = {};
      int cnt = 0;
      for (int i = 10; i < 80; ++i) {
        if (!C(i, 0) || !P(i, 3) || !C(i + 1, 0)) break;
        s[0] += C(i, 1) - C(i, 0);      // loop
        s[1] += C(i, 2) - C(i, 1);      // post
        s[2] += C(i + 1, 0) - C(i, 2);  // top of next tile (waits)
        s[3] += C(i, 0) - P(i, 3);      // loop start after planes signalled
        s[4] += P(i, 1) - P(i, 0);      // producer audio
        s[5] += P(i, 2) - P(i, 1);      // producer window + planesFree wait
        s[6] += P(i, 3) - P(i, 2);      // producer convert + writes + signal
        s[7] += P(i, 2) - C(i - 2, 1);  // planesFree seen after consumer loop i-2 end
        s[8] += C(i + 1, 0) - C(i, 0);  // period
        s[9] += C(i + 1, 0) - C(i + 1, 3);  // from the readiness check to the loop start
        ++cnt;
      }
      if (cnt) {
        const char* nm[9] = {"C loop", "C post", "C top-wait", "C start - P planesFull", "P audio", "P window+planesFree wait",
                             "P convert", "P planesFree seen - C loop(i-2) end", "period"};
        printf("   trace (block 128, tiles 10-%d, mean cycles):", 10 + cnt - 1);
        for (int k = 0; k < 9; ++k) printf(" %s %.0f;", nm[k], s[k] / cnt);
        printf(" ready->loop %.0f\n", s[9] / cnt);
        int nr = 0, npf = 0, npp = 0;
        for (int i = 10; i < 10 + cnt; ++i) {
          const unsigned long long f = tr[i * 4 + 3] & 7ull;
          nr += (f & 1) ? 0 : 1; npf += (f & 2) ? 0 : 1; npp += (f & 4) ? 0 : 1;
        }
        printf("   not ready at the top: %d of %d tiles (planesFull not reached %d, partsFull %d)\n", nr, cnt, npf, npp);
        printf("   tiles 20-27 (cycles from C(20) loop start): \n");
        const double t0 = C(20, 0);
        for (int i = 20; i < 28; ++i)
          printf("     %d: C %7.0f %7.0f %7.0f | P %7.0f %7.0f %7.0f %7.0f\n", i, C(i, 0) - t0, C(i, 1) - t0, C(i, 2) - t0,
                 P(i, 0) - t0, P(i, 1) - t0, P(i, 2) - t0, P(i, 3) - t0);
      }
    }
    if (vars[v].waits) {  // GSDR_WS_WAITS build: one more launch with the counters reset
      const size_t nw = 256 * 12 * 13;
      std::vector<unsigned long long> w(nw, 0);
      vars[v].waits(w.data(), nw, 1);
      std::fill(w.begin(), w.end(), 0ull);
      vars[v].fn(&a, ksteps, 0);
      vars[v].waits(w.data(), nw, 1);
      const char* kinds[13] = {"planesFull", "planesFree", "partsFull", "partsFree", "pstat", "tapsRead", "amSlot",
                               "amFree", "span", "count", "MFMA loop", "partials write", "epilogue"};
      for (int role = 0; role < 2; ++role) {
        double tot[13] = {};
        for (int g = 0; g < 256; ++g)
          for (int wv = 4 * role; wv < 4 * role + 4; ++wv)
            for (int k = 0; k < 13; ++k) tot[k] += (double)w[(g * 12 + wv) * 13 + k];
        printf("   %s: span %.0f cycles/wave;", role ? "producers" : "consumers", tot[8] / 1024.0);
        for (int k = 0; k < 13; ++k)
          if (k != 8 && tot[k] > 0)
            printf(" %s %.1f%%", role && k >= 9 ? (k == 9 ? "convert+writes" : k == 10 ? "audio" : k == 11 ? "window wait" : "planesFree wait")
                                                : kinds[k], 100.0 * tot[k] / tot[8]);
        printf("\n");
      }
    }
  }
  return 0;
}
