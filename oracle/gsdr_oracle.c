/*
 * gsdr_oracle.c - CPU restatement of the reference hot path. TEST INFRASTRUCTURE ONLY
 * (see gsdr_oracle.h for what may link it and which reference lines each function follows).
 *
 * Build: oracle/Makefile (-O2/-O3, -ffp-contract=off so every fmaf below is the only fused
 * operation, exactly as in the kernels' expressions).
 */
#include "gsdr_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* Fir.cpp:178-186: first output needs (T - D + 1) inputs (size_t arithmetic), then
 * floor((N - (T - 1)) / D). The size_t wrap when D > T + 1 (and the over-read when
 * N < T - 1) are guarded: no output until at least T - 1 + 1 inputs are buffered. */
size_t orc_fir_output_count(size_t numInputs, size_t tapCount, size_t decimation) {
  const size_t D = decimation == 0 ? 1 : decimation;
  /* T = 0: T - D + 1 wraps in the reference, so it never produces output. */
  if (tapCount == 0) return 0;
  /* For T-1 <= N the reference's floor((N - (T-1)) / D) is 0 at N = T-1; below that it wraps
   * (over-read). Requiring N >= T gives the same counts wherever the reference is defined. */
  if (numInputs < tapCount) return 0;
  return (numInputs - (tapCount - 1)) / D;
}

/* gsdrFir* semantics (Fir.cpp:229-269 call sites; FirTests.cpp:81-84 / :196-202 pin the
 * correlation orientation): y[k] = sum_{j<T} h[j] * x[k*D + j]. Non-conjugated complex MAC. */
void orc_fir_f64(int tapsComplex, int inputComplex, size_t decimation, const float* taps, size_t tapCount,
                 const float* input, double* out, double* bound, size_t numOutputs) {
  const size_t D = decimation == 0 ? 1 : decimation;
  for (size_t k = 0; k < numOutputs; ++k) {
    double re = 0.0, im = 0.0, b = 0.0;
    for (size_t j = 0; j < tapCount; ++j) {
      const size_t n = k * D + j;
      const double hr = tapsComplex ? taps[2 * j] : taps[j];
      const double hi = tapsComplex ? taps[2 * j + 1] : 0.0;
      const double xr = inputComplex ? input[2 * n] : input[n];
      const double xi = inputComplex ? input[2 * n + 1] : 0.0;
      re += hr * xr - hi * xi;
      im += hr * xi + hi * xr;
      b += sqrt(hr * hr + hi * hi) * sqrt(xr * xr + xi * xi);
    }
    out[2 * k] = re;
    out[2 * k + 1] = im;
    if (bound) bound[k] = b;
  }
}

/* include/gsdr/conversion.h definition (Int8ToFloat.cpp:89-94 calls gsdrInt8ToNormFloat). */
float orc_int8_to_norm(int8_t v) { return fmaxf(-1.0f, (float)v / 127.0f); }

void orc_int8_to_float(const int8_t* in, float* out, size_t n) {
  for (size_t i = 0; i < n; ++i) out[i] = orc_int8_to_norm(in[i]);
}

/* include/gsdr/gsdr.h definition (QuadAmDemod.cpp:93-98 calls gsdrQuadAmDemod). */
static inline float am_envelope(float re, float im) { return sqrtf(fmaf(re, re, im * im)); }

void orc_quad_am_demod(const float* inComplex, float* out, size_t n) {
  for (size_t i = 0; i < n; ++i) out[i] = am_envelope(inComplex[2 * i], inComplex[2 * i + 1]);
}

/* include/gsdr/gsdr.h gsdrMultiplyCC (Multiply.cpp:145): non-conjugate complex product. */
void orc_multiply_cc(const float* a, const float* b, float* out, size_t n) {
  for (size_t i = 0; i < n; ++i) {
    const float ar = a[2 * i], ai = a[2 * i + 1], br = b[2 * i], bi = b[2 * i + 1];
    out[2 * i] = fmaf(ar, br, -(ai * bi));
    out[2 * i + 1] = fmaf(ar, bi, ai * br);
  }
}

/* include/gsdr/gsdr.h gsdrQuadFmDemod (QuadFmDemod.cpp:80-115): the float32 discriminator product
 * exactly as the kernel forms it, then gain * atan2 in float64 (the kernel's atan2f is checked
 * against this within its ulp bound). */
void orc_quad_fm_demod_f64(const float* in, double gain, double* out, size_t nOut) {
  for (size_t i = 0; i < nOut; ++i) {
    const float r0 = in[2 * i], i0 = in[2 * i + 1], r1 = in[2 * i + 2], i1 = in[2 * i + 3];
    const float re = fmaf(r1, r0, i1 * i0);
    const float im = fmaf(i1, r0, -(r1 * i0));
    out[i] = gain * atan2((double)im, (double)re);
  }
}

/* CosineSource.cpp:70-83: the source passes (phi, phi + n * delta) and the kernel spreads
 * the phase linearly over n samples. */
void orc_cosine_f(float phiBegin, float phiEnd, float* out, size_t n) {
  if (n == 0) return;
  const float step = (phiEnd - phiBegin) / (float)n;
  for (size_t i = 0; i < n; ++i) out[i] = cosf(fmaf((float)i, step, phiBegin));
}

void orc_cosine_c(float phiBegin, float phiEnd, float* outComplex, size_t n) {
  if (n == 0) return;
  const float step = (phiEnd - phiBegin) / (float)n;
  for (size_t i = 0; i < n; ++i) {
    const float phi = fmaf((float)i, step, phiBegin);
    outComplex[2 * i] = cosf(phi);
    outComplex[2 * i + 1] = sinf(phi);
  }
}

/* ---- synthetic sources (same definitions as include/gsdr/gsdr_amd.h) -------------------- */
static inline uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

static inline double uniform_pm1(uint64_t seed, uint64_t key) {
  return (double)(splitmix64(seed ^ key) >> 11) * (1.0 / 9007199254740992.0) * 2.0 - 1.0;
}

static inline float cycle_phase(double cyclesPerSample, uint64_t n) {
  const double c = cyclesPerSample * (double)n;
  return (float)(6.283185307179586 * (c - floor(c)));
}

static inline int8_t quantize_iq(double v) {
  double r = v < 0.0 ? -floor(-v + 0.5) : floor(v + 0.5);
  r = r > 127.0 ? 127.0 : (r < -127.0 ? -127.0 : r);
  return (int8_t)(int)r;
}

void orc_synth_iq_int8(uint64_t seed, double sampleRate, double amToneHz, double carrierHz, uint64_t firstSample,
                       int8_t* outIq, size_t n) {
  const double fAm = amToneHz / sampleRate, fC = carrierHz / sampleRate;
  for (size_t i = 0; i < n; ++i) {
    const uint64_t s = firstSample + i;
    const float am = 100.0f * (1.0f + 0.5f * cosf(cycle_phase(fAm, s)));
    const float ph = cycle_phase(fC, s);
    const double re = (double)(am * cosf(ph)) + 3.0 * uniform_pm1(seed, 2 * s);
    const double im = (double)(am * sinf(ph)) + 3.0 * uniform_pm1(seed, 2 * s + 1);
    outIq[2 * i] = quantize_iq(re);
    outIq[2 * i + 1] = quantize_iq(im);
  }
}

void orc_synth_wideband_cf32(uint64_t seed, double f1, double f2, uint64_t firstSample, float* outComplex, size_t n) {
  for (size_t i = 0; i < n; ++i) {
    const uint64_t s = firstSample + i;
    const float p1 = cycle_phase(f1, s), p2 = cycle_phase(f2, s);
    const float ur = (float)uniform_pm1(seed, 2 * s), ui = (float)uniform_pm1(seed, 2 * s + 1);
    outComplex[2 * i] = cosf(p1) + 0.5f * cosf(p2) + 0.01f * ur;
    outComplex[2 * i + 1] = sinf(p1) + 0.5f * sinf(p2) + 0.01f * ui;
  }
}

/* ---- CPU baseline: float32 direct form, one time shard per thread ------------------------ */
enum { kTile = 1024, kReg = 32 };

typedef struct {
  size_t D, T, k0, k1;
  const float* taps;
  const int8_t* iq;      /* one of iq / cf32 */
  const float* cf32;
  float* out;
} ShardJob;

static void* run_shard(void* arg) {
  const ShardJob* j = (const ShardJob*)arg;
  const size_t D = j->D, T = j->T;
  const size_t perPhase = kTile + (T + D - 1) / D + kReg;
  float* re = (float*)calloc(D * perPhase, sizeof(float));
  float* im = (float*)calloc(D * perPhase, sizeof(float));
  float* accr = (float*)malloc(kTile * sizeof(float));
  float* acci = (float*)malloc(kTile * sizeof(float));
  for (size_t kb = j->k0; kb < j->k1; kb += kTile) {
    const size_t nt = (j->k1 - kb) < kTile ? (j->k1 - kb) : kTile;
    const size_t n0 = kb * D;
    const size_t len = (nt - 1) * D + T;
    /* polyphase de-interleave (and int8 -> float) of the tile's input window */
    for (size_t i = 0; i < len; ++i) {
      const size_t p = i % D, m = i / D;
      float xr, xi;
      if (j->iq) {
        xr = orc_int8_to_norm(j->iq[2 * (n0 + i)]);
        xi = orc_int8_to_norm(j->iq[2 * (n0 + i) + 1]);
      } else {
        xr = j->cf32[2 * (n0 + i)];
        xi = j->cf32[2 * (n0 + i) + 1];
      }
      re[p * perPhase + m] = xr;
      im[p * perPhase + m] = xi;
    }
    for (size_t i0 = 0; i0 < nt; i0 += kReg) {
      float ar[kReg], ai[kReg];
      for (int i = 0; i < kReg; ++i) ar[i] = ai[i] = 0.0f;
      for (size_t p = 0; p < D && p < T; ++p) {
        const float* xr = re + p * perPhase + i0;
        const float* xi = im + p * perPhase + i0;
        for (size_t q = 0; q * D + p < T; ++q) {
          const float h = j->taps[q * D + p];
          for (int i = 0; i < kReg; ++i) {
            ar[i] = fmaf(h, xr[q + i], ar[i]);
            ai[i] = fmaf(h, xi[q + i], ai[i]);
          }
        }
      }
      for (int i = 0; i < kReg && i0 + i < nt; ++i) j->out[kb + i0 + i] = am_envelope(ar[i], ai[i]);
    }
  }
  free(re);
  free(im);
  free(accr);
  free(acci);
  return NULL;
}

static void run_chain(size_t decimation, const float* taps, size_t tapCount, const int8_t* iq, const float* cf32,
                      float* out, size_t numOutputs, int threads) {
  if (numOutputs == 0 || tapCount == 0) return;
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  pthread_t tids[256];
  ShardJob jobs[256];
  const size_t D = decimation == 0 ? 1 : decimation;
  for (int t = 0; t < threads; ++t) {
    jobs[t].D = D;
    jobs[t].T = tapCount;
    jobs[t].k0 = numOutputs * (size_t)t / (size_t)threads;
    jobs[t].k1 = numOutputs * (size_t)(t + 1) / (size_t)threads;
    jobs[t].taps = taps;
    jobs[t].iq = iq;
    jobs[t].cf32 = cf32;
    jobs[t].out = out;
  }
  for (int t = 1; t < threads; ++t) pthread_create(&tids[t], NULL, run_shard, &jobs[t]);
  run_shard(&jobs[0]);
  for (int t = 1; t < threads; ++t) pthread_join(tids[t], NULL);
}

void orc_chain_i8_fc_am_f32(size_t decimation, const float* taps, size_t tapCount, const int8_t* inIq, float* out,
                            size_t numOutputs, int threads) {
  run_chain(decimation, taps, tapCount, inIq, NULL, out, numOutputs, threads);
}

void orc_chain_fc_am_f32(size_t decimation, const float* taps, size_t tapCount, const float* inComplex, float* out,
                         size_t numOutputs, int threads) {
  run_chain(decimation, taps, tapCount, NULL, inComplex, out, numOutputs, threads);
}

/* ---- C1 CPU baseline: real float32 FIR (CosineSource -> 63-tap FF) ----- */
typedef struct {
  size_t D, T, k0, k1;
  const float* taps;
  const float* x;
  float* out;
} FfJob;

static void* run_ff_shard(void* arg) {
  const FfJob* j = (const FfJob*)arg;
  for (size_t kb = j->k0; kb < j->k1; kb += kReg) {
    float acc[kReg];
    const size_t nt = (j->k1 - kb) < kReg ? (j->k1 - kb) : kReg;
    for (int i = 0; i < kReg; ++i) acc[i] = 0.0f;
    if (nt == kReg) {
      for (size_t q = 0; q < j->T; ++q) {
        const float h = j->taps[q];
        const float* xs = j->x + kb * j->D + q;
        for (int i = 0; i < kReg; ++i) acc[i] = fmaf(h, xs[(size_t)i * j->D], acc[i]);
      }
    } else {
      for (size_t i = 0; i < nt; ++i)
        for (size_t q = 0; q < j->T; ++q) acc[i] = fmaf(j->taps[q], j->x[(kb + i) * j->D + q], acc[i]);
    }
    for (size_t i = 0; i < nt; ++i) j->out[kb + i] = acc[i];
  }
  return NULL;
}

void orc_fir_ff_f32(size_t decimation, const float* taps, size_t tapCount, const float* x, float* out,
                    size_t numOutputs, int threads) {
  if (numOutputs == 0 || tapCount == 0) return;
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  pthread_t tids[256];
  FfJob jobs[256];
  for (int t = 0; t < threads; ++t) {
    jobs[t].D = decimation == 0 ? 1 : decimation;
    jobs[t].T = tapCount;
    jobs[t].k0 = numOutputs * (size_t)t / (size_t)threads;
    jobs[t].k1 = numOutputs * (size_t)(t + 1) / (size_t)threads;
    jobs[t].taps = taps;
    jobs[t].x = x;
    jobs[t].out = out;
  }
  for (int t = 1; t < threads; ++t) pthread_create(&tids[t], NULL, run_ff_shard, &jobs[t]);
  run_ff_shard(&jobs[0]);
  for (int t = 1; t < threads; ++t) pthread_join(tids[t], NULL);
}
