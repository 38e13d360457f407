/*
 * gsdr_oracle.h - CPU restatement of the reference hot path. TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
 * library, and only as the checker / the timed CPU baseline - never as the product path.
 *
 * What it restates (kernrj/cuda-sdr @ /root/reference):
 *   - FIR count / consume rule       src/filters/Fir.cpp:141-197, :270-276
 *   - FIR arithmetic                 gsdrFir{FF,FC,CC,CF} call sites Fir.cpp:229-269; the
 *                                    orientation is pinned by tests/FirTests.cpp:81-84, :196-202
 *   - AM envelope                    QuadAmDemod.cpp:93-98 (gsdr arithmetic absent: this build's
 *                                    definition, see include/gsdr/gsdr.h)
 *   - int8 -> float                  Int8ToFloat.cpp:89-94 (scale absent: include/gsdr/conversion.h)
 *   - phase cosines                  CosineSource.cpp:70-83, ComplexCosineSource.cpp:70-83
 *
 * Pinning: the FIR restatement reproduces the reference's two FIR known-answer tests and
 * the cosine KAT (tests/test_oracle_golden.py); the AM and int8 scale definitions are
 * "parity unpinned" (no reference test, arithmetic in the absent gsdr library).
 */
#ifndef GSDR_ORACLE_H
#define GSDR_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* FIR output count for `numInputs` buffered inputs (Fir.cpp:178-186), with the size_t wrap
 * of `tapCount - decimation + 1` guarded. */
size_t orc_fir_output_count(size_t numInputs, size_t tapCount, size_t decimation);

/* Float64 reference of y[k] = sum_j h[j] x[kD+j].
 * tapsComplex / inputComplex select the FF/FC/CC/CF variant; complex data is interleaved.
 * out: 2 doubles per output (re, im; im = 0 for FF). bound (may be NULL): per output
 * sum_j |h_j| |x_{kD+j}| (complex moduli), the scale of the parity tolerance. */
void orc_fir_f64(int tapsComplex, int inputComplex, size_t decimation, const float* taps, size_t tapCount,
                 const float* input, double* out, double* bound, size_t numOutputs);

/* int8 -> normalised float, identical expression to the kernel. */
float orc_int8_to_norm(int8_t v);
void orc_int8_to_float(const int8_t* in, float* out, size_t n);

/* AM envelope of cf32, identical expression to the kernel. */
void orc_quad_am_demod(const float* inComplex, float* out, size_t n);

/* cos / exp(j phi) over phi_i = phiBegin + i * (phiEnd - phiBegin) / n (float arithmetic). */
void orc_cosine_f(float phiBegin, float phiEnd, float* out, size_t n);
void orc_cosine_c(float phiBegin, float phiEnd, float* outComplex, size_t n);

/* Synthetic sources, same definitions as gsdrSynthIqInt8 / gsdrSynthWidebandCf32. */
void orc_synth_iq_int8(uint64_t seed, double sampleRate, double amToneHz, double carrierHz, uint64_t firstSample,
                       int8_t* outIq, size_t n);
void orc_synth_wideband_cf32(uint64_t seed, double f1, double f2, uint64_t firstSample, float* outComplex, size_t n);

/* ---- CPU baseline ("port"): float32 direct form, threads = time shards ---------------- */
/* int8 IQ -> cf32 -> FC FIR (real taps) -> AM envelope, the BASELINE metric's chain. */
void orc_chain_i8_fc_am_f32(size_t decimation, const float* taps, size_t tapCount, const int8_t* inIq, float* out,
                            size_t numOutputs, int threads);
/* cf32 -> FC FIR -> AM envelope. */
void orc_chain_fc_am_f32(size_t decimation, const float* taps, size_t tapCount, const float* inComplex, float* out,
                         size_t numOutputs, int threads);

/* real f32 -> FF FIR, float32 direct form (the C1 CPU configuration). */
void orc_fir_ff_f32(size_t decimation, const float* taps, size_t tapCount, const float* x, float* out,
                    size_t numOutputs, int threads);

void orc_multiply_cc(const float* a, const float* b, float* out, size_t n);
void orc_quad_fm_demod_f64(const float* in, double gain, double* out, size_t nOut);

#ifdef __cplusplus
}
#endif

#endif /* GSDR_ORACLE_H */
