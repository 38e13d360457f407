/*
 * gsdr.h - MI355X (gfx950) kernel library behind the gpusdrpipeline filters.
 *
 * The reference filters (kernrj/cuda-sdr, src/filters) call exactly one
 * entry point of the external, un-vendored `gsdr` CUDA library per readOutput().
 * This header declares HIP-native replacements with the argument order and
 * meaning implied by those call sites, so the filter layer (and any other
 * gsdr caller) links against this library unchanged apart from the
 * cudaStream_t -> hipStream_t / cuComplex -> hipFloatComplex type names.
 *
 * Conventions (all entry points):
 *   - asynchronous on `stream`; nothing is synchronised, nothing is allocated;
 *     every call is graph-capture safe.
 *   - `device` is the HIP device the pointers live on; the call sets it for the
 *     duration of the launch and restores the caller's device.
 *   - returns hipSuccess, hipErrorInvalidValue for bad arguments, or the launch
 *     error.
 *   - complex samples are interleaved float pairs {re, im} (8 bytes).
 *   - a count of 0 is a no-op that returns hipSuccess.
 */
#ifndef GSDR_GSDR_H
#define GSDR_GSDR_H

#include <hip/hip_complex.h>
#include <hip/hip_runtime_api.h>
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#if defined(__GNUC__)
#define GSDR_API __attribute__((visibility("default")))
#else
#define GSDR_API
#endif

/*
 * Decimating FIR (correlation orientation, taps applied in the order given):
 *
 *     output[k] = sum_{j < tapCount} taps[j] * input[k * decimation + j],  k < outputCount
 *
 * The caller must supply (outputCount - 1) * decimation + tapCount input
 * elements. decimation 0 is treated as 1 (Fir.cpp:119 clamps the same way).
 * Orientation pinned by the reference KATs tests/FirTests.cpp:81-84, :196-202.
 *
 *   FF: real taps,    real input    -> real output      (Fir.cpp:230-238)
 *   FC: real taps,    complex input -> complex output   (Fir.cpp:240-248)
 *   CC: complex taps, complex input -> complex output   (Fir.cpp:250-258), non-conjugated MAC
 *   CF: complex taps, real input    -> complex output   (Fir.cpp:260-268)
 *
 * Complex taps are `tapCount` interleaved {re, im} float pairs.
 */
GSDR_API hipError_t gsdrFirFF(size_t decimation, const float* taps, size_t tapCount, const float* input,
                              float* output, size_t outputCount, int32_t device, hipStream_t stream);
GSDR_API hipError_t gsdrFirFC(size_t decimation, const float* taps, size_t tapCount,
                              const hipFloatComplex* input, hipFloatComplex* output, size_t outputCount,
                              int32_t device, hipStream_t stream);
GSDR_API hipError_t gsdrFirCC(size_t decimation, const hipFloatComplex* taps, size_t tapCount,
                              const hipFloatComplex* input, hipFloatComplex* output, size_t outputCount,
                              int32_t device, hipStream_t stream);
GSDR_API hipError_t gsdrFirCF(size_t decimation, const hipFloatComplex* taps, size_t tapCount, const float* input,
                              hipFloatComplex* output, size_t outputCount, int32_t device, hipStream_t stream);

/*
 * AM envelope detector (QuadAmDemod.cpp:93-98):
 *     output[i] = sqrtf(fmaf(re, re, im * im))
 * The reference's arithmetic lives in the absent gsdr library; this expression
 * is this build's definition (parity unpinned) and the CPU oracle
 * uses the identical expression, so the comparison is bit-exact.
 */
GSDR_API hipError_t gsdrQuadAmDemod(const hipFloatComplex* input, float* output, size_t numElements, int32_t device,
                                    hipStream_t stream);

/*
 * Phase cosines (CosineSource.cpp:74-80, ComplexCosineSource.cpp:74-80):
 *     phi_i = phiBegin + i * (phiEnd - phiBegin) / numElements
 *     F: output[i] = cosf(phi_i)          C: output[i] = {cosf(phi_i), sinf(phi_i)}
 * Pinned (1e-4) by tests/CosineSourceTests.cpp:49-55.
 */
GSDR_API hipError_t gsdrCosineF(float phiBegin, float phiEnd, float* output, size_t numElements, int32_t device,
                                hipStream_t stream);
GSDR_API hipError_t gsdrCosineC(float phiBegin, float phiEnd, hipFloatComplex* output, size_t numElements,
                                int32_t device, hipStream_t stream);

/*
 * Complex multiply (Multiply.cpp:145, MultiplyCcc::readOutput), non-conjugate:
 *     out[i] = { fmaf(a.re, b.re, -(a.im * b.im)), fmaf(a.re, b.im, a.im * b.re) }
 * The expression is this build's definition (gsdr is absent); the oracle uses the same one.
 */
GSDR_API hipError_t gsdrMultiplyCC(const hipFloatComplex* a, const hipFloatComplex* b, hipFloatComplex* output,
                                   size_t numElements, int32_t device, hipStream_t stream);

/*
 * Quadrature FM discriminator (QuadFmDemod.cpp:80-115): numOutputs = inputs - 1,
 *     p = input[i + 1] * conj(input[i]) = { fmaf(r1, r0, i1 * i0), fmaf(i1, r0, -(r1 * i0)) }
 *     output[i] = gain * atan2f(p.im, p.re)
 * with gain = sampleRate / (2 pi fskDeviation 5) from QuadDemodFactory (QuadDemodFactory.h:111).
 */
GSDR_API hipError_t gsdrQuadFmDemod(const hipFloatComplex* input, float* output, float gain, size_t numOutputs,
                                    int32_t device, hipStream_t stream);

#ifdef __cplusplus
}
#endif

#endif /* GSDR_GSDR_H */
