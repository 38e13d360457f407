/*
 * conversion.h - sample-format conversion kernels (MI355X / gfx950).
 *
 * Replaces gsdr's <gsdr/conversion.h>, included by Int8ToFloat.cpp:20 and
 * called at Int8ToFloat.cpp:89-94.
 */
#ifndef GSDR_CONVERSION_H
#define GSDR_CONVERSION_H

#include <hip/hip_runtime_api.h>
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#if defined(__GNUC__)
#define GSDR_CONV_API __attribute__((visibility("default")))
#else
#define GSDR_CONV_API
#endif

/*
 * int8 -> normalised float, element-wise over BYTES, so interleaved int8 IQ
 * becomes interleaved cf32:
 *
 *     output[i] = fmaxf(-1.0f, (float)input[i] / 127.0f)
 *
 * The scale lives in gsdr, which is not in the reference tree (SURVEY.md 8c:
 * parity unpinned). This single expression is the build's definition; the
 * kernel and the CPU oracle evaluate it identically (IEEE division, no
 * reciprocal), and tests check all 256 codes bit-exactly.
 */
GSDR_CONV_API hipError_t gsdrInt8ToNormFloat(const int8_t* input, float* output, size_t numElements, int32_t device,
                                             hipStream_t stream);

/* float -> int8 with the inverse scale, saturating and rounding to nearest even:
 *     output[i] = (int8_t)clamp(rintf(input[i] * 127.0f), -128, 127)
 * (format conversion for the egress side; not in the reference path). */
GSDR_CONV_API hipError_t gsdrFloatToInt8(const float* input, int8_t* output, size_t numElements, int32_t device,
                                         hipStream_t stream);

#ifdef __cplusplus
}
#endif

#endif /* GSDR_CONVERSION_H */
