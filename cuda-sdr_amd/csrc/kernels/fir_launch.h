// Host-side FIR launch geometry shared by the kernel launchers and the filter layer.
#pragma once

#include <stddef.h>

namespace gsdr_amd {

enum FirMode : int { kFirFF = 0, kFirFC = 1, kFirCC = 2, kFirCF = 3 };
enum FirEpilogue : int { kEpiComplex = 0, kEpiPair = 1, kEpiAm = 2, kEpiFm = 3 };

struct FirPlanShape {
  size_t decimation;        // clamped to >= 1
  size_t deff;              // phases that carry taps: min(decimation, tapCount)
  size_t gtot;              // 8-tap groups summed over phases
  size_t gmax;              // 8-tap groups in the longest phase
  int waveOutputSlices;     // WO: 4, 2 or 1 waves along the outputs; 0 = direct (no-LDS) kernel
  size_t regionRows;        // LDS rows per phase region (64*WO + gmax)
  size_t ldsBytes;          // dynamic LDS per block
  size_t tileOutputs;       // outputs per block tile (per stream for FF)
};

// Geometry the LDS kernel uses for a (tapCount, decimation) pair.
FirPlanShape planFirShape(size_t tapCount, size_t decimation);

}  // namespace gsdr_amd

#include <hip/hip_runtime_api.h>
#include <stdint.h>

namespace gsdr_amd {

// int8 IQ -> FC FIR on the exact int8 MFMA path (fir_i8_mfma.hip).
bool firI8MfmaEligible(size_t tapCount, size_t decimation, const void* in);
// carryDst != nullptr: the launch also copies the last tapCount - 1 input samples there (the
// streaming history); it may alias the first tapCount - 1 input samples. Needs nOut >= tapCount - 1.
hipError_t launchFirI8Mfma(const int8_t* iq, const float* taps, size_t tapCount, void* out, size_t nOut, int epi,
                           hipStream_t stream, int8_t* carryDst = nullptr);

// cf32 input x real taps -> FC FIR on split-precision bf16 MFMA (fir_cf_mfma.hip).
bool firCfMfmaEligible(size_t tapCount, size_t decimation, const void* in);
hipError_t launchFirCfMfma(const float* x, const float* taps, size_t tapCount, size_t decimation, void* out,
                           size_t nOut, int epi, hipStream_t stream);

// int8 IQ input (2-byte aligned) x real taps, D <= 16, 31 D + T <= 1408, T >= 5 D, on f16 MFMA
// (fir_cf_mfma.hip).
bool firI8DecMfmaEligible(size_t tapCount, size_t decimation, const void* in);
hipError_t launchFirI8DecMfma(const int8_t* iq, const float* taps, size_t tapCount, size_t decimation, void* out,
                              size_t nOut, int epi, hipStream_t stream);
// The same RF stage with the AM -> FF audio FIR fused into the launch (gsdrInt8FirFCAmDemodFirFF);
// hipErrorNotSupported when the wave-specialised kernel does not take the shape / policy.
hipError_t launchFirI8DecMfmaAudio(const int8_t* iq, const float* taps, size_t tapCount, size_t decimation,
                                   float* amOut, size_t nOut, const float* amHist, size_t amH, const float* aTaps,
                                   size_t aT, size_t aD, float* aOut, size_t aN, hipStream_t stream);

// cf32 (16-byte aligned) or int8 IQ (4-byte aligned) x real taps, long filters, D in {2,4,6,8,10}:
// polyphase overlap-save FFT fast convolution (fir_fft.hip).
// mixed: the fused frequency shifter (gsdr*MixFirFC*) - D >= 2 only, and for int8 IQ the FFT is then
// the long-filter kernel (the int8 MFMA kernels need unmixed integer samples).
struct FftMix {
  bool on = false;
  uint64_t phase0 = 0, step = 0;  // theta(n) = 2 pi (phase0 + n step) / 2^64
};
bool firFftEligible(size_t tapCount, size_t decimation, const void* in, bool int8Iq, bool mixed = false);
hipError_t launchFirFft(const void* in, bool int8Iq, const float* taps, size_t tapCount, size_t decimation,
                        void* out, size_t nOut, int epi, hipStream_t stream, FftMix mix = FftMix{},
                        bool complexTaps = false);

// Kernel-selection policy bits (gsdrAmdSetKernelPolicy).
uint32_t kernelPolicy();

}  // namespace gsdr_amd
