// Element-wise kernels of the hot path (gfx950): int8 -> normalised float
// (Int8ToFloat.cpp:89-94), float -> int8, the AM envelope (QuadAmDemod.cpp:93-98),
// phase cosines (CosineSource.cpp:74-80, ComplexCosineSource.cpp:74-80) and the
// deterministic synthetic sources used by the benchmark.
//
// All of these are HBM-bound: 16-byte accesses per lane where the pointers allow it,
// grid-stride loops capped at 8 blocks per CU, a scalar path for ragged heads/tails or
// misaligned pointers (the filter layer hands over buffer write pointers at arbitrary
// byte offsets).
#include "kcommon.h"

#include <algorithm>

#include <gsdr/conversion.h>
#include <gsdr/gsdr.h>
#include <gsdr/gsdr_amd.h>

namespace gsdr_amd {

namespace {

constexpr int kBlock = 256;
constexpr unsigned kMaxBlocks = 256 * 8;

unsigned blocksFor(size_t work) {
  const size_t b = (work + kBlock - 1) / kBlock;
  return (unsigned)(b < kMaxBlocks ? (b == 0 ? 1 : b) : kMaxBlocks);
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

struct DevicePush {
  int prev = -1;
  bool ok = true;
  explicit DevicePush(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) ok = hipSetDevice(dev) == hipSuccess;
  }
  ~DevicePush() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

}  // namespace

// ---- int8 -> float --------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void int8ToFloatVec(const int4* __restrict__ in, f4* __restrict__ out,
                                                         size_t n16) {
  for (size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x; i < n16; i += (size_t)gridDim.x * kBlock) {
    const int4 v = in[i];
    const int words[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const int x = words[w];
      f4 o;
      o.x = int8ToNorm((int8_t)(x & 0xff));
      o.y = int8ToNorm((int8_t)((x >> 8) & 0xff));
      o.z = int8ToNorm((int8_t)((x >> 16) & 0xff));
      o.w = int8ToNorm((int8_t)((x >> 24) & 0xff));
      out[4 * i + w] = o;
    }
  }
}

__global__ __launch_bounds__(kBlock) void int8ToFloatScalar(const int8_t* __restrict__ in, float* __restrict__ out,
                                                            size_t n) {
  for (size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (size_t)gridDim.x * kBlock)
    out[i] = int8ToNorm(in[i]);
}

__global__ __launch_bounds__(kBlock) void floatToInt8Scalar(const float* __restrict__ in, int8_t* __restrict__ out,
                                                            size_t n) {
  for (size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (size_t)gridDim.x * kBlock) {
    const float v = fminf(127.0f, fmaxf(-128.0f, rintf(in[i] * 127.0f)));
    out[i] = (int8_t)v;
  }
}

// ---- AM envelope -------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void amDemodVec(const f4* __restrict__ in, f2* __restrict__ out, size_t n2) {
  for (size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x; i < n2; i += (size_t)gridDim.x * kBlock) {
    const f4 v = in[i];
    out[i] = f2{amEnvelope(v.xy), amEnvelope(v.zw)};
  }
}

__global__ __launch_bounds__(kBlock) void amDemodScalar(const f2* __restrict__ in, float* __restrict__ out, size_t n) {
  for (size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (size_t)gridDim.x * kBlock)
    out[i] = amEnvelope(in[i]);
}

// ---- cosines -----------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void cosineF(float phi0, float step, float* __restrict__ out, size_t n) {
  for (size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (size_t)gridDim.x * kBlock)
    out[i] = cosf(fmaf((float)i, step, phi0));
}

__global__ __launch_bounds__(kBlock) void cosineC(float phi0, float step, f2* __restrict__ out, size_t n) {
  for (size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (size_t)gridDim.x * kBlock) {
    const float phi = fmaf((float)i, step, phi0);
    float s, c;
    sincosf(phi, &s, &c);
    out[i] = f2{c, s};
  }
}

// ---- complex multiply / FM discriminator --------------------------------------------------------------
__device__ __forceinline__ f2 cmul(f2 a, f2 b) {
  return f2{fmaf(a.x, b.x, -(a.y * b.y)), fmaf(a.x, b.y, a.y * b.x)};
}

__global__ __launch_bounds__(kBlock) void multiplyCC(const f2* __restrict__ a, const f2* __restrict__ b,
                                                     f2* __restrict__ out, size_t n) {
  for (size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (size_t)gridDim.x * kBlock)
    out[i] = cmul(a[i], b[i]);
}

// each thread reads its sample and the next one (the neighbour's read hits L1/L2)
__global__ __launch_bounds__(kBlock) void quadFmDemod(const f2* __restrict__ in, float* __restrict__ out, float gain,
                                                      size_t n) {
  for (size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (size_t)gridDim.x * kBlock) {
    const f2 z0 = in[i], z1 = in[i + 1];
    out[i] = fmDiscriminate(z0, z1, gain);
  }
}

// ---- synthetic sources ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// uniform in [-1, 1)
__device__ __forceinline__ double uniformPm1(uint64_t seed, uint64_t key) {
  return (double)(splitmix64(seed ^ key) >> 11) * (1.0 / 9007199254740992.0) * 2.0 - 1.0;
}

// 2 pi * frac(f * n), argument reduction in double
__device__ __forceinline__ float cyclePhase(double cyclesPerSample, uint64_t n) {
  const double c = cyclesPerSample * (double)n;
  return (float)(6.283185307179586 * (c - floor(c)));
}

__device__ __forceinline__ int8_t quantizeIq(double v) {
  double r = v < 0.0 ? -floor(-v + 0.5) : floor(v + 0.5);  // half away from zero
  r = r > 127.0 ? 127.0 : (r < -127.0 ? -127.0 : r);
  return (int8_t)(int)r;
}

__global__ __launch_bounds__(kBlock) void synthIqInt8(uint64_t seed, double fAm, double fCarrier, uint64_t first,
                                                      char2* __restrict__ out, size_t n) {
  for (size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (size_t)gridDim.x * kBlock) {
    const uint64_t s = first + i;
    const float am = 100.0f * (1.0f + 0.5f * cosf(cyclePhase(fAm, s)));
    float sc, cc;
    sincosf(cyclePhase(fCarrier, s), &sc, &cc);
    const double re = (double)(am * cc) + 3.0 * uniformPm1(seed, 2 * s);
    const double im = (double)(am * sc) + 3.0 * uniformPm1(seed, 2 * s + 1);
    out[i] = char2{quantizeIq(re), quantizeIq(im)};
  }
}

__global__ __launch_bounds__(kBlock) void synthWideband(uint64_t seed, double f1, double f2c, uint64_t first,
                                                        f2* __restrict__ out, size_t n) {
  for (size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (size_t)gridDim.x * kBlock) {
    const uint64_t s = first + i;
    float s1, c1, s2, c2;
    sincosf(cyclePhase(f1, s), &s1, &c1);
    sincosf(cyclePhase(f2c, s), &s2, &c2);
    const float ur = (float)uniformPm1(seed, 2 * s);
    const float ui = (float)uniformPm1(seed, 2 * s + 1);
    out[i] = f2{c1 + 0.5f * c2 + 0.01f * ur, s1 + 0.5f * s2 + 0.01f * ui};
  }
}

}  // namespace gsdr_amd

using namespace gsdr_amd;

// ---- HBM bandwidth probe (diagnostics: the measured read / copy bandwidth the bench reports the
// roofline against, beside the 8 TB/s spec) -------------------------------------------------------
template <int MODE>
__global__ __launch_bounds__(kBlock) void hbmProbeKernel(const f4* __restrict__ in, f4* __restrict__ out, size_t n4) {
  float acc = 0.0f;
  for (size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x; i < n4; i += (size_t)gridDim.x * kBlock) {
    const f4 v = in[i];
    if (MODE == 1) out[i] = v;
    else acc += v.x + v.y + v.z + v.w;
  }
  // read mode: the sum must look used; it is never equal to this for finite data of the probe
  if (MODE == 0 && acc == -1.2345e-38f) out[0] = f4{acc, acc, acc, acc};
}

// ---- copies between mapped pinned host memory and the device as kernels (the host-fed chain) ---------
// 16-byte loads from a 16-byte aligned source, stores at any 4-byte aligned destination (global stores
// of 16 bytes need dword alignment only); the dword kernel for the rest.
__global__ __launch_bounds__(kBlock) void copyVec16(const uint4* __restrict__ src, uint8_t* __restrict__ dst, size_t n16) {
  for (size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x; i < n16; i += (size_t)gridDim.x * kBlock) {
    const uint4 v = src[i];
    uint32_t* d = reinterpret_cast<uint32_t*>(dst + 16 * i);
    d[0] = v.x;
    d[1] = v.y;
    d[2] = v.z;
    d[3] = v.w;
  }
}
__global__ __launch_bounds__(kBlock) void copyDword(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst, size_t n4) {
  for (size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x; i < n4; i += (size_t)gridDim.x * kBlock) dst[i] = src[i];
}

// ---- LDS poison (tests): fill every CU's LDS with a pattern so a kernel that reads LDS it never
// wrote shows it (a NaN pattern turns 0 * stale into NaN) ------------------------------------------
constexpr int kPoisonLdsBytes = 160 * 1024 - 256;
__global__ __launch_bounds__(1024) void ldsPoisonKernel(uint32_t pattern) {
  extern __shared__ uint32_t poisonLds[];
  for (int i = threadIdx.x; i < kPoisonLdsBytes / 4; i += 1024) poisonLds[i] = pattern;
  __syncthreads();
}

extern "C" {

hipError_t gsdrAmdCopyKernel(void* dst, const void* src, size_t bytes, hipStream_t stream) {
  if (bytes == 0) return hipSuccess;
  const auto d = reinterpret_cast<uintptr_t>(dst), s = reinterpret_cast<uintptr_t>(src);
  if ((d & 3) != 0 || (s & 3) != 0 || (bytes & 3) != 0) return hipErrorInvalidValue;
  if ((s & 15) == 0 && (bytes & 15) == 0) {
    const size_t n16 = bytes / 16;
    const unsigned grid = (unsigned)std::min<size_t>((n16 + kBlock - 1) / kBlock, 2048);
    hipLaunchKernelGGL(copyVec16, dim3(grid), dim3(kBlock), 0, stream, static_cast<const uint4*>(src),
                       static_cast<uint8_t*>(dst), n16);
  } else {
    const size_t n4 = bytes / 4;
    const unsigned grid = (unsigned)std::min<size_t>((n4 + kBlock - 1) / kBlock, 2048);
    hipLaunchKernelGGL(copyDword, dim3(grid), dim3(kBlock), 0, stream, static_cast<const uint32_t*>(src),
                       static_cast<uint32_t*>(dst), n4);
  }
  return hipGetLastError();
}

hipError_t gsdrAmdPoisonLds(uint32_t pattern, int32_t device, hipStream_t stream) {
  DevicePush push(device);
  if (!push.ok) return hipErrorInvalidDevice;
  const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&ldsPoisonKernel),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, kPoisonLdsBytes);
  if (e != hipSuccess) return e;
  int n = 256;
  (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, device);
  hipLaunchKernelGGL(ldsPoisonKernel, dim3((unsigned)(4 * n)), dim3(1024), kPoisonLdsBytes, stream, pattern);
  return hipGetLastError();
}

hipError_t gsdrAmdHbmProbe(const void* input, void* output, size_t bytes, int32_t mode, int32_t device,
                           hipStream_t stream) {
  if (bytes < 16 || input == nullptr || output == nullptr || !aligned16(input) || !aligned16(output) ||
      (mode != 0 && mode != 1))
    return hipErrorInvalidValue;
  DevicePush push(device);
  if (!push.ok) return hipErrorInvalidDevice;
  const size_t n4 = bytes / 16;
  int n = 256;
  (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, device);
  const dim3 grid((unsigned)(n * 8));  // 8 blocks of 256 per CU: the grid-stride sweep's best (fft_bench readBw)
  if (mode == 0)
    hipLaunchKernelGGL(hbmProbeKernel<0>, grid, dim3(kBlock), 0, stream, reinterpret_cast<const f4*>(input),
                       reinterpret_cast<f4*>(output), n4);
  else
    hipLaunchKernelGGL(hbmProbeKernel<1>, grid, dim3(kBlock), 0, stream, reinterpret_cast<const f4*>(input),
                       reinterpret_cast<f4*>(output), n4);
  return hipGetLastError();
}

hipError_t gsdrInt8ToNormFloat(const int8_t* input, float* output, size_t numElements, int32_t device,
                               hipStream_t stream) {
  if (numElements == 0) return hipSuccess;
  if (input == nullptr || output == nullptr) return hipErrorInvalidValue;
  DevicePush push(device);
  if (!push.ok) return hipErrorInvalidDevice;
  size_t done = 0;
  if (aligned16(input) && aligned16(output) && numElements >= 16) {
    const size_t n16 = numElements / 16;
    hipLaunchKernelGGL(int8ToFloatVec, dim3(blocksFor(n16)), dim3(kBlock), 0, stream,
                       reinterpret_cast<const int4*>(input), reinterpret_cast<f4*>(output), n16);
    done = n16 * 16;
  }
  if (done < numElements) {
    hipLaunchKernelGGL(int8ToFloatScalar, dim3(blocksFor(numElements - done)), dim3(kBlock), 0, stream,
                       input + done, output + done, numElements - done);
  }
  return hipGetLastError();
}

hipError_t gsdrFloatToInt8(const float* input, int8_t* output, size_t numElements, int32_t device,
                           hipStream_t stream) {
  if (numElements == 0) return hipSuccess;
  if (input == nullptr || output == nullptr) return hipErrorInvalidValue;
  DevicePush push(device);
  if (!push.ok) return hipErrorInvalidDevice;
  hipLaunchKernelGGL(floatToInt8Scalar, dim3(blocksFor(numElements)), dim3(kBlock), 0, stream, input, output,
                     numElements);
  return hipGetLastError();
}

hipError_t gsdrQuadAmDemod(const hipFloatComplex* input, float* output, size_t numElements, int32_t device,
                           hipStream_t stream) {
  if (numElements == 0) return hipSuccess;
  if (input == nullptr || output == nullptr) return hipErrorInvalidValue;
  DevicePush push(device);
  if (!push.ok) return hipErrorInvalidDevice;
  size_t done = 0;
  if (aligned16(input) && (reinterpret_cast<uintptr_t>(output) & 7u) == 0 && numElements >= 2) {
    const size_t n2 = numElements / 2;
    hipLaunchKernelGGL(amDemodVec, dim3(blocksFor(n2)), dim3(kBlock), 0, stream, reinterpret_cast<const f4*>(input),
                       reinterpret_cast<f2*>(output), n2);
    done = n2 * 2;
  }
  if (done < numElements) {
    hipLaunchKernelGGL(amDemodScalar, dim3(blocksFor(numElements - done)), dim3(kBlock), 0, stream,
                       reinterpret_cast<const f2*>(input) + done, output + done, numElements - done);
  }
  return hipGetLastError();
}

hipError_t gsdrCosineF(float phiBegin, float phiEnd, float* output, size_t numElements, int32_t device,
                       hipStream_t stream) {
  if (numElements == 0) return hipSuccess;
  if (output == nullptr) return hipErrorInvalidValue;
  DevicePush push(device);
  if (!push.ok) return hipErrorInvalidDevice;
  const float step = (phiEnd - phiBegin) / (float)numElements;
  hipLaunchKernelGGL(cosineF, dim3(blocksFor(numElements)), dim3(kBlock), 0, stream, phiBegin, step, output,
                     numElements);
  return hipGetLastError();
}

hipError_t gsdrCosineC(float phiBegin, float phiEnd, hipFloatComplex* output, size_t numElements, int32_t device,
                       hipStream_t stream) {
  if (numElements == 0) return hipSuccess;
  if (output == nullptr) return hipErrorInvalidValue;
  DevicePush push(device);
  if (!push.ok) return hipErrorInvalidDevice;
  const float step = (phiEnd - phiBegin) / (float)numElements;
  hipLaunchKernelGGL(cosineC, dim3(blocksFor(numElements)), dim3(kBlock), 0, stream, phiBegin, step,
                     reinterpret_cast<f2*>(output), numElements);
  return hipGetLastError();
}

hipError_t gsdrMultiplyCC(const hipFloatComplex* a, const hipFloatComplex* b, hipFloatComplex* output,
                          size_t numElements, int32_t device, hipStream_t stream) {
  if (numElements == 0) return hipSuccess;
  if (a == nullptr || b == nullptr || output == nullptr) return hipErrorInvalidValue;
  DevicePush push(device);
  if (!push.ok) return hipErrorInvalidDevice;
  hipLaunchKernelGGL(multiplyCC, dim3(blocksFor(numElements)), dim3(kBlock), 0, stream,
                     reinterpret_cast<const f2*>(a), reinterpret_cast<const f2*>(b), reinterpret_cast<f2*>(output),
                     numElements);
  return hipGetLastError();
}

hipError_t gsdrQuadFmDemod(const hipFloatComplex* input, float* output, float gain, size_t numOutputs, int32_t device,
                           hipStream_t stream) {
  if (numOutputs == 0) return hipSuccess;
  if (input == nullptr || output == nullptr) return hipErrorInvalidValue;
  DevicePush push(device);
  if (!push.ok) return hipErrorInvalidDevice;
  hipLaunchKernelGGL(quadFmDemod, dim3(blocksFor(numOutputs)), dim3(kBlock), 0, stream,
                     reinterpret_cast<const f2*>(input), output, gain, numOutputs);
  return hipGetLastError();
}

hipError_t gsdrSynthIqInt8(uint64_t seed, double sampleRate, double amToneHz, double carrierHz, uint64_t firstSample,
                           int8_t* outputIq, size_t numSamples, int32_t device, hipStream_t stream) {
  if (numSamples == 0) return hipSuccess;
  if (outputIq == nullptr || !(sampleRate > 0.0)) return hipErrorInvalidValue;
  DevicePush push(device);
  if (!push.ok) return hipErrorInvalidDevice;
  hipLaunchKernelGGL(synthIqInt8, dim3(blocksFor(numSamples)), dim3(kBlock), 0, stream, seed, amToneHz / sampleRate,
                     carrierHz / sampleRate, firstSample, reinterpret_cast<char2*>(outputIq), numSamples);
  return hipGetLastError();
}

hipError_t gsdrSynthWidebandCf32(uint64_t seed, double f1, double f2Cycles, uint64_t firstSample, hipFloatComplex* output,
                                 size_t numSamples, int32_t device, hipStream_t stream) {
  if (numSamples == 0) return hipSuccess;
  if (output == nullptr) return hipErrorInvalidValue;
  DevicePush push(device);
  if (!push.ok) return hipErrorInvalidDevice;
  hipLaunchKernelGGL(synthWideband, dim3(blocksFor(numSamples)), dim3(kBlock), 0, stream, seed, f1, f2Cycles, firstSample,
                     reinterpret_cast<f2*>(output), numSamples);
  return hipGetLastError();
}

}  // extern "C"
