// Shared device helpers for the gfx950 kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gsdr_amd {

typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));

constexpr int kWave = 64;  // CDNA wavefront width

// The int8 -> float normalisation of gsdrInt8ToNormFloat (include/gsdr/conversion.h).
// IEEE division on purpose: the CPU oracle evaluates the same expression.
__device__ __forceinline__ float int8ToNorm(int8_t v) { return fmaxf(-1.0f, (float)v / 127.0f); }

// AM envelope (include/gsdr/gsdr.h, gsdrQuadAmDemod).
__device__ __forceinline__ float amEnvelope(f2 z) { return sqrtf(fmaf(z.x, z.x, z.y * z.y)); }

// Map a launch-order block index to a tile so that tiles t and t+1 run on the same XCD
// (blocks b and b+8 share an XCD under round-robin dispatch). Bijective for any grid size;
// only affects L2 locality of the (taps-1) input halo, never correctness.
__device__ __forceinline__ uint32_t xcdTile(uint32_t b, uint32_t nb) {
  const uint32_t xcd = b & 7u;
  const uint32_t idx = b >> 3;
  const uint32_t q = nb >> 3;
  const uint32_t rem = nb & 7u;
  const uint32_t start = xcd < rem ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q;
  return start + idx;
}

__device__ __forceinline__ int waveUniform(int v) { return __builtin_amdgcn_readfirstlane(v); }

}  // namespace gsdr_amd
