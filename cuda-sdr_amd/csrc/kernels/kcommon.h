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

typedef _Float16 h2 __attribute__((ext_vector_type(2)));

// Four interleaved int8 IQ words (I0 Q0 I1 Q1 each) -> the clamped samples x' = max(x, -127) of
// gsdrInt8ToNormFloat's numerator as f16 I and Q units (8 samples each), exactly.
// u = x ^ 0x80 = x + 128 lands in the low byte of the f16 1024 + u (high byte 0x64); adding
// -1152 gives x exactly, and max(., -127) is the reference's fmaxf(-1, x/127) clamp.
__device__ __forceinline__ void int8IqToF16Units(const uint32_t (&w)[4], uint4& iu, uint4& qu) {
  const h2 bias = {(_Float16)-1152.0f, (_Float16)-1152.0f};
  const h2 lo = {(_Float16)-127.0f, (_Float16)-127.0f};
  uint32_t ri[4], rq[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint32_t u = w[q] ^ 0x80808080u;
    const uint32_t pi = __builtin_amdgcn_perm(0x64646464u, u, 0x04020400u);
    const uint32_t pq = __builtin_amdgcn_perm(0x64646464u, u, 0x04030401u);
    h2 fi = __builtin_bit_cast(h2, pi) + bias;
    h2 fq = __builtin_bit_cast(h2, pq) + bias;
    fi = __builtin_elementwise_max(fi, lo);
    fq = __builtin_elementwise_max(fq, lo);
    ri[q] = __builtin_bit_cast(uint32_t, fi);
    rq[q] = __builtin_bit_cast(uint32_t, fq);
  }
  iu = uint4{ri[0], ri[1], ri[2], ri[3]};
  qu = uint4{rq[0], rq[1], rq[2], rq[3]};
}

}  // namespace gsdr_amd
