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

// FM discriminator (gsdrQuadFmDemod, QuadFmDemod.cpp:80-115): gain * arg(z1 conj(z0)).
__device__ __forceinline__ float fmDiscriminate(f2 z0, f2 z1, float gain) {
  const float re = fmaf(z1.x, z0.x, z1.y * z0.y);
  const float im = fmaf(z1.y, z0.x, -(z1.x * z0.y));
  return gain * atan2f(im, re);
}

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

// Cross-lane reductions on DPP (VALU) instead of ds_bpermute: no LDS round trip, which matters in
// waves whose LDS queue is shared with MFMA operand reads. dpp_ctrl encodings (gfx9):
// quad_perm [1,0,3,2] = 0xB1, [2,3,0,1] = 0x4E, row_mirror = 0x140, row_half_mirror = 0x141.
template <int CTRL>
__device__ __forceinline__ float dppF(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xf, 0xf, false));
}
// max over each aligned group of 8 lanes (the result in every lane of the group)
__device__ __forceinline__ float dppMax8(float v) {
  v = fmaxf(v, dppF<0x141>(v));
  v = fmaxf(v, dppF<0xB1>(v));
  return fmaxf(v, dppF<0x4E>(v));
}
__device__ __forceinline__ float dppMin8(float v) {
  v = fminf(v, dppF<0x141>(v));
  v = fminf(v, dppF<0xB1>(v));
  return fminf(v, dppF<0x4E>(v));
}
// The same on unsigned words (bit patterns of |x|: they order like the values, and NaN patterns
// sort above +inf, so a max over them also flags non-finite samples). bound_ctrl lets the
// compiler fold each DPP move into the max.
template <int CTRL>
__device__ __forceinline__ uint32_t dppU(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xf, 0xf, true);
}
__device__ __forceinline__ uint32_t dppMax8u(uint32_t v) {
  v = max(v, dppU<0x141>(v));
  v = max(v, dppU<0xB1>(v));
  return max(v, dppU<0x4E>(v));
}
__device__ __forceinline__ uint32_t waveMaxU(uint32_t v) {
  v = dppMax8u(v);
  v = max(v, dppU<0x140>(v));
  uint32_t m = __builtin_amdgcn_readlane(v, 0);
  m = max(m, (uint32_t)__builtin_amdgcn_readlane(v, 16));
  m = max(m, (uint32_t)__builtin_amdgcn_readlane(v, 32));
  return max(m, (uint32_t)__builtin_amdgcn_readlane(v, 48));
}
__device__ __forceinline__ uint32_t waveMinU(uint32_t v) {
  v = min(v, dppU<0x141>(v));
  v = min(v, dppU<0xB1>(v));
  v = min(v, dppU<0x4E>(v));
  v = min(v, dppU<0x140>(v));
  uint32_t m = __builtin_amdgcn_readlane(v, 0);
  m = min(m, (uint32_t)__builtin_amdgcn_readlane(v, 16));
  m = min(m, (uint32_t)__builtin_amdgcn_readlane(v, 32));
  return min(m, (uint32_t)__builtin_amdgcn_readlane(v, 48));
}

// wave-wide max / min of NON-NEGATIVE floats (+inf allowed, no NaN): 8-lane groups by DPP, the
// rows' halves by row_mirror, the four rows through SGPRs (bit patterns order like the values)
__device__ __forceinline__ float waveMaxNonNeg(float v) {
  v = dppMax8(v);
  v = fmaxf(v, dppF<0x140>(v));
  const uint32_t u = __builtin_bit_cast(uint32_t, v);
  uint32_t m = __builtin_amdgcn_readlane(u, 0);
  m = max(m, (uint32_t)__builtin_amdgcn_readlane(u, 16));
  m = max(m, (uint32_t)__builtin_amdgcn_readlane(u, 32));
  m = max(m, (uint32_t)__builtin_amdgcn_readlane(u, 48));
  return __builtin_bit_cast(float, m);
}
__device__ __forceinline__ float waveMinNonNeg(float v) {
  v = dppMin8(v);
  v = fminf(v, dppF<0x140>(v));
  const uint32_t u = __builtin_bit_cast(uint32_t, v);
  uint32_t m = __builtin_amdgcn_readlane(u, 0);
  m = min(m, (uint32_t)__builtin_amdgcn_readlane(u, 16));
  m = min(m, (uint32_t)__builtin_amdgcn_readlane(u, 32));
  m = min(m, (uint32_t)__builtin_amdgcn_readlane(u, 48));
  return __builtin_bit_cast(float, m);
}

// wave-wide sum of a float (butterfly over lane xor 1..32; the result in every lane)
__device__ __forceinline__ float waveSum(float v) {
#pragma unroll
  for (int m = 1; m < 64; m <<= 1) v += __shfl_xor(v, m);
  return v;
}

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

// The same four words -> the clamped samples as int8 I and Q halves-units (8 samples each, for the
// int8 x int8 MFMA planes): x = -128 (0x80) becomes -127 (0x81), the reference's clamp. Per byte,
// t = x ^ 0x80 is zero exactly for 0x80; (t - 1) & ~t & 0x80 flags it (the borrow can also flag a byte
// t = 1, x = 0x81, above a flagged one - setting bit 0 of 0x81 changes nothing), and the flag shifted
// to bit 0 turns 0x80 into 0x81.
__device__ __forceinline__ uint32_t clampInt8x4(uint32_t x) {
  const uint32_t t = x ^ 0x80808080u;
  const uint32_t z = (t - 0x01010101u) & ~t & 0x80808080u;
  return x | (z >> 7);
}
__device__ __forceinline__ void int8IqToI8Units(const uint32_t (&w)[4], uint2& iu, uint2& qu) {
  uint32_t c[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) c[q] = clampInt8x4(w[q]);
  // bytes I0 Q0 I1 Q1 | I2 Q2 I3 Q3 of two words -> I0 I1 I2 I3 and Q0 Q1 Q2 Q3
  iu = uint2{__builtin_amdgcn_perm(c[1], c[0], 0x06040200u), __builtin_amdgcn_perm(c[3], c[2], 0x06040200u)};
  qu = uint2{__builtin_amdgcn_perm(c[1], c[0], 0x07050301u), __builtin_amdgcn_perm(c[3], c[2], 0x07050301u)};
}

}  // namespace gsdr_amd
