// Fast-convolution (polyphase overlap-save FFT) decimating FIR for gfx950: the long-filter
// path of gsdrFirFC / gsdrFirFCAmDemod / gsdrInt8FirFC / gsdrInt8FirFCAmDemod.
//
// Semantics are the reference's (src/filters/Fir.cpp:229-269; orientation pinned by
// tests/FirTests.cpp:81-84, :196-202):  y[k] = sum_{j<T} h[j] x[kD + j].
//
// Algorithm:
//   * Polyphase: with j = qD + p, y[k] = sum_p sum_q h_p[q] x_p[k + q], where
//     x_p[m] = x[mD + p] and h_p[q] = h[qD + p] (Q = ceil(T / D) taps per phase).
//   * Overlap-save per phase with M = 512-point FFTs: for a block of 512 rows (a row is the D
//     consecutive samples x[mD .. mD + D - 1]), c_p[t] = sum_q h_p[q] x_p[t + q] equals the
//     circular correlation IDFT(X_p . conj(H_p)) / M for t <= M - Q, so one block yields
//     V = M - Q + 1 outputs (T = 1023, D = 10: Q = 103, V = 410) and the D phase spectra are
//     summed BEFORE the single inverse FFT:  Y = sum_p X_p . G_p,  G_p = conj(DFT(h_p)) / M.
//   * Per input sample: 5 log2(M) flops of forward FFT + 8 of spectral MAC + (5 log2 M) / D of
//     inverse FFT, times the overlap factor M / V (~70 flops/sample at C3) - against 4 T / D =
//     409 for the direct form: the kernel is HBM-bound, not VALU-bound.
//   * One wave owns one block at a time: lane l holds rows l + 64 j (j = 0..7) of the block, so
//     each phase's 512-point FFT is 8 points per lane: a radix-8 pass in registers, an 8x8
//     digit transpose through a per-wave LDS scratch, radix-8, transpose, radix-8 (packed
//     v_pk_* complex arithmetic). The inverse FFT runs the mirrored passes so neither direction
//     needs a bit reversal: the spectra stay in the forward FFT's digit order (G is stored in it).
//   * Input: coalesced 16-byte loads of the whole block (a buffer resource clipped at the input's
//     end, so the last block reads zeros instead of faulting), transposed to rows through the
//     same LDS scratch. int8 IQ input (the fused int8 -> cf32 -> FIR chain) carries the clamped
//     integers x' = max(x, -127) and folds the 1/127 of gsdrInt8ToNormFloat into G.
//   * The G table (D x 512 complex, 40 KB at D = 10) and the 512-entry twiddle table are built
//     by each workgroup in LDS (prologue: one forward FFT per phase), so the entry points stay
//     stateless like the reference's gsdr calls.
//   * Epilogue: the first V outputs of the inverse FFT, AM envelope (|y|, the gsdrQuadAmDemod
//     expression) or complex, coalesced stores.
//
// Accuracy: fp32 FFT round-off is relative to the block's signal level, not to each output's
// own window (the tolerance's scale sum_j |h_j||x_kD+j|). Each block therefore measures the
// spread of its rows' magnitudes; a block whose quietest row group is far below its loudest
// (a burst edge, silence next to signal, inf/NaN) is recomputed in the direct fp32 form by the
// same wave (see blockNeedsDirect and DESIGN.md 3.7 for the error model and its calibration).
#include "kcommon.h"
#include "fir_launch.h"

#include <gsdr/gsdr.h>
#include <gsdr/gsdr_amd.h>

#include <atomic>
#include <cmath>


namespace gsdr_amd {
namespace fftfir {

// Blocks computed in the direct form by the accuracy guard since the last reset (diagnostics:
// gsdrAmdFftDirectBlocks; one vector atomic per fallback block).
__device__ unsigned long long gDirectBlocks;

// In-kernel clock stamps, diagnostic builds only (tools/exp/run_fft_variants.sh stamps; the product
// build compiles none): per wave of the first 256 workgroups, the shader-clock and the 100 MHz
// real-time counters after the prologue and after the wave's last block, so the clock the kernel
// runs at is read inside it (MI355X_MICROARCH.md, DVFS give-back item 6). The stamps go to this
// array only; nothing in the kernel reads them.
#ifndef GSDR_FFT_STAMPS
#define GSDR_FFT_STAMPS 0
#endif
// Attribution switches, diagnostic builds only (0 in the product build: every test below folds away):
// bit 1 no FFT math, 2 no global loads (synthetic rows), 4 no LDS transposition, 8 no accuracy
// guard, 16 no output stores.
#ifndef GSDR_FFT_EXP
#define GSDR_FFT_EXP 0
#endif
#if GSDR_FFT_STAMPS
constexpr int kStampWaves = 256 * 8;
__device__ unsigned long long gFftStamps[kStampWaves * 4];
#endif

constexpr int kM = 512;      // FFT points per phase per block
constexpr int kWaves = 8;     // waves per workgroup (one workgroup per CU)
constexpr int kThreads = kWaves * kWave;
constexpr int kSA = 10;       // pattern-A exchange row stride (complex): see exchangeA

enum Input : int { kCf32 = 0, kI8 = 1 };
enum Epi : int { kComplex = 0, kAm = 1 };

struct Args {
  const void* in;
  const float* taps;
  void* out;
  int64_t nOut;
  int64_t inBytes;      // readable input bytes from `in` (loads past this return zeros)
  int64_t nBlocks;
  int64_t inRows;       // rows (D samples) wholly inside the input
  int32_t T;
  int32_t Q;            // taps per phase, ceil(T / D)
  int32_t V;            // outputs per block
  float inScale;        // 1 (cf32) or 1/127 (int8 IQ): folded into G
  float guardRatio;     // direct-form fallback when max/min row-group level exceeds this
  uint64_t mixPhase0;   // fused frequency shifter (kernels with MIX): sample n of `in` is multiplied
  uint64_t mixStep;     // by exp(j theta(n)), theta(n) = 2 pi (mixPhase0 + n mixStep) / 2^64
  int32_t outAligned;   // `out` is 16-byte aligned (the D = 1 kernel's row-unit stores)
  int32_t complexTaps;  // taps are {re, im} pairs (gsdrFirCC / gsdrFirCCAmDemod), else real
};

// Tap j (real taps: imaginary part 0).
__device__ __forceinline__ f2 tapAt(const Args& a, int j) {
  return a.complexTaps ? reinterpret_cast<const f2*>(a.taps)[j] : f2{a.taps[j], 0.0f};
}

// ---- fused frequency shifter -----------------------------------------------------------------------
// Sample n = (b V + r) D + p of block b (row r, phase p) is multiplied by
//     exp(j theta(n)) = E_b . T_r . c_p,   E_b = exp(j 2 pi (phase0 + b V D step) / 2^64),
//     T_r = exp(j 2 pi r D step / 2^64),   c_p = exp(j 2 pi p step / 2^64)
// (all phases reduced exactly in 64-bit fixed point, the exponentials in double, rounded once):
// T_r is a per-lane table (rows l + 64 j) applied to the loaded rows - one complex multiply per
// sample; c_p is a constant per phase, folded into G_p; E_b is a constant per block, which the
// linear transform carries to the outputs (|E_b y| = |y|: the AM epilogue needs nothing).
__device__ __forceinline__ f2 turnExp(uint64_t frac) {  // exp(j 2 pi frac / 2^64)
  double sn, cs;
  sincospi((double)(int64_t)frac * 1.0842021724855044e-19, &sn, &cs);  // 2 / 2^64
  return f2{(float)cs, (float)sn};
}
// The same in float at ~2 ulp, cheap on registers (the per-block factor): the top 24 bits of the
// phase are an exact float fraction of a turn (sincospif), the low 40 bits a rotation below
// 2 pi 2^-24 rad, where exp(j d) = 1 - d^2 / 2 + j d to float precision.
__device__ __forceinline__ f2 turnExpF(uint64_t frac) {
  const int32_t hi = (int32_t)(frac >> 40) << 8 >> 8;  // signed top 24 bits: turns * 2^24
  float sh, ch;
  sincospif((float)hi * 1.1920928955078125e-7f, &sh, &ch);  // 2 * hi / 2^24 half-turns
  const float d = (float)(int64_t)(frac & 0xFFFFFFFFFFull) * 3.4061215800865545e-19f;  // 2 pi / 2^64
  const float cl = fmaf(-0.5f * d, d, 1.0f);
  return f2{fmaf(ch, cl, -(sh * d)), fmaf(sh, cl, ch * d)};
}
// The VALU kernels' per-sample rotation (fir.hip mixSample): the direct-form fallback block.
__device__ __forceinline__ f2 mixOne(const Args& a, int64_t n, f2 z) {
  const uint64_t ph = a.mixPhase0 + (uint64_t)n * a.mixStep;
  const float th = (float)((double)(int64_t)ph * 3.4061215800865545e-19);  // 2 pi / 2^64
  float sn, cs;
  sincosf(th, &sn, &cs);
  return f2{fmaf(z.x, cs, -(z.y * sn)), fmaf(z.x, sn, z.y * cs)};
}

// ---------------------------------------------------------------- packed complex arithmetic
// Written as VOP3P with op_sel / neg modifiers: the compiler otherwise builds the swapped /
// negated operand with v_xor + v_mov (two extra VALU per complex product).
__device__ __forceinline__ f2 cmul(f2 a, f2 b) {  // a * b
  f2 t, r;
  asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[1,0]" : "=v"(t) : "v"(a), "v"(b));
  asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[0,1,1] neg_lo:[0,1,0]" : "=v"(r) : "v"(a), "v"(b), "v"(t));
  return r;
}
// the two halves of cmul / cmac, so independent products can be issued stage-interleaved (a
// dependent v_pk_fma right behind the v_pk_* that writes its operand costs an s_nop on gfx950)
__device__ __forceinline__ f2 cmul1(f2 a, f2 b) {
  f2 t;
  asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[1,0]" : "=v"(t) : "v"(a), "v"(b));
  return t;
}
__device__ __forceinline__ f2 cmac1(f2 a, f2 b, f2 acc) {
  f2 t;
  asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[1,0,1]" : "=v"(t) : "v"(a), "v"(b), "v"(acc));
  return t;
}
__device__ __forceinline__ f2 cmul2(f2 a, f2 b, f2 t) {
  f2 r;
  asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[0,1,1] neg_lo:[0,1,0]" : "=v"(r) : "v"(a), "v"(b), "v"(t));
  return r;
}
// second half of a * conj(b) (the first half is cmul1)
__device__ __forceinline__ f2 cmulc2(f2 a, f2 b, f2 t) {
  f2 r;
  asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[0,1,1] neg_hi:[0,1,0]" : "=v"(r) : "v"(a), "v"(b), "v"(t));
  return r;
}
__device__ __forceinline__ f2 cmac(f2 a, f2 b, f2 acc) {  // acc + a * b
  f2 t, r;
  asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[1,0,1]" : "=v"(t) : "v"(a), "v"(b), "v"(acc));
  asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[0,1,1] neg_lo:[0,1,0]" : "=v"(r) : "v"(a), "v"(b), "v"(t));
  return r;
}
__device__ __forceinline__ f2 addMi(f2 a, f2 b) {  // a - i b
  f2 r;
  asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ f2 addPi(f2 a, f2 b) {  // a + i b
  f2 r;
  asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1]" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ f2 rotM(f2 v) {  // (1 - i) v
  f2 r;
  asm("v_pk_add_f32 %0, %1, %1 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]" : "=v"(r) : "v"(v));
  return r;
}
__device__ __forceinline__ f2 rotP(f2 v) {  // (1 + i) v
  f2 r;
  asm("v_pk_add_f32 %0, %1, %1 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1]" : "=v"(r) : "v"(v));
  return r;
}

// In-register 8-point DFT: z[k] <- sum_n z[n] W8^{+-nk}, W8 = exp(-2 pi i / 8) (INV: conjugate).
template <bool INV>
__device__ __forceinline__ void dft8(f2 (&z)[8]) {
  constexpr float s = 0.70710678118654752440f;
  const f2 a0 = z[0] + z[4], a1 = z[0] - z[4], a2 = z[2] + z[6], a3 = z[2] - z[6];
  const f2 a4 = z[1] + z[5], a5 = z[1] - z[5], a6 = z[3] + z[7], a7 = z[3] - z[7];
  const f2 b0 = a0 + a2, b2 = a0 - a2, b4 = a4 + a6, b6 = a4 - a6;
  const f2 b1 = INV ? addPi(a1, a3) : addMi(a1, a3);
  const f2 b3 = INV ? addMi(a1, a3) : addPi(a1, a3);
  const f2 b5 = INV ? addPi(a5, a7) : addMi(a5, a7);
  const f2 b7 = INV ? addMi(a5, a7) : addPi(a5, a7);
  const f2 t5 = INV ? rotP(b5) : rotM(b5);
  const f2 t7 = INV ? rotM(b7) : rotP(b7);
  const f2 sv = {s, s};
  z[0] = b0 + b4;
  z[4] = b0 - b4;
  z[2] = INV ? addPi(b2, b6) : addMi(b2, b6);
  z[6] = INV ? addMi(b2, b6) : addPi(b2, b6);
  z[1] = b1 + t5 * sv;
  z[5] = b1 - t5 * sv;
  z[3] = b3 - t7 * sv;
  z[7] = b3 + t7 * sv;
}

// LDS layout (complex units): [G: D x 8 x 64][twiddles: 4 x 8 x 64][scratch: kWaves x scratch].
// Every table is read 16 bytes per lane (ds_read_b128, lanes 16 B apart: conflict free, 256 B/clk;
// two 8-byte reads would be fused by the compiler into ds_read2_b64 / ds_read2st64_b64 at half
// that rate). G: f4 (G_p[d], G_p[d + 1]) at (p 4 + d / 2) 64 + l. Twiddles: per-lane tables for the
// four stage boundaries of the forward / inverse 512-point DFT, f4 (t_k, t_k+1) at
// (stage 4 + k / 2) 64 + l, t_k = W^(e r) with r = k + 1 = 1..7 (slot 7 unused).
constexpr int kTw = 4 * 8 * 64;
struct Lds {
  f4* g;
  const f4* tw;  // tw + l: this lane's column
  f2* scratch;   // this wave's
};

// Cross-lane hand-offs through the wave's own LDS scratch need no s_waitcnt between the writes
// and the reads: one wave's DS instructions execute in issue order, so a ds_read issued after a
// ds_write sees it (and a ds_write after a ds_read does not overtake it). Only the compiler must
// not reorder them (it reasons per lane and would move a read above a write it proves disjoint).
__device__ __forceinline__ void ldsOrder() { asm volatile("" ::: "memory"); }

// Digit transposes of NP independent columns through the wave's scratch (NP areas of kXch
// complex): register r of lane l = (a = l & 7, hi = l >> 3) is written to one row, then every lane
// reads its own row of 8 (row l) as four 16-byte reads. The NP columns' writes and reads are
// issued back to back, so one column's LDS latency overlaps the other's. Both layouts are
// bank-conflict free for the 8-byte writes (16-lane groups, 32 banks) and the 16-byte reads
// (ds_read_b128 lane groups, 64 banks) - MI355X_MICROARCH.md LDS table.
//   pattern A: r -> row a + 8 r, col hi; rows kSA = 10 complex apart.
//   pattern B: r -> row 8 hi + r, col a; rows 8 complex apart plus 8 after every 8th row, and
//              the column pairs XOR-swizzled by row & 3: (row, col) at 9 row - row % 8 + (col ^ 2 (row & 3)).
constexpr int kXch = 64 * kSA;  // >= pattern B's 72 x 8
template <int NP>
__device__ __forceinline__ void readRows(f2 (&z)[NP][8], const f2* s, int rowOff, int sw) {
#pragma unroll
  for (int n = 0; n < NP; ++n)
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const f4 v = *reinterpret_cast<const f4*>(s + n * kXch + rowOff + ((2 * c) ^ sw));
      z[n][2 * c] = f2{v.x, v.y};
      z[n][2 * c + 1] = f2{v.z, v.w};
    }
}
// exchangeA in registers (GSDR_FFT_XA_REG): the same permutation - lane a + 8 b, register c receives
// lane a + 8 c, register b - as three butterfly stages of an 8 x 8 transpose over lane bits 3, 4, 5:
// DPP row_ror:8 with bank masks (lane ^ 8, register bit 0), v_permlane16_swap (lane ^ 16, register
// bit 1), v_permlane32_swap (lane ^ 32, register bit 2); no LDS traffic. The swaps are inline asm
// (the builtins lost their second result under this compiler); s_nop 1 covers the VALU-write ->
// v_permlane read hazard.
#ifndef GSDR_FFT_XA_REG
#define GSDR_FFT_XA_REG 0
#endif
template <int BANKS>
__device__ __forceinline__ float dppRor8(float old, float src) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, old), __builtin_bit_cast(int, src),
                                                                0x128, 0xF, BANKS, false));
}
__device__ __forceinline__ void permSwap16(float& a, float& b) {
  asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(a), "+v"(b));
}
__device__ __forceinline__ void permSwap32(float& a, float& b) {
  asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(a), "+v"(b));
}
template <int W>
__device__ __forceinline__ void permSwapC(f2& a, f2& b) {  // both components of two complex registers
  float ax = a.x, ay = a.y, bx = b.x, by = b.y;
  if (W == 16) {
    permSwap16(ax, bx);
    permSwap16(ay, by);
  } else {
    permSwap32(ax, bx);
    permSwap32(ay, by);
  }
  a = f2{ax, ay};
  b = f2{bx, by};
}
template <int NP>
__device__ __forceinline__ void exchangeAReg(f2 (&z)[NP][8]) {
#pragma unroll
  for (int n = 0; n < NP; ++n) {
#pragma unroll
    for (int r = 0; r < 8; r += 2) {
      const f2 p = z[n][r], q = z[n][r + 1];
      z[n][r] = f2{dppRor8<0xC>(p.x, q.x), dppRor8<0xC>(p.y, q.y)};
      z[n][r + 1] = f2{dppRor8<0x3>(q.x, p.x), dppRor8<0x3>(q.y, p.y)};
    }
  }
#pragma unroll
  for (int n = 0; n < NP; ++n)
#pragma unroll
    for (int r : {0, 1, 4, 5}) permSwapC<16>(z[n][r], z[n][r + 2]);
#pragma unroll
  for (int n = 0; n < NP; ++n)
#pragma unroll
    for (int r = 0; r < 4; ++r) permSwapC<32>(z[n][r], z[n][r + 4]);
}

template <int NP>
__device__ __forceinline__ void exchangeA(f2 (&z)[NP][8], f2* s, int l) {
  if constexpr (GSDR_FFT_XA_REG != 0) {
    exchangeAReg<NP>(z);
    return;
  }
  const int a = l & 7, hi = l >> 3;
#pragma unroll
  for (int n = 0; n < NP; ++n)
#pragma unroll
    for (int r = 0; r < 8; ++r) s[n * kXch + (a + 8 * r) * kSA + hi] = z[n][r];
  ldsOrder();
  readRows<NP>(z, s, l * kSA, 0);
  ldsOrder();
}
template <int NP>
__device__ __forceinline__ void exchangeB(f2 (&z)[NP][8], f2* s, int l) {
  const int a = l & 7, hi = l >> 3;
#pragma unroll
  for (int n = 0; n < NP; ++n)
#pragma unroll
    for (int r = 0; r < 8; ++r) s[n * kXch + 72 * hi + 8 * r + (a ^ (2 * (r & 3)))] = z[n][r];
  ldsOrder();
  readRows<NP>(z, s, 72 * hi + 8 * a, 2 * (l & 3));
  ldsOrder();
}

template <int NP>
__device__ __forceinline__ void loadTw(f2 (&t)[7], const Lds& L, int stage) {
#pragma unroll
  for (int kp = 0; kp < 4; ++kp) {
    const f4 v = L.tw[(stage * 4 + kp) * 64];
    t[2 * kp] = f2{v.x, v.y};
    if (2 * kp + 1 < 7) {
      t[2 * kp + 1] = f2{v.z, v.w};
    } else {
      // keep the unused slot 7 live: a whole ds_read_b128 (lanes 16 B apart, conflict free). Loading
      // only t[6], the compiler paired two stages' 8-byte reads into ds_read2st64_b64, whose 16-lane
      // accesses 16 B apart hit every bank pair twice (r05: 2-way conflicts in every FFT)
      float zw0 = v.z, zw1 = v.w;
      asm volatile("" : "+v"(zw0), "+v"(zw1));
    }
  }
}

template <int NP>
__device__ __forceinline__ void twiddleAll(f2 (&z)[NP][8], const f2 (&t)[7]) {
  f2 u[NP][7];
#pragma unroll
  for (int n = 0; n < NP; ++n)
#pragma unroll
    for (int r = 1; r < 8; ++r) u[n][r - 1] = cmul1(z[n][r], t[r - 1]);
#pragma unroll
  for (int n = 0; n < NP; ++n)
#pragma unroll
    for (int r = 1; r < 8; ++r) z[n][r] = cmul2(z[n][r], t[r - 1], u[n][r - 1]);
}

// Forward 512-point DFTs of NP block columns: in: z[n][j] = x_n[l + 64 j];
// out: lane L = 8 k0 + c, z[n][d] = X_n[k0 + 8 c + 64 d] (layout F). Each stage's twiddles are
// loaded a stage ahead (before the exchange that precedes their use) and shared by the columns.
template <int NP>
__device__ __forceinline__ void fftFwd(f2 (&z)[NP][8], const Lds& L, int l) {
  f2 t[7];
  loadTw<NP>(t, L, 0);  // W512^(m1 k0), m1 = l
#pragma unroll
  for (int n = 0; n < NP; ++n) dft8<false>(z[n]);  // over m2 -> k0
  twiddleAll<NP>(z, t);
  loadTw<NP>(t, L, 1);  // W64^(a c)
  exchangeA<NP>(z, L.scratch, l);  // -> lane 8 k0 + a, reg b
#pragma unroll
  for (int n = 0; n < NP; ++n) dft8<false>(z[n]);  // over b -> c
  twiddleAll<NP>(z, t);
  exchangeB<NP>(z, L.scratch, l);  // -> lane 8 k0 + c, reg a
#pragma unroll
  for (int n = 0; n < NP; ++n) dft8<false>(z[n]);  // over a -> d
}

// Inverse (unscaled) 512-point DFTs of NP columns from layout F: out lane L, z[n][h] = y_n[L + 64 h].
// NP = 2 issues both columns' exchange writes before their reads, so one column's LDS round trip
// overlaps the other's (the D = 1 kernel runs one wave per SIMD: nothing else hides it).
template <int NP = 1>
__device__ __forceinline__ void ifft512(f2 (&zz)[NP][8], const Lds& L, int l) {
  f2 t[7];
  loadTw<NP>(t, L, 2);  // W512^-((k0 + 8 c) e)
#pragma unroll
  for (int n = 0; n < NP; ++n) dft8<true>(zz[n]);  // over d -> e (lane 8 k0 + c)
  twiddleAll<NP>(zz, t);
  loadTw<NP>(t, L, 3);  // W64^-(k0 g)
  exchangeB<NP>(zz, L.scratch, l);  // -> lane 8 k0 + e, reg c
#pragma unroll
  for (int n = 0; n < NP; ++n) dft8<true>(zz[n]);  // over c -> g
  twiddleAll<NP>(zz, t);
  exchangeA<NP>(zz, L.scratch, l);  // -> lane e + 8 g, reg k0
#pragma unroll
  for (int n = 0; n < NP; ++n) dft8<true>(zz[n]);  // over k0 -> h
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t blockRsrc(const void* base, int64_t bytes) {
  const int n = bytes <= 0 ? 0 : (bytes > 0x7fffffff ? 0x7fffffff : (int)bytes);
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, n, 0x00020000);
}

// cf32 row-group image: row r of the group at 16-byte unit r kRowUnits<D> (D / 2 units of data).
// Rows D * 8 bytes apart put the ds_read_b128 of lanes 64 / (D / 2) apart on the same banks when D / 2
// is a power of two (D = 8, the D = 1 kernel: 4-way, 15 % of its LDS cycles in SQ_LDS_BANK_CONFLICT).
// D = 4: one pad unit per row spreads a 16-lane group over 16 distinct bank quads. D = 8 (r05): no pad,
// the units of row r XOR-swizzled by (r >> 2) & 3 instead - the padded image (5 units per row) left the
// ds_write_b128 of the transposition 2-way conflicted (8-lane groups over 32 banks: lanes 0 and 7 of
// every group on one bank quad), 8 extra LDS cycles per write, ~260 of the D = 1 kernel's ~350 conflict
// cycles per block (SQ_LDS_BANK_CONFLICT 11.6 % of SQ_LDS_IDX_ACTIVE, r04). With the swizzle a write's
// 8 lanes cover two whole consecutive rows (32 distinct banks) and a ds_read_b128 lane group's 16 lanes
// hit 16 distinct bank quads (the four lanes of a group that share l mod 4 get four distinct swizzles).
#ifndef GSDR_FFT_PADROWS
#define GSDR_FFT_PADROWS 1
#endif
template <int D>
constexpr int kRowUnits = D / 2 + ((GSDR_FFT_PADROWS && D == 4) ? 1 : 0);
template <int D>
__device__ __forceinline__ int rowSwizzle(int row) {
  return D == 8 ? (row >> 2) & 3 : 0;
}

template <int D>
constexpr int scratchComplex(int input) {
  // two exchange areas (2 x kXch) | cf32 row-group image (64 rows x kRowUnits 16-byte units) | int8
  // block image (512 D x 2 B + 16)
  return input == kCf32 ? (128 * kRowUnits<D> > 2 * kXch ? 128 * kRowUnits<D> : 2 * kXch)
                        : ((1024 * D + 16) / 8 > 2 * kXch ? (1024 * D + 16 + 7) / 8 : 2 * kXch);
}

constexpr int kMixT = 8 * 64;  // the row-chirp table T_r, per-lane float4 pairs like G

template <int D, int IN, bool MIX = false>
constexpr size_t ldsBytes() {
  return (size_t)(D * 8 * 64 + kTw + kWaves * scratchComplex<D>(IN) + (MIX ? kMixT : 0)) * sizeof(f2);
}

// Prologue: the twiddle tables and G_p = inScale * conj(DFT_512(h_p)) / 512 in layout F (MIX: times
// c_p, and the row-chirp table T at mixT: f4 (T_j, T_j+1) at (j / 2) 64 + l, rows r = l + 64 j).
template <int D, int IN, int NW = kWaves, bool MIX = false>
__device__ void buildTables(const Args& a, f2* twAll, const Lds& L, int w, int l, f2* mixT = nullptr) {
  if constexpr (MIX) {
    for (int n = threadIdx.x; n < kMixT; n += NW * kWave) {
      const int lane = (n >> 1) & 63, j = 2 * (n >> 7) + (n & 1);
      mixT[n] = turnExp((uint64_t)((lane + 64 * j) * D) * a.mixStep);
    }
  }
  for (int n = threadIdx.x; n < kTw; n += NW * kWave) {
    // complex n = ((stage 4 + kp) 64 + lane) 2 + (k & 1), k = 2 kp + (n & 1), r = k + 1
    const int stage = n >> 9, kp = (n >> 7) & 3, lane = (n >> 1) & 63, r = 2 * kp + (n & 1) + 1;
    const int lo = lane & 7, hi = lane >> 3;
    int e;  // exponent of W512 = exp(-2 pi i / 512)
    switch (stage) {
      case 0: e = lane * r; break;                  // forward: W512^(m1 k0)
      case 1: e = 8 * lo * r; break;                // forward: W64^(a c)
      case 2: e = -(hi + 8 * lo) * r; break;        // inverse: W512^-((k0 + 8 c) e)
      default: e = -8 * hi * r; break;              // inverse: W64^-(k0 g)
    }
    double sn, cs;
    sincospi(-2.0 * e / kM, &sn, &cs);
    twAll[n] = r == 8 ? f2{0.0f, 0.0f} : f2{(float)cs, (float)sn};
  }
  __syncthreads();
  const float sc = a.inScale / (float)kM;
  for (int p = w; p < D; p += NW) {
    f2 z[1][8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int q = l + 64 * j;
      const int t = q * D + p;
      // the correlation y = sum_q h_p[q] x_p[t + q] has the spectrum X . sum_q h_p[q] W^-qk = X . conj(DFT(conj h_p)):
      // the FFT of conj(h_p), conjugated below with the scale (real taps: conj h = h)
      const f2 h = (q < a.Q && t < a.T) ? tapAt(a, t) : f2{0.0f, 0.0f};
      z[0][j] = f2{h.x, -h.y};
    }
    fftFwd<1>(z, L, l);
    if constexpr (MIX) {  // G_p c_p, the product in double and rounded once
      double sn, cs;
      sincospi((double)(int64_t)((uint64_t)p * a.mixStep) * 1.0842021724855044e-19, &sn, &cs);
#pragma unroll
      for (int d = 0; d < 8; ++d) {
        const double gr = (double)z[0][d].x * sc, gi = -(double)z[0][d].y * sc;
        z[0][d] = f2{(float)(gr * cs - gi * sn), (float)(gr * sn + gi * cs)};
      }
#pragma unroll
      for (int d = 0; d < 8; d += 2)
        L.g[(p * 4 + d / 2) * 64 + l] = f4{z[0][d].x, z[0][d].y, z[0][d + 1].x, z[0][d + 1].y};
    } else {
#pragma unroll
      for (int d = 0; d < 8; d += 2)
        L.g[(p * 4 + d / 2) * 64 + l] = f4{z[0][d].x * sc, -z[0][d].y * sc, z[0][d + 1].x * sc, -z[0][d + 1].y * sc};
    }
  }
  __syncthreads();
}

// This lane's row-chirp factors T_{l + 64 j}, j = 0..7.
__device__ __forceinline__ void loadMixT(f2 (&t)[8], const f4* mixT4, int l) {
#pragma unroll
  for (int jp = 0; jp < 4; ++jp) {
    const f4 v = mixT4[jp * 64 + l];
    t[2 * jp] = f2{v.x, v.y};
    t[2 * jp + 1] = f2{v.z, v.w};
  }
}

// The block's rows in registers: rows[j][p] = x[(l + 64 j) D + p] (cf32), or the raw int8 IQ
// words of row l + 64 j (int8: D/2 dwords per row, D even).
template <int D, int IN>
struct Rows;

template <int D>
struct Rows<D, kCf32> {
  f2 v[8][D];
  __device__ __forceinline__ f2 point(int j, int p) const { return v[j][p]; }
};

template <int D>
struct Rows<D, kI8> {
  uint32_t v[8][D / 2];
  // x' = max(x, -127) as float (the 1/127 lives in G)
  __device__ __forceinline__ f2 point(int j, int p) const {
    const uint32_t w = v[j][p >> 1];
    const int sh = (p & 1) * 16;
    const float re = (float)(int)(int8_t)(w >> sh);
    const float im = (float)(int)(int8_t)(w >> (sh + 8));
    return __builtin_elementwise_max(f2{re, im}, f2{-127.0f, -127.0f});
  }
};

// Row group j of the block as loaded (16-byte unit 64 i + l of the group in R.v[j][2i..2i+1]) ->
// rows (R.v[j][p] = x[(l + 64 j) D + p]) through the wave's scratch.
// Row groups transposed per LDS round trip: two images fit the wave's scratch (2 x 64 RU units =
// 2 kXch complex at D = 8, 10), so group j + 1's writes are issued before group j's reads and one
// round trip's latency hides the other's (GSDR_FFT_TPAIR 1). Measured r04: bit-identical and 0.6 %
// slower on C3, 1 % on C4 (the power cap, not LDS latency, sets the pace), so off.
#ifndef GSDR_FFT_TPAIR
#define GSDR_FFT_TPAIR 0
#endif
template <int D>
__device__ __forceinline__ void transposeRows(Rows<D, kCf32>& R, f2* s, int l) {
  constexpr int H = D / 2, RU = kRowUnits<D>;
  constexpr int NG = (GSDR_FFT_TPAIR && 2 * 64 * RU * 2 <= 2 * kXch) ? 2 : 1;  // images per round trip
#pragma unroll
  for (int j0 = 0; j0 < 8; j0 += NG) {
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      f4* s4 = reinterpret_cast<f4*>(s) + g * 64 * RU;
      const int j = j0 + g;
#pragma unroll
      for (int i = 0; i < H; ++i) {  // unit u = 64 i + l of the group: row u / H, unit u % H of it
        const int u = i * 64 + l;
        s4[RU == H ? (u ^ rowSwizzle<D>(u / H)) : (u / H) * RU + u % H] =
            f4{R.v[j][2 * i].x, R.v[j][2 * i].y, R.v[j][2 * i + 1].x, R.v[j][2 * i + 1].y};
      }
    }
    ldsOrder();
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      const f4* s4 = reinterpret_cast<const f4*>(s) + g * 64 * RU;
      const int j = j0 + g;
#pragma unroll
      for (int p = 0; p < D; p += 2) {  // row l: 16-byte reads (D even), lanes 16 RU bytes apart
        const f4 u = s4[l * RU + ((p / 2) ^ rowSwizzle<D>(l))];
        R.v[j][p] = f2{u.x, u.y};
        R.v[j][p + 1] = f2{u.z, u.w};
      }
    }
    ldsOrder();
  }
}

// Row groups loaded non-temporal (bit j: group j), see loadRows.
#ifndef GSDR_FFT_NT_GROUPS
#define GSDR_FFT_NT_GROUPS 0x3C
#endif

// Load block b (rows b V .. b V + 511) and transpose to rows. Loads past the input's end read 0.
template <int D>
__device__ __forceinline__ void loadRows(const Args& a, int64_t b, Rows<D, kCf32>& R, f2* s, int l) {
  static_assert(D % 2 == 0, "cf32 rows: D even (whole 16-byte units per row group)");
  const int64_t off = b * (int64_t)a.V * D * 8;  // byte offset of the block (16-byte aligned)
  const auto rs = blockRsrc((const char*)a.in + off, a.inBytes - off);
  // coalesced: instruction i, lane l -> 16-byte unit 64 i + l; row group j = instructions
  // [j D/2, (j + 1) D/2)
#pragma unroll
  for (int j = 0; j < 8; ++j) {
#pragma unroll
    for (int i = 0; i < D / 2; ++i) {
      // row groups 2-5 are read by this block only: non-temporal (aux 2), which saves fabric energy
      // under the board power cap (C3 runs at 1400 W: time ~ energy); groups 0-1
      // (the previous block's tail) and 6-7 (re-read by the next block) keep the default policy so
      // the overlap stays an L2 hit. C3 490 -> 485 us, profiles/r03/exp/fft_nt_mid_ab.log
      const int off = ((j * D / 2 + i) * 64 + l) * 16;
      const f4 u = (GSDR_FFT_EXP & 2) ? f4{(float)(l + i), (float)j, (float)(b & 7), 1.0f}
                   : ((GSDR_FFT_NT_GROUPS >> j) & 1) ? __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 2))
                                                     : __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
      R.v[j][2 * i] = f2{u.x, u.y};
      R.v[j][2 * i + 1] = f2{u.z, u.w};
    }
  }
  if (GSDR_FFT_EXP & 4) return;
  transposeRows<D>(R, s, l);
}

template <int D>
__device__ __forceinline__ void loadRows(const Args& a, int64_t b, Rows<D, kI8>& R, f2* s, int l) {
  static_assert(D % 2 == 0, "int8 rows: D even (dword-aligned rows)");
  const int64_t off = b * (int64_t)a.V * D * 2;        // byte offset of the block
  const char* base = (const char*)a.in + off;
  const int mis = (int)((uintptr_t)base & 15);         // 0, 4, 8 or 12 (4-byte aligned input)
  const char* abase = base - mis;
  // the range check is per dword: round the readable range up to whole dwords so the final
  // 2-byte sample is not dropped with its dword (the extra <= 2 bytes share that dword, so the
  // load stays inside the allocation's last page; they only feed rows past the input's end)
  const auto rs = blockRsrc(abase, (a.inBytes - off + mis + 3) & ~(int64_t)3);
  constexpr int kUnits = (1024 * D + 16) / 16;         // covers mis + 1024 D bytes
  constexpr int kInstr = (kUnits + 63) / 64;
  f4* s4 = reinterpret_cast<f4*>(s);
  uint4 u[kInstr];
#pragma unroll
  for (int i = 0; i < kInstr; ++i) {
    const int unit = i * 64 + l;
    u[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, unit * 16, 0, 0));
  }
#pragma unroll
  for (int i = 0; i < kInstr; ++i) {
    const int unit = i * 64 + l;
    if (unit < kUnits) s4[unit] = __builtin_bit_cast(f4, u[i]);
  }
  ldsOrder();
  const uint32_t* s1 = reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(s) + mis);
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int p = 0; p < D / 2; ++p) R.v[j][p] = s1[(l + 64 * j) * (D / 2) + p];
  ldsOrder();
}

// Accuracy guard. The FFT's round-off is relative to the block's level; the tolerance is relative to
// each output's own window sum_j |h_j||x_kD+j|. The block is split into segments of >= 16
// consecutive samples (GL adjacent rows, i.e. adjacent lanes); if the loudest segment's level
// (root of its energy sum |x|^2) exceeds guardRatio times the quietest, or the block holds inf / NaN, the
// block is recomputed in the direct form. Rows past the input's end (the last block) are ignored.
template <int D>
constexpr int guardLanes() {
  return D >= 16 ? 1 : (D >= 8 ? 2 : (D >= 4 ? 4 : 8));  // GL rows = GL * D >= 16 samples
}

template <int D, int IN>
__device__ __forceinline__ bool blockNeedsDirect(const Args& a, const Rows<D, IN>& R, int64_t b, int l) {
  constexpr int GL = guardLanes<D>();
  // rows of this block inside the input, as a 32-bit wave-uniform bound (lane math stays 32-bit:
  // no 64-bit per-lane constants for the compiler to keep live across the block loop)
  const int64_t vr64 = a.inRows - b * (int64_t)a.V;
  const int validRows = __builtin_amdgcn_readfirstlane((int)(vr64 < kM ? vr64 : kM));
  float lo = INFINITY, hi = 0.0f;
  bool nonFinite = false;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    f2 e2 = {0.0f, 0.0f};  // segment energy sum |x|^2, one packed FMA per sample
#pragma unroll
    for (int p = 0; p < D; ++p) {
      const f2 z = R.point(j, p);
      e2 = __builtin_elementwise_fma(z, z, e2);
    }
    float lvl = e2.x + e2.y;
#pragma unroll
    for (int m = 1; m < GL; m <<= 1) lvl += __shfl_xor(lvl, m);
    // the segment = lanes (l & ~(GL-1)) .. + GL - 1 of row group j; whole inside the input?
    if (((l | (GL - 1)) + 64 * j) < validRows) {
      nonFinite |= !(lvl < INFINITY);  // inf or NaN (fminf / fmaxf would drop a NaN)
      lo = fminf(lo, lvl);
      hi = fmaxf(hi, lvl);
    }
  }
  lo = waveMinNonNeg(lo);
  hi = waveMaxNonNeg(hi);
  return __any(nonFinite) || !(hi <= a.guardRatio * a.guardRatio * lo);
}

// Direct-form fallback for one block (outputs b V + m, m < V): lane l computes m = l + 64 h.
template <int D, int IN, int EPI, bool MIX = false>
__device__ void directBlock(const Args& a, int64_t b, int l) {
  const int64_t k0 = b * (int64_t)a.V;
  const int64_t left = a.nOut - k0;
  const int nv = __builtin_amdgcn_readfirstlane((int)(left < a.V ? left : a.V));  // outputs of this block
  const int64_t base = k0 * D;  // the block's first input sample (scalar)
  for (int h = 0; h < 8; ++h) {
    const int m = l + 64 * h;
    if (m >= nv) continue;
    // blocked sums (64 taps per partial, then added to the running total), as the other direct
    // forms: a plain 1023-term chain can exceed the 1e-6 sum|h||x| tolerance
    float re = 0.0f, im = 0.0f;
    for (int t0 = 0; t0 < a.T; t0 += 64) {
      const int t1 = t0 + 64 < a.T ? t0 + 64 : a.T;
      float pr = 0.0f, pi = 0.0f;
      for (int t = t0; t < t1; ++t) {
        const f2 hc = tapAt(a, t);
        float xr, xi;
        if (IN == kCf32) {
          const f2 x = (reinterpret_cast<const f2*>(a.in) + base)[m * D + t];
          xr = x.x;
          xi = x.y;
        } else {
          const int8_t* iq = reinterpret_cast<const int8_t*>(a.in) + 2 * base + 2 * (m * D + t);
          xr = int8ToNorm(iq[0]);
          xi = int8ToNorm(iq[1]);
        }
        if constexpr (MIX) {
          const f2 zm = mixOne(a, base + m * D + t, f2{xr, xi});
          xr = zm.x;
          xi = zm.y;
        }
        pr = fmaf(hc.x, xr, fmaf(-hc.y, xi, pr));
        pi = fmaf(hc.x, xi, fmaf(hc.y, xr, pi));
      }
      re += pr;
      im += pi;
    }
    if (EPI == kAm)
      (reinterpret_cast<float*>(a.out) + k0)[m] = amEnvelope(f2{re, im});
    else
      (reinterpret_cast<f2*>(a.out) + k0)[m] = f2{re, im};
  }
}

// The block's outputs from its rows: D forward FFTs (two phases at a time), Y = sum_p X_p G_p,
// one inverse FFT, the first V outputs stored (AM envelope or complex).
// MIX with int8 rows: `t` holds this lane's row-chirp factors, applied as the points are formed
// (cf32 rows were rotated when they landed).
template <int D, int IN, int EPI, bool MIX = false>
__device__ __forceinline__ void convolveBlock(const Args& a, const Rows<D, IN>& R, int64_t b, const Lds& L, int l,
                                              const f2* t = nullptr) {
  constexpr int NP = (D % 2 == 0) ? 2 : 1;  // phases transformed together
  f2 acc[1][8];
#pragma unroll
  for (int d = 0; d < 8; ++d) acc[0][d] = f2{0.0f, 0.0f};
#pragma unroll
  for (int p = 0; p < D; p += NP) {
    f2 z[NP][8];
#pragma unroll
    for (int n = 0; n < NP; ++n)
#pragma unroll
      for (int j = 0; j < 8; ++j) z[n][j] = (MIX && IN == kI8) ? cmul(R.point(j, p + n), t[j]) : R.point(j, p + n);
    if (!(GSDR_FFT_EXP & 1)) fftFwd<NP>(z, L, l);
#pragma unroll
    for (int n = 0; n < NP; ++n) {
      f2 g[8], u[8];
#pragma unroll
      for (int d = 0; d < 8; d += 2) {
        const f4 v = L.g[((p + n) * 4 + d / 2) * 64 + l];
        g[d] = f2{v.x, v.y};
        g[d + 1] = f2{v.z, v.w};
      }
#pragma unroll
      for (int d = 0; d < 8; ++d) u[d] = cmac1(z[n][d], g[d], acc[0][d]);
#pragma unroll
      for (int d = 0; d < 8; ++d) acc[0][d] = cmul2(z[n][d], g[d], u[d]);
    }
  }
  if (!(GSDR_FFT_EXP & 1)) ifft512(acc, L, l);
  if constexpr (MIX && EPI != kAm) {  // the block's factor E_b (|E_b y| = |y|: AM needs none)
    const f2 eb = turnExpF(a.mixPhase0 + (uint64_t)(b * (int64_t)a.V * D) * a.mixStep);
#pragma unroll
    for (int h = 0; h < 8; ++h) acc[0][h] = cmul(acc[0][h], eb);
  }
  // outputs k0 + m, m < nv: the bound and the base are wave-uniform, so the lane math stays
  // 32-bit (per-lane 64-bit output indices were spilled to scratch, and each reload between the
  // stores waited for the stores before it: s_waitcnt vmcnt(0))
  const int64_t k0 = b * (int64_t)a.V;
  const int64_t left = a.nOut - k0;
  const int nv = __builtin_amdgcn_readfirstlane((int)(left < a.V ? left : a.V));
#pragma unroll
  for (int h = 0; h < 8; ++h) {
    const int m = l + 64 * h;
    if (m < nv && !((GSDR_FFT_EXP & 16) && a.T > 0)) {
      if (EPI == kAm)
        (reinterpret_cast<float*>(a.out) + k0)[m] = amEnvelope(acc[0][h]);
      else
        (reinterpret_cast<f2*>(a.out) + k0)[m] = acc[0][h];
    }
  }
}

// Workgroup i runs on XCD i mod 8 (round-robin dispatch). Logical group (i mod 8) n / 8 + i / 8 puts
// consecutive logical groups - whose blocks share their overlap rows - on one XCD, so the re-read
// rows meet in that XCD's L2 rather than travelling from the fabric twice.
#ifndef GSDR_FFT_XCD
#define GSDR_FFT_XCD 1
#endif
__device__ __forceinline__ int xcdGroup(int i, int n) {
  if (!GSDR_FFT_XCD || (n & 7) != 0) return i;
  return (i & 7) * (n >> 3) + (i >> 3);
}
// The D >= 2 kernel's workgroup order (1: xcdGroup, A/B builds; r02 measured it neutral at C3).
#ifndef GSDR_FFT_XCD_D
#define GSDR_FFT_XCD_D 0
#endif

template <int D, int IN, int EPI, bool MIX = false>
__global__ void __launch_bounds__(kThreads) firFftKernel(Args a) {
  extern __shared__ __attribute__((aligned(16))) f2 lds[];
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), l = threadIdx.x & 63;
  f2* twAll = lds + D * 8 * 64;
  f2* mixT = twAll + kTw + kWaves * scratchComplex<D>(IN);
  Lds L;
  L.g = reinterpret_cast<f4*>(lds);
  L.tw = reinterpret_cast<const f4*>(twAll) + l;
  L.scratch = twAll + kTw + w * scratchComplex<D>(IN);
  buildTables<D, IN, kWaves, MIX>(a, twAll, L, w, l, mixT);
#if GSDR_FFT_STAMPS
  const unsigned long long st0 = __builtin_amdgcn_s_memtime(), rt0 = __builtin_amdgcn_s_memrealtime();
#endif

  // round r: workgroup g's wave w takes block (r * groups + g) * kWaves + w, so in every round
  // the grid streams one contiguous stretch of the input (DRAM-friendly, like a grid-stride copy)
  // and a workgroup's waves read adjacent blocks (their overlapping rows are L2 hits). The two waves
  // of a SIMD do not progress alike (r04 stamps: waves 0-3 of a workgroup span ~414 us, waves 4-7
  // ~452 us of a 478 us launch), but evening that out does not pay: handing the workgroup's blocks to
  // its waves from an LDS counter, or the last rounds to any free wave from a grid-wide counter, made
  // every span ~the old maximum and the launch 1.5-5 % slower (the SIMD's throughput is the same
  // whether one or two waves run it at the end).
  const int64_t stride = (int64_t)gridDim.x * kWaves;
  const int grp = GSDR_FFT_XCD_D ? xcdGroup((int)blockIdx.x, (int)gridDim.x) : (int)blockIdx.x;
  for (int64_t b = (int64_t)grp * kWaves + w; b < a.nBlocks; b += stride) {
    Rows<D, IN> R;
    loadRows<D>(a, b, R, L.scratch, l);
    f2 t[8];
    if constexpr (MIX) {  // the row chirp: cf32 rows rotated here, int8 rows as they become points
      loadMixT(t, reinterpret_cast<const f4*>(mixT), l);
      if constexpr (IN == kCf32) {
#pragma unroll
        for (int j = 0; j < 8; ++j)
#pragma unroll
          for (int p = 0; p < D; ++p) R.v[j][p] = cmul(R.v[j][p], t[j]);
      }
    }
    if (!(GSDR_FFT_EXP & 8) && blockNeedsDirect<D, IN>(a, R, b, l)) {
      if (l == 0) atomicAdd(&gDirectBlocks, 1ull);
      directBlock<D, IN, EPI, MIX>(a, b, l);
      continue;
    }
    // The two waves of a SIMD overlap one's loads with the other's FFTs only while they are out
    // of phase. The wave in its FFT part runs at raised issue priority, so it is not slowed by
    // the other wave's transposition and guard work: it finishes first and the pair settles into
    // alternation - C3 513 -> 487 us per launch (tools/exp/run_fft_variants.sh, bit-identical).
    // This replaces the start-up stagger (s_sleep for half the waves) of earlier builds, which
    // is neutral on top of it.
    __builtin_amdgcn_s_setprio(2);
    convolveBlock<D, IN, EPI, MIX>(a, R, b, L, l, t);
    __builtin_amdgcn_s_setprio(0);
  }
#if GSDR_FFT_STAMPS
  const unsigned long long st1 = __builtin_amdgcn_s_memtime(), rt1 = __builtin_amdgcn_s_memrealtime();
  const int slot = (int)blockIdx.x * kWaves + w;
  if (l == 0 && slot < kStampWaves) {
    unsigned long long* s = gFftStamps + 4 * slot;
    s[0] = st0;
    s[1] = rt0;
    s[2] = st1;
    s[3] = rt1;
  }
#endif
}

// ---- one wave per SIMD with the next block's loads in flight (D = 1) ---------------------------
// The 8-wave kernels overlap loads with FFT math only through their two waves per SIMD running out
// of phase (the rows take 128-160 VGPRs). firFftD1PfKernel runs ONE wave per SIMD (the whole
// 512-entry register file) and loads the next block (32 buffer_load_dwordx4 per lane, 128
// registers) while the current block is transformed: the compiler places the in-flight block in
// AGPRs (the half of the file VALU code does not otherwise use) and waits for it only when the
// next iteration drains it into VGPRs. Measured (tools/exp/run_fft_variants.sh, one box): C4
// 892 -> 850 us per 2^27 samples, bit-identical. The same scheme at D = 10 (C3) is SLOWER (543 ->
// 640 us): one wave per SIMD exposes the LDS latency of the transposes and FFT exchanges, which
// the 8-wave kernel hides behind its second wave, and the D = 10 block has 6x less FFT work per
// loaded byte to hide the loads under.
constexpr int kPfWaves = 4;

template <int D>
struct PrefetchCf {
  f4 u[8][D / 2];  // 16-byte unit 64 i + l of row group j, in AGPRs
};

// Issue block b's loads (past the input's end, or past the last block, they read zeros).
template <int D>
__device__ __forceinline__ void issueBlockLoads(const Args& a, int64_t b, PrefetchCf<D>& P, int l) {
  const int64_t off = b < a.nBlocks ? b * (int64_t)a.V * D * 8 : 0;
  const auto rs = blockRsrc((const char*)a.in + off, b < a.nBlocks ? a.inBytes - off : 0);
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int i = 0; i < D / 2; ++i)
      P.u[j][i] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rs, ((j * D / 2 + i) * 64 + l) * 16, 0, 0));
}

template <int D>
__device__ __forceinline__ void drainBlockLoads(const PrefetchCf<D>& P, Rows<D, kCf32>& R) {
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int i = 0; i < D / 2; ++i) {
      const f4 u = P.u[j][i];
      R.v[j][2 * i] = f2{u.x, u.y};
      R.v[j][2 * i + 1] = f2{u.z, u.w};
    }
}

// ---- D = 1: a 4096-point overlap-save FFT as eight 512-point FFTs and a radix-8 phase stage ------
// With k = 8m + r and j = 8q + p (p, r < 8), y[8m + r] = sum_p sum_q h_p[q] x_{(p+r) mod 8}[m + q + c],
// c = (p + r >= 8), x_t[n] = x[8n + t], h_p[q] = h[8q + p]: each output phase r is an 8-phase
// polyphase correlation of the SAME input phases, some advanced by one row. A block of 512 rows (8
// samples each) is transformed once per input phase (8 forward 512-point FFTs X_t, in registers in
// place of the rows). Per frequency k, Y_r = sum_t X_t G_{(t - r) mod 8} (w^k if t < r), w^k =
// exp(+2 pi i k / 512) the one-row advance. With alpha = exp(+2 pi i k / 4096) (alpha^8 = w^k) the
// twist X~_t = alpha^-t X_t, G~_s = alpha^s G_s turns that into a plain circular correlation over
// the phase index, alpha^-r Y_r = sum_s X~_{(r + s) mod 8} G~_s, which an 8-point DFT over the
// phases diagonalises: A_f = DFT8_t(X~_t), B_f = (1/8) sum_s G~_s W8^-fs (built once per launch, in
// place of G), alpha^-r Y_r = IDFT8_f(A_f B_f). Per frequency 7 + 8 + 7 complex products and two
// in-register 8-point DFTs instead of 64 complex MACs and 7 twists (r02-r03a), and 88 instead of 256
// table reads per lane and block. (This is the decimation-in-time radix-8 stage of a 4096-point
// FFT of the block and its decimation-in-frequency inverse: the same overlap-save, valid for
// m < V = 512 - Q.) Then one inverse 512-point FFT per output phase.
constexpr int kTwD1 = 7 * 8 * 64;  // alpha^-t, t = 1..7: per-lane float4 pairs like G


template <int EPI>
__device__ void directBlockD1(const Args& a, int64_t b, int l) {
  const int64_t k0 = b * (int64_t)a.V * 8;  // first output of the block
  const int64_t left = a.nOut - k0;
  const int nv = __builtin_amdgcn_readfirstlane((int)(left < 8 * a.V ? left : 8 * a.V));
  for (int i = l; i < nv; i += 64) {
    float re = 0.0f, im = 0.0f;
    for (int t0 = 0; t0 < a.T; t0 += 64) {  // blocked sums, as the other direct forms
      const int t1 = t0 + 64 < a.T ? t0 + 64 : a.T;
      float pr = 0.0f, pi = 0.0f;
      for (int t = t0; t < t1; ++t) {
        const f2 x = reinterpret_cast<const f2*>(a.in)[k0 + i + t];
        const f2 hc = tapAt(a, t);
        pr = fmaf(hc.x, x.x, fmaf(-hc.y, x.y, pr));
        pi = fmaf(hc.x, x.y, fmaf(hc.y, x.x, pi));
      }
      re += pr;
      im += pi;
    }
    if (EPI == kAm)
      reinterpret_cast<float*>(a.out)[k0 + i] = amEnvelope(f2{re, im});
    else
      reinterpret_cast<f2*>(a.out)[k0 + i] = f2{re, im};
  }
}

// After buildTables (G_s in layout F at gAll, barrier passed): G_s -> B_f in place and the twist
// table alpha^-t, in double, rounded once. Complex slot n of a phase's 512 (layout F: n = ((d / 2)
// 64 + lane) 2 + (d & 1), frequency k = k0 + 8 c + 64 d for lane 8 k0 + c) is read and written only
// by thread n mod threads, so no barrier is needed between the reads and the writes.
__device__ __forceinline__ void buildPhaseTablesD1(f2* gAll, f2* twist, int threads) {
  for (int n = threadIdx.x; n < kM; n += threads) {
    const int lane = (n >> 1) & 63, d = 2 * (n >> 7) + (n & 1);
    const int k = (lane >> 3) + 8 * (lane & 7) + 64 * d;
    double gr[8], gi[8];
#pragma unroll
    for (int s = 0; s < 8; ++s) {  // G~_s = alpha^s G_s
      double sn, cs;
      sincospi(2.0 * (double)(k * s) / 4096.0, &sn, &cs);
      const f2 g = gAll[s * kM + n];
      gr[s] = (double)g.x * cs - (double)g.y * sn;
      gi[s] = (double)g.x * sn + (double)g.y * cs;
    }
#pragma unroll
    for (int f = 0; f < 8; ++f) {  // B_f = (1/8) sum_s G~_s exp(+2 pi i f s / 8)
      double br = 0.0, bi = 0.0;
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        double sn, cs;
        sincospi((double)((f * s) & 7) / 4.0, &sn, &cs);
        br += gr[s] * cs - gi[s] * sn;
        bi += gr[s] * sn + gi[s] * cs;
      }
      gAll[f * kM + n] = f2{(float)(br * 0.125), (float)(bi * 0.125)};
    }
#pragma unroll
    for (int t = 1; t < 8; ++t) {
      double sn, cs;
      sincospi(-2.0 * (double)(k * t) / 4096.0, &sn, &cs);
      twist[(t - 1) * kM + n] = f2{(float)cs, (float)sn};
    }
  }
}

// Eight factors of one table row (t, or f for B) for this lane: f4 pairs at (row 4 + d / 2) 64 from
// tab, which already points at this lane's column.
__device__ __forceinline__ void loadRow8(f2 (&v)[8], const f4* tab, int row) {
#pragma unroll
  for (int d = 0; d < 8; d += 2) {
    const f4 u = tab[(row * 4 + d / 2) * 64];
    v[d] = f2{u.x, u.y};
    v[d + 1] = f2{u.z, u.w};
  }
}

// One D = 1 block: the eight input-phase spectra, the phase stage, then per output phase one
// inverse FFT and the stores.
template <int EPI>
__device__ __forceinline__ void convolveBlockD1(const Args& a, const Rows<8, kCf32>& R, int64_t b, const Lds& L,
                                                const f4* twist, int l) {
  constexpr int D = 8;
  // the eight input-phase spectra, in place of the rows
  f2 X[D][8];
#pragma unroll
  for (int p = 0; p < D; p += 2) {
    f2 z[2][8];
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int j = 0; j < 8; ++j) z[n][j] = R.point(j, p + n);
    fftFwd<2>(z, L, l);
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int d = 0; d < 8; ++d) X[p + n][d] = z[n][d];
  }
  // X~_t = alpha^-t X_t (the halves of each row's eight products issued stage-interleaved: a
  // v_pk_fma right behind the one that writes its operand costs an s_nop, and one wave per SIMD
  // has nothing to hide it behind)
#pragma unroll
  for (int t = 1; t < D; ++t) {
    f2 w[8], u[8];
    loadRow8(w, twist, t - 1);
#pragma unroll
    for (int d = 0; d < 8; ++d) u[d] = cmul1(X[t][d], w[d]);
#pragma unroll
    for (int d = 0; d < 8; ++d) X[t][d] = cmul2(X[t][d], w[d], u[d]);
  }
  // A_f = DFT8 over the phases, times B_f, inverse DFT8: alpha^-r Y_r in X[r]
#pragma unroll
  for (int d = 0; d < 8; ++d) {
    f2 z[8];
#pragma unroll
    for (int t = 0; t < D; ++t) z[t] = X[t][d];
    dft8<false>(z);
#pragma unroll
    for (int f = 0; f < D; ++f) X[f][d] = z[f];
  }
#pragma unroll
  for (int f = 0; f < D; ++f) {
    f2 g[8], u[8];
    loadRow8(g, L.g + l, f);
#pragma unroll
    for (int d = 0; d < 8; ++d) u[d] = cmul1(X[f][d], g[d]);
#pragma unroll
    for (int d = 0; d < 8; ++d) X[f][d] = cmul2(X[f][d], g[d], u[d]);
  }
#pragma unroll
  for (int d = 0; d < 8; ++d) {
    f2 z[8];
#pragma unroll
    for (int f = 0; f < D; ++f) z[f] = X[f][d];
    dft8<true>(z);
#pragma unroll
    for (int r = 0; r < D; ++r) X[r][d] = z[r];
  }
  const int64_t row0 = b * (int64_t)a.V;
  // outputs 8 (row0 + m) + r: row m = l + 64 h of output phase r lands in lane l, register h
  float am[D][8];  // EPI == kAm: the envelopes (the complex results go back into X[r])
  // Output phases inverse-transformed together. Pairs (their exchanges' LDS round trips overlapped)
  // measured SLOWER: C4 678 -> 752 us per 2^27 samples (profiles/r04/exp/fft_d1_ifft_pairs_ab.log;
  // the larger live set costs the one-wave-per-SIMD schedule more than the overlap gains). The wave's
  // scratch holds two exchange columns, so at most 2.
#ifndef GSDR_FFT_D1_IFFT_NP
#define GSDR_FFT_D1_IFFT_NP 1
#endif
  constexpr int INP = GSDR_FFT_D1_IFFT_NP;
  static_assert(INP == 1 || INP == 2, "the wave's scratch holds two exchange columns");
#pragma unroll
  for (int r0 = 0; r0 < D; r0 += INP) {
    f2 acc[INP][8];
#pragma unroll
    for (int n = 0; n < INP; ++n) {
      const int r = r0 + n;
      if (r > 0) {  // Y_r = alpha^r (alpha^-r Y_r): times the conjugate of the twist row r
        f2 w[8], u[8];
        loadRow8(w, twist, r - 1);
#pragma unroll
        for (int d = 0; d < 8; ++d) u[d] = cmul1(X[r][d], w[d]);
#pragma unroll
        for (int d = 0; d < 8; ++d) acc[n][d] = cmulc2(X[r][d], w[d], u[d]);
      } else {
#pragma unroll
        for (int d = 0; d < 8; ++d) acc[n][d] = X[0][d];
      }
    }
    ifft512<INP>(acc, L, l);
#pragma unroll
    for (int n = 0; n < INP; ++n)
#pragma unroll
      for (int h = 0; h < 8; ++h) {
        if (EPI == kAm) am[r0 + n][h] = amEnvelope(acc[n][h]);
        else X[r0 + n][h] = acc[n][h];
      }
  }
  // row m's eight phases are 8 consecutive outputs: stored as 16-byte units (lanes 32 / 64 bytes
  // apart, the whole row range of a register h in one sweep) - phase-strided 4-byte stores left
  // lines partially written and cost 1.31x the output bytes in WRITE_SIZE (C4, r03 profile)
  const int64_t left = a.nOut - 8 * row0;
  const int64_t rows = left <= 0 ? 0 : (left + 7) / 8;
  const int nv = __builtin_amdgcn_readfirstlane((int)(rows < a.V ? rows : a.V));
  const bool whole = left >= 8 * (int64_t)a.V;  // wave-uniform: every row of the block is complete
#pragma unroll
  for (int h = 0; h < 8; ++h) {
    const int m = l + 64 * h;
    if (m >= nv) continue;
    const int64_t k0 = 8 * (row0 + m);
    if (EPI == kAm) {
      float* o = reinterpret_cast<float*>(a.out) + k0;
      if (whole && a.outAligned) {
        reinterpret_cast<f4*>(o)[0] = f4{am[0][h], am[1][h], am[2][h], am[3][h]};
        reinterpret_cast<f4*>(o)[1] = f4{am[4][h], am[5][h], am[6][h], am[7][h]};
      } else {
#pragma unroll
        for (int r = 0; r < D; ++r)
          if (k0 + r < a.nOut) o[r] = am[r][h];
      }
    } else {
      f2* o = reinterpret_cast<f2*>(a.out) + k0;
      if (whole && a.outAligned) {
#pragma unroll
        for (int r = 0; r < D; r += 2) reinterpret_cast<f4*>(o)[r / 2] = f4{X[r][h].x, X[r][h].y, X[r + 1][h].x, X[r + 1][h].y};
      } else {
#pragma unroll
        for (int r = 0; r < D; ++r)
          if (k0 + r < a.nOut) o[r] = X[r][h];
      }
    }
  }
}

// D = 1 with one wave per SIMD and the next block's loads in flight into AGPRs (as firFftPfKernel).
template <int EPI>
__global__ void __launch_bounds__(kPfWaves * kWave) __attribute__((amdgpu_waves_per_eu(1, 1)))
firFftD1PfKernel(Args a) {
  constexpr int D = 8;
  extern __shared__ __attribute__((aligned(16))) f2 lds[];
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), l = threadIdx.x & 63;
  f2* twAll = lds + D * 8 * 64;
  f2* twistAll = twAll + kTw + kPfWaves * scratchComplex<D>(kCf32);
  Lds L;
  L.g = reinterpret_cast<f4*>(lds);
  L.tw = reinterpret_cast<const f4*>(twAll) + l;
  L.scratch = twAll + kTw + w * scratchComplex<D>(kCf32);
  buildTables<D, kCf32, kPfWaves>(a, twAll, L, w, l);
  buildPhaseTablesD1(lds, twistAll, kPfWaves * kWave);
  __syncthreads();
  const f4* twist = reinterpret_cast<const f4*>(twistAll) + l;
  const int64_t stride = (int64_t)gridDim.x * kPfWaves;
  int64_t b = (int64_t)xcdGroup((int)blockIdx.x, (int)gridDim.x) * kPfWaves + w;
  PrefetchCf<D> P;
  issueBlockLoads<D>(a, b, P, l);
  for (; b < a.nBlocks; b += stride) {
    Rows<D, kCf32> R;
    drainBlockLoads<D>(P, R);
    issueBlockLoads<D>(a, b + stride, P, l);
    transposeRows<D>(R, L.scratch, l);
    if (blockNeedsDirect<D, kCf32>(a, R, b, l)) {
      if (l == 0) atomicAdd(&gDirectBlocks, 1ull);
      directBlockD1<EPI>(a, b, l);
      continue;
    }
    convolveBlockD1<EPI>(a, R, b, L, twist, l);
  }
}

}  // namespace fftfir

// ------------------------------------------------------------------------------------ host
namespace {

std::atomic<float> gFftGuard{8.0f};

int cuCount() {
  int dev = 0, n = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
    return 256;
  return n;
}

template <int D, int IN, int EPI, bool MIX>
hipError_t launchD(fftfir::Args a, hipStream_t stream) {
  using namespace fftfir;
  auto kernel = firFftKernel<D, IN, EPI, MIX>;
  const size_t lds = ldsBytes<D, IN, MIX>();
  // set per launch (cheap): a once-per-process flag would race between threads and miss other devices
  const hipError_t e = hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  const int64_t maxGroups = cuCount();
  int64_t groups = (a.nBlocks + kWaves - 1) / kWaves;
  if (groups > maxGroups) groups = maxGroups;

  hipLaunchKernelGGL(kernel, dim3((unsigned)groups), dim3(kThreads), lds, stream, a);
  return hipGetLastError();
}

template <int EPI>
hipError_t launchD1(fftfir::Args a, hipStream_t stream) {
  using namespace fftfir;
  auto kernel = firFftD1PfKernel<EPI>;
  const size_t lds = (size_t)(8 * 8 * 64 + kTw + kPfWaves * scratchComplex<8>(kCf32) + kTwD1) * sizeof(f2);
  // set per launch (cheap): a once-per-process flag would race between threads and miss other devices
  const hipError_t e = hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  const int64_t maxGroups = cuCount();
  int64_t groups = (a.nBlocks + kPfWaves - 1) / kPfWaves;
  if (groups > maxGroups) groups = maxGroups;
  hipLaunchKernelGGL(kernel, dim3((unsigned)groups), dim3(kPfWaves * kWave), lds, stream, a);
  return hipGetLastError();
}

template <int IN, int EPI, bool MIX = false>
hipError_t launchFft(fftfir::Args a, size_t D, hipStream_t stream) {
  switch (D) {
    case 2: return launchD<2, IN, EPI, MIX>(a, stream);
    case 4: return launchD<4, IN, EPI, MIX>(a, stream);
    case 6: return launchD<6, IN, EPI, MIX>(a, stream);
    case 8: return launchD<8, IN, EPI, MIX>(a, stream);
    case 10: return launchD<10, IN, EPI, MIX>(a, stream);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace

#if GSDR_FFT_STAMPS
// Diagnostic builds: the stamps of the last firFftKernel launch (4 per wave, kStampWaves waves).
hipError_t fftStampsRead(unsigned long long* host, size_t count) {
  if (count > (size_t)fftfir::kStampWaves * 4) count = (size_t)fftfir::kStampWaves * 4;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(fftfir::gFftStamps), count * sizeof(unsigned long long));
}
#endif

// Eligible: real taps (FC), D in {2,4,6,8,10}, enough taps that the FFT beats the direct forms,
// at least 64 outputs per block, and the loads' alignment (cf32: 16-byte input; int8 IQ: 4-byte).
bool firFftEligible(size_t tapCount, size_t decimation, const void* in, bool int8Iq, bool mixed) {
  const size_t D = decimation < 1 ? 1 : decimation;
  if (D == 1) {  // cf32: eight output phases per block (firFftD1PfKernel), up to 3 584 taps
    if (mixed) return false;
    const size_t Q = (tapCount + 7) / 8;
    return !int8Iq && tapCount >= 256 && Q <= (size_t)fftfir::kM - 64 && ((uintptr_t)in & 15) == 0;
  }
  if (!(D == 2 || D == 4 || D == 6 || D == 8 || D == 10)) return false;
  const size_t Q = (tapCount + D - 1) / D;
  if (tapCount < 256 || Q > (size_t)fftfir::kM - 63) return false;
  const uintptr_t p = (uintptr_t)in;
  // int8 IQ: the exact f16 MFMA kernels are faster where they apply (C5 RF stage, 125 M samples:
  // 195 us wave-specialised MFMA vs 263 us FFT); the FFT takes the shapes they cannot
  if (int8Iq)
    return (p & 3) == 0 && (mixed || (kernelPolicy() & GSDR_POLICY_PREFER_FFT) != 0 ||
                            (!firI8MfmaEligible(tapCount, decimation, in) && !firI8DecMfmaEligible(tapCount, decimation, in)));
  return (p & 15) == 0;
}

hipError_t launchFirFft(const void* in, bool int8Iq, const float* taps, size_t tapCount, size_t decimation,
                        void* out, size_t nOut, int epi, hipStream_t stream, FftMix mix, bool complexTaps) {
  using namespace fftfir;
  if (nOut == 0) return hipSuccess;
  if (complexTaps && (int8Iq || mix.on)) return hipErrorInvalidValue;
  const size_t D = decimation < 1 ? 1 : decimation;
  if (D == 1) {
    if (int8Iq || mix.on) return hipErrorInvalidValue;
    Args a{};
    a.in = in;
    a.taps = taps;
    a.out = out;
    a.nOut = (int64_t)nOut;
    a.T = (int32_t)tapCount;
    a.Q = (int32_t)((tapCount + 7) / 8);
    a.V = kM - a.Q;  // rows per block: the one-row advance costs one
    a.inBytes = (int64_t)(nOut - 1 + tapCount) * 8;
    a.nBlocks = ((int64_t)nOut + 8 * (int64_t)a.V - 1) / (8 * (int64_t)a.V);
    a.inRows = (int64_t)((nOut - 1 + tapCount) / 8);
    a.inScale = 1.0f;
    a.guardRatio = gFftGuard.load(std::memory_order_relaxed);
    a.outAligned = ((uintptr_t)out & 15) == 0;
    a.complexTaps = complexTaps ? 1 : 0;
    return epi == kEpiAm ? launchD1<kAm>(a, stream) : launchD1<kComplex>(a, stream);
  }
  Args a{};
  a.in = in;
  a.taps = taps;
  a.out = out;
  a.nOut = (int64_t)nOut;
  a.T = (int32_t)tapCount;
  a.Q = (int32_t)((tapCount + D - 1) / D);
  a.V = kM - a.Q + 1;
  a.inBytes = (int64_t)((nOut - 1) * D + tapCount) * (int8Iq ? 2 : 8);
  a.nBlocks = ((int64_t)nOut + a.V - 1) / a.V;
  a.inRows = (int64_t)(((nOut - 1) * D + tapCount) / D);
  a.inScale = int8Iq ? 1.0f / 127.0f : 1.0f;
  a.guardRatio = gFftGuard.load(std::memory_order_relaxed);
  a.complexTaps = complexTaps ? 1 : 0;
  const bool am = epi == kEpiAm;
  if (mix.on) {
    a.mixPhase0 = mix.phase0;
    a.mixStep = mix.step;
    if (int8Iq) return am ? launchFft<kI8, kAm, true>(a, D, stream) : launchFft<kI8, kComplex, true>(a, D, stream);
    return am ? launchFft<kCf32, kAm, true>(a, D, stream) : launchFft<kCf32, kComplex, true>(a, D, stream);
  }
  if (int8Iq) return am ? launchFft<kI8, kAm>(a, D, stream) : launchFft<kI8, kComplex>(a, D, stream);
  return am ? launchFft<kCf32, kAm>(a, D, stream) : launchFft<kCf32, kComplex>(a, D, stream);
}

}  // namespace gsdr_amd

extern "C" {
// Test / tuning hook (include/gsdr/gsdr_amd.h): the FFT FIR's direct-form fallback threshold on
// the ratio of a block's loudest to quietest row level. 0 forces the direct form for every block.
void gsdrAmdSetFftGuard(float ratio) { gsdr_amd::gFftGuard.store(ratio, std::memory_order_relaxed); }
float gsdrAmdGetFftGuard(void) { return gsdr_amd::gFftGuard.load(std::memory_order_relaxed); }

// Blocks the FFT FIR computed in the direct form since the last reset on `device` (synchronises
// the device); reset != 0 zeroes the counter afterwards.
hipError_t gsdrAmdFftDirectBlocks(int32_t device, uint64_t* count, int reset) {
  int prev = 0;
  hipError_t e = hipGetDevice(&prev);
  if (e != hipSuccess) return e;
  if ((e = hipSetDevice(device)) != hipSuccess) return e;
  unsigned long long v = 0;
  e = hipDeviceSynchronize();
  if (e == hipSuccess) e = hipMemcpyFromSymbol(&v, HIP_SYMBOL(gsdr_amd::fftfir::gDirectBlocks), sizeof(v));
  if (e == hipSuccess && reset) {
    const unsigned long long z = 0;
    e = hipMemcpyToSymbol(HIP_SYMBOL(gsdr_amd::fftfir::gDirectBlocks), &z, sizeof(z));
  }
  if (count) *count = v;
  (void)hipSetDevice(prev);
  return e;
}
}
