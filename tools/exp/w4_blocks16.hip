// r05 A/B source (tools/exp/run_w4_variants.sh, third field): the 4-way kernel with 16 x 16 x 32 f16 blocks
// (four independent accumulators, K-steps of 32) and the reduction two tiles behind over three partial
// buffers; measured 146-151 vs 143-147 us for the product form (profiles/r05/exp/w4_variants_r05b16.log).
// 4-way split-K wave-specialised int8 IQ decimating MFMA kernel (r05): gsdrInt8FirFC /
// gsdrInt8FirFCAmDemod with D > 1 or T > 129, and the fused C5 receive chain
// (gsdrInt8FirFCAmDemodFirFF: RF FIR -> AM -> audio FIR in one launch).
//
// Same decimating Toeplitz tiles as firI8WsKernel (fir_cf_mfma.hip): a 512-output tile is
// C[m][n] = sum_kappa x'[32 D m + kappa] h[kappa - n D] on v_mfma_f32_32x32x16_f16, x' exact in f16,
// the taps as two scaled f16 limbs. What changes is the work split. firI8WsKernel splits K over 8
// consumer waves (2 per SIMD, 22 MFMAs each per tile): every tile is one round of hand-offs among 8
// waves, the partial sums of 8 waves (32 KB per tile) cross the LDS, and the matrix pipe sat 34 %
// busy behind that per-tile chain (r04). Here a 512-thread block has ONE consumer wave
// per SIMD, each holding a quarter of K: 2 x KS K-steps of B fragments (hi / lo limbs, up to 176
// VGPRs at KS = 22 - a wave may use 256 with two waves per SIMD), 2 KS MFMAs per tile back to back
// (42 at C5's shape), and 4 partials per output (16 KB per tile) instead of 8. The producers (one
// wave per SIMD) are firI8WsKernel's: int8 window loads, f16 planes, the fused audio stage.
//
// r05 product form (GSDR_W4_Q8 = 1, below): the int8 x int8 MFMA with the taps as three signed-byte limbs
// of a 22-bit integer - 33 v_mfma_i32_32x32x32_i8 per consumer wave and tile at C5 instead of 42
// v_mfma_f32_32x32x16_f16, three independent accumulator chains (a single dependent 32x32 chain issues
// every ~48 cycles, interleaved chains every ~33: tools/exp/mfma_valu_overlap.hip), int8 planes (half
// the plane bytes and A-fragment reads), and the K sums of a wave exact in int32.
//
// Summation: each consumer wave sums its K range (exactly, Q8), and the reduction adds the 4 partials in
// wave order; the plain and the fused entry points run the same consumer code, so the fused chain's AM
// samples equal gsdrInt8FirFCAmDemod's bit for bit (the 8-way kernel and the barrier-synchronous one
// group the K sums differently and round the taps to f16 limbs: same error bound, other rounding).
#include <algorithm>
#include <mutex>
#include <vector>

#include "fir_launch.h"
#include "kcommon.h"
// the waits profile (-DGSDR_WS_WAITS=1) counts the consumer waves 0-3 only: the producers' counted
// vmcnt waits must not see its global atomics
#define GSDR_WS_WAIT_WAVES 4
#ifdef GSDR_W4_STAMPS
// harness builds: per-phase cycle sums (below) and a per-tile event trace of one block's wave 0
// (consumer) and wave 4 (producer) after them
namespace gsdr_amd {
constexpr int kW4TraceBlock = 128, kW4TraceTiles = 128, kW4StampWords = 256 * 8 * 9;
static __device__ unsigned long long gW4Stamps[kW4StampWords + 2 * kW4TraceTiles * 4];
// the trace goes to LDS (a global store would sit in the producers' counted vmcnt waits), copied out at
// the end of the launch
__shared__ unsigned long long w4Trace[2 * kW4TraceTiles * 4];
}  // namespace gsdr_amd
#define W4TR(role, tile, ev)                                                       \
  if ((threadIdx.x & 63) == 0 && (tile) >= 0 && (tile) < kW4TraceTiles)            \
    w4Trace[((role) * kW4TraceTiles + (tile)) * 4 + (ev)] = __builtin_amdgcn_s_memtime();
#define W4TRV(role, tile, ev, val)                                                 \
  if ((threadIdx.x & 63) == 0 && (tile) >= 0 && (tile) < kW4TraceTiles)            \
    w4Trace[((role) * kW4TraceTiles + (tile)) * 4 + (ev)] = (__builtin_amdgcn_s_memtime() & ~7ull) | (val);
#endif
#include "ws_common.h"

#include <gsdr/gsdr_amd.h>

namespace gsdr_amd {

constexpr int kW4Consumers = 4;                                    // one per SIMD
#ifndef GSDR_W4_SETS
#define GSDR_W4_SETS 2
#endif
constexpr int kW4Sets = GSDR_W4_SETS;  // plane sets: the producers fill tile i while tiles i - kW4Sets + 1 .. i - 1 wait
constexpr int kW4Threads = (kW4Consumers + kWsProducers) * kWave;  // 512
constexpr int kW4PartialBytes = kW4Consumers * 16 * kWave * 4;     // 16 KB per partial buffer
#ifndef GSDR_W4_Q8
#define GSDR_W4_Q8 0
#endif
// Q8: the int8 x int8 form - v_mfma_i32_32x32x32_i8 on the int8 samples (the reference's clamp of -128
// applied), the taps as one 24-bit integer H = round(h 2^sh) (|H| < 2^23) split into three signed bytes
// H = 65536 H0 + 256 H1 + H2, one int32 accumulator per limb (exact: |x H_l| sums over a wave's K
// quarter stay below 2^24, so each converts to float exactly), combined in fp32 per wave. A K-step is
// 32 wide (K-steps of 16 below otherwise): 3 MFMAs per 32 taps instead of 2 per 16, int8 planes.
constexpr bool kW4Q8 = GSDR_W4_Q8 != 0;
// f16 form (the default): v_mfma_f32_16x16x32_f16 on 2 x 2 blocks of the 32 x 32 tile (I / Q rows x two
// column halves), four independent accumulators - one 32 x 32 x 16 accumulator chain issued its
// dependent MFMAs every ~48 cycles instead of ~33 (r05, tools/exp/mfma_valu_overlap.hip). Both forms take
// K-steps of 32 taps.
constexpr int kW4KStep = 32;                                         // taps per consumer K-step
constexpr int kW4MaxKS = 11;                                         // K <= 4 x 11 x 32 = 1408
typedef int v16i __attribute__((ext_vector_type(16)));

// A-fragment reads in flight ahead of the MFMAs (K-steps)
#ifndef GSDR_W4_PF
#define GSDR_W4_PF 1
#endif
#ifndef GSDR_W4_ADDR_INC
#define GSDR_W4_ADDR_INC 0
#endif

// Phase stamps, harness builds only (-DGSDR_W4_STAMPS, tools/exp/run_w4_variants.sh): per wave of the first
// 256 workgroups the s_memtime cycles of each phase, summed in registers and stored once at the end
// (plain stores: no atomics beside the producers' counted vmcnt waits). Consumers: 0 planesFull wait,
// 1 partsFull wait, 2 MFMA loop (with the previous tile's partial reads and sums), 3 the two signals after
// it, 4 partsFree / tapsRead waits, 5 partials write + signal, 6 epilogue, 7 the last tile's reduction;
// producers: 0 audio stage, 1 window (vmcnt) wait, 2 planesFree wait, 3 convert + plane writes + loads.
#ifdef GSDR_W4_STAMPS
#define W4ST(k)                                              \
  {                                                          \
    const unsigned long long now__ = __builtin_amdgcn_s_memtime(); \
    cst[k] += now__ - tlast;                                 \
    tlast = now__;                                           \
  }
#else
#define W4ST(k)
#endif

// Partial sums in LDS (two buffers of 16 KB, tile i in buffer i & 1): writer wave v stores for reducer
// wave r = 0..3 one float4 per lane, {acc[r], acc[r + 4], acc[r + 8], acc[r + 12]} at float4 index
// (v 4 + r) 64 + lane - 4 ds_write_b128 per lane instead of 16 ds_write_b32, and the reducer reads its
// four values of one writer with one ds_read_b128 (lanes 16 B apart: conflict free both ways). Reducer
// r finishes accumulator registers r, r + 4 (I, output rows r + 4 half and r + 8 + 4 half) and r + 8,
// r + 12 (Q of the same outputs): yi = ((p0 + p1) + p2) + p3 in writer order.
__device__ __forceinline__ const f4* w4Part(const float* part, int b, int v, int r, int lane) {
  return reinterpret_cast<const f4*>(part + b * (kW4PartialBytes / 4)) + (v * 4 + r) * kWave + lane;
}

// Tile-local output index (32 row + column) of the sums a reducer wave holds in lane `lane`, slot h:
// 32 x 32 accumulators (Q8): register i = wave + 4 h is row (i & 3) + 8 (i >> 2) + 4 half; 16 x 16 blocks
// (f16): register `wave` of column block h is row 4 (lane >> 4) + wave, column 16 h + lane % 16.
__device__ __forceinline__ int w4OutIndex(int wave, int lane, int h) {
  if constexpr (kW4Q8) return 32 * (wave + 8 * h + 4 * (lane >> 5)) + (lane & 31);
  return 32 * (4 * (lane >> 4) + wave) + 16 * h + (lane & 15);
}

// The epilogue values of block-local tile j from its sums y = {yi0, yi1, yq0, yq1}: the two AM samples of
// this lane (AUD: held for the ring, and stored when the caller asked for the AM samples), or the outputs
// stored right away. Accumulator register i = wave + 4 h holds row (i & 3) + 8 (i >> 2) + 4 half of the
// 32 x 32 tile.
template <int EPI, bool AUD>
__device__ __forceinline__ void w4Outputs(const I8DecArgs& a, float outScale, int tile, int j, int tid, f4 y, bool lead,
                                          float (&am)[2]) {
  const int lane = tid & (kWave - 1);
  const int wave = tid >> 6;
  const float yi[2] = {y.x, y.y}, yq[2] = {y.z, y.w};
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int64_t k = (int64_t)tile * kCfTileOut + w4OutIndex(wave, lane, h);
    if constexpr (AUD) {
      const float v = __builtin_amdgcn_sqrtf(fmaf(yi[h], yi[h], yq[h] * yq[h])) * outScale;
      am[h] = k < a.nOut ? v : 0.0f;
      // the lead tile belongs to the previous block (computed here only for the audio windows)
      if (a.out != nullptr && k < a.nOut && !(lead && j == 0)) reinterpret_cast<float*>(a.out)[k] = v;
    } else if (k < a.nOut) {
      if (EPI == kEpiAm)
        reinterpret_cast<float*>(a.out)[k] = __builtin_amdgcn_sqrtf(fmaf(yi[h], yi[h], yq[h] * yq[h])) * outScale;
      else
        reinterpret_cast<f2*>(a.out)[k] = f2{yi[h], yq[h]} * outScale;
    }
  }
}

// AUD: tile j's AM samples of this lane into ring slot j mod kAmRing (and its mirror). The slot must be
// free - the producers done with the audio of tile j - kAmRing + 1 - which the caller waits for.
__device__ __forceinline__ void w4RingWrite(float* ring, int j, int tid, const float (&am)[2]) {
  const int lane = tid & (kWave - 1);
  const int wave = tid >> 6;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int pos = (j & (kAmRing - 1)) * kCfTileOut + w4OutIndex(wave, lane, h);
#if GSDR_WS_DIAG
    wsDiag(3, pos < 0 || pos >= kAmRing * kCfTileOut);
#endif
    ring[pos] = am[h];
    if (pos < kAmRingMirror) ring[kAmRing * kCfTileOut + pos] = am[h];
  }
}

__device__ __forceinline__ void w4AmFreeWait(WsCtl* c, int j) {  // ring slot of tile j reusable
  if (j - kAmRing + 2 > 0) wsWait(c, &c->amFree, kWsProducers * (j - kAmRing + 2));
}

#ifndef GSDR_W4_CPRIO  // Q8: 0 (r05: 128.9-131.4 vs 130.4-136.4 us at priority 1); f16 form: 1
#define GSDR_W4_CPRIO (GSDR_W4_Q8 ? 0 : 1)
#endif
// Partial-sum buffers: tile i's partials go to buffer i % 3 and are reduced in tile i + 2's K loop, so a
// wave never waits for the other consumer waves' partials of the tile it has just finished (r05 trace:
// with the reduction one tile behind, the four waves met every tile, ~600 cycles of waiting per tile).
constexpr int kW4PartBufs = 3;
// the producers compute the audio of tile p - kW4AudioLag at their tile p: the ring holds tile j once the
// consumers are past tile j + 3, and a producer at tile p has seen the consumers past tile p - 3
constexpr int kW4AudioLag = 6;

// The three hand-off counters a consumer tile starts on (planesFull, partsFull, amFree) checked in ONE LDS
// round trip (the loads issued together, one wait): true when all have reached their targets (the
// caller then skips the individual waits, three serial round trips; they are almost always satisfied).
__device__ __forceinline__ bool w4Ready(const int* p0, int g0, const int* p1, int g1, const int* p2, int g2) {
  const int v0 = __hip_atomic_load(p0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  const int v1 = __hip_atomic_load(p1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  const int v2 = __hip_atomic_load(p2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  return waveUniform(v0) >= g0 && waveUniform(v1) >= g1 && waveUniform(v2) >= g2;
}

// The consumer waves: B fragments of this wave's K quarter in VGPRs for the whole launch, then per tile i
// its K-quarter MFMAs with tile i - 2's reduction folded in - its four partial reads issued and summed in
// the gaps between the MFMAs - and, for the fused chain, the AM ring writes of tile i - 3; then tile i's
// partials (signalled at the top of tile i + 1, whose readiness check has drained them) and tile i - 2's
// outputs formed in registers. (r05 stamps: as separate phases the reduction, the partial writes and the
// epilogue took ~40 % of a consumer wave's span beside 43 % for its MFMAs: with one consumer wave per
// SIMD nothing hid their LDS round trips.)
template <int KS, int EPI, bool AUD>
__device__ __forceinline__ void w4Consumers(const I8DecArgs& a, const int8_t* smem, float* part, WsCtl* c, int sh,
                                            int t0, int n, int tid, float* ring, bool lead) {
  constexpr int PF = GSDR_W4_PF < KS ? GSDR_W4_PF : KS;
  const int lane = tid & (kWave - 1);
  const int wave = waveUniform(tid >> 6);
  const int D = a.D;
  const int off0 = 31 * D;
  const int half = lane >> 5;
  const int col = lane & 31;
#if GSDR_W4_Q8
  i4v b0[KS], b1[KS], b2[KS];  // limbs H0, H1, H2 of B[k = 32 s' + 16 half + e][col] = H[k - col D], e < 16
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int kap = 32 * (wave * KS + s) + 16 * half;
    uint32_t w0[4] = {0, 0, 0, 0}, w1[4] = {0, 0, 0, 0}, w2[4] = {0, 0, 0, 0};
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int H = (int)rintf(ldexpf(part[off0 + kap + e - col * D], sh));  // |H| <= 8 355 711
      const int h2 = (int)(int8_t)(H & 0xff);
      const int r1 = (H - h2) >> 8;
      const int h1 = (int)(int8_t)(r1 & 0xff);
      const int h0 = (r1 - h1) >> 8;  // in [-128, 127]
      w0[e >> 2] |= (uint32_t)(h0 & 0xff) << (8 * (e & 3));
      w1[e >> 2] |= (uint32_t)(h1 & 0xff) << (8 * (e & 3));
      w2[e >> 2] |= (uint32_t)(h2 & 0xff) << (8 * (e & 3));
    }
    b0[s] = i4v{(int)w0[0], (int)w0[1], (int)w0[2], (int)w0[3]};
    b1[s] = i4v{(int)w1[0], (int)w1[1], (int)w1[2], (int)w1[3]};
    b2[s] = i4v{(int)w2[0], (int)w2[1], (int)w2[2], (int)w2[3]};
  }
#else
  // 16 x 16 x 32 blocks: lane l holds B[k = 8 (l >> 4) + e][column l % 16 of block cb] = h[k - (16 cb + l % 16) D]
  h8 bh[KS][2], bl[KS][2];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int kap = 32 * (wave * KS + s) + 8 * (lane >> 4);
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) {
      const int colb = 16 * cb + (lane & 15);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float hs = ldexpf(part[off0 + kap + e - colb * D], sh);
        const _Float16 hi = (_Float16)hs;
        bh[s][cb][e] = hi;
        bl[s][cb][e] = (_Float16)(hs - (float)hi);
      }
    }
  }
#endif
  // the tap staging area becomes the partial-sum area once every consumer wave has its fragments
  wsSignal(&c->tapsRead, lane);
  // the consumer (MFMA) wave's issue priority over its SIMD's producer wave: r05 A/B at C5, 5 runs,
  // 142.9-146.7 vs 144.3-149.6 us per launch (4 of 5 faster); the producers at priority 1 instead: 161.8
  if (GSDR_W4_CPRIO > 0) __builtin_amdgcn_s_setprio(GSDR_W4_CPRIO);

  const int arow = lane & 15;
  const int comp = (lane >> 4) & 1;
  // A row arow: 32 D samples = 2 D int8 / 4 D f16 slots; Q8 (32 x 32 x 32): lanes 0-15 / 16-31 rows of
  // the I / Q plane, k = 16 half + e; f16 (16 x 16 x 32): row l % 16 of both planes, k = 8 (l >> 4) + e
  const int uRow = kW4Q8 ? 2 * D * arow + half : 4 * D * arow + (lane >> 4);
  const float outScale = ldexpf(1.0f / 127.0f, -sh);
  float am[2] = {0.0f, 0.0f};  // AUD: AM samples of tile i - 3 (this lane's), written to the ring in tile i's loop
#ifdef GSDR_W4_STAMPS
  unsigned long long cst[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long tlast = __builtin_amdgcn_s_memtime();
  const unsigned long long tspan = tlast;
#endif
  for (int i = 0; i < n; ++i) {
    const int set = i % kW4Sets;
    const int jr = i - 2;                           // the tile reduced in this tile's K loop
    const bool red = jr >= 0;
    const int rb = (i + 1) % kW4PartBufs;           // = jr mod 3
    const int jw = i - 3;                           // the tile whose AM samples go to the ring in it
    const bool ringW = AUD && jw >= 0;
    const int b = i % kW4PartBufs;                  // this tile's partial buffer: tile i - 3's, reduced in tile i - 1
    const int gFull = kWsProducers * (i / kW4Sets + 1);
    const int gParts = red ? kW4Consumers * (jr / kW4PartBufs + 1) : 0;
    const int gAm = ringW && jw - kAmRing + 2 > 0 ? kWsProducers * (jw - kAmRing + 2) : 0;
    // before tile i - 3 exists the buffer is free once every wave has read the taps staged there
    int* const pFree = i >= kW4PartBufs ? &c->partsFree[b] : &c->tapsRead;
    const int gFree = i >= kW4PartBufs ? kW4Consumers * (i / kW4PartBufs) : kW4Consumers;
    // the partial buffer's counter is read here and checked after the K loop, where it is needed (the
    // other waves free it at the end of their tile i - 1: folded into the check above, it failed whenever
    // one of them was a little behind, and the slow path cost three more round trips)
    const int vFree = __hip_atomic_load(pFree, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    const bool ready = w4Ready(&c->planesFull[set], gFull, &c->partsFull[rb], gParts, &c->amFree, gAm);
#ifdef GSDR_W4_STAMPS
    if (wave == 0) {
      const int pf = waveUniform(__hip_atomic_load(&c->planesFull[set], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) >= gFull;
      const int pp = waveUniform(__hip_atomic_load(&c->partsFull[rb], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) >= gParts;
      W4TRV(0, i, 3, (ready ? 1 : 0) | (pf ? 2 : 0) | (pp ? 4 : 0))
    }
#endif
    // tile i - 1's partials, written before the check above (its wait drained them: the fence costs nothing
    // more), for the waves that reduce them in tile i + 1 - signalled before any wait of this wave
    if (i >= 1) wsSignal(&c->partsFull[(i - 1) % kW4PartBufs], lane);
    if (ready) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
    } else {
      wsWait(c, &c->planesFull[set], gFull);
      if (red) wsWait(c, &c->partsFull[rb], gParts);
      if (ringW) w4AmFreeWait(c, jw);
    }
    W4ST(0)
    W4ST(1)
#ifdef GSDR_W4_STAMPS
    if (wave == 0) { W4TR(0, i, 0) }
#endif
#if GSDR_W4_Q8
    const int8_t* pI = smem + set * 2 * a.planeStride + comp * a.planeStride;
    v16i acc0 = v16i{}, acc1 = v16i{}, acc2 = v16i{};
    typedef i4v AFrag;  // 16 int8 samples
    AFrag xa[KS];
#else
    const int8_t* pI = smem + set * 2 * a.planeStride;  // the I plane; Q at + planeStride
    f4 acc4[2][2] = {{f4{}, f4{}}, {f4{}, f4{}}};       // [I / Q rows][column block]
    typedef h8 AFrag;  // 8 f16 samples
    AFrag xa[KS][2];
#endif
    f4 pv[kW4Consumers];
    f4 y = f4{0.0f, 0.0f, 0.0f, 0.0f};
    auto readA = [&](int s) {
#if GSDR_W4_Q8
      xa[s] = *reinterpret_cast<const AFrag*>(pI + 16 * cfPhys(uRow + 2 * (wave * KS + s), a.padShift));
#else
#if GSDR_W4_ADDR_INC  // the slot formed per read (3 VALU) instead of KS address registers held all launch
      int v = uRow + 4 * (wave * KS + s);
      asm volatile("" : "+v"(v));
      const int8_t* pa = pI + 16 * cfPhys(v, a.padShift);
#else
      const int8_t* pa = pI + 16 * cfPhys(uRow + 4 * (wave * KS + s), a.padShift);
#endif
      xa[s][0] = *reinterpret_cast<const AFrag*>(pa);
      xa[s][1] = *reinterpret_cast<const AFrag*>(pa + a.planeStride);
#endif
    };
    // (the partial reads are unconditional - no branch in the K loop; for i < 2 they read a buffer
    // whatever it holds, and the sums are not used)
    auto readP = [&](int v) { pv[v] = *w4Part(part, rb, v, wave, lane); };
#pragma unroll
    for (int s = 0; s < PF; ++s) readA(s);
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      if (s + PF < KS) readA(s + PF);
      if (s < kW4Consumers) readP(s);
      if (s == 0 && ringW) w4RingWrite(ring, jw, tid, am);
      asm volatile("" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
#if GSDR_W4_Q8
      acc0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(xa[s], b0[s], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(xa[s], b1[s], acc1, 0, 0, 0);
      acc2 = __builtin_amdgcn_mfma_i32_32x32x32_i8(xa[s], b2[s], acc2, 0, 0, 0);
#else
      // hi limb then lo limb over the four blocks: an accumulator's next MFMA is four instructions later
#pragma unroll
      for (int rb = 0; rb < 2; ++rb)
#pragma unroll
        for (int cb = 0; cb < 2; ++cb)
          acc4[rb][cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(xa[s][rb], bh[s][cb], acc4[rb][cb], 0, 0, 0);
#pragma unroll
      for (int rb = 0; rb < 2; ++rb)
#pragma unroll
        for (int cb = 0; cb < 2; ++cb)
          acc4[rb][cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(xa[s][rb], bl[s][cb], acc4[rb][cb], 0, 0, 0);
#endif
      __builtin_amdgcn_sched_barrier(0);
      if (s >= 2 && s - 2 < kW4Consumers) y += pv[s - 2];  // writer order: v = s - 2
    }
#pragma unroll
    for (int v = 0; v < kW4Consumers; ++v) {  // shares the K loop did not reach (KS < 6)
      if (v >= KS) readP(v);
      if (v >= KS - 2) y += pv[v];
    }
#if GSDR_W4_Q8
    // the limbs in fp32: 256 S1 + S2 exact in int32 (|S1|, |S2| < 2^24), rounded once to float, then
    // 65536 S0 (exact) added with one more rounding - 4 VALU per value
    v16f acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = fmaf((float)acc0[r], 65536.0f, (float)(acc1[r] * 256 + acc2[r]));
#endif
    W4ST(2)
#ifdef GSDR_W4_STAMPS
    if (wave == 0) { W4TR(0, i, 1) }
#endif
    // one release for the three hand-offs (their LDS reads and writes were all waited for in the loop)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    wsSignalNF(&c->planesFree[set], lane);                           // this wave's A reads are complete
    if (red) wsSignalNF(&c->partsFree[rb], lane);                    // and its reads of tile i - 2's partials
    if (ringW) wsSignalNF(&c->amSlot[jw & (kAmRing - 1)], lane);     // tile i - 3 is in the ring
    W4ST(3)
    if (waveUniform(vFree) < gFree) wsWait(c, pFree, gFree);  // tile i - 3 reduced by every wave
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
    W4ST(4)
    f4* pb = reinterpret_cast<f4*>(part + b * (kW4PartialBytes / 4));
    // reducer r gets {I h0, I h1, Q h0, Q h1} of its outputs (w4OutIndex)
#pragma unroll
    for (int r = 0; r < kW4Consumers; ++r)
#if GSDR_W4_Q8
      pb[(wave * 4 + r) * kWave + lane] = f4{acc[r], acc[r + 4], acc[r + 8], acc[r + 12]};
#else
      pb[(wave * 4 + r) * kWave + lane] = f4{acc4[0][0][r], acc4[0][1][r], acc4[1][0][r], acc4[1][1][r]};
#endif
    W4ST(5)
    if (red) w4Outputs<EPI, AUD>(a, outScale, t0 + jr, jr, tid, y, lead, am);
    W4ST(6)
#ifdef GSDR_W4_STAMPS
    if (wave == 0) { W4TR(0, i, 2) }
#endif
  }
  if (n >= 1) wsSignal(&c->partsFull[(n - 1) % kW4PartBufs], lane);  // the last tile's partials
  if constexpr (AUD) {  // tile n - 3 (pending) into the ring
    if (n >= 3) {
      w4AmFreeWait(c, n - 3);
      w4RingWrite(ring, n - 3, tid, am);
      wsSignal(&c->amSlot[(n - 3) & (kAmRing - 1)], lane);
    }
  }
  for (int j = n >= 2 ? n - 2 : 0; j < n; ++j) {  // the last two tiles' reductions on their own
    const int rbj = j % kW4PartBufs;
    wsWait(c, &c->partsFull[rbj], kW4Consumers * (j / kW4PartBufs + 1));
    f4 y = f4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int v = 0; v < kW4Consumers; ++v) y += *w4Part(part, rbj, v, wave, lane);
    wsSignal(&c->partsFree[rbj], lane);
    w4Outputs<EPI, AUD>(a, outScale, t0 + j, j, tid, y, lead, am);
    if constexpr (AUD) {
      w4AmFreeWait(c, j);
      w4RingWrite(ring, j, tid, am);
      wsSignal(&c->amSlot[j & (kAmRing - 1)], lane);
    }
  }
  W4ST(7)
#ifdef GSDR_W4_STAMPS
  if ((int)blockIdx.x == kW4TraceBlock && wave == 0 && lane == 0)
    for (int k = 0; k < kW4TraceTiles * 4; ++k) gW4Stamps[kW4StampWords + k] = w4Trace[k];
  if ((int)blockIdx.x < 256 && lane == 0) {
    for (int k = 0; k < 8; ++k) gW4Stamps[((int)blockIdx.x * 8 + wave) * 9 + k] = cst[k];
    gW4Stamps[((int)blockIdx.x * 8 + wave) * 9 + 8] = __builtin_amdgcn_s_memtime() - tspan;
  }
#endif
}

template <int KS, int G, int EPI, bool AUD>
__global__ __launch_bounds__(kW4Threads, 1) void firI8Ws4Kernel(I8DecArgs a8, int Wl) {
  extern __shared__ __attribute__((aligned(16))) int8_t smem[];
  float* part = reinterpret_cast<float*>(smem + 2 * kW4Sets * a8.planeStride);
  float* ring = AUD ? reinterpret_cast<float*>(smem + 2 * kW4Sets * a8.planeStride + kW4PartBufs * kW4PartialBytes) : nullptr;
  __shared__ WsCtl ctl;
  __shared__ float waveMax[kW4Consumers + kWsProducers];
  WsCtl* c = &ctl;

  const int tid = threadIdx.x;
  const int lane = tid & (kWave - 1);
  const int wave = waveUniform(tid >> 6);
  const int D = a8.D, T = a8.T;

  // contiguous tile range of this block
  const int q = a8.tiles / (int)gridDim.x, r = a8.tiles % (int)gridDim.x;
  int t0 = (int)blockIdx.x * q + min((int)blockIdx.x, r);
  int n = q + ((int)blockIdx.x < r ? 1 : 0);
  if (n <= 0) return;
  // fused audio: every block but the first also computes the tile before its range (the lead) into
  // its AM ring, so each audio window it owns is complete on chip
  bool lead = false;
  if (AUD && t0 > 0) {
    --t0;
    ++n;
    lead = true;
  }

  // ---- taps -> LDS (zero-padded to [-31 D, 64 KS)), block max; zero both plane sets and the ring --
  if (tid < kWsCtlZeroWords) reinterpret_cast<int*>(c)[tid] = 0;
  if (tid == 0) {
    c->spinLimit = a8.spinLimit;
    c->abortOut = a8.abortOut;
  }
  const int off0 = 31 * D;
  const int span = off0 + 4 * kW4KStep * KS;
  float hm = 0.0f;
  for (int i = tid; i < span; i += kW4Threads) {
    const int j = i - off0;
    const float h = (j >= 0 && j < T) ? a8.taps[j] : 0.0f;
    part[i] = h;
    hm = fmaxf(hm, fabsf(h));
  }
  for (int i = tid; i < 2 * kW4Sets * a8.planeStride / 16; i += kW4Threads) reinterpret_cast<uint4*>(smem)[i] = uint4{0, 0, 0, 0};
  // the AM ring starts zeroed: an audio window reads 256 ring samples whatever the tap count (the ones
  // past its taps times zero, and 0 * NaN is NaN: r04's stale-LDS defect)
  if constexpr (AUD && GSDR_WS_RING_ZERO)
    for (int i = tid; i < (kAmRing * kCfTileOut + kAmRingMirror) / 4; i += kW4Threads)
      reinterpret_cast<uint4*>(ring)[i] = uint4{0, 0, 0, 0};
  hm = waveMaxNonNeg(hm);
  if (lane == 0) waveMax[wave] = hm;
  __syncthreads();
  float hMax = waveMax[0];
#pragma unroll
  for (int v = 1; v < kW4Consumers + kWsProducers; ++v) hMax = fmaxf(hMax, waveMax[v]);
  // max |h 2^sh| in [2^14, 2^15) (f16 limbs) / below 127 (65536 + 256 + 1) = 8 355 711 (Q8: three signed
  // bytes; [2^22, 2^23) unless that would overflow the top limb, then half of it)
  int sh = hMax > 0.0f ? (kW4Q8 ? 22 : 14) - ilogbf(hMax) : 0;
  if (kW4Q8 && hMax > 0.0f && ldexpf(hMax, sh) > 8355711.0f) --sh;
#if GSDR_WS_WAITS
  const unsigned long long span0 = __builtin_amdgcn_s_memtime();
#endif

  if (wave >= kW4Consumers) {
    // ================= producers (firI8WsKernel's, signalling 4 consumer waves) =================
    const int ptid = tid - kW4Consumers * kWave;
#ifdef GSDR_W4_PPRIO  // A/B builds only: the producer wave's issue priority over its SIMD's consumer
    __builtin_amdgcn_s_setprio(GSDR_W4_PPRIO);
#endif
    float ht[kAudioTapsPerLane];  // audio taps (lane % 8) + 8 u
    AudioBounds ab = AUD ? audioBounds(a8, t0, n, lead) : AudioBounds{0, 0, 0};
#pragma unroll
    for (int u = 0; u < kAudioTapsPerLane; ++u) {
      const int tp = (lane & 7) + 8 * u;
      ht[u] = AUD && tp < a8.aT ? a8.aTaps[tp] : 0.0f;
    }
    // the taps in registers before the first window load: the compiler does not count the window loads
    // (inline asm), so a first use of ht inside the loop got a full s_waitcnt vmcnt(0) - in every audio
    // batch, which also waited for the window loads in flight (r05 ISA)
#pragma unroll
    for (int u = 0; u < kAudioTapsPerLane; ++u) asm volatile("" ::"v"(ht[u]));
    I8WsWindow<G> wA, wB;
    const i4v r0 = wsI8TileRsrc(a8, t0, true);
#pragma unroll
    for (int j = 0; j < G; ++j) wsI8LoadGroup<G>(r0, Wl, ptid, j, wA);
    const i4v r1 = wsI8TileRsrc(a8, t0 + 1, n > 1);
#pragma unroll
    for (int j = 0; j < G; ++j) wsI8LoadGroup<G>(r1, Wl, ptid, j, wB);
#if GSDR_WS_WAITS || defined(GSDR_W4_STAMPS)
    unsigned long long st[5] = {0, 0, 0, 0, 0};
    unsigned long long* stp = st;
#ifdef GSDR_W4_STAMPS
    const unsigned long long tspanP = __builtin_amdgcn_s_memtime();
#endif
#else
    unsigned long long* stp = nullptr;
#endif
    for (int i = 0;; i += 2) {
      wsI8ProducerTile<G, kW4Consumers, kW4Sets, kW4Q8>(a8, Wl, smem, c, n, t0 + i, i, ptid, wA, [&] {
        if (AUD && i >= kW4AudioLag) wsAudioTile<kW4Consumers>(a8, ring, c, t0, n, lead, i - kW4AudioLag, ptid, ht, ab, stp);
      }, stp);
      if (i + 1 >= n) break;
      wsI8ProducerTile<G, kW4Consumers, kW4Sets, kW4Q8>(a8, Wl, smem, c, n, t0 + i + 1, i + 1, ptid, wB, [&] {
        if (AUD && i + 1 >= kW4AudioLag) wsAudioTile<kW4Consumers>(a8, ring, c, t0, n, lead, i + 1 - kW4AudioLag, ptid, ht, ab, stp);
      }, stp);
      if (i + 2 >= n) break;
    }
    (void)stp;
    if constexpr (AUD)
      for (int t = n > kW4AudioLag ? n - kW4AudioLag : 0; t < n; ++t)
        wsAudioTile<kW4Consumers>(a8, ring, c, t0, n, lead, t, ptid, ht, ab);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no load outlives the wave
#ifdef GSDR_W4_STAMPS
    if ((int)blockIdx.x == kW4TraceBlock && wave == kW4Consumers && lane == 0)
      for (int k = 0; k < kW4TraceTiles * 4; ++k) gW4Stamps[kW4StampWords + kW4TraceTiles * 4 + k] = w4Trace[kW4TraceTiles * 4 + k];
    if ((int)blockIdx.x < 256 && lane == 0) {
      for (int k = 0; k < 5; ++k) gW4Stamps[((int)blockIdx.x * 8 + wave) * 9 + k] = st[k];
      gW4Stamps[((int)blockIdx.x * 8 + wave) * 9 + 8] = __builtin_amdgcn_s_memtime() - tspanP;
    }
#endif
#if GSDR_WS_WAITS
    wsSpanStore(__builtin_amdgcn_s_memtime() - span0);
    {  // the producer phases into its slots 10-13 (plain stores after the final vmcnt(0))
      const int wg = (int)blockIdx.x;
      if (wg < 256 && lane == 0)
        for (int k = 0; k < 3; ++k) gWsWaits[(wg * 12 + wave) * kWaitSlots + 10 + k] = st[k];
      if (wg < 256 && lane == 0) gWsWaits[(wg * 12 + wave) * kWaitSlots + 9] = st[3];
    }
#endif
    return;
  }
  w4Consumers<KS, EPI, AUD>(a8, smem, part, c, sh, t0, n, tid, ring, lead);
#if GSDR_WS_WAITS
  wsSpanStore(__builtin_amdgcn_s_memtime() - span0);
#endif
}

// ---- host side ---------------------------------------------------------------------------------

uint32_t cachedAudioSlotPerm(int aD) {  // ~40 k permutations scored once per audio decimation
  static std::mutex mu;
  static std::vector<std::pair<int, uint32_t>> cache;
  std::lock_guard<std::mutex> lock(mu);
  for (const auto& [d, p] : cache)
    if (d == aD) return p;
  const uint32_t p = audioSlotPerm(aD);
  if (cache.size() >= 16) cache.erase(cache.begin());
  cache.emplace_back(aD, p);
  return p;
}

namespace {

template <int KS, int G, int EPI, bool AUD>
hipError_t launchW4G(const I8DecArgs& a, int Wl, size_t lds, int grid, hipStream_t stream) {
  auto kernel = &firI8Ws4Kernel<KS, G, EPI, AUD>;
#ifdef GSDR_W4_STAMPS
  constexpr int kDynMax = kCfDynLdsMax - (int)sizeof(w4Trace);  // the trace is static LDS
#else
  constexpr int kDynMax = kCfDynLdsMax;
#endif
  if (lds > (size_t)kDynMax) return hipErrorNotSupported;
  const hipError_t attrErr =
      hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize, kDynMax);
  if (attrErr != hipSuccess) return attrErr;
  hipLaunchKernelGGL(kernel, dim3(grid), dim3(kW4Threads), lds, stream, a, Wl);
  return hipGetLastError();
}

template <int KS>
hipError_t launchW4KS(const I8DecArgs& a, int Wl, size_t lds, int grid, int epi, bool audio, hipStream_t stream) {
  const int G = (Wl + kWsPThreads - 1) / kWsPThreads;
#define GSDR_W4_G(g)                                                                   \
  case g:                                                                              \
    if (audio) return launchW4G<KS, g, kEpiAm, true>(a, Wl, lds, grid, stream);        \
    return epi == kEpiAm ? launchW4G<KS, g, kEpiAm, false>(a, Wl, lds, grid, stream)   \
                         : launchW4G<KS, g, kEpiComplex, false>(a, Wl, lds, grid, stream);
  switch (G) {
    GSDR_W4_G(1)
    GSDR_W4_G(2)
    GSDR_W4_G(3)
    default:
      GSDR_W4_G(4)
  }
#undef GSDR_W4_G
  return hipErrorNotSupported;
}

// Instantiated K quarters (K-steps of kW4KStep per consumer wave): a shape runs on the smallest one that
// covers it (the extra K-steps meet zero taps). C5 (1023 taps, D = 10: K = 1333): 21 steps of 16 per
// wave, or 11 of 32 (Q8).
constexpr int kW4KS[] = {1, 2, 3, 4, 6, 8, 11};
constexpr int kW4HarnessKS = 11;

// ksteps: K-steps of 16 the shape needs ((31 D + T) / 16 rounded up)
int w4PickKS(int ksteps) {
  const int steps = (ksteps * 16 + kW4KStep - 1) / kW4KStep;
  const int need = (steps + kW4Consumers - 1) / kW4Consumers;
  for (int k : kW4KS)
    if (k >= need) return k;
  return 0;
}

hipError_t launchW4Any(const I8DecArgs& a, int Wl, size_t lds, int grid, int epi, bool audio, hipStream_t stream) {
#ifdef GSDR_W4_HARNESS  // variant builds of tools/exp/run_w4_variants.sh: C5's fused shape only
  if (a.KS != kW4HarnessKS || !audio || (Wl + kWsPThreads - 1) / kWsPThreads != 3) return hipErrorNotSupported;
  return launchW4G<kW4HarnessKS, 3, kEpiAm, true>(a, Wl, lds, grid, stream);
#endif
  switch (a.KS) {
    case 1: return launchW4KS<1>(a, Wl, lds, grid, epi, audio, stream);
    case 3: return launchW4KS<3>(a, Wl, lds, grid, epi, audio, stream);
    case 2: return launchW4KS<2>(a, Wl, lds, grid, epi, audio, stream);
    case 4: return launchW4KS<4>(a, Wl, lds, grid, epi, audio, stream);
    case 6: return launchW4KS<6>(a, Wl, lds, grid, epi, audio, stream);
    case 8: return launchW4KS<8>(a, Wl, lds, grid, epi, audio, stream);
    case 11: return launchW4KS<11>(a, Wl, lds, grid, epi, audio, stream);
    default: return hipErrorNotSupported;
  }
}

}  // namespace

// The 4-way kernel for an int8 decimating launch `a` (its iq4 / sub / taps / out / T / D / nOut / nIn /
// tiles filled in; audio fields too when `audio`): hipErrorNotSupported when the shape does not fit
// (the caller then takes the 8-way kernel).
hipError_t launchFirI8Ws4(I8DecArgs a, int ksteps, int epi, bool audio, hipStream_t stream) {
  static_assert(kCfTileOut == 512, "the audio ring indexes AM samples by k >> 9");
  a.KS = w4PickKS(ksteps);
  if (a.KS == 0 || a.KS > kW4MaxKS) return hipErrorNotSupported;
  a.Wu = 60 * a.D + kW4KStep / 2 * a.KS;  // window units (8 samples) per tile: 480 D + 4 kW4KStep KS samples
  const int Wl = std::min(a.Wu, (511 * a.D + a.T + 7) / 8);
  if (Wl > 4 * kWsPThreads) return hipErrorNotSupported;
  const size_t ringBytes = audio ? sizeof(float) * (kAmRing * kCfTileOut + kAmRingMirror) : 0;
  const size_t extra = kW4PartBufs * (size_t)kW4PartialBytes + ringBytes;
  // the layout search costs ~1 ms of host time: cached per (D, KS, audio)
  static std::mutex mu;
  static std::vector<std::pair<uint64_t, CfLayout>> cache;
  const uint64_t key = ((uint64_t)(uint32_t)a.D << 32) | ((uint64_t)(uint32_t)a.KS << 8) | (audio ? 1u : 0u);
  CfLayout lay{};
  {
    std::lock_guard<std::mutex> lock(mu);
    bool found = false;
    for (const auto& [k, v] : cache)
      if (k == key) {
        lay = v;
        found = true;
      }
    if (!found) {
      // Q8: int8 planes, 16-byte slots of 16 samples (Wu / 2 per plane), A rows 2 D slots apart
      lay = kW4Q8 ? cfPlaneLayout(a.D, a.KS, a.Wu / 2, 2 * kW4Sets, extra, kW4Consumers * a.KS, 2 * a.D)
                  : cfPlaneLayout(a.D, a.KS, a.Wu, 2 * kW4Sets, extra, kW4Consumers * a.KS, 4 * a.D, true);
      if (cache.size() >= 16) cache.erase(cache.begin());
      cache.emplace_back(key, lay);
    }
  }
  if (lay.planeStride == 0) return hipErrorNotSupported;
  a.padShift = lay.padShift;
  a.planeStride = lay.planeStride;
  a.dbp = 1;
#ifdef GSDR_W4_IDPERM  // A/B builds only: consecutive outputs in slot order
  if (audio) a.audioPerm = 0x76543210u;
#else
  if (audio) a.audioPerm = cachedAudioSlotPerm(a.aD);
#endif
  const size_t lds = 2 * kW4Sets * (size_t)a.planeStride + extra;
  if (lds > (size_t)kCfDynLdsMax) return hipErrorNotSupported;
  const int grid = (int)(a.tiles < 256 ? a.tiles : 256);
  if (hipError_t e = wsPrepareLaunch(stream, a.spinLimit, a.abortOut); e != hipSuccess) return e;
  return launchW4Any(a, Wl, lds, grid, epi, audio, stream);
}

#ifdef GSDR_W4_HARNESS
// tools/exp/run_w4_variants.sh: this variant build's entry point (-DGSDR_W4_HARNESS=<name>)
extern "C" hipError_t GSDR_W4_HARNESS(const void* args, int ksteps, hipStream_t stream) {
  return launchFirI8Ws4(*static_cast<const I8DecArgs*>(args), ksteps, kEpiAm, true, stream);
}
#endif

#if GSDR_WS_DIAG
// this translation unit's counters (ws_common.h keeps one copy per unit), added to fir_cf_mfma.hip's
hipError_t w4DiagRead(unsigned long long* out8, int reset) {
  unsigned long long v[8];
  hipError_t e = hipMemcpyFromSymbol(v, HIP_SYMBOL(gWsDiag), sizeof v);
  if (e == hipSuccess)
    for (int i = 0; i < 8; ++i) out8[i] += v[i];
  if (e == hipSuccess && reset) {
    const unsigned long long z[8] = {};
    e = hipMemcpyToSymbol(HIP_SYMBOL(gWsDiag), z, sizeof z);
  }
  return e;
}
#endif
#if defined(GSDR_W4_HARNESS_STAMPS) && defined(GSDR_W4_STAMPS)
extern "C" hipError_t GSDR_W4_HARNESS_STAMPS(unsigned long long* out, size_t n, int reset) {
  hipError_t e = hipDeviceSynchronize();
  const size_t m = n < (size_t)(kW4StampWords + 2 * kW4TraceTiles * 4) ? n : (size_t)(kW4StampWords + 2 * kW4TraceTiles * 4);
  if (e == hipSuccess) e = hipMemcpyFromSymbol(out, HIP_SYMBOL(gW4Stamps), m * sizeof(unsigned long long));
  if (e == hipSuccess && reset) {
    void* p = nullptr;
    e = hipGetSymbolAddress(&p, HIP_SYMBOL(gW4Stamps));
    if (e == hipSuccess) e = hipMemset(p, 0, sizeof(unsigned long long) * (kW4StampWords + 2 * kW4TraceTiles * 4));
  }
  return e;
}
#endif
#if defined(GSDR_W4_HARNESS_WAITS) && GSDR_WS_WAITS
hipError_t w4WaitsRead(unsigned long long* out, size_t n, int reset);
extern "C" hipError_t GSDR_W4_HARNESS_WAITS(unsigned long long* out, size_t n, int reset) {
  hipError_t e = hipDeviceSynchronize();
  if (e == hipSuccess) e = w4WaitsRead(out, n, reset);
  return e;
}
#endif
#if GSDR_WS_WAITS
hipError_t w4WaitsRead(unsigned long long* out, size_t n, int reset) {
  std::vector<unsigned long long> v(n);
  hipError_t e = hipMemcpyFromSymbol(v.data(), HIP_SYMBOL(gWsWaits), n * sizeof(unsigned long long));
  if (e == hipSuccess)
    for (size_t i = 0; i < n; ++i) out[i] += v[i];
  if (e == hipSuccess && reset) {
    void* p = nullptr;
    e = hipGetSymbolAddress(&p, HIP_SYMBOL(gWsWaits));
    if (e == hipSuccess) e = hipMemset(p, 0, sizeof(unsigned long long) * 256 * 12 * kWaitSlots);
  }
  return e;
}
#endif

}  // namespace gsdr_amd
