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
// Summation: each consumer wave accumulates its K range in one MFMA chain, and the reduction adds
// the 4 partials in wave order; the plain and the fused entry points run the same consumer code, so
// the fused chain's AM samples equal gsdrInt8FirFCAmDemod's bit for bit (the 8-way kernel and the
// barrier-synchronous one group the K sums differently: same error bound, other rounding).
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
constexpr int kW4RingBytes = 4 * (kAmRing * kCfTileOut + kAmRingMirror);  // the fused chain's AM ring
constexpr int kW4ZlaneBytes = 4 * 2 * kWsPThreads;                 // the zero-window guard's pair minima, 2 sets
#ifndef GSDR_W4_Q8
#define GSDR_W4_Q8 0
#endif
// Q8 (build option, not the product: DESIGN.md 5.1): the int8 x int8 form - v_mfma_i32_32x32x32_i8 on the
// int8 samples (the reference's clamp of -128 applied), the taps as one 24-bit integer H = round(h 2^sh)
// (|H| < 2^23) split into three signed bytes H = 65536 H0 + 256 H1 + H2, one int32 accumulator per limb
// (exact: |x H_l| sums over a wave's K quarter stay below 2^24, so each converts to float exactly),
// combined in fp32 per wave. A K-step is 32 wide (16 otherwise): 3 MFMAs per 32 taps instead of 2 per 16,
// three independent accumulator chains, int8 planes - 11-13 % faster at C5, but the tap rounding is
// relative to the largest tap, and for long filters with wide passbands the output's relative L2 error
// reaches the 1e-6 bar (1.03e-6 at T = 1023, D = 3; 4.8e-7 at C5's filter), where the f16 limbs keep
// each tap to 2^-22 of itself.
constexpr bool kW4Q8 = GSDR_W4_Q8 != 0;
constexpr int kW4KStep = kW4Q8 ? 32 : 16;                            // taps per consumer K-step
constexpr int kW4MaxKS = kW4Q8 ? 11 : 22;                            // K <= 4 x 11 x 32 = 4 x 22 x 16 = 1408
typedef int v16i __attribute__((ext_vector_type(16)));

// A-fragment reads in flight ahead of the MFMAs (K-steps)
#ifndef GSDR_W4_PF
#define GSDR_W4_PF 3
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

// The epilogue values of block-local tile j from its sums y = {yi0, yi1, yq0, yq1}: the two AM samples of
// this lane (AUD: held for the ring, and stored when the caller asked for the AM samples), or the outputs
// stored right away. Accumulator register i = wave + 4 h holds row (i & 3) + 8 (i >> 2) + 4 half of the
// 32 x 32 tile.
// skip: the zero-window guard's tile (its outputs are the producers', w4DirectTile / w4PatchRing): no
// global store (AUD: the AM samples still go to the ring, where the producers overwrite them).
template <int EPI, bool AUD>
__device__ __forceinline__ void w4Outputs(const I8DecArgs& a, float outScale, int tile, int j, int tid, f4 y, bool lead,
                                          float (&am)[2], bool skip) {
  const int lane = tid & (kWave - 1);
  const int wave = tid >> 6;
  const int half = lane >> 5, col = lane & 31;
  const float yi[2] = {y.x, y.y}, yq[2] = {y.z, y.w};
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int orow = wave + 8 * h + 4 * half;
    const int64_t k = (int64_t)tile * kCfTileOut + 32 * orow + col;
    if constexpr (AUD) {
      const float v = __builtin_amdgcn_sqrtf(fmaf(yi[h], yi[h], yq[h] * yq[h])) * outScale;
      am[h] = k < a.nOut ? v : 0.0f;
      // the lead tile belongs to the previous block (computed here only for the audio windows)
      if (a.out != nullptr && k < a.nOut && !(lead && j == 0) && !skip) reinterpret_cast<float*>(a.out)[k] = v;
    } else if (k < a.nOut && !skip) {
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
  const int half = lane >> 5, col = lane & 31;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int pos = (j & (kAmRing - 1)) * kCfTileOut + 32 * (wave + 8 * h + 4 * half) + col;
#if GSDR_WS_DIAG
    wsDiag(3, pos < 0 || pos >= kAmRing * kCfTileOut);
#endif
    ring[pos] = am[h];
    if (pos < kAmRingMirror) ring[kAmRing * kCfTileOut + pos] = am[h];
  }
}

// The zero-window guard (ws_common.h wsI8ZeroRun) in this kernel: a flagged tile's outputs come from the
// PRODUCER waves in the direct form (double sums), the consumers skip their stores of it. (r06: the direct
// form inside the consumer loop cost registers the 168 VGPRs of tap fragments leave no room for - spills
// in the K loop, C5 0.160 -> 0.202 ms per step.) Plain launches: each producer wave that flags a tile
// writes all 512 outputs right after handing its planes over (several flagging waves write the same
// values). Fused chain: the AM samples must be right in the ring before the audio FIR reads them, so
// the tile's flag goes to a bit mask (zhist, by block-local tile mod 64) and at the audio stage of that
// tile the four producer waves overwrite its ring slot (and store the AM samples) - after the consumers
// wrote it, before any window reads it. (The wait in w4PatchRing is then already satisfied.)
__device__ __forceinline__ float w4DirectValue(const I8DecArgs& a, int64_t k, int epi, float& im) {
  double si, sq;
  wsI8DirectSums<1>(a.iq4 + a.sub, a.taps, a.T, a.D, k, si, sq);
  si *= 1.0 / 127.0;
  sq *= 1.0 / 127.0;
  im = (float)sq;
  // the envelope in double: the guard's outputs can be far below 1 (squares below the fp32 normals)
  return epi == kEpiAm ? (float)__builtin_sqrt(fma(si, si, sq * sq)) : (float)si;
}

template <int EPI>
__device__ __forceinline__ void w4DirectTile(const I8DecArgs& a, int tile, int lane) {
#pragma unroll 1
  for (int r = 0; r < kCfTileOut / kWave; ++r) {
    const int64_t k = (int64_t)tile * kCfTileOut + kWave * r + lane;
    if (k >= a.nOut) break;
    float im;
    const float v = w4DirectValue(a, k, EPI, im);
    if (EPI == kEpiAm) reinterpret_cast<float*>(a.out)[k] = v;
    else reinterpret_cast<f2*>(a.out)[k] = f2{v, im};
  }
}

// zhist: two words of WsCtl's zflag area the 4-way kernel's two plane sets leave free
static_assert(kW4Sets <= 2, "zhist / zsync use zflag[2] and zflag[3]");
__device__ __forceinline__ int* w4Zhist(WsCtl* c) { return &c->zflag[2][0]; }
__device__ __forceinline__ int* w4Zsync(WsCtl* c) { return &c->zflag[3][0]; }

// Fused chain, producer wave pw, before the audio outputs of block-local tile t: when t was flagged, its
// AM samples in the direct form into the ring (the 4 waves 128 each), stored when the caller asked for
// them (not the lead tile's), then all 4 waves meet (zsync, nz flagged tiles so far) before a window
// reads the slot.
__device__ __forceinline__ void w4PatchRing(const I8DecArgs& a, float* ring, WsCtl* c, int t0, int t,
                                                      bool lead, int ptid, int nz) {
  const int lane = ptid & (kWave - 1);
  const int pw = ptid >> 6;
  const bool aborted = wsWaitAb(c, &c->amSlot[t & (kAmRing - 1)], kW4Consumers * (t / kAmRing + 1));
  if (!aborted) {
#pragma unroll 1
    for (int r = 0; r < 2; ++r) {
      const int idx = 128 * pw + kWave * r + lane;
      const int64_t k = (int64_t)(t0 + t) * kCfTileOut + idx;
      float im;
      const float v = k < a.nOut ? w4DirectValue(a, k, kEpiAm, im) : 0.0f;
      const int pos = (t & (kAmRing - 1)) * kCfTileOut + idx;
      ring[pos] = v;
      if (pos < kAmRingMirror) ring[kAmRing * kCfTileOut + pos] = v;
      if (a.out != nullptr && k < a.nOut && !(lead && t == 0)) reinterpret_cast<float*>(a.out)[k] = v;
    }
  }
  wsSignal(w4Zsync(c), lane);
  wsWait(c, w4Zsync(c), kWsProducers * nz);
}

__device__ __forceinline__ void w4AmFreeWait(WsCtl* c, int j) {  // ring slot of tile j reusable
  if (j - kAmRing + 2 > 0) wsWait(c, &c->amFree, kWsProducers * (j - kAmRing + 2));
}

#ifndef GSDR_W4_LATESIG
#define GSDR_W4_LATESIG 1  // A/B switch: outputs formed between the partial writes and their signal
#endif
#ifndef GSDR_W4_CPRIO  // f16 form: 1 (r05: 142.9-146.7 vs 144.3-149.6 us); Q8: 0 (128.9-131.4 vs 130.4-136.4)
#define GSDR_W4_CPRIO (GSDR_W4_Q8 ? 0 : 1)
#endif
#ifndef GSDR_W4_NOFENCE  // A/B: hand-offs ordered by the LDS queue alone (no lgkmcnt(0) before a signal)
#define GSDR_W4_NOFENCE 0
#endif
#ifndef GSDR_W4_READY
#define GSDR_W4_READY 1  // A/B switch of the one-round-trip readiness check below
#endif
// Up to four hand-off counters checked in ONE LDS round trip (the four loads issued together, one wait):
// true when every counter has reached its target (the caller then skips the individual waits). A
// consumer wave starts each tile waiting on planesFull, partsFull, amFree and partsFree - one after the
// other that was four serial LDS round trips per tile, and they are almost always already satisfied.
__device__ __forceinline__ bool w4Ready(WsCtl* c, const int* p0, int g0, const int* p1, int g1, const int* p2, int g2,
                                        const int* p3, int g3) {
  const int v0 = __hip_atomic_load(p0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  const int v1 = __hip_atomic_load(p1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  const int v2 = __hip_atomic_load(p2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  const int v3 = __hip_atomic_load(p3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  return waveUniform(v0) >= g0 && waveUniform(v1) >= g1 && waveUniform(v2) >= g2 && waveUniform(v3) >= g3;
}

// The consumer waves: B fragments of this wave's K quarter in VGPRs for the whole launch, then per tile
// 2 KS MFMAs with the previous tile's reduction folded in - its four partial reads issued and summed in
// the gaps between this tile's MFMAs - and, for the fused chain, the AM ring writes of the tile before
// that (r05 stamps: as separate phases the reduction, the partial writes and the epilogue took ~40 % of a
// consumer wave's span beside 43 % for its MFMAs: with one consumer wave per SIMD nothing hid their LDS
// round trips); then the partials of this tile, and the previous tile's outputs formed in registers.
template <int KS, int EPI, bool AUD>
__device__ __forceinline__ void w4Consumers(const I8DecArgs& a, const int8_t* smem, float* part, WsCtl* c, int sh,
                                            int t0, int n, int tid, float* ring, bool lead, const uint32_t* zlane) {
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
  h8 bh[KS], bl[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int kap = 16 * (wave * KS + s) + 8 * half;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float hs = ldexpf(part[off0 + kap + e - col * D], sh);
      const _Float16 hi = (_Float16)hs;
      bh[s][e] = hi;
      bl[s][e] = (_Float16)(hs - (float)hi);
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
  const int uRow = (kW4Q8 ? 2 : 4) * D * arow + half;  // A row arow: 32 D samples = 2 D int8 / 4 D f16 slots
  const float outScale = ldexpf(1.0f / 127.0f, -sh);
  float am[2] = {0.0f, 0.0f};  // AUD: AM samples of tile i - 2 (this lane's), written to the ring in tile i's loop
  bool zPrev = false, zCur = false;  // zero-window guard: tiles i - 1 and i take the direct form
#ifdef GSDR_W4_STAMPS
  unsigned long long cst[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long tlast = __builtin_amdgcn_s_memtime();
  const unsigned long long tspan = tlast;
#endif
  for (int i = 0; i < n; ++i) {
    const int set = i % kW4Sets;
    const bool red = i >= 1;           // tile i - 1's partials (all four waves': each wrote them before its tile i)
    const int rb = (i - 1) & 1;
    const bool ringW = AUD && i >= 2;  // tile i - 2's AM samples go to the ring in this loop
    const int b = i & 1;               // this tile's partial buffer: free once tile i - 2 is reduced
    const int gFull = kWsProducers * (i / kW4Sets + 1);
    const int gParts = red ? kW4Consumers * (((i - 1) >> 1) + 1) : 0;
    const int gAm = ringW && i - 2 - kAmRing + 2 > 0 ? kWsProducers * (i - 2 - kAmRing + 2) : 0;
    // the partial buffer: free once tile i - 2 is reduced (before that: once the tap staging area is read)
    int* const pFree = i >= 2 ? &c->partsFree[b] : &c->tapsRead;
    const int gFree = i >= 2 ? kW4Consumers * (i >> 1) : kW4Consumers;
    const bool ready = GSDR_W4_READY && w4Ready(c, &c->planesFull[set], gFull, &c->partsFull[rb], gParts, &c->amFree, gAm, pFree, gFree);
    if (ready) {
      if (GSDR_W4_NOFENCE) asm volatile("" ::: "memory");
      else __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
    } else {
      wsWait(c, &c->planesFull[set], gFull);
      if (red) wsWait(c, &c->partsFull[rb], gParts);
      if (ringW) w4AmFreeWait(c, i - 2);
    }
    W4ST(0)
    W4ST(1)
#ifdef GSDR_W4_STAMPS
    if (wave == 0) { W4TR(0, i, 0) }
#endif
    zPrev = zCur;
    if (GSDR_WS_ZGUARD & 2) {  // read before this tile's planesFree lets the producers rewrite it
      // the producer threads' pair minima (ws_common.h wsI8ZeroPair), four waves' per ds_read_b128
      const u4v zl = *reinterpret_cast<const u4v*>(zlane + set * kWsPThreads + 4 * lane);
      zCur = __ballot(min(min(zl.x, zl.y), min(zl.z, zl.w)) == 0u) != 0;
      if (zCur && wave == 0 && lane == 0)  // for the producers (direct outputs / ring patch), before planesFree
        __hip_atomic_fetch_or(&w4Zhist(c)[(i >> 5) & 1], 1 << (i & 31), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    const int8_t* pI = smem + set * 2 * a.planeStride + comp * a.planeStride;
#if GSDR_W4_Q8
    v16i acc0 = v16i{}, acc1 = v16i{}, acc2 = v16i{};
    typedef i4v AFrag;  // 16 int8 samples
#else
    v16f acc = v16f{};
    typedef h8 AFrag;  // 8 f16 samples
#endif
    AFrag xa[KS];
    f4 pv[kW4Consumers];
    f4 y = f4{0.0f, 0.0f, 0.0f, 0.0f};
    auto readA = [&](int s) {
      xa[s] = *reinterpret_cast<const AFrag*>(pI + 16 * cfPhys(uRow + 2 * (wave * KS + s), a.padShift));
    };
    // (the partial reads are unconditional - no branch in the K loop; at i = 0 they read buffer 1,
    // whatever it holds, and the sums are not used)
    auto readP = [&](int v) { pv[v] = *w4Part(part, rb, v, wave, lane); };
#pragma unroll
    for (int s = 0; s < PF; ++s) readA(s);
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      if (s + PF < KS) readA(s + PF);
      if (s < kW4Consumers) readP(s);
      if (s == 0 && ringW) w4RingWrite(ring, i - 2, tid, am);
      asm volatile("" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
#if GSDR_W4_Q8
      acc0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(xa[s], b0[s], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(xa[s], b1[s], acc1, 0, 0, 0);
      acc2 = __builtin_amdgcn_mfma_i32_32x32x32_i8(xa[s], b2[s], acc2, 0, 0, 0);
#else
      if (!(GSDR_WS_ABL & 1)) {
#pragma unroll
        for (int rep = 0; rep < GSDR_WS_MFREP; ++rep) {  // timing experiments: MFMA work x MFREP
          acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(xa[s], bh[s], acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(xa[s], bl[s], acc, 0, 0, 0);
        }
      } else {
        asm volatile("" ::"v"(xa[s]));
        acc[s & 15] += 1.0f;
      }
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
    // one release for the three hand-offs (their LDS reads and writes were all waited for in the loop);
    // fenced one by one, each signal waited out the previous one's LDS atomic
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    wsSignalNF(&c->planesFree[set], lane);         // this wave's A reads are complete
    if (red) wsSignalNF(&c->partsFree[rb], lane);  // and its reads of tile i - 1's partials
    if (ringW) wsSignalNF(&c->amSlot[(i - 2) & (kAmRing - 1)], lane);  // tile i - 2 is in the ring
    W4ST(3)
    if (!ready) wsWait(c, pFree, gFree);  // tile i - 2 reduced by every wave (almost always seen above)
    W4ST(4)
    f4* pb = reinterpret_cast<f4*>(part + b * (kW4PartialBytes / 4));
#pragma unroll
    for (int r = 0; r < kW4Consumers; ++r)
      if (!(GSDR_WS_ABL & 2)) pb[(wave * 4 + r) * kWave + lane] = f4{acc[r], acc[r + 4], acc[r + 8], acc[r + 12]};
      else asm volatile("" ::"v"(acc[r]), "v"(acc[r + 4]), "v"(acc[r + 8]), "v"(acc[r + 12]));
#if GSDR_W4_LATESIG  // the previous tile's outputs while the partial writes land
    if (red) w4Outputs<EPI, AUD>(a, outScale, t0 + i - 1, i - 1, tid, y, lead, am, zPrev);
    W4ST(6)
    if (GSDR_W4_NOFENCE) {
      asm volatile("" ::: "memory");
      wsSignalNF(&c->partsFull[b], lane);
    } else {
      wsSignal(&c->partsFull[b], lane);
    }
    W4ST(5)
#else
    wsSignal(&c->partsFull[b], lane);
    W4ST(5)
    if (red) w4Outputs<EPI, AUD>(a, outScale, t0 + i - 1, i - 1, tid, y, lead, am, zPrev);
    W4ST(6)
#endif
#ifdef GSDR_W4_STAMPS
    if (wave == 0) { W4TR(0, i, 2) }
#endif
  }
  if constexpr (AUD) {  // tile n - 2 (pending) into the ring
    if (n >= 2) {
      w4AmFreeWait(c, n - 2);
      w4RingWrite(ring, n - 2, tid, am);
      wsSignal(&c->amSlot[(n - 2) & (kAmRing - 1)], lane);
    }
  }
  if (n >= 1) {  // the last tile's reduction on its own
    const int j = n - 1, rb = j & 1;
    wsWait(c, &c->partsFull[rb], kW4Consumers * ((j >> 1) + 1));
    f4 y = f4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int v = 0; v < kW4Consumers; ++v) y += *w4Part(part, rb, v, wave, lane);
    wsSignal(&c->partsFree[rb], lane);
    w4Outputs<EPI, AUD>(a, outScale, t0 + j, j, tid, y, lead, am, zCur);
    if constexpr (AUD) {
      w4AmFreeWait(c, j);
      w4RingWrite(ring, j, tid, am);
      wsSignal(&c->amSlot[j & (kAmRing - 1)], lane);
    }
    W4ST(7)
  }
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
  float* ring = AUD ? reinterpret_cast<float*>(smem + 2 * kW4Sets * a8.planeStride + 2 * kW4PartialBytes) : nullptr;
  uint32_t* zlane = reinterpret_cast<uint32_t*>(smem + 2 * kW4Sets * a8.planeStride + 2 * kW4PartialBytes +
                                                (AUD ? kW4RingBytes : 0));
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
    int nz = 0;  // AUD: flagged tiles patched so far (the zsync target)
    // AUD: the audio outputs of block-local tile t, after patching its ring slot when it was flagged
    // (the bit is read once the consumers have put tile t in the ring - its producers set it before the
    // planes went over; the slot count and the mask in one LDS round trip, the count almost always reached)
    auto audio = [&](int t) {
      if (t < n) {
        int* slot = &c->amSlot[t & (kAmRing - 1)];
        const int target = kW4Consumers * (t / kAmRing + 1);
        const int v = __hip_atomic_load(slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        int zh = __hip_atomic_load(&w4Zhist(c)[(t >> 5) & 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (waveUniform(v) < target) {
          wsWait(c, slot, target);
          zh = __hip_atomic_load(&w4Zhist(c)[(t >> 5) & 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        if (waveUniform(zh) & (1 << (t & 31))) w4PatchRing(a8, ring, c, t0, t, lead, ptid, ++nz);
      }
      wsAudioTile<kW4Consumers>(a8, ring, c, t0, n, lead, t, ptid, ht, ab, stp);
    };
    // after tile i's planes: the zhist bit of tile i - 32 cleared (AUD: its audio is long done - production leads
    // the audio stage by fewer than kAmRing + kW4Sets + kAudioLag tiles); plain: tile i - 2's direct outputs when
    // the consumers flagged it (they did at its top, before the planesFree this tile waited for)
    auto zbit = [&](int t) {
      return (waveUniform(__hip_atomic_load(&w4Zhist(c)[(t >> 5) & 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) >>
              (t & 31)) & 1;
    };
    auto guard = [&](int i) {
      if (ptid == 0)
        __hip_atomic_fetch_and(&w4Zhist(c)[((i >> 5) & 1) ^ 1], ~(1 << (i & 31)), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_WORKGROUP);
      if constexpr (!AUD)
        if (i >= 2 && zbit(i - 2)) w4DirectTile<EPI>(a8, t0 + i - 2, lane);
    };
    static_assert(kAmRing + kW4Sets + kAudioLag + 2 < 32, "zhist: a bit is cleared 32 tiles after it was set");
    for (int i = 0;; i += 2) {
      wsI8ProducerTile<G, kW4Consumers, kW4Sets, kW4Q8>(a8, Wl, smem, c, n, t0 + i, i, ptid, wA, [&] {
        if (AUD && i >= kAudioLag) audio(i - kAudioLag);
      }, stp, zlane);
      guard(i);
      if (i + 1 >= n) break;
      wsI8ProducerTile<G, kW4Consumers, kW4Sets, kW4Q8>(a8, Wl, smem, c, n, t0 + i + 1, i + 1, ptid, wB, [&] {
        if (AUD && i + 1 >= kAudioLag) audio(i + 1 - kAudioLag);
      }, stp, zlane);
      guard(i + 1);
      if (i + 2 >= n) break;
    }
    (void)stp;
    wsI8DrainWindows<G>(wA, wB);  // before the registers can go to the tail's code
    if constexpr (!AUD)  // the last two tiles, once the consumers are past their tops
      for (int t = n > 2 ? n - 2 : 0; t < n; ++t) {
        wsWait(c, &c->planesFree[t % kW4Sets], kW4Consumers * (t / kW4Sets + 1));
        if (zbit(t)) w4DirectTile<EPI>(a8, t0 + t, lane);
      }
    if constexpr (AUD)
      for (int t = n > kAudioLag ? n - kAudioLag : 0; t < n; ++t) audio(t);
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
  w4Consumers<KS, EPI, AUD>(a8, smem, part, c, sh, t0, n, tid, ring, lead, zlane);
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
#if GSDR_W4_Q8
constexpr int kW4KS[] = {1, 2, 3, 4, 6, 8, 11};
constexpr int kW4HarnessKS = 11;
#else
constexpr int kW4KS[] = {2, 4, 6, 8, 11, 14, 17, 21, 22};
constexpr int kW4HarnessKS = 21;
#endif

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
#if GSDR_W4_Q8
    case 1: return launchW4KS<1>(a, Wl, lds, grid, epi, audio, stream);
    case 3: return launchW4KS<3>(a, Wl, lds, grid, epi, audio, stream);
#else
    case 14: return launchW4KS<14>(a, Wl, lds, grid, epi, audio, stream);
    case 17: return launchW4KS<17>(a, Wl, lds, grid, epi, audio, stream);
    case 21: return launchW4KS<21>(a, Wl, lds, grid, epi, audio, stream);
    case 22: return launchW4KS<22>(a, Wl, lds, grid, epi, audio, stream);
#endif
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
  const size_t ringBytes = audio ? (size_t)kW4RingBytes : 0;
  const size_t extra = 2 * (size_t)kW4PartialBytes + ringBytes + kW4ZlaneBytes;
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
                  : cfPlaneLayout(a.D, a.KS, a.Wu, 2 * kW4Sets, extra, kW4Consumers * a.KS);
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
