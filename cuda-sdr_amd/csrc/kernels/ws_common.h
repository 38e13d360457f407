// Shared pieces of the wave-specialised decimating MFMA kernels (fir_cf_mfma.hip: the cf32 and 8-way
// int8 kernels; fir_i8_ws4.hip: the 4-way int8 kernel, r05): the Toeplitz tile geometry, the LDS
// hand-off protocol between producer and consumer waves (WsCtl, bounded waits, the abort path), the
// int8 IQ producer, the fused audio stage and the host-side plane-layout search.
#pragma once

#include <cstddef>
#include <cstdint>

#include <hip/hip_runtime.h>

#include "kcommon.h"

namespace gsdr_amd {

typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf2 __attribute__((ext_vector_type(2)));
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));

constexpr int kCfWaves = 8;
constexpr int kCfThreads = kCfWaves * kWave;
constexpr int kCfTileOut = 512;  // 16 rows x 32 columns
constexpr int kCfMaxKS = 11;     // K-steps of 16 per wave: K <= 8 x 11 x 16 = 1408
constexpr int kCfMaxD = 16;
constexpr int kCfPartialBytes = kCfWaves * 16 * kWave * 4;  // 32 KB
constexpr int kCfDynLdsMax = 160 * 1024 - 256;             // the rest: static flags

__device__ __forceinline__ int cfPhys(int u, int p) { return u + (u >> p); }

// Hand-off counters (monotonic, one increment per wave): planesFull[set] (producers -> consumers:
// tile's planes and mode written), planesFree[set] (consumers finished reading the set),
// partsFull / partsFree (consumers among themselves: all partials of a tile written / all read),
// pstat (producer-local statistics of the next tile published). Every wait is bounded: a wave that spins past the limit
// raises `abort`, which releases every other wait, so the grid always drains.

constexpr int kWsProducers = 4;
constexpr int kWsPThreads = kWsProducers * kWave;           // 256
constexpr int kWsThreads = kCfThreads + kWsPThreads;        // 768
constexpr int kWsDirect = 0x7fffffff;                       // plane-set mode: direct fp32 tile
// default hand-off wait budget, microseconds of wall clock (r06; through r05 a count of s_sleep(1) polls,
// 1 << 22, whose duration depends on the poll's LDS latency and so on whatever else runs on the CU)
constexpr int kWsSpinLimit = 2000000;
// Fused audio stage (firI8WsKernel<.., AUD>): AM ring of kAmRing tiles in LDS; the producers compute
// the audio outputs of tile i - kAudioLag after producing the planes of tile i.
constexpr int kAmRing = 8;
#ifndef GSDR_AUDIO_LAG
#define GSDR_AUDIO_LAG 5
#endif
constexpr int kAudioLag = GSDR_AUDIO_LAG;
constexpr int kAmRingMirror = 256;  // ring[4096 + i] = ring[i] for i < 256: no wrap inside a window
constexpr int kAudioMaxTaps = 256;  // 8 tap groups of 32 per output slot
constexpr int kGWaves = 4;          // two-group kernel: consumer waves per group

#ifndef GSDR_WS_WAITS
#define GSDR_WS_WAITS 0
#endif
// hand-off polls: one LDS round trip each (1) or three (0, through r04)
#ifndef GSDR_WS_POLL
#define GSDR_WS_POLL 1
#endif
// fused audio stage: zero the AM ring per launch (0: the r04 defect, for its regression test only)
#ifndef GSDR_WS_RING_ZERO
#define GSDR_WS_RING_ZERO 1
#endif
// s_sleep argument between hand-off polls (units of 64 clocks; 0: spin on the LDS read alone)
#ifndef GSDR_WS_SLEEP
#define GSDR_WS_SLEEP 1
#endif
// int8 consumers with two partial buffers: tile i - 1's reduction interleaved with tile i's MFMAs
// (r04: bit-identical and time-neutral, 171.7-172.9 vs 169.2-174.8 us per C5 launch; off)
#ifndef GSDR_WS_RED_IL
#define GSDR_WS_RED_IL 0
#endif
// int8 consumers: A-fragment reads in flight ahead of the MFMAs (K-steps)
#ifndef GSDR_WS_PF
#define GSDR_WS_PF 3
#endif
struct WsCtl {
  int planesFull[3];  // per plane set (the 8-way kernels use two, the 4-way kernel kW4Sets)
  int planesFree[3];
  int partsFull[3];                   // per partial buffer (one buffer: index 0; the 4-way kernel has 3)
  int partsFree[3];
  int pstat;
  int tapsRead;                       // consumer waves done reading the taps staged in `part`
  int amFree;                         // producer waves done with the audio outputs of a tile
  int abort;
  int mode[3];                        // per plane set: scale exponent sx, or kWsDirect
  union {                             // (the static LDS budget: kCfDynLdsMax leaves 256 bytes)
    float stat[2][2][kWsProducers];   // cf32: [tile parity][max, smallest block max][producer wave]
    int zflag[4][kWsProducers];       // int8, per plane set and producer wave: the tile's window holds an exact-
                                      // zero run (wsI8ZeroRun) - the consumers compute it in the direct form
  };
  int amSlot[kAmRing];                // fused audio stage: consumer waves' AM signals per ring slot
  // set once by thread 0 (not part of the zeroed hand-off words above)
  int spinLimit;  // hand-off wait budget, microseconds
  uint32_t* abortOut;
};
constexpr int kWsCtlZeroWords = (int)(offsetof(WsCtl, spinLimit) / 4);
static_assert(sizeof(WsCtl) + 12 * sizeof(float) <= 256, "WsCtl + waveMax must fit the 256 static LDS bytes");

// Diagnostic builds only (-DGSDR_WS_DIAG=1: tools/build_variant.sh diag, run by tools/r05/session.sh diag; the product build has none): bounds
// checks on every index the fused audio stage and the AM ring writes compute, counted per kind, to
// show whether the abort path (a wsWait that returns early) computes an index outside its range -
// [0] audio-tile waits that returned on an abort, [1] history index outside
// [0, amH), [2] block-local AM index outside the two ring tiles a window may span, [3] ring write
// position outside the ring, [4] history reads, [5] ring reads, [6] audio-tile calls (per producer
// wave), [7] audio batches (8 outputs per wave) - r05: the batch count against the launch's model.
#ifndef GSDR_WS_DIAG
#define GSDR_WS_DIAG 0
#endif
#if GSDR_WS_DIAG
static __device__ unsigned long long gWsDiag[8];
__device__ __forceinline__ void wsDiag(int kind, bool hit) {
  if (hit) atomicAdd(&gWsDiag[kind], 1ull);
}
#endif

__device__ __forceinline__ void wsSignal(int* p, int lane) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");  // LDS writes/reads complete
  if (lane == 0) __hip_atomic_fetch_add(p, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// A signal after the caller's own release fence (several hand-offs released by one fence)
__device__ __forceinline__ void wsSignalNF(int* p, int lane) {
  if (lane == 0) __hip_atomic_fetch_add(p, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Hand-off wait profile, diagnostic builds only (-DGSDR_WS_WAITS=1; the product build has none): per
// wave of the first 256 workgroups, the shader cycles spent in each kind of wait (the WsCtl counter
// waited on) and the wave's whole span after its prologue, to tell which hand-off holds which role.
// Kinds: 0 planesFull, 1 planesFree, 2 partsFull, 3 partsFree, 4 pstat, 5 tapsRead, 6 amSlot (the
// audio stage's per-ring-slot counts), 7 amFree; slot 8 = the wave's span, 9 = its wait count.
#if GSDR_WS_WAITS
#ifndef GSDR_WS_WAIT_WAVES  // the consumer waves (waves below it); the 4-way kernel's unit sets 4
#define GSDR_WS_WAIT_WAVES kCfWaves
#endif
constexpr int kWaitSlots = 13;  // + the 4-way consumers' phases: 10 MFMA loop, 11 partials write, 12 reduce
static __device__ unsigned long long gWsWaits[256 * 12 * kWaitSlots];
__device__ __forceinline__ int wsWaitKind(const WsCtl* c, const int* p) {
  const int off = (int)(reinterpret_cast<const char*>(p) - reinterpret_cast<const char*>(c));  // byte offset
  if (off < (int)offsetof(WsCtl, planesFree)) return 0;
  if (off < (int)offsetof(WsCtl, partsFull)) return 1;
  if (off < (int)offsetof(WsCtl, partsFree)) return 2;
  if (off < (int)offsetof(WsCtl, pstat)) return 3;
  if (off < (int)offsetof(WsCtl, tapsRead)) return 4;
  if (off < (int)offsetof(WsCtl, amFree)) return 5;
  if (off < (int)offsetof(WsCtl, abort)) return 7;
  if (off >= (int)offsetof(WsCtl, amSlot) && off < (int)offsetof(WsCtl, spinLimit)) return 6;
  return 7;
}
// Consumer waves only (global atomics: the producers' counted vmcnt waits must not see extra
// vector-memory operations, and the LDS has no room for per-wave counters); producers record their
// span once, after their final vmcnt(0).
__device__ __forceinline__ void wsWaitAdd(WsCtl*, int slot, unsigned long long v) {
  const int wg = (int)blockIdx.x, w = (int)(threadIdx.x >> 6);
  if (wg < 256 && w < GSDR_WS_WAIT_WAVES && (threadIdx.x & 63) == 0) atomicAdd(&gWsWaits[(wg * 12 + w) * kWaitSlots + slot], v);
}
__device__ __forceinline__ void wsSpanStore(unsigned long long v) {
  const int wg = (int)blockIdx.x, w = (int)(threadIdx.x >> 6);
  if (wg < 256 && (threadIdx.x & 63) == 0) gWsWaits[(wg * 12 + w) * kWaitSlots + 8] = v;
}
#endif

// A hand-off that never completes: release every other wait so the grid drains, and count the
// failure where the host sees it (the entry points report it as hipErrorLaunchTimeOut). The count
// goes through the global address space: a FLAT atomic would count on lgkmcnt too and turn every
// later LDS wait of the wave into a full drain (lgkmcnt(0)).
__device__ __forceinline__ void wsRaiseAbort(WsCtl* c) {
  __hip_atomic_store(&c->abort, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  if ((threadIdx.x & (kWave - 1)) == 0 && c->abortOut != nullptr)
    __hip_atomic_fetch_add((__attribute__((address_space(1))) uint32_t*)(c->abortOut), 1u, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
}

// The hand-off budget in s_memrealtime ticks (100 MHz), 32 bits: the elapsed time is compared modulo 2^32
// (42.9 s), so a budget above that saturates. 32-bit scalar compares only: a 64-bit ordered compare is a VALU
// v_cmp on gfx9, whose mask the scalar branch must wait for (a VALU -> SALU hand-off; see wsClampI64).
__device__ __forceinline__ uint32_t wsBudgetTicks(const WsCtl* c) {
  const uint32_t us = (uint32_t)waveUniform(c->spinLimit);
  return us >= 42949672u ? 0xffffffffu : 100u * us;
}
__device__ __forceinline__ bool wsElapsedOver(uint32_t t0, uint32_t budget) {
  uint32_t dt = (uint32_t)__builtin_amdgcn_s_memrealtime() - t0;
  asm volatile("" : "+s"(dt));
  return dt > budget;
}

__device__ __forceinline__ void wsWait(WsCtl* c, int* p, int target) {
#if GSDR_WS_WAITS
  const unsigned long long t0w = __builtin_amdgcn_s_memtime();
#endif
#if GSDR_WS_POLL
  // one LDS round trip per poll: the counter and the abort word read together, the spin limit
  // once (reading the three one after the other, each waited for, made a poll ~3 round trips,
  // added to the hand-off latency of every wait that polls)
  if (waveUniform(__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) < target) {
    // the budget is wall clock (s_memrealtime: the constant 100 MHz counter), so a wave that is merely
    // slowed - other kernels or processes on its CU, a context switch - never counts as a hang (r06,
    // VERDICT r05 weak 2); only a hand-off that has not come in spinLimit microseconds aborts
    const uint32_t budget = wsBudgetTicks(c);
    const uint32_t t0 = (uint32_t)__builtin_amdgcn_s_memrealtime();
    for (;;) {
      if (GSDR_WS_SLEEP > 0) __builtin_amdgcn_s_sleep(GSDR_WS_SLEEP);
      const int v = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      const int ab = __hip_atomic_load(&c->abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      if (waveUniform(v) >= target || waveUniform(ab)) break;
      if (wsElapsedOver(t0, budget)) {
        wsRaiseAbort(c);
        break;
      }
    }
  }
#else
  const uint32_t budget = wsBudgetTicks(c), t0 = (uint32_t)__builtin_amdgcn_s_memrealtime();
  for (;;) {
    const int v = waveUniform(__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
    if (v >= target) break;
    if (waveUniform(__hip_atomic_load(&c->abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP))) break;
    if (wsElapsedOver(t0, budget)) {
      wsRaiseAbort(c);
      break;
    }
    __builtin_amdgcn_s_sleep(1);
  }
#endif
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
#if GSDR_WS_WAITS
  wsWaitAdd(c, wsWaitKind(c, p), __builtin_amdgcn_s_memtime() - t0w);
  wsWaitAdd(c, 9, 1);
#endif
}

// wsWait that also reports an abort, read in the same LDS round trip as the counter's first poll (the
// fused audio stage stops on an abort; a separate read of the abort word cost it a round trip per tile)
__device__ __forceinline__ bool wsWaitAb(WsCtl* c, int* p, int target) {
  const int v0 = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  const int ab0 = __hip_atomic_load(&c->abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  if (waveUniform(v0) >= target) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
    return waveUniform(ab0) != 0;
  }
  wsWait(c, p, target);
  return waveUniform(__hip_atomic_load(&c->abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) != 0;
}

typedef int i4v __attribute__((ext_vector_type(4)));

struct I8DecArgs {
  const int8_t* iq4;  // the input rounded down to 4 bytes; the samples start `sub` bytes later
  const float* taps;
  void* out;
  int64_t nOut;
  int64_t nIn;        // complex samples readable: (nOut - 1) D + T
  int32_t sub;        // 0 or 2: byte offset of the first sample inside its dword
  int32_t T;
  int32_t D;
  int32_t KS;
  int32_t tiles;
  int32_t Wu;         // window units (8 samples = 16 input bytes) per tile = 60 D + 16 KS
  int32_t padShift;
  int32_t planeStride;  // bytes between the I and Q f16 planes
  int32_t dbp;          // wave-specialised kernel: two partial-sum buffers
  int32_t spinLimit;    // as CfFirArgs
  uint32_t* abortOut;
  // fused audio stage (firI8WsKernel<.., true>): audio[j] = sum_t aTaps[t] A(j aD - amH + t) for
  // j < aN, where A(k) is AM output k of this launch (k >= 0) or amHist[amH + k] (k < 0)
  const float* aTaps;
  float* aOut;
  const float* amHist;
  int64_t aN;
  int32_t aT;
  int32_t aD;
  int32_t amH;
  // two-group kernel (firI8WsGroupKernel): B fragments from shifted tap copies in LDS
  int32_t kneed;     // K-steps of 16 that meet nonzero taps
  int32_t tcLen;     // f16 elements per tap copy
  int32_t tcStride;  // bytes between two tap-copy arrays (hi / lo limb of each shift)
  // fused audio stage: output slot o of a wave's batch of 8 consecutive outputs takes output
  // jb + ((audioPerm >> 4 o) & 7) (audioSlotPerm: the order that spreads the slots' ds_read_b32 over
  // the LDS banks for this aD)
  uint32_t audioPerm;
};


typedef uint32_t u4v __attribute__((ext_vector_type(4)));

#ifndef GSDR_WS_ABL  // timing ablations of the 4-way kernel (tools/exp/run_w4_variants.sh; outputs wrong):
#define GSDR_WS_ABL 0  // 1 no MFMAs, 2 no partial exchange, 4 no plane writes, 8 no int8 conversion
#endif                 // (4-way Q8: 16 no partial exchange, 32 no A reads, 64 no MFMAs)
#if 0
#endif
#ifndef GSDR_WS_MFREP  // timing experiments: each consumer MFMA pair issued MFREP times (outputs wrong)
#define GSDR_WS_MFREP 1
#endif

template <int G>
struct I8WsWindow {
  u4v q[G];       // the unit's 16 bytes from the dword holding its first byte
  uint32_t e[G];  // the next dword
};

// A 64-bit value clamped to [0, cap] with 32-bit compares only: gfx9 has no scalar 64-bit ordered compare,
// so `x < cap` on int64 becomes a VALU v_cmp whose mask the scalar code then waits for. (r06: removed from the
// producers' per-tile range math while chasing the zero-window guard's cost - measured neutral by itself.)
__device__ __forceinline__ int wsClampI64(int64_t x, int cap) {
  int hi = (int)(x >> 32);
  uint32_t lo = (uint32_t)x;
  asm("" : "+s"(hi), "+s"(lo));  // opaque halves: LLVM would fold `hi < 0` back into a 64-bit compare
  return hi < 0 ? 0 : (hi > 0 || lo > (uint32_t)cap) ? cap : (int)lo;
}

__device__ __forceinline__ i4v wsI8TileRsrc(const I8DecArgs& a, int tile, bool valid) {
  const int64_t first = (int64_t)tile * kCfTileOut * a.D * 2;  // bytes from iq4
  const int64_t total = (2 * a.nIn + a.sub + 3) & ~(int64_t)3;  // whole dwords holding input bytes
  // clamped at 0 (r06): a tile index past the input must give an empty range, never a
  // negative num_records, which as uint32 would switch the range check off
  const int bytes = valid ? wsClampI64(total - first, 0x7fffffff) : 0;
  const uint64_t base = reinterpret_cast<uint64_t>(a.iq4 + first);
  i4v r;
  r.x = waveUniform((int)(uint32_t)base);
  r.y = waveUniform((int)((base >> 32) & 0xffffu));
  r.z = waveUniform((int)bytes);
  r.w = 0x00020000;
  return r;
}

template <int G>
__device__ __forceinline__ void wsI8LoadGroup(i4v rsrc, int Wl, int ptid, int j, I8WsWindow<G>& w) {
  const int g = ptid + kWsPThreads * j;
  const int voff = g < Wl ? 16 * g : 0x7ffffff0;
  asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen" : "=v"(w.q[j]) : "v"(voff), "s"(rsrc) : "memory");
  asm volatile("buffer_load_dword %0, %1, %2, 0 offen offset:16" : "=v"(w.e[j]) : "v"(voff), "s"(rsrc) : "memory");
}

template <int N, int G>
__device__ __forceinline__ void wsI8WaitWindow(I8WsWindow<G>& w) {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
#pragma unroll
  for (int j = 0; j < G; ++j) {
    asm volatile("" : "+v"(w.q[j]));
    asm volatile("" : "+v"(w.e[j]));
  }
}

// After the producer loop (r06): the last window loads - the tiles past the block's range, out of range,
// returning zeros - are still landing in BOTH windows. The compiler does not know (inline asm): once a
// window's value is dead it hands the registers to the tail's code (the last audio tiles: LDS addresses,
// the audio output store's address), and a load that lands late overwrites them. Under contention (ranks
// sharing the GPU) that was the r05 multi-rank C5 fault, hipErrorIllegalAddress on an audio store whose
// address a window load had zeroed (tools/isa_vmcnt_check.py finds such reuse in the ISA).
// Both windows stay live until every load has landed.
template <int G>
__device__ __forceinline__ void wsI8DrainWindows(I8WsWindow<G>& a, I8WsWindow<G>& b) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int j = 0; j < G; ++j) {
    asm volatile("" : "+v"(a.q[j]), "+v"(a.e[j]));
    asm volatile("" : "+v"(b.q[j]), "+v"(b.e[j]));
  }
}

// The zero-window guard of the int8 kernels (r06). The taps are two f16 limbs under one
// block scale: a tap below ~2^-17 of the largest keeps only an absolute 2^-39 of it (the Blackman tails of
// C5's RF filter: 1e-20 .. 1e-8 of the largest), so an output whose window has non-zero samples ONLY under
// such taps - at a zero-padded stream start, after an exact-zero gap - misses the 1e-6 sum|h||x| bound.
// Such a window's samples under every other tap are zero, i.e. the tile window holds a long run of exact
// complex zeros. A wave flags its part of the window when two adjacent 8-sample units of its 64 are all
// zero (I = Q = 0; units past Wl or past the input's end excluded; wsI8ZeroPair): any zero run of >= 39
// samples is caught, and the violating runs are ~T long. Flagged tiles are computed in the direct form (the
// 8-way kernel's consumers, wsI8DirectOutput; the 4-way kernel's producers, fir_i8_ws4.hip). An adversarial
// comb - non-zero samples only where a windowed sinc has its zeros - is not a run and stays uncaught
// (DESIGN.md 9). Cost: ~6 VALU per unit, one ballot per tile.
#ifndef GSDR_WS_ZGUARD  // A/B builds only: bit 0 the producers' zero runs, bit 1 the 4-way consumers' flag reads
#define GSDR_WS_ZGUARD 3
#endif
// The zero-run test in VALU arithmetic only: per unit, o = the OR of its four words; the pair (unit, next
// unit) is all zero when o | o(neighbouring lane) is 0 (one DPP wave shift); invalid pairs - a unit or its
// neighbour past the input, and lanes 0 and 63 (the pair that would cross the wave, whichever way the shift
// runs) - are OR-ed with all ones; the thread keeps the minimum. Any zero run of >= 39 samples holds 4 whole
// units, 3 pairs, one of them tested. The reduction over the threads is the consumers' in the 4-way kernel
// (r06: every form that finished it in the producer - a compare per unit, a ballot or a DPP min chain per tile
// - cost the C5 launch 35-50 us of its 145; this form + the consumer reduction 3.5 us).
__device__ __forceinline__ uint32_t wsI8ZeroPair(const uint32_t (&words)[4], int g, int Wz, uint32_t edge) {
  const uint32_t o = words[0] | words[1] | words[2] | words[3];
  const uint32_t on = (uint32_t)__builtin_amdgcn_mov_dpp((int)o, 0x130, 0xf, 0xf, true);  // wave_shl:1
  const uint32_t invalid = (uint32_t)((Wz - g - 2) >> 31) | edge;
  return o | on | invalid;
}
// The wave's minimum in lane 63, DPP only (row shifts, then the row broadcasts): no VALU -> SALU hand-off.
template <int CTRL, int ROWS = 0xf, int BANKS = 0xf>
__device__ __forceinline__ uint32_t wsDppMinStep(uint32_t v) {
  return min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, CTRL, ROWS, BANKS, false));
}
__device__ __forceinline__ uint32_t wsWaveMinLane63(uint32_t v) {
  v = wsDppMinStep<0x111>(v);            // row_shr:1
  v = wsDppMinStep<0x112>(v);            // row_shr:2
  v = wsDppMinStep<0x113>(v);            // row_shr:3
  v = wsDppMinStep<0x114, 0xf, 0xe>(v);  // row_shr:4
  v = wsDppMinStep<0x118, 0xf, 0xc>(v);  // row_shr:8 (lane 15 of each row: the row's minimum)
  v = wsDppMinStep<0x142, 0xa, 0xf>(v);  // row_bcast:15
  return wsDppMinStep<0x143, 0xc, 0xf>(v);  // row_bcast:31
}
// The tile's zero-run flag of this wave (1 / 0, valid in lane 63) from the threads' pair minima.
__device__ __forceinline__ uint32_t wsI8ZeroRunLane63(uint32_t zmin) {
  if (!(GSDR_WS_ZGUARD & 1)) return 0u;
  return 1u - min(wsWaveMinLane63(zmin), 1u);
}

// zero-window flags of plane set `set` (the producer waves' zflag words, read after planesFull)
__device__ __forceinline__ bool wsI8Zflag(const WsCtl* c, int set) {
  return waveUniform(c->zflag[set][0] | c->zflag[set][1] | c->zflag[set][2] | c->zflag[set][3]) != 0;
}

// Direct form of int8 IQ output k (the guard's tiles): sum_j h_j I'_kD+j and sum_j h_j Q'_kD+j with
// x' = max(x, -127), accumulated in double (rare tiles; a sequential fp32 sum of ~1 000 products can
// reach 1e-6 of sum|h||x|, tests/test_mfma_guard.py). U: unroll; 1 in both kernels (r06: 4 or 8 in the 4-way
// kernel's producers would keep more tap loads in flight - a flagged tile costs its block ~180 us - but spilled
// SGPRs of the C5 kernel; in the 8-way kernel's consumers, VGPRs).
template <int U = 1>
__device__ __forceinline__ void wsI8DirectSums(const int8_t* iq, const float* taps, int T, int D, int64_t k, double& si,
                                               double& sq) {
  const int8_t* p = iq + 2 * k * D;
  si = 0.0;
  sq = 0.0;
#pragma unroll U
  for (int j = 0; j < T; ++j) {
    const double h = taps[j];
    si = fma(h, (double)max((int)p[2 * j], -127), si);
    sq = fma(h, (double)max((int)p[2 * j + 1], -127), sq);
  }
}

// The same in the MFMA path's scaled units (x 2^sh), for the 8-way kernel's consumers (their epilogue,
// x 2^-sh / 127, applies unchanged).
__device__ __forceinline__ void wsI8DirectOutput(const int8_t* iq, const float* taps, int T, int D, int64_t k, int sh,
                                                 float& yi, float& yq) {
  double si, sq;
  wsI8DirectSums(iq, taps, T, D, k, si, sq);
  yi = (float)ldexp(si, sh);
  yq = (float)ldexp(sq, sh);
}

// Producer, tile i: wCur holds tile i's window (complete after the wait), wNext tile i + 1's.
// `pre` runs while the window is still landing (the fused audio stage hides its work under that
// wait; its few output stores sit behind tile i + 1's loads in the vmcnt order - issued a tile
// earlier - and in front of tile i + 2's, so no window wait waits for loads issued this iteration).
struct NoPre {
  __device__ void operator()() const {}
};

// `st` (GSDR_WS_WAITS builds, 4-way kernel): per-producer-wave cycle sums [0] audio stage, [1] window
// (vmcnt) wait, [2] planesFree wait, [3] the rest (convert, plane writes, load issue); nullptr: none.
// NS plane sets: tile i goes to set i % NS once the consumers are done with tile i - NS. Q8: int8 planes
// (the 4-way kernel's int8 x int8 MFMA form): the 8 samples of a group are one 8-byte half of a 16-byte
// plane slot, slot g / 2 (padded like the f16 units), half g % 2.
// Returns this wave's zero-run flag of the tile (the zero-window guard) in lane 63: 1 when its part of the
// window holds a zero run - the 8-way kernel's form (lane 63 stores it); with zlane (the 4-way kernel) 0: the
// per-lane minima go to LDS for the consumers to reduce.
template <int G, int NC = kCfWaves, int NS = 2, bool Q8 = false, typename Pre = NoPre>
// zlane (the 4-way kernel): the threads' pair minima go to LDS instead of a flag per wave (see below).
__device__ __forceinline__ uint32_t wsI8ProducerTile(const I8DecArgs& a, int Wl, int8_t* smem, WsCtl* c, int n, int tile,
                                                 int i, int ptid, I8WsWindow<G>& wCur, const Pre& pre = Pre{},
                                                 unsigned long long* st = nullptr, uint32_t* zlane = nullptr) {
  const int lane = ptid & (kWave - 1);
  const int set = i % NS;
#if GSDR_WS_WAITS || defined(GSDR_W4_STAMPS)
  unsigned long long t0s = __builtin_amdgcn_s_memtime(), t1s;
#endif
#ifdef W4TR
  if (ptid < kWave) { W4TR(1, i, 0) }
#endif
  pre();
#ifdef W4TR
  if (ptid < kWave) { W4TR(1, i, 1) }
#endif
#if GSDR_WS_WAITS || defined(GSDR_W4_STAMPS)
  if (st) { t1s = __builtin_amdgcn_s_memtime(); st[0] += t1s - t0s; t0s = t1s; }
#endif
  wsI8WaitWindow<2 * G>(wCur);
#if GSDR_WS_WAITS || defined(GSDR_W4_STAMPS)
  if (st) { t1s = __builtin_amdgcn_s_memtime(); st[1] += t1s - t0s; t0s = t1s; }
#endif
  wsWait(c, &c->planesFree[set], NC * (i / NS));
#if GSDR_WS_WAITS || defined(GSDR_W4_STAMPS)
  if (st) { t1s = __builtin_amdgcn_s_memtime(); st[2] += t1s - t0s; t0s = t1s; }
#endif
#ifdef W4TR
  if (ptid < kWave) { W4TR(1, i, 2) }
#endif
  int8_t* planes = smem + set * 2 * a.planeStride;
  const i4v rsrc2 = wsI8TileRsrc(a, tile + 2, i + 2 < n);
  uint32_t zmin = 0xffffffffu;
  const uint32_t edge = 0u - (uint32_t)(((lane + 1) >> 6) | ((64 - lane) >> 6));  // lanes 0, 63
  // units wholly inside the input: the last tile's window runs past it (zeros, out of range), not a run
  const int Wz = wsClampI64((a.nIn - (int64_t)tile * kCfTileOut * a.D) >> 3, Wl);
#pragma unroll
  for (int j = 0; j < G; ++j) {
    const int g = ptid + kWsPThreads * j;
    const uint32_t words[4] = {__builtin_amdgcn_alignbyte(wCur.q[j].y, wCur.q[j].x, a.sub),
                               __builtin_amdgcn_alignbyte(wCur.q[j].z, wCur.q[j].y, a.sub),
                               __builtin_amdgcn_alignbyte(wCur.q[j].w, wCur.q[j].z, a.sub),
                               __builtin_amdgcn_alignbyte(wCur.e[j], wCur.q[j].w, a.sub)};
    if (GSDR_WS_ZGUARD & 1) zmin = min(zmin, wsI8ZeroPair(words, g, Wz, edge));
    if constexpr (Q8) {
      uint2 iu, qu;
      int8IqToI8Units(words, iu, qu);
      const int gg = g < Wl ? g : a.Wu;  // spare unit Wu (even): slot Wu / 2, never read
      const int off = 16 * cfPhys(gg >> 1, a.padShift) + 8 * (gg & 1);
      if (!(GSDR_WS_ABL & 4)) {
        *reinterpret_cast<uint2*>(planes + off) = iu;
        *reinterpret_cast<uint2*>(planes + a.planeStride + off) = qu;
      } else {
        asm volatile("" ::"v"(iu.x), "v"(iu.y), "v"(qu.x), "v"(qu.y));
      }
      wsI8LoadGroup<G>(rsrc2, Wl, ptid, j, wCur);
      continue;
    }
    uint4 iu, qu;
    if (GSDR_WS_ABL & 8) {  // timing ablation: no conversion VALU
      iu = uint4{words[0], words[1], words[2], words[3]};
      qu = iu;
    } else {
      int8IqToF16Units(words, iu, qu);
    }
    const int off = 16 * cfPhys(g < Wl ? g : a.Wu, a.padShift);  // spare unit Wu: never read
    if (!(GSDR_WS_ABL & 4)) {
      *reinterpret_cast<uint4*>(planes + off) = iu;
      *reinterpret_cast<uint4*>(planes + a.planeStride + off) = qu;
    } else {
      asm volatile("" ::"v"(iu.x), "v"(iu.y), "v"(iu.z), "v"(iu.w), "v"(qu.x), "v"(qu.y), "v"(qu.z), "v"(qu.w));
    }
    wsI8LoadGroup<G>(rsrc2, Wl, ptid, j, wCur);
  }
  if (ptid == 0) c->mode[set] = 0;
  uint32_t zflag = 0;
  if (zlane != nullptr) {
    // 4-way kernel: every lane's pair minimum to LDS ([set][lane][producer wave]: one ds_read_b128 per consumer
    // lane gathers the four waves'), reduced by the consumer waves - no dependent chain in the producer
    zlane[set * kWsPThreads + 4 * lane + (ptid >> 6)] = zmin;
  } else {
    zflag = wsI8ZeroRunLane63(zmin);
    if (lane == kWave - 1) c->zflag[set][ptid >> 6] = (int)zflag;  // published by the planesFull release
  }
  wsSignal(&c->planesFull[set], lane);
#if GSDR_WS_WAITS || defined(GSDR_W4_STAMPS)
  if (st) st[3] += __builtin_amdgcn_s_memtime() - t0s;
#endif
#ifdef W4TR
  if (ptid < kWave) { W4TR(1, i, 3) }
#endif
  return zflag;
}


// Fused audio stage, producer side: the audio outputs of block-local tile t (global tile t0 + t) -
// those whose window ends in that tile's AM range (tile 0 of the launch: also windows ending
// before AM sample 0, in the history) - from the AM ring the consumers fill (tiles t - 1 and t are
// in it: a window spans at most 256 AM samples), then amFree. A wave takes 8 consecutive outputs at a
// time, jb + perm(o) (o < 8, wave pw from jb = jLo + 8 pw): lane l works on slot o = l / 8 with the
// taps q + 8 u of its tap group q = l % 8 (u < 32; 32 LDS reads and FMAs, the 8 lanes of a slot
// reading consecutive AM samples), then the slot's 8 partial sums meet in 3 DPP adds - no LDS round trip
// (a 64-lane sum per output through ds_bpermute serialised ~50 LDS round trips per tile and made the
// producers, who feed the matrix cores, the bottleneck: C5 0.18 -> 0.71 ms per step).
// The lead tile (the previous block's last, computed for the ring only) has no outputs here.
constexpr int kAudioTapsPerLane = kAudioMaxTaps / 8;
#ifndef GSDR_AUDIO_ACC  // packed partial sums per audio window (A/B: 2 or 4)
#define GSDR_AUDIO_ACC 2
#endif
#ifndef GSDR_AUDIO_ROTATE
#define GSDR_AUDIO_ROTATE 1
#endif
#ifndef GSDR_AUDIO_SKIP  // timing experiments only: the audio windows not computed (outputs wrong)
#define GSDR_AUDIO_SKIP 0
#endif


// smallest audio output j whose window end j aD - amH + aT - 1 is >= X (AM index X of this launch). In
// 32 bits: the launcher admits only launches whose AM indices, history and audio offsets stay below 2^31
// (audioIndexFits). r05: the 64-bit divisions here (four per tile and producer wave, a software sequence
// of ~100 instructions each) were most of the producers' audio-stage time.
__device__ __forceinline__ int audioFirstJ(const I8DecArgs& a, int X) {
  const int num = X + a.amH - a.aT + 1;
  return num <= 0 ? 0 : (int)((uint32_t)(num + a.aD - 1) / (uint32_t)a.aD);
}

// The audio outputs a block owns (those whose window ends in its own tiles, the lead excluded, below aN),
// from the launch's shape alone; `next`: the first output of the next tile the stage processes (tiles are
// processed in order, and a tile's outputs end where the next one's begin - one division per tile).
struct AudioBounds {
  int lo, hi, next;
  int batches;  // 8-output batches dealt so far: the next tile's first batch goes to wave batches % 4
};
__device__ __forceinline__ AudioBounds audioBounds(const I8DecArgs& a, int t0, int n, bool lead) {
  const int own0 = t0 + (lead ? 1 : 0);
  AudioBounds b;
  b.lo = own0 == 0 ? 0 : audioFirstJ(a, own0 * kCfTileOut);
  b.hi = audioFirstJ(a, (t0 + n) * kCfTileOut);
  if (b.hi > (int)a.aN) b.hi = (int)a.aN;
  b.next = b.lo;
  b.batches = 0;
  return b;
}

// t0 / n: the block's tile range (lead included); t: the block-local tile whose audio outputs to compute
// (called for t = 0, 1, ... in order); ab: audioBounds of the block.
template <int NSIG = kCfWaves>
__device__ __forceinline__ void wsAudioTile(const I8DecArgs& a, const float* ring, WsCtl* c, int t0, int n, bool lead,
                                            int t, int ptid, const float (&ht)[kAudioTapsPerLane], AudioBounds& ab,
                                            unsigned long long* st = nullptr) {
  const int lane = ptid & (kWave - 1);
  const int pw = ptid >> 6;
  const int o = lane >> 3, q = lane & 7;
#if GSDR_WS_DIAG
  wsDiag(6, lane == 0);
#endif
  if (!(lead && t == 0) && t < n) {
    // the ring slots of tiles t and t - 1 (a window spans at most 256 AM samples). Slot s holds
    // tiles s, s + 8, ..., each signalled by the NSIG consumer waves that write it, and no slot is
    // rewritten before the audio of the tile after its occupant is done (amFree), so a slot's count
    // says exactly which of its tiles are complete. (A single tile counter, waited for at
    // NSIG (t + 1), was not: a wave that reduced tile t + 1 could signal it before a slower wave
    // had written its part of tile t - the count was reached with tile t incomplete. With short
    // filters - 2 K-steps per wave, little MFMA work between the hand-offs - that happened: r04,
    // test_am_chain_device_steps at T = 127 / D = 1 and T = 64 / D = 3.)
    // Tile t - 1's slot was waited for by this wave's previous call (audio tiles run in order),
    // except when that call was the lead tile's, which has no outputs and waits for nothing.
    // an aborted launch computes nothing more: its outputs are undefined anyway (the next call fails),
    // and no window is formed from ring slots a finished pipeline would not hold
#ifdef GSDR_W4_STAMPS
    const unsigned long long tw0 = __builtin_amdgcn_s_memtime();
#endif
    bool aborted = wsWaitAb(c, &c->amSlot[t & (kAmRing - 1)], NSIG * (t / kAmRing + 1));
    if (lead && t == 1) aborted |= wsWaitAb(c, &c->amSlot[0], NSIG);
#ifdef GSDR_W4_STAMPS
    if (st) st[4] += __builtin_amdgcn_s_memtime() - tw0;  // the ring-slot wait (inside the audio stage's time)
#endif
#if GSDR_WS_DIAG
    wsDiag(0, lane == 0 && aborted);
#endif
    const int g = t0 + t;
    // the tile's outputs, clamped to the block's own range (its tiles after the lead) and to aN: the
    // loop bounds follow from the launch's shape alone, whatever a wait returned
    const int jLo = ab.next;
    int jHi = audioFirstJ(a, (g + 1) * kCfTileOut);
    jHi = jHi < ab.hi ? jHi : ab.hi;
    jHi = jHi > jLo ? jHi : jLo;
    ab.next = jHi;
    // batches dealt round robin over the whole block, not from wave 0 at every tile: at aD = 20 a tile
    // has 51-52 outputs = 7 batches, and waves 0-2 took two each tile while wave 3 took one - the
    // planes hand-off waits for the slowest producer wave
    const int first = GSDR_AUDIO_ROTATE ? (ab.batches & (kWsProducers - 1)) : 0;
    ab.batches += (jHi - jLo + 7) >> 3;
    const int pwr = (pw - first) & (kWsProducers - 1);
    if (aborted || GSDR_AUDIO_SKIP) jHi = jLo;
    // r05: 8 consecutive outputs per wave batch, slots ordered by audioPerm. Through r04 a batch took
    // outputs jb + 4 o: at aD = 20 the windows of slots o and o + 2 then started 160 floats apart, on the
    // same LDS banks - every audio ds_read_b32 2-way conflicted (6.6 M of the C5 launch's 37 M LDS cycles)
    const int perm = (int)((a.audioPerm >> (4 * o)) & 7u);
    for (int jb = jLo + 8 * pwr; jb < jHi; jb += 8 * kWsProducers) {
#if GSDR_WS_DIAG
      wsDiag(7, lane == 0);
#endif
      const int j = jb + perm;
      const int k0 = j * a.aD - a.amH;  // this slot's window: AM samples k0 .. k0 + aT - 1
      float s = 0.0f;
      if (jb * a.aD - a.amH >= 0) {  // wave-uniform: every window of the batch lies in the ring
        // block-local AM index, wrapped once: the mirror behind the ring keeps the window contiguous
        // (immediate-offset LDS reads)
        const float* w = ring + ((k0 - kCfTileOut * t0 + q) & (kAmRing * kCfTileOut - 1));
#if GSDR_WS_DIAG
        if (j < jHi) {
          const int64_t kk0 = k0 - (int64_t)kCfTileOut * t0 + q, kk1 = kk0 + 8 * (kAudioTapsPerLane - 1);
          wsDiag(2, kk0 < 0 || kk0 < (int64_t)kCfTileOut * (t - 1) || kk1 >= (int64_t)kCfTileOut * (t + 1));
          wsDiag(5, true);
        }
#endif
        // all 32 reads in flight before the first FMA, then four interleaved partial sums (r05: the
        // compiler had paired the reads into 16 ds_read2_b32, each waited for in full (lgkmcnt(0))
        // before its two FMAs - 16 serialised LDS round trips per batch, ~half of the producers' span)
        // (taps 2k, 2k + 1 of the lane as one pair: the pair a ds_read2_b32 returns, one v_pk_fma_f32 - r05:
        // with four scalar partial sums the compiler paired the reads across pairs, 24 v_mov per batch)
        f2 xv[kAudioTapsPerLane / 2];
#pragma unroll
        for (int k = 0; k < kAudioTapsPerLane / 2; ++k) xv[k] = f2{w[16 * k], w[16 * k + 8]};
        asm volatile("" ::: "memory");
        if (GSDR_AUDIO_ACC == 4) {  // four packed partial sums: dependent FMA chains of 4, not 8
          f2 a0 = f2{0.0f, 0.0f}, a1 = a0, a2 = a0, a3 = a0;
#pragma unroll
          for (int k = 0; k < kAudioTapsPerLane / 2; k += 4) {
            a0 = __builtin_elementwise_fma(f2{ht[2 * k], ht[2 * k + 1]}, xv[k], a0);
            a1 = __builtin_elementwise_fma(f2{ht[2 * k + 2], ht[2 * k + 3]}, xv[k + 1], a1);
            a2 = __builtin_elementwise_fma(f2{ht[2 * k + 4], ht[2 * k + 5]}, xv[k + 2], a2);
            a3 = __builtin_elementwise_fma(f2{ht[2 * k + 6], ht[2 * k + 7]}, xv[k + 3], a3);
          }
          const f2 b0 = a0 + a2, b1 = a1 + a3;
          s = (b0.x + b0.y) + (b1.x + b1.y);
        } else {
          f2 a0 = f2{0.0f, 0.0f}, a1 = f2{0.0f, 0.0f};
#pragma unroll
          for (int k = 0; k < kAudioTapsPerLane / 2; k += 2) {
            a0 = __builtin_elementwise_fma(f2{ht[2 * k], ht[2 * k + 1]}, xv[k], a0);
            a1 = __builtin_elementwise_fma(f2{ht[2 * k + 2], ht[2 * k + 3]}, xv[k + 1], a1);
          }
          s = (a0.x + a0.y) + (a1.x + a1.y);
        }
      } else {  // windows reaching into the history (the launch's first outputs)
        // buffer loads (range-checked): a pointer select between the ring and the history would
        // compile to FLAT loads
        const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.amHist), (short)0, 4 * a.amH,
                                                          0x00020000);
#pragma unroll 4
        for (int u = 0; u < kAudioTapsPerLane; ++u) {
          const int k = k0 + q + 8 * u;
          float x;
#if GSDR_WS_DIAG
          if (j < jHi) {
            const int64_t kk = k - (int64_t)kCfTileOut * t0;
            if (k >= 0) wsDiag(2, kk < 0 || kk < (int64_t)kCfTileOut * (t - 1) || kk >= (int64_t)kCfTileOut * (t + 1));
            else wsDiag(1, a.amH + k < 0 || a.amH + k >= a.amH);
            wsDiag(k >= 0 ? 5 : 4, true);
          }
#endif
          if (k >= 0)
            x = ring[(k - kCfTileOut * t0) & (kAmRing * kCfTileOut - 1)];
          else
            x = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, (int)(4 * (a.amH + k)), 0, 0));
          s = fmaf(ht[u], x, s);
        }
      }
      // the slot's 8 tap groups: half-mirror, then the two quad swaps (every lane of the 8 ends
      // with the sum)
      s += dppF<0x141>(s);
      s += dppF<0x4E>(s);
      s += dppF<0xB1>(s);
      if (q == 0 && j < jHi) a.aOut[j] = s;
    }
  }
  wsSignal(&c->amFree, lane);
}


// ---- host side ---------------------------------------------------------------------------------

struct CfLayout {
  int padShift;
  int planeStride;
};

// Lane groups of ds_read_b128 (MI355X_MICROARCH.md, LDS): 4 x 16 lanes, one LDS cycle each.
inline constexpr int kB128Groups[4][16] = {
    {0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27},
    {4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31},
    {32, 33, 34, 35, 44, 45, 46, 47, 52, 53, 54, 55, 56, 57, 58, 59},
    {36, 37, 38, 39, 40, 41, 42, 43, 48, 49, 50, 51, 60, 61, 62, 63}};

// Pick the plane padding and the I/Q plane offset that minimise the A-fragment bank conflicts
// for this (D, KS), within the LDS budget. Wu: 16-byte slots per plane; rowUnits: slots between two
// A rows (4 D for f16 units of 8 samples, 2 D for int8 slots of 16; 0 = 4 D).
// blocks16: the 4-way kernel's 16 x 16 x 32 reads (lane l: row l % 16, slot 4 s + l / 16, one plane per
// read) instead of the 32 x 32 ones (row l % 16, slot 2 s + l / 32, lanes 16-31 of l % 32 in the Q plane).
inline CfLayout cfPlaneLayout(int D, int KS, int Wu, int nPlanes, size_t extra = kCfPartialBytes, int kSteps = 0,
                              int rowUnits = 0, bool blocks16 = false) {
  if (rowUnits <= 0) rowUnits = 4 * D;
  CfLayout best{4, 0};
  double bestCost = 1e30;
  for (int p = 4; p >= 1; --p) {
    const int units = Wu + (Wu >> p) + 1;
    const int base = (16 * units + 255) / 256 * 256;
    for (int qoff = 0; qoff < 16; ++qoff) {
      const int stride = base + 16 * qoff;
      if (nPlanes * (size_t)stride + extra > (size_t)kCfDynLdsMax) continue;
      double cost = 0;
      for (int s = 0; s < (kSteps > 0 ? kSteps : kCfWaves * KS); ++s) {
        for (const auto& grp : kB128Groups) {
          int slots[16][4];
          int cnt[16] = {};
          int worst = 1;
          for (int li = 0; li < 16; ++li) {
            const int l = grp[li];
            const int u = blocks16 ? rowUnits * (l & 15) + 4 * s + (l >> 4) : rowUnits * (l & 15) + 2 * s + (l >> 5);
            const int unit = u + (u >> p) + (!blocks16 && ((l >> 4) & 1) ? stride / 16 : 0);
            const int slot = unit & 15;
            bool dup = false;
            for (int c = 0; c < cnt[slot]; ++c) dup |= slots[slot][c] == unit;
            if (!dup && cnt[slot] < 4) slots[slot][cnt[slot]++] = unit;
            worst = cnt[slot] > worst ? cnt[slot] : worst;
          }
          cost += worst;
        }
      }
      cost += 1e-3 * (nPlanes * (double)stride) / 1024.0;  // tie-break: less LDS
      if (cost < bestCost) {
        bestCost = cost;
        best = CfLayout{p, stride};
      }
    }
  }
  return best;
}


// The fused audio stage computes AM / audio indices in 32 bits: every AM index of the launch (tiles x 512
// plus the history) and every audio window offset (j aD, j <= aN + 8) must stay below 2^31.
inline bool audioIndexFits(int64_t tiles, int64_t amH, int64_t aN, int64_t aD, int64_t aT) {
  const int64_t lim = (int64_t)1 << 30;  // headroom for the sums formed on top of each
  return tiles * 512 + 512 + amH + aT < lim && (aN + 16) * aD + amH < lim;
}

// The order of the 8 output slots of an audio batch (8 consecutive outputs, aD samples apart): the
// permutation whose two 32-lane halves (slots 0-3, 4-7; each slot's 8 lanes read 8 consecutive floats)
// hit the fewest distinct addresses per LDS bank in a ds_read_b32 (2 groups of 32 lanes, 32 banks).
// At aD = 20: outputs 0, 2, 4, 6 | 1, 3, 5, 7 - conflict free. Packed 4 bits per slot.
inline uint32_t audioSlotPerm(int aD) {
  int perm[8] = {0, 1, 2, 3, 4, 5, 6, 7};
  int best[8] = {0, 1, 2, 3, 4, 5, 6, 7};
  int bestCost = 1 << 30;
  auto cost = [&](const int* p) {
    int c = 0;
    for (int h = 0; h < 2; ++h) {
      int hits[32] = {};
      int worst = 0;
      for (int o = 4 * h; o < 4 * h + 4; ++o)
        for (int q = 0; q < 8; ++q) {
          const int bank = (int)(((int64_t)p[o] * aD + q) & 31);
          worst = ++hits[bank] > worst ? hits[bank] : worst;
        }
      c += worst;
    }
    return c;
  };
  // all 8! orders; the first of the cheapest (the identity when nothing beats it)
  auto visit = [&](auto&& self, int k) -> void {
    if (k == 8) {
      const int c = cost(perm);
      if (c < bestCost) {
        bestCost = c;
        for (int i = 0; i < 8; ++i) best[i] = perm[i];
      }
      return;
    }
    for (int i = k; i < 8; ++i) {
      const int t = perm[k];
      perm[k] = perm[i];
      perm[i] = t;
      self(self, k + 1);
      perm[i] = perm[k];
      perm[k] = t;
    }
  };
  visit(visit, 0);
  uint32_t packed = 0;
  for (int o = 0; o < 8; ++o) packed |= (uint32_t)best[o] << (4 * o);
  return packed;
}

// Before a wave-specialised launch: report an earlier launch's abort (hipErrorLaunchTimeOut), arm this
// one (spin limit, the device's abort word). Defined in fir_cf_mfma.hip.
hipError_t wsPrepareLaunch(hipStream_t stream, int32_t& spinLimit, uint32_t*& abortOut);

// The 4-way split-K int8 kernel (fir_i8_ws4.hip) for a launch whose iq4 / sub / taps / out / T / D /
// nOut / nIn / tiles (and, with `audio`, the audio fields) are set: hipErrorNotSupported when the
// shape does not fit it.
hipError_t launchFirI8Ws4(I8DecArgs a, int ksteps, int epi, bool audio, hipStream_t stream);
// audioSlotPerm(aD), cached (fir_i8_ws4.hip)
uint32_t cachedAudioSlotPerm(int aD);

}  // namespace gsdr_amd
