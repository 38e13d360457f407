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
#include "ws_common.h"

#include <gsdr/gsdr_amd.h>

namespace gsdr_amd {

constexpr int kW4Consumers = 4;                                    // one per SIMD
constexpr int kW4Threads = (kW4Consumers + kWsProducers) * kWave;  // 512
constexpr int kW4PartialBytes = kW4Consumers * 16 * kWave * 4;     // 16 KB per partial buffer
constexpr int kW4MaxKS = 22;                                       // K <= 4 x 22 x 16 = 1408

// A-fragment reads in flight ahead of the MFMAs (K-steps)
#ifndef GSDR_W4_PF
#define GSDR_W4_PF 3
#endif

// Consumer wave `wave` reduces accumulator registers wave, wave + 4 (I) and wave + 8, wave + 12 (Q)
// of block-local tile j over the 4 waves' partials (wave order), then the epilogue: the AM ring and
// the audio hand-off (AUD), or the output store.
template <int EPI, bool AUD>
__device__ __forceinline__ void w4Reduce(const I8DecArgs& a, const float* part, WsCtl* c, float outScale, int tile,
                                         int j, int tid, float* ring, bool lead) {
  const int lane = tid & (kWave - 1);
  const int wave = tid >> 6;
  const int half = lane >> 5, col = lane & 31;
  const int b = j & 1;
  wsWait(c, &c->partsFull[b], kW4Consumers * ((j >> 1) + 1));
  const float* pb = part + b * (kW4PartialBytes / 4);
  float yi[2] = {0.0f, 0.0f}, yq[2] = {0.0f, 0.0f};
#pragma unroll
  for (int v = 0; v < kW4Consumers; ++v)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      yi[h] += pb[(v * 16 + wave + 4 * h) * kWave + lane];
      yq[h] += pb[(v * 16 + wave + 4 * h + 8) * kWave + lane];
    }
  wsSignal(&c->partsFree[b], lane);
  // slot j mod kAmRing is free once the producers finished the audio outputs of tile j - kAmRing + 1
  if (AUD && j - kAmRing + 2 > 0) wsWait(c, &c->amFree, kWsProducers * (j - kAmRing + 2));
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    // accumulator register i = wave + 4 h holds row (i & 3) + 8 (i >> 2) + 4 half of the 32 x 32 tile
    const int orow = wave + 8 * h + 4 * half;
    const int64_t k = (int64_t)tile * kCfTileOut + 32 * orow + col;
    if constexpr (AUD) {
      const float v = __builtin_amdgcn_sqrtf(fmaf(yi[h], yi[h], yq[h] * yq[h])) * outScale;
      const int pos = (j & (kAmRing - 1)) * kCfTileOut + 32 * orow + col;
#if GSDR_WS_DIAG
      wsDiag(3, pos < 0 || pos >= kAmRing * kCfTileOut);
#endif
      const float rv = k < a.nOut ? v : 0.0f;
      ring[pos] = rv;
      if (pos < kAmRingMirror) ring[kAmRing * kCfTileOut + pos] = rv;
      // the lead tile belongs to the previous block (computed here only for the audio windows)
      if (a.out != nullptr && k < a.nOut && !(lead && j == 0)) reinterpret_cast<float*>(a.out)[k] = v;
    } else if (k < a.nOut) {
      if (EPI == kEpiAm)
        reinterpret_cast<float*>(a.out)[k] = __builtin_amdgcn_sqrtf(fmaf(yi[h], yi[h], yq[h] * yq[h])) * outScale;
      else
        reinterpret_cast<f2*>(a.out)[k] = f2{yi[h], yq[h]} * outScale;
    }
  }
  if constexpr (AUD) wsSignal(&c->amSlot[j & (kAmRing - 1)], lane);
}

// The consumer waves: B fragments of this wave's K quarter in VGPRs for the whole launch, then per
// tile 2 KS MFMAs, the partials into buffer i & 1, and the reduction of the previous tile (so no wave
// waits for the slowest one before its next MFMAs).
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
  // the tap staging area becomes the partial-sum area once every consumer wave has its fragments
  wsSignal(&c->tapsRead, lane);

  const int arow = lane & 15;
  const int comp = (lane >> 4) & 1;
  const int uRow = 4 * D * arow + half;
  const float outScale = ldexpf(1.0f / 127.0f, -sh);
  for (int i = 0; i < n; ++i) {
    const int set = i & 1;
    wsWait(c, &c->planesFull[set], kWsProducers * ((i >> 1) + 1));
    const int8_t* pI = smem + set * 2 * a.planeStride + comp * a.planeStride;
    v16f acc = v16f{};
    h8 xa[KS];
    auto readA = [&](int s) {
      xa[s] = *reinterpret_cast<const h8*>(pI + 16 * cfPhys(uRow + 2 * (wave * KS + s), a.padShift));
    };
#pragma unroll
    for (int s = 0; s < PF; ++s) readA(s);
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      if (s + PF < KS) readA(s + PF);
      asm volatile("" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(xa[s], bh[s], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(xa[s], bl[s], acc, 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    wsSignal(&c->planesFree[set], lane);  // this wave's A reads are complete
    const int b = i & 1;
    wsWait(c, &c->partsFree[b], kW4Consumers * (i >> 1));  // tile i - 2 reduced by every wave
    if (i < 2) wsWait(c, &c->tapsRead, kW4Consumers);
    float* pb = part + b * (kW4PartialBytes / 4);
#pragma unroll
    for (int k = 0; k < 16; ++k) pb[(wave * 16 + k) * kWave + lane] = acc[k];
    wsSignal(&c->partsFull[b], lane);
    if (i >= 1) w4Reduce<EPI, AUD>(a, part, c, outScale, t0 + i - 1, i - 1, tid, ring, lead);
  }
  if (n >= 1) w4Reduce<EPI, AUD>(a, part, c, outScale, t0 + n - 1, n - 1, tid, ring, lead);
}

template <int KS, int G, int EPI, bool AUD>
__global__ __launch_bounds__(kW4Threads, 1) void firI8Ws4Kernel(I8DecArgs a8, int Wl) {
  extern __shared__ __attribute__((aligned(16))) int8_t smem[];
  float* part = reinterpret_cast<float*>(smem + 4 * a8.planeStride);
  float* ring = AUD ? reinterpret_cast<float*>(smem + 4 * a8.planeStride + 2 * kW4PartialBytes) : nullptr;
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
  const int span = off0 + 64 * KS;
  float hm = 0.0f;
  for (int i = tid; i < span; i += kW4Threads) {
    const int j = i - off0;
    const float h = (j >= 0 && j < T) ? a8.taps[j] : 0.0f;
    part[i] = h;
    hm = fmaxf(hm, fabsf(h));
  }
  for (int i = tid; i < 4 * a8.planeStride / 16; i += kW4Threads) reinterpret_cast<uint4*>(smem)[i] = uint4{0, 0, 0, 0};
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
  const int sh = hMax > 0.0f ? 14 - ilogbf(hMax) : 0;  // max |h 2^sh| in [2^14, 2^15)

  if (wave >= kW4Consumers) {
    // ================= producers (firI8WsKernel's, signalling 4 consumer waves) =================
    const int ptid = tid - kW4Consumers * kWave;
    I8WsWindow<G> wA, wB;
    const i4v r0 = wsI8TileRsrc(a8, t0, true);
#pragma unroll
    for (int j = 0; j < G; ++j) wsI8LoadGroup<G>(r0, Wl, ptid, j, wA);
    const i4v r1 = wsI8TileRsrc(a8, t0 + 1, n > 1);
#pragma unroll
    for (int j = 0; j < G; ++j) wsI8LoadGroup<G>(r1, Wl, ptid, j, wB);
    float ht[kAudioTapsPerLane];  // audio taps (lane % 8) + 8 u
#pragma unroll
    for (int u = 0; u < kAudioTapsPerLane; ++u) {
      const int tp = (lane & 7) + 8 * u;
      ht[u] = AUD && tp < a8.aT ? a8.aTaps[tp] : 0.0f;
    }
    for (int i = 0;; i += 2) {
      wsI8ProducerTile<G, kW4Consumers>(a8, Wl, smem, c, n, t0 + i, i, ptid, wA, [&] {
        if (AUD && i >= kAudioLag) wsAudioTile<kW4Consumers>(a8, ring, c, t0, n, lead, i - kAudioLag, ptid, ht);
      });
      if (i + 1 >= n) break;
      wsI8ProducerTile<G, kW4Consumers>(a8, Wl, smem, c, n, t0 + i + 1, i + 1, ptid, wB, [&] {
        if (AUD && i + 1 >= kAudioLag) wsAudioTile<kW4Consumers>(a8, ring, c, t0, n, lead, i + 1 - kAudioLag, ptid, ht);
      });
      if (i + 2 >= n) break;
    }
    if constexpr (AUD)
      for (int t = n > kAudioLag ? n - kAudioLag : 0; t < n; ++t)
        wsAudioTile<kW4Consumers>(a8, ring, c, t0, n, lead, t, ptid, ht);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no load outlives the wave
    return;
  }
  w4Consumers<KS, EPI, AUD>(a8, smem, part, c, sh, t0, n, tid, ring, lead);
}

// ---- host side ---------------------------------------------------------------------------------

namespace {

template <int KS, int G, int EPI, bool AUD>
hipError_t launchW4G(const I8DecArgs& a, int Wl, size_t lds, int grid, hipStream_t stream) {
  auto kernel = &firI8Ws4Kernel<KS, G, EPI, AUD>;
  const hipError_t attrErr =
      hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize, kCfDynLdsMax);
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

// Instantiated K quarters (K-steps of 16 per consumer wave): a shape runs on the smallest one that
// covers it (the extra K-steps meet zero taps). 21 is C5's (1023 taps, D = 10: K = 1333 -> 84 steps).
constexpr int kW4KS[] = {2, 4, 6, 8, 11, 14, 17, 21, 22};

int w4PickKS(int ksteps) {
  const int need = (ksteps + kW4Consumers - 1) / kW4Consumers;
  for (int k : kW4KS)
    if (k >= need) return k;
  return 0;
}

hipError_t launchW4Any(const I8DecArgs& a, int Wl, size_t lds, int grid, int epi, bool audio, hipStream_t stream) {
  switch (a.KS) {
    case 2: return launchW4KS<2>(a, Wl, lds, grid, epi, audio, stream);
    case 4: return launchW4KS<4>(a, Wl, lds, grid, epi, audio, stream);
    case 6: return launchW4KS<6>(a, Wl, lds, grid, epi, audio, stream);
    case 8: return launchW4KS<8>(a, Wl, lds, grid, epi, audio, stream);
    case 11: return launchW4KS<11>(a, Wl, lds, grid, epi, audio, stream);
    case 14: return launchW4KS<14>(a, Wl, lds, grid, epi, audio, stream);
    case 17: return launchW4KS<17>(a, Wl, lds, grid, epi, audio, stream);
    case 21: return launchW4KS<21>(a, Wl, lds, grid, epi, audio, stream);
    case 22: return launchW4KS<22>(a, Wl, lds, grid, epi, audio, stream);
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
  a.Wu = 60 * a.D + 8 * a.KS;  // window units (8 samples) per tile: 480 D + 64 KS samples
  const int Wl = std::min(a.Wu, (511 * a.D + a.T + 7) / 8);
  if (Wl > 4 * kWsPThreads) return hipErrorNotSupported;
  const size_t ringBytes = audio ? sizeof(float) * (kAmRing * kCfTileOut + kAmRingMirror) : 0;
  const size_t extra = 2 * (size_t)kW4PartialBytes + ringBytes;
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
      lay = cfPlaneLayout(a.D, a.KS, a.Wu, 4, extra, kW4Consumers * a.KS);
      if (cache.size() >= 16) cache.erase(cache.begin());
      cache.emplace_back(key, lay);
    }
  }
  if (lay.planeStride == 0) return hipErrorNotSupported;
  a.padShift = lay.padShift;
  a.planeStride = lay.planeStride;
  a.dbp = 1;
  const size_t lds = 4 * (size_t)a.planeStride + extra;
  if (lds > (size_t)kCfDynLdsMax) return hipErrorNotSupported;
  const int grid = (int)(a.tiles < 256 ? a.tiles : 256);
  if (hipError_t e = wsPrepareLaunch(stream, a.spinLimit, a.abortOut); e != hipSuccess) return e;
  return launchW4Any(a, Wl, lds, grid, epi, audio, stream);
}

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
