// Exact int8 MFMA FIR for interleaved int8 IQ input (the C2 chain: int8 IQ -> cf32 -> FC FIR
// [-> AM envelope]), decimation 1, up to 129 real taps.
//
// Arithmetic. gsdrInt8ToNormFloat maps x to fmaxf(-1, x/127) = x'/127 with x' = max(x, -127), so
//     y[k] = sum_j h_j x'[k+j] / 127.
// The taps are quantised once to a 30-bit fixed point H_j = rint(h_j 2^sc) (sc from max|h|, error
// <= max|h| 2^-31 per tap) and split into four signed base-256 digits (limbs) H = L0 + L1 2^8 +
// L2 2^16 + L3 2^24, |L| <= 128. Every sum_j L_lj x'[k+j] is then an EXACT int32 dot product of
// int8 values - what v_mfma_i32_32x32x32_i8 computes - and
//     y = ((S0 + S1 2^8) + (S2 + S3 2^8) 2^16) 2^-sc / 127
// is rounded once or twice in fp32. The result is closer to the float64 oracle than the fp32
// direct form (error ~1e-7 of sum|h||x| vs ~T^0.5 eps); tests/test_gpu_parity.py checks it.
//
// GEMM shape (Toeplitz). Output k = 32 m + n (row m, column n < 32):
//     C[m][n] = sum_kappa A[m][kappa] B[kappa][n],  A[m][kappa] = x'[32 m + kappa],
//     B[kappa][n] = H[kappa - n] (0 <= kappa - n < T, else 0),  kappa < K = 32 S >= T + 31.
// One 32x32x32 MFMA tile holds 16 rows of the I stream and the same 16 rows of the Q stream
// (A rows 0-15 read the I plane, rows 16-31 the Q plane), so a lane ends with I and Q of the
// same output in registers i and i+8: the AM envelope needs no data movement.
// Per wave tile: 512 complex outputs = S K-steps x 4 limbs MFMAs; the B fragments (taps) live in
// registers for the whole kernel (16 S VGPRs), the A fragment is one ds_read_b128 per K-step
// from the block's staged, clamped, I/Q-deinterleaved LDS window.
//
// Cost per complex output: 4 limbs x K/32 MFMA-cycles: at T = 127 (S = 5) 1.25 SIMD-cycles per
// output, ~2 Tsamples/s of MFMA throughput on 1024 SIMDs - above the ~1 Tsample/s the
// 6-byte-per-sample HBM stream allows, so the chain becomes HBM-bound.
#include "kcommon.h"
#include "fir_launch.h"

namespace gsdr_amd {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

constexpr int kI8Waves = 4;
constexpr int kI8Threads = kI8Waves * kWave;
constexpr int kI8TileOut = 512;                  // 16 rows x 32 columns per wave
constexpr int kI8ChunkOut = kI8Waves * kI8TileOut;  // 2048 outputs per block iteration
constexpr int kI8MaxS = 5;                       // K <= 160 -> T <= 129

// Lane -> k map of the 16 bytes of an A / B fragment of v_mfma_i32_32x32x32_i8. Only its
// consistency between A and B matters (a dot product is invariant under a common permutation
// of k); tools/probes/mfma_i8_layout.hip confirms A/B/C maps with exact integers on gfx950.
__device__ __forceinline__ int i8FragK(int half, int j) { return 16 * half + j; }

struct I8FirArgs {
  const int8_t* iq;   // interleaved I, Q
  const float* taps;
  void* out;
  int64_t nOut;
  int64_t nIn;        // complex samples readable
  int32_t T;
  int32_t chunks;
};

// 0x80 (-128) -> 0x81 (-127) in every byte: fmaxf(-1, x/127) == max(x, -127)/127.
__device__ __forceinline__ uint32_t clampMinByte(uint32_t w) {
  const uint32_t low7 = w & 0x7F7F7F7Fu;
  const uint32_t nonzeroLow = (low7 + 0x7F7F7F7Fu) & 0x80808080u;  // no carries: 0x7F + 0x7F < 0x100
  const uint32_t isMin = (w & 0x80808080u) & ~nonzeroLow;
  return w | (isMin >> 7);
}

__device__ __forceinline__ int8_t byteAt(int v, int i) { return (int8_t)((v >> (8 * i)) & 0xFF); }

// 16 interleaved IQ bytes at p as four little-endian words, for a pointer aligned to ALIGN bytes.
template <int ALIGN>
__device__ __forceinline__ void load16(const int8_t* p, uint32_t (&w)[4]) {
  if (ALIGN >= 16) {
    const int4 v = *reinterpret_cast<const int4*>(p);
    w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
  } else if (ALIGN >= 4) {
#pragma unroll
    for (int q = 0; q < 4; ++q) w[q] = reinterpret_cast<const uint32_t*>(p)[q];
  } else {
    const uint16_t* h = reinterpret_cast<const uint16_t*>(p);
#pragma unroll
    for (int q = 0; q < 4; ++q) w[q] = (uint32_t)h[2 * q] | ((uint32_t)h[2 * q + 1] << 16);
  }
}

// Raw (not yet clamped) staging words of one chunk window held by one thread: groups tid and
// tid + 256 of 8 IQ samples each.
template <int kPlane>
struct StageRegs {
  static constexpr int kGroups = kPlane / 8;
  static constexpr int kPerThread = (kGroups + kI8Threads - 1) / kI8Threads;
  uint32_t w[kPerThread][4];
};

// SAFE = false: the whole window lies inside the input (every chunk but the last ones), pure
// vector loads that stay in flight until storeStage; SAFE = true: byte-guarded tail.
template <int ALIGN, int kPlane, bool SAFE>
__device__ __forceinline__ void loadStageImpl(const I8FirArgs& a, int64_t s0, int tid, StageRegs<kPlane>& r) {
#pragma unroll
  for (int u = 0; u < StageRegs<kPlane>::kPerThread; ++u) {
    // every lane issues every load (surplus lanes re-read the last group, which storeStage
    // skips): branch-free issue keeps the vmcnt bookkeeping exact across the pipeline
    const int g = SAFE ? tid + u * kI8Threads : min(tid + u * kI8Threads, StageRegs<kPlane>::kGroups - 1);
    if (SAFE && g >= StageRegs<kPlane>::kGroups) break;
    const int64_t smp = s0 + 8 * g;
    if (!SAFE || smp + 8 <= a.nIn) {
      load16<ALIGN>(a.iq + 2 * smp, r.w[u]);
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        uint32_t acc = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const int64_t byteIdx = 2 * smp + 4 * q + b;
          const uint32_t v = byteIdx < 2 * a.nIn ? (uint8_t)a.iq[byteIdx] : 0u;
          acc |= v << (8 * b);
        }
        r.w[u][q] = acc;
      }
    }
  }
}


// Clamp, split I and Q and write the thread's groups to the LDS planes.
template <int kPlane>
__device__ __forceinline__ void storeStage(const StageRegs<kPlane>& r, int8_t* planes, int tid) {
#pragma unroll
  for (int u = 0; u < StageRegs<kPlane>::kPerThread; ++u) {
    const int g = tid + u * kI8Threads;
    if (g >= StageRegs<kPlane>::kGroups) break;
    uint32_t w[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) w[q] = clampMinByte(r.w[u][q]);
    // bytes: I0 Q0 I1 Q1 | I2 Q2 I3 Q3 | ...
    const uint32_t i01 = __builtin_amdgcn_perm(w[1], w[0], 0x06040200u);
    const uint32_t i23 = __builtin_amdgcn_perm(w[3], w[2], 0x06040200u);
    const uint32_t q01 = __builtin_amdgcn_perm(w[1], w[0], 0x07050301u);
    const uint32_t q23 = __builtin_amdgcn_perm(w[3], w[2], 0x07050301u);
    *reinterpret_cast<uint2*>(planes + 8 * g) = uint2{i01, i23};
    *reinterpret_cast<uint2*>(planes + kPlane + 8 * g) = uint2{q01, q23};
  }
}

// One wave's 16 rows x 32 columns of I and Q: S K-steps x 4 limbs MFMAs, then the epilogue.
// FULL: every output of the chunk exists (interior chunks), so the stores need no guard and
// the waitcnt pass can count them exactly instead of draining all loads at the next stage.
template <int S, int EPI, int kPlane, bool FULL>
__device__ __forceinline__ void computeTile(const I8FirArgs& a, const int8_t* planes, const v4i (&bf)[S][4],
                                            int64_t s0, int wave, int lane, float outScale, float hiScale) {
  const int half = lane >> 5;
  const int col = lane & 31;
  const int row = lane & 31;  // A row: 0-15 read the I plane, 16-31 the Q plane
  v16i acc[4];
#pragma unroll
  for (int l = 0; l < 4; ++l) acc[l] = v16i{};
  const int8_t* rowBase = planes + (row >> 4) * kPlane + 32 * (wave * 16 + (row & 15)) + 16 * half;
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const v4i av = *reinterpret_cast<const v4i*>(rowBase + 32 * s);
#pragma unroll
    for (int l = 0; l < 4; ++l) acc[l] = __builtin_amdgcn_mfma_i32_32x32x32_i8(av, bf[s][l], acc[l], 0, 0, 0);
  }
  // limbs -> float; I and Q of one output sit in registers i and i + 8 of the same lane
  const int64_t tileOut = s0 + (int64_t)wave * kI8TileOut;
  const bool full = FULL || tileOut + kI8TileOut <= a.nOut;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int mrow = (i & 3) + 8 * (i >> 2) + 4 * half;
    const int64_t k = tileOut + 32 * mrow + col;
    const int loI = acc[0][i] + (acc[1][i] << 8), hiI = acc[2][i] + (acc[3][i] << 8);
    const int loQ = acc[0][i + 8] + (acc[1][i + 8] << 8), hiQ = acc[2][i + 8] + (acc[3][i + 8] << 8);
    const float yi = fmaf((float)hiI, hiScale, (float)loI * outScale);
    const float yq = fmaf((float)hiQ, hiScale, (float)loQ * outScale);
    if (full || k < a.nOut) {
      if (EPI == kEpiAm) reinterpret_cast<float*>(a.out)[k] = amEnvelope(f2{yi, yq});
      else reinterpret_cast<f2*>(a.out)[k] = f2{yi, yq};
    }
  }
}

template <int S, int EPI, int ALIGN>
__global__ __launch_bounds__(kI8Threads) void firI8MfmaKernel(I8FirArgs a) {
  constexpr int kWin = kI8ChunkOut - 32 + 32 * S;  // samples a block iteration reads
  constexpr int kPlane = (kWin + 15) / 16 * 16;
  __shared__ __attribute__((aligned(16))) int8_t planes[2 * kPlane];
  __shared__ int hq[32 * kI8MaxS];
  __shared__ float waveMax[kI8Waves];

  const int tid = threadIdx.x;
  const int lane = tid & (kWave - 1);
  const int wave = waveUniform(tid >> 6);
  const int T = a.T;

  // ---- taps -> 30-bit fixed point (block-uniform scale) -----------------------------------
  float hv = tid < T ? a.taps[tid] : 0.0f;
  float m = fabsf(hv);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off));
  if (lane == 0) waveMax[wave] = m;
  __syncthreads();
  const float maxAbs = fmaxf(fmaxf(waveMax[0], waveMax[1]), fmaxf(waveMax[2], waveMax[3]));
  const int sc = maxAbs > 0.0f ? 29 - ilogbf(maxAbs) : 0;  // max|H| < 2^30
  if (tid < 32 * S) hq[tid] = tid < T ? (int)rintf(ldexpf(hv, sc)) : 0;
  __syncthreads();
  const float outScale = ldexpf(1.0f / 127.0f, -sc);
  const float hiScale = outScale * 65536.0f;

  // ---- B fragments: bf[s][l] holds limb l of H[kappa - n] for this lane's 16 kappas ----------
  const int half = lane >> 5;
  const int col = lane & 31;
  v4i bf[S][4];
#pragma unroll
  for (int s = 0; s < S; ++s) {
    int packed[4][4] = {};
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int idx = 32 * s + i8FragK(half, j) - col;
      int v = (idx >= 0 && idx < T) ? hq[idx] : 0;
#pragma unroll
      for (int l = 0; l < 4; ++l) {
        const int digit = l < 3 ? (int)(int8_t)(v & 0xFF) : v;  // signed base-256 digit
        v = (v - digit) >> 8;
        packed[l][j >> 2] |= (digit & 0xFF) << (8 * (j & 3));
      }
    }
#pragma unroll
    for (int l = 0; l < 4; ++l) bf[s][l] = v4i{packed[l][0], packed[l][1], packed[l][2], packed[l][3]};
  }

  // Software pipeline over this block's chunks c, c + G, c + 2G, ... (G = gridDim.x): the raw
  // window of chunk c + 2G is loaded into registers while chunk c is multiplied, so the HBM
  // latency of the staging loads overlaps two chunks of MFMA work; the window of chunk c + G
  // (loaded one iteration earlier) is written to the LDS planes between the two barriers.
  // Only "interior" chunks (window wholly inside the input) take this path; their prefetch is
  // unconditional, clamped to the last interior chunk (an L2 hit), so no register set is ever
  // conditionally live and the loads stay in flight across the MFMA work.
  const int G = gridDim.x;
  const int interior = a.nIn >= kPlane ? (int)min((int64_t)a.chunks, (a.nIn - kPlane) / kI8ChunkOut + 1) : 0;
  const int lastInterior = interior - 1;
  int c = blockIdx.x;
  if (c < interior) {
    StageRegs<kPlane> ra, rb;
    loadStageImpl<ALIGN, kPlane, false>(a, (int64_t)c * kI8ChunkOut, tid, ra);
    loadStageImpl<ALIGN, kPlane, false>(a, (int64_t)min(c + G, lastInterior) * kI8ChunkOut, tid, rb);
    storeStage<kPlane>(ra, planes, tid);
    __syncthreads();
    for (;;) {
      // even half: compute c from the planes, prefetch c + 2G into ra, then stage rb (c + G)
      loadStageImpl<ALIGN, kPlane, false>(a, (int64_t)min(c + 2 * G, lastInterior) * kI8ChunkOut, tid, ra);
      computeTile<S, EPI, kPlane, true>(a, planes, bf, (int64_t)c * kI8ChunkOut, wave, lane, outScale, hiScale);
      __syncthreads();
      c += G;
      if (c >= interior) break;
      storeStage<kPlane>(rb, planes, tid);
      __syncthreads();
      // odd half: same with the register sets swapped
      loadStageImpl<ALIGN, kPlane, false>(a, (int64_t)min(c + 2 * G, lastInterior) * kI8ChunkOut, tid, rb);
      computeTile<S, EPI, kPlane, true>(a, planes, bf, (int64_t)c * kI8ChunkOut, wave, lane, outScale, hiScale);
      __syncthreads();
      c += G;
      if (c >= interior) break;
      storeStage<kPlane>(ra, planes, tid);
      __syncthreads();
    }
  }
  // edge chunks (window runs past the input end): byte-guarded loads, no pipelining
  for (; c < a.chunks; c += G) {
    StageRegs<kPlane> r;
    loadStageImpl<ALIGN, kPlane, true>(a, (int64_t)c * kI8ChunkOut, tid, r);
    storeStage<kPlane>(r, planes, tid);
    __syncthreads();
    computeTile<S, EPI, kPlane, false>(a, planes, bf, (int64_t)c * kI8ChunkOut, wave, lane, outScale, hiScale);
    __syncthreads();
  }
}

namespace {
template <int S, int ALIGN>
hipError_t launchI8Aligned(const I8FirArgs& a, int epi, hipStream_t stream, int grid) {
  if (epi == kEpiAm)
    hipLaunchKernelGGL((firI8MfmaKernel<S, kEpiAm, ALIGN>), dim3(grid), dim3(kI8Threads), 0, stream, a);
  else
    hipLaunchKernelGGL((firI8MfmaKernel<S, kEpiComplex, ALIGN>), dim3(grid), dim3(kI8Threads), 0, stream, a);
  return hipGetLastError();
}

template <int S>
hipError_t launchI8(const I8FirArgs& a, int epi, hipStream_t stream, int grid) {
  const uintptr_t p = reinterpret_cast<uintptr_t>(a.iq);
  if ((p & 15u) == 0) return launchI8Aligned<S, 16>(a, epi, stream, grid);
  if ((p & 3u) == 0) return launchI8Aligned<S, 4>(a, epi, stream, grid);
  return launchI8Aligned<S, 2>(a, epi, stream, grid);
}
}  // namespace

bool firI8MfmaEligible(size_t tapCount, size_t decimation, const void* in) {
  // IQ samples are 2-byte pairs: any sample-aligned pointer works (16/4/2-byte load variants)
  return tapCount >= 1 && tapCount <= 32 * kI8MaxS - 31 && decimation <= 1 &&
         (reinterpret_cast<uintptr_t>(in) & 1u) == 0;
}

hipError_t launchFirI8Mfma(const int8_t* iq, const float* taps, size_t tapCount, void* out, size_t nOut, int epi,
                           hipStream_t stream) {
  I8FirArgs a{};
  a.iq = iq;
  a.taps = taps;
  a.out = out;
  a.nOut = (int64_t)nOut;
  a.nIn = (int64_t)nOut - 1 + (int64_t)tapCount;
  a.T = (int32_t)tapCount;
  const int64_t chunks = ((int64_t)nOut + kI8ChunkOut - 1) / kI8ChunkOut;
  if (chunks > 0x7fffffff) return hipErrorInvalidValue;
  a.chunks = (int32_t)chunks;
  // enough blocks for 3 per CU; each block then amortises its tap preparation over its chunks
  const int grid = (int)(chunks < 256 * 2 ? chunks : 256 * 2);  // 2 resident blocks per CU (252 VGPRs)
  const int S = (int)((tapCount + 31 + 31) / 32);
  switch (S) {
    case 1: return launchI8<1>(a, epi, stream, grid);
    case 2: return launchI8<2>(a, epi, stream, grid);
    case 3: return launchI8<3>(a, epi, stream, grid);
    case 4: return launchI8<4>(a, epi, stream, grid);
    default: return launchI8<5>(a, epi, stream, grid);
  }
}

}  // namespace gsdr_amd
