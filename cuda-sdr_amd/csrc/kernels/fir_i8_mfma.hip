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
//
// Data movement (v3). Each block owns a contiguous range of 4096-output chunks (its windows
// overlap by T - 1 samples, so the overlap is an L2 hit). The raw interleaved window of a chunk
// goes HBM -> LDS by LDS-DMA (global_load_lds_dwordx4, no VGPRs) into a ring of kRing slots
// filled kRing - 1 chunks ahead, so ~25 KB of loads per block stay in flight across the MFMA
// work and the barriers; one pass per chunk then clamps and splits the slot into the I / Q
// planes the A fragments read. The DMA is issued from inline asm and retired with counted
// `s_waitcnt vmcnt(N)` (the compiler does not see it): N counts the DMA pieces and the epilogue
// stores issued after the slot being waited for (see vmWaitFor).
#include "kcommon.h"
#include "fir_launch.h"

namespace gsdr_amd {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

constexpr int kI8Waves = 4;
constexpr int kI8Threads = kI8Waves * kWave;
constexpr int kI8TileOut = 512;                                   // 16 rows x 32 columns
constexpr int kI8TilesPerWave = 2;
constexpr int kI8ChunkOut = kI8Waves * kI8TilesPerWave * kI8TileOut;  // 4096 outputs per chunk
constexpr int kI8MaxS = 5;                                        // K <= 160 -> T <= 129
constexpr int kRing = 4;                                          // LDS-DMA ring slots
constexpr int kPiece = 64 * 16;                                   // bytes per wave DMA instruction
// Epilogue stores per wave per chunk (one store instruction per lane output, 8 per tile).
constexpr int kStoresPerChunk = kI8TilesPerWave * 8;

// Lane -> k map of the 16 bytes of an A / B fragment of v_mfma_i32_32x32x32_i8. Only its
// consistency between A and B matters (a dot product is invariant under a common permutation
// of k); tools/probes/mfma_i8_layout.hip confirms A/B/C maps with exact integers on gfx950.
__device__ __forceinline__ int i8FragK(int half, int j) { return 16 * half + j; }

struct I8FirArgs {
  const int8_t* iq;   // interleaved I, Q (2-byte aligned)
  const float* taps;
  void* out;
  int64_t nOut;
  int64_t nIn;        // complex samples readable: nOut - 1 + T
  int32_t T;
  int32_t chunks;
  int8_t* carryDst;     // nullptr, or where the last T - 1 input samples go (may alias iq[0 .. T-1))
};

template <int S>
struct I8Geom {
  static constexpr int kWin = kI8ChunkOut - 32 + 32 * S;        // samples one chunk reads
  static constexpr int kPlane = (kWin + 15) / 16 * 16;           // bytes per I / Q plane
  static constexpr int kGroups = kPlane / 8;                     // 8-sample staging groups
  // slot: up to 14 bytes of alignment shift + the window + one dword of read-ahead
  static constexpr int kPieces = (14 + 2 * kPlane + 4 + kPiece - 1) / kPiece;
  static constexpr int kSlot = kPieces * kPiece;
};

// 0x80 (-128) -> 0x81 (-127) in every byte: fmaxf(-1, x/127) == max(x, -127)/127.
__device__ __forceinline__ uint32_t clampMinByte(uint32_t w) {
  const uint32_t low7 = w & 0x7F7F7F7Fu;
  const uint32_t nonzeroLow = (low7 + 0x7F7F7F7Fu) & 0x80808080u;  // no carries: 0x7F + 0x7F < 0x100
  const uint32_t isMin = (w & 0x80808080u) & ~nonzeroLow;
  return w | (isMin >> 7);
}

// Tap-limb table: 4 rows of kLimbRow bytes, tap j of limb l at l * kLimbRow + kLimbPad + j.
constexpr int kLimbPad = 32;
constexpr int kLimbRow = 256;
static_assert(kLimbPad + 32 * kI8MaxS + 20 <= kLimbRow && 4 * kLimbRow == 4 * kI8Threads, "limb table");

__device__ __forceinline__ float loadF32Async(const float* p) {
  float v;
  asm volatile("global_load_dword %0, %1, off" : "=v"(v) : "v"(p) : "memory");
  return v;
}

template <int N>
__device__ __forceinline__ void vmWait() {
  static_assert(N >= 0 && N <= 63, "vmcnt is 6 bits on gfx950");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// s_waitcnt vmcnt(n) for a wave-uniform runtime n in [LO, HI] (binary dispatch on constants).
template <int LO, int HI>
__device__ __forceinline__ void vmWaitDyn(int n) {
  if constexpr (LO == HI) {
    vmWait<LO>();
  } else {
    constexpr int MID = (LO + HI) / 2;
    if (n <= MID) vmWaitDyn<LO, MID>(n);
    else vmWaitDyn<MID + 1, HI>(n);
  }
}

// LDS barrier that leaves vector-memory operations (the DMA ring, the epilogue stores) in flight.
__device__ __forceinline__ void ldsBarrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// One LDS-DMA wave instruction: 64 lanes x 16 bytes from per-lane `src` to ldsDst + 16 lane.
__device__ __forceinline__ void dmaPiece(const void* src, uint32_t ldsDst) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(src), "s"(ldsDst)
      : "memory");
}

// Issue this wave's DMA pieces of chunk c's raw window into ring slot `slotLds` (LDS byte
// address). Lanes past the input end re-read the last 16-byte block that holds input bytes (it
// never crosses a page); the bytes they land only feed outputs >= nOut, which are not stored.
template <int S>
__device__ __forceinline__ void issueChunk(const I8FirArgs& a, uintptr_t alignedBase, uintptr_t lastBlock, int c,
                                           uint32_t slotLds, int wave, int lane) {
  using G = I8Geom<S>;
  const uintptr_t chunkBase = alignedBase + (uintptr_t)c * (2 * kI8ChunkOut);
#pragma unroll
  for (int p0 = 0; p0 < G::kPieces; p0 += kI8Waves) {
    const int p = p0 + wave;
    if (p < G::kPieces) {  // wave-uniform
      uintptr_t src = chunkBase + (uintptr_t)p * kPiece + 16 * lane;
      src = src < lastBlock ? src : lastBlock;
      dmaPiece(reinterpret_cast<const void*>(src), slotLds + p * kPiece);
    }
  }
}

// Clamp and split one landed slot into the I / Q planes: group g = samples [8g, 8g + 8) of the
// window, at slot bytes [shift + 16 g, shift + 16 g + 16).
template <int S>
__device__ __forceinline__ void splitSlot(const int8_t* slot, int8_t* planes, int shift, int tid) {
  using G = I8Geom<S>;
  const uint32_t* words = reinterpret_cast<const uint32_t*>(slot + (shift & ~3));
  const int sub = shift & 3;  // 0 or 2
#pragma unroll
  for (int u = 0; u < (G::kGroups + kI8Threads - 1) / kI8Threads; ++u) {
    const int g = tid + u * kI8Threads;
    if (g < G::kGroups) {
      uint32_t d[5];
#pragma unroll
      for (int q = 0; q < 5; ++q) d[q] = words[4 * g + q];
      uint32_t w[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) w[q] = clampMinByte(__builtin_amdgcn_alignbyte(d[q + 1], d[q], sub));
      // bytes: I0 Q0 I1 Q1 | I2 Q2 I3 Q3 | ...
      const uint32_t i01 = __builtin_amdgcn_perm(w[1], w[0], 0x06040200u);
      const uint32_t i23 = __builtin_amdgcn_perm(w[3], w[2], 0x06040200u);
      const uint32_t q01 = __builtin_amdgcn_perm(w[1], w[0], 0x07050301u);
      const uint32_t q23 = __builtin_amdgcn_perm(w[3], w[2], 0x07050301u);
      *reinterpret_cast<uint2*>(planes + 8 * g) = uint2{i01, i23};
      *reinterpret_cast<uint2*>(planes + G::kPlane + 8 * g) = uint2{q01, q23};
    }
  }
}

// AM epilogue: the same expression as amEnvelope with the hardware square root (v_sqrt_f32,
// <= 1 ulp) instead of the correctly rounded sequence - the MFMA outputs are not bit-identical to
// the fp32 chain anyway, and the 12-instruction IEEE fix-up was ~1/3 of the epilogue.
template <int EPI>
__device__ __forceinline__ void storeOut(void* out, int64_t k, f2 y) {
  if (EPI == kEpiAm) reinterpret_cast<float*>(out)[k] = __builtin_amdgcn_sqrtf(fmaf(y.x, y.x, y.y * y.y));
  else reinterpret_cast<f2*>(out)[k] = y;
}

// One 16-row x 32-column tile (512 outputs, I and Q): S K-steps x 4 limbs MFMAs, then the
// epilogue. Exactly 8 store instructions per lane whenever the tile is complete.
template <int S, int EPI>
__device__ __forceinline__ void computeTile(const I8FirArgs& a, const int8_t* planes, const v4i (&bf)[S][4],
                                            int64_t chunkOut, int tile, int lane, float outScale,
                                            float hiScale) {
  constexpr int kPlane = I8Geom<S>::kPlane;
  const int half = lane >> 5;
  const int col = lane & 31;
  const int row = lane & 31;  // A row: 0-15 read the I plane, 16-31 the Q plane
  v16i acc[4];
#pragma unroll
  for (int l = 0; l < 4; ++l) acc[l] = v16i{};
  const int8_t* rowBase = planes + (row >> 4) * kPlane + 32 * (tile * 16 + (row & 15)) + 16 * half;
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const v4i av = *reinterpret_cast<const v4i*>(rowBase + 32 * s);
#pragma unroll
    for (int l = 0; l < 4; ++l) acc[l] = __builtin_amdgcn_mfma_i32_32x32x32_i8(av, bf[s][l], acc[l], 0, 0, 0);
  }
  // limbs -> float; I and Q of one output sit in registers i and i + 8 of the same lane
  const int64_t tileOut = chunkOut + (int64_t)tile * kI8TileOut;
  f2 y[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const f2 lo = {(float)(acc[0][i] + (acc[1][i] << 8)), (float)(acc[0][i + 8] + (acc[1][i + 8] << 8))};
    const f2 hi = {(float)(acc[2][i] + (acc[3][i] << 8)), (float)(acc[2][i + 8] + (acc[3][i + 8] << 8))};
    y[i] = hi * hiScale + lo * outScale;  // packed: v_pk_mul_f32 + v_pk_fma_f32
  }
  const int64_t rowOut = tileOut + 4 * half * 32 + col;  // output of register i: rowOut + 32 mrow(i)
  if (tileOut + kI8TileOut <= a.nOut) {  // wave-uniform: complete tile, straight-line stores
#pragma unroll
    for (int i = 0; i < 8; ++i) storeOut<EPI>(a.out, rowOut + 32 * ((i & 3) + 8 * (i >> 2)), y[i]);
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int64_t k = rowOut + 32 * ((i & 3) + 8 * (i >> 2));
      if (k < a.nOut) storeOut<EPI>(a.out, k, y[i]);
    }
  }
}

template <int S, int EPI>
__global__ __launch_bounds__(kI8Threads, 3) void firI8MfmaKernel(I8FirArgs a) {
  using G = I8Geom<S>;
  __shared__ __attribute__((aligned(16))) int8_t ring[kRing * G::kSlot];
  __shared__ __attribute__((aligned(16))) int8_t planes[2 * G::kPlane];
  __shared__ __attribute__((aligned(16))) int8_t limbTab[4 * kLimbRow];
  __shared__ float waveMax[kI8Waves];

  const int tid = threadIdx.x;
  const int lane = tid & (kWave - 1);
  const int wave = waveUniform(tid >> 6);
  const int T = a.T;

  // this block's contiguous chunk range
  const int G0 = (int)(((int64_t)blockIdx.x * a.chunks) / gridDim.x);
  const int G1 = (int)(((int64_t)(blockIdx.x + 1) * a.chunks) / gridDim.x);
  const int n = G1 - G0;
  if (n <= 0) return;  // block-uniform, before any barrier or DMA

  // ---- tap load, then the ring prologue (chunks 0 .. kRing-2 of the range) -------------------
  // The tap load is an asm load too, so no compiler-inserted vmcnt(0) drains the DMA: it is
  // retired below by a counted wait that leaves the prologue pieces in flight.
  float hv = loadF32Async(a.taps + min(tid, T - 1));
  const uintptr_t base = reinterpret_cast<uintptr_t>(a.iq);
  const int shift = (int)(base & 15u);
  const uintptr_t alignedBase = base - shift;
  const uintptr_t lastBlock = (base + 2 * (uintptr_t)a.nIn - 1) & ~(uintptr_t)15;
  const uint32_t ringLds = waveUniform((int)(uint32_t)reinterpret_cast<uintptr_t>(ring));
  // DMA instructions this wave issues per chunk
  const int perChunk = (G::kPieces - wave + kI8Waves - 1) / kI8Waves;
  constexpr int kMaxPerChunk = (G::kPieces + kI8Waves - 1) / kI8Waves;
#pragma unroll
  for (int j = 0; j < kRing - 1; ++j)
    if (j < n) issueChunk<S>(a, alignedBase, lastBlock, G0 + j, ringLds + j * G::kSlot, wave, lane);
  reinterpret_cast<uint32_t*>(limbTab)[tid] = 0u;  // 4 rows x 256 bytes = one dword per thread
  vmWaitDyn<0, (kRing - 1) * kMaxPerChunk>(waveUniform(min(kRing - 1, n) * perChunk));
  asm volatile("" : "+v"(hv));  // hv is defined only after the wait
  hv = tid < T ? hv : 0.0f;

  // ---- taps -> 30-bit fixed point (block-uniform scale), split into signed base-256 limbs ---
  float m = fabsf(hv);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off));
  if (lane == 0) waveMax[wave] = m;
  __syncthreads();
  const float maxAbs = fmaxf(fmaxf(waveMax[0], waveMax[1]), fmaxf(waveMax[2], waveMax[3]));
  const int sc = maxAbs > 0.0f ? 29 - ilogbf(maxAbs) : 0;  // max|H| < 2^30
  if (tid < T) {
    int v = (int)rintf(ldexpf(hv, sc));
#pragma unroll
    for (int l = 0; l < 4; ++l) {
      const int digit = l < 3 ? (int)(int8_t)(v & 0xFF) : v;  // signed base-256 digit
      v = (v - digit) >> 8;
      limbTab[l * kLimbRow + kLimbPad + tid] = (int8_t)digit;
    }
  }
  __syncthreads();
  const float outScale = ldexpf(1.0f / 127.0f, -sc);
  const float hiScale = outScale * 65536.0f;

  // ---- B fragments: bf[s][l] holds limb l of H[kappa - n] for this lane's 16 kappas ----------
  // kappa = 32 s + i8FragK(half, j), n = col: 16 consecutive table bytes from
  // kLimbPad + 32 s + 16 half - col (zero outside [0, T)), re-aligned with v_alignbyte.
  const int half = lane >> 5;
  const int col = lane & 31;
  v4i bf[S][4];
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const int b0 = kLimbPad + 32 * s + i8FragK(half, 0) - col;
#pragma unroll
    for (int l = 0; l < 4; ++l) {
      const uint32_t* wsrc = reinterpret_cast<const uint32_t*>(limbTab + l * kLimbRow + (b0 & ~3));
      uint32_t d[5];
#pragma unroll
      for (int q = 0; q < 5; ++q) d[q] = wsrc[q];
      bf[s][l] = v4i{(int)__builtin_amdgcn_alignbyte(d[1], d[0], b0 & 3),
                     (int)__builtin_amdgcn_alignbyte(d[2], d[1], b0 & 3),
                     (int)__builtin_amdgcn_alignbyte(d[3], d[2], b0 & 3),
                     (int)__builtin_amdgcn_alignbyte(d[4], d[3], b0 & 3)};
    }
  }
  // from here on the only vector-memory operations are the DMA pieces and the epilogue stores

  for (int i = 0; i < n; ++i) {
    // Retire slot i: after its pieces this wave issued min(kRing-2, n-1-i) later chunks' pieces
    // and the stores of min(i, kRing-1) chunks (stores of chunk j follow the pieces of j+kRing-1).
    const int later = min(kRing - 2, n - 1 - i) * perChunk + min(i, kRing - 1) * kStoresPerChunk;
    vmWaitDyn<0, (kRing - 2) * ((G::kPieces + kI8Waves - 1) / kI8Waves) + (kRing - 1) * kStoresPerChunk>(
        waveUniform(later));
    ldsBarrier();  // every wave's pieces of slot i landed; compute(i-1) done with the planes
    const int slot = i % kRing;
    splitSlot<S>(ring + slot * G::kSlot, planes, shift, tid);
    if (a.carryDst != nullptr && G0 == 0 && i == 0) {
      // streaming history: the only block that reads samples [0, T - 1) has them in LDS now,
      // so the carry may overwrite them in place (source [nOut, nIn) is disjoint: nOut >= T - 1)
      const uint16_t* src = reinterpret_cast<const uint16_t*>(a.iq) + (a.nIn - (T - 1));
      for (int t = tid; t < T - 1; t += kI8Threads) reinterpret_cast<uint16_t*>(a.carryDst)[t] = src[t];
    }
    // refill the slot chunk i-1 used (its split finished before the barrier above)
    if (i + kRing - 1 < n)
      issueChunk<S>(a, alignedBase, lastBlock, G0 + i + kRing - 1, ringLds + ((i + kRing - 1) % kRing) * G::kSlot,
                    wave, lane);
    ldsBarrier();  // planes complete
    const int64_t chunkOut = (int64_t)(G0 + i) * kI8ChunkOut;
#pragma unroll
    for (int t = 0; t < kI8TilesPerWave; ++t)
      computeTile<S, EPI>(a, planes, bf, chunkOut, wave * kI8TilesPerWave + t, lane, outScale, hiScale);
  }
  vmWait<0>();  // no DMA may still target this block's LDS when it exits
}

namespace {
template <int S>
hipError_t launchI8(const I8FirArgs& a, int epi, hipStream_t stream, int grid) {
  if (epi == kEpiAm)
    hipLaunchKernelGGL((firI8MfmaKernel<S, kEpiAm>), dim3(grid), dim3(kI8Threads), 0, stream, a);
  else
    hipLaunchKernelGGL((firI8MfmaKernel<S, kEpiComplex>), dim3(grid), dim3(kI8Threads), 0, stream, a);
  return hipGetLastError();
}
}  // namespace

bool firI8MfmaEligible(size_t tapCount, size_t decimation, const void* in) {
  // IQ samples are 2-byte pairs; any sample-aligned pointer works (the split pass re-aligns)
  return tapCount >= 1 && tapCount <= 32 * kI8MaxS - 31 && decimation <= 1 &&
         (reinterpret_cast<uintptr_t>(in) & 1u) == 0;
}

hipError_t launchFirI8Mfma(const int8_t* iq, const float* taps, size_t tapCount, void* out, size_t nOut, int epi,
                           hipStream_t stream, int8_t* carryDst) {
  if (carryDst != nullptr && nOut + 1 < tapCount) return hipErrorInvalidValue;
  I8FirArgs a{};
  a.carryDst = tapCount > 1 ? carryDst : nullptr;
  a.iq = iq;
  a.taps = taps;
  a.out = out;
  a.nOut = (int64_t)nOut;
  a.nIn = (int64_t)nOut - 1 + (int64_t)tapCount;
  a.T = (int32_t)tapCount;
  const int64_t chunks = ((int64_t)nOut + kI8ChunkOut - 1) / kI8ChunkOut;
  if (chunks > 0x7fffffff) return hipErrorInvalidValue;
  a.chunks = (int32_t)chunks;
  // 3 resident blocks per CU (<= 168 VGPRs, 46 KB LDS); each streams a contiguous chunk range
  const int grid = (int)(chunks < 256 * 3 ? chunks : 256 * 3);
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
