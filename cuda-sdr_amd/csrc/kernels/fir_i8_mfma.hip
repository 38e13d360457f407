// MFMA FIR for interleaved int8 IQ input (the C2 chain: int8 IQ -> cf32 -> FC FIR [-> AM
// envelope]), decimation 1, up to 129 real taps.
//
// Arithmetic. gsdrInt8ToNormFloat maps x to fmaxf(-1, x/127) = x'/127 with x' = max(x, -127), so
//     y[k] = sum_j h_j x'[k+j] / 127.
// x' is an integer in [-127, 127]: exact in f16. The taps are scaled by a block-uniform power of
// two 2^sc (max |h 2^sc| in [2^14, 2^15)) and split into two f16 limbs, hs = hi + lo + e with
// hi = f16(hs), lo = f16(hs - hi), |e| <= 2^-22 |hs| (2^-25 absolute once lo is subnormal, i.e.
// below 2^-39 of the largest tap). v_mfma_f32_32x32x16_f16 forms the products x' * limb exactly
// and accumulates both limbs into ONE fp32 accumulator, so
//     y = acc * 2^-sc / 127
// carries the rounding of an fp32 accumulation of exact terms - the same class as the fp32
// direct form the reference computes; tests/test_gpu_parity.py bounds it against float64.
//
// GEMM shape (Toeplitz). Output k = 32 m + n (row m, column n < 32):
//     C[m][n] = sum_kappa A[m][kappa] B[kappa][n],  A[m][kappa] = x'[32 m + kappa],
//     B[kappa][n] = h[kappa - n] (0 <= kappa - n < T, else 0),  kappa < K = 32 S >= T + 31.
// One 32x32 MFMA tile holds 16 rows of the I stream and the same 16 rows of the Q stream (A
// rows 0-15 read the I plane, rows 16-31 the Q plane), so a lane ends with I and Q of the same
// output in accumulator registers i and i+8: the AM envelope needs no data movement.
// Per wave tile: 512 complex outputs = S K-blocks x 2 K-halves (16 each) x 2 limbs MFMAs; the B
// fragments (taps) live in registers for the whole kernel (16 S VGPRs), the A fragments are
// ds_read_b128 from the block's f16 I/Q planes. Only the consistency of the lane -> k map of A
// and B matters (a dot product is invariant under a common permutation of k).
//
// Cost: 4 S MFMAs of 32 cycles per 512 outputs: at T = 127 (S = 5) 1.25 SIMD-cycles per output
// (~10 us of matrix-core time for 20 M outputs), below the ~20 us the 6-byte-per-sample HBM
// stream takes; the epilogue is 4 VALU operations per output.
//
// Data movement. Each block owns a contiguous range of 512-output tiles (the ranges differ by at
// most one tile, so no block runs a whole chunk longer than another) and walks it in chunks of
// up to 4096 outputs (their windows overlap by T - 1 samples, an L2 hit). The raw interleaved window of a chunk goes HBM -> LDS by
// LDS-DMA (global_load_lds_dwordx4, no VGPRs) into a ring of kRing slots filled kRing - 1 chunks
// ahead, so the loads of the next chunks stay in flight across the MFMA work and the barriers;
// one pass per chunk then clamps, converts and splits the slot into the f16 I / Q planes. The
// DMA is issued from inline asm and retired with counted `s_waitcnt vmcnt(N)` (the compiler
// does not see it): N counts the DMA pieces and the epilogue stores issued after the slot waited
// for.
#include "kcommon.h"
#include "fir_launch.h"

namespace gsdr_amd {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));

constexpr int kI8Waves = 4;
constexpr int kI8Threads = kI8Waves * kWave;
constexpr int kI8TileOut = 512;                                        // 16 rows x 32 columns
// Tuning knobs (tools/exp builds variants of this file with -D overrides; the product uses the
// defaults).
#ifndef GSDR_I8_TILES_PER_WAVE
#define GSDR_I8_TILES_PER_WAVE 2
#endif
#ifndef GSDR_I8_RING
#define GSDR_I8_RING 3
#endif
#ifndef GSDR_I8_BLOCKS_PER_CU
#define GSDR_I8_BLOCKS_PER_CU 3
#endif
constexpr int kI8TilesPerWave = GSDR_I8_TILES_PER_WAVE;
constexpr int kI8ChunkTiles = kI8Waves * kI8TilesPerWave;              // 8 tiles per chunk
constexpr int kI8ChunkOut = kI8ChunkTiles * kI8TileOut;                // 4096 outputs per chunk
constexpr int kI8MaxS = 5;                                             // K <= 160 -> T <= 129
constexpr int kRing = GSDR_I8_RING;                                    // LDS-DMA ring slots
constexpr int kPiece = 64 * 16;                                        // bytes per wave DMA instruction
constexpr int kRingPad = 16;                                           // room for the DMA re-alignment
// Epilogue stores per wave per chunk (one store instruction per lane output, 8 per tile).
constexpr int kStoresPerChunk = kI8TilesPerWave * 8;

// Tap-limb table: 2 rows (hi, lo) of kLimbRow f16, tap j at kLimbPad + j, zero elsewhere.
constexpr int kLimbPad = 32;
constexpr int kLimbRow = 256;
static_assert(kLimbPad + 32 * kI8MaxS + 16 <= kLimbRow && 2 * kLimbRow * 2 == 4 * kI8Threads, "limb table");

struct I8FirArgs {
  const int8_t* iq;   // interleaved I, Q (2-byte aligned)
  const float* taps;
  void* out;
  int64_t nOut;
  int64_t nIn;        // complex samples readable: nOut - 1 + T
  int32_t T;
  int32_t tiles;      // ceil(nOut / 512)
  int8_t* carryDst;   // nullptr, or where the last T - 1 input samples go (may alias iq[0 .. T-1))
};

template <int S>
struct I8Geom {
  static constexpr int kWin = kI8ChunkOut - 32 + 32 * S;  // samples one chunk reads (multiple of 32)
  static constexpr int kBlocks = kWin / 32;                // 32-sample blocks per plane
  static constexpr int kGroups = kWin / 8;                 // 8-sample split groups
  // f16 plane: block b, 16-byte unit q (8 samples) at planeUnit(b, q), the Q plane a multiple of 256
  // bytes after the I plane.
  static constexpr int kPlaneBytes = (64 * kBlocks + 255) / 256 * 256;
  // slot: the window + up to 12 bytes of DMA re-alignment + a dword of read-ahead
  static constexpr int kPieces = (2 * kWin + 18 + kPiece - 1) / kPiece;
  static constexpr int kSlot = kPieces * kPiece;
};

// Block b's four units, swizzled within the block by (b >> 2) & 3 (r06). MI355X_MICROARCH.md's LDS banking:
// the split pass's ds_write_b128 (8 groups of 8 contiguous lanes = blocks 2k, 2k + 1, bank (a/4) mod 32) hit
// 8 distinct 16-byte slots, and every ds_read_b128 lane group of the A fragments (rows r and r + 12 of
// one plane, r + 4 and r + 8 of the other: their swizzles differ by 3, 1 and 2) 16 distinct ones of 64
// banks. Through r05 the layout was 5 b + q (one pad unit per block): conflict-free reads, but every split
// write group 2-way conflicted (units 0 and 8 of a group on one bank) - 17.9 % of C2's LDS cycles were
// bank conflicts (r05 pmc_sq_c2); the model (tools/exp/c2_lds_model.py) gives 5.5 extra cycles per
// write then, 0 now.
__device__ __forceinline__ int planeUnit(int b, int q) { return 4 * b + (q ^ ((b >> 2) & 3)); }

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

// Issue this wave's DMA pieces of the raw window of the chunk starting at tile `tile` into the
// slot at `slotLds` (LDS byte address, moved down by the dword part of the input's misalignment,
// so the window starts at the slot's nominal start + (shift & 3)). Lanes past the last 16-byte
// block this block's outputs need (`lastBlock`) re-read it (it never crosses a page); those
// bytes only feed outputs of other blocks or >= nOut, which this block does not store.
template <int S>
__device__ __forceinline__ void issueChunk(uintptr_t alignedBase, uintptr_t lastBlock, int tile, uint32_t slotLds,
                                           int wave, int lane) {
  using G = I8Geom<S>;
  const uintptr_t chunkBase = alignedBase + (uintptr_t)tile * (2 * kI8TileOut);
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

// Split one landed slot into the f16 I / Q planes: group g = samples [8g, 8g + 8) of the window
// at window bytes [16 g, 16 g + 16); `win` is 4-byte aligned when sub = 0, else 2-byte aligned.
template <int S>
__device__ __forceinline__ void splitSlot(const int8_t* win, int8_t* planes, int sub, int tid) {
  using G = I8Geom<S>;
#pragma unroll
  for (int u = 0; u < (G::kGroups + kI8Threads - 1) / kI8Threads; ++u) {
    const int g = tid + u * kI8Threads;
    if (g < G::kGroups) {
      uint32_t w[4];
      if (sub == 0) {  // kernel-uniform: 4-byte aligned input -> the window is 16-byte aligned
        const uint4 v = *reinterpret_cast<const uint4*>(win + 16 * g);
        w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
      } else {
        const uint32_t* d = reinterpret_cast<const uint32_t*>(win - 2 + 16 * g);
        uint32_t e[5];
#pragma unroll
        for (int q = 0; q < 5; ++q) e[q] = d[q];
#pragma unroll
        for (int q = 0; q < 4; ++q) w[q] = __builtin_amdgcn_alignbyte(e[q + 1], e[q], 2);
      }
      uint4 iu, qu;
      int8IqToF16Units(w, iu, qu);
      const int unit = planeUnit(g >> 2, g & 3);
      *reinterpret_cast<uint4*>(planes + 16 * unit) = iu;
      *reinterpret_cast<uint4*>(planes + G::kPlaneBytes + 16 * unit) = qu;
    }
  }
}

// Tile MFMAs: 16 rows x 32 columns (512 outputs, I and Q) = S K-blocks x 2 K-halves x 2 limbs,
// both limbs accumulating into one fp32 accumulator.
template <int S>
__device__ __forceinline__ void tileMfma(const int8_t* planes, const h8 (&bf)[S][2][2], int tile, int lane,
                                         v16f& acc) {
  constexpr int kPlaneBytes = I8Geom<S>::kPlaneBytes;
  const int row = lane & 31;  // A row: 0-15 read the I plane, 16-31 the Q plane
  const int half = lane >> 5;
  const int8_t* plane = planes + (row >> 4) * kPlaneBytes;
  const int b0 = tile * 16 + (row & 15);
  acc = v16f{};
#pragma unroll
  for (int s = 0; s < S; ++s) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const h8 av = *reinterpret_cast<const h8*>(plane + 16 * planeUnit(b0 + s, 2 * u + half));
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(av, bf[s][u][0], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(av, bf[s][u][1], acc, 0, 0, 0);
    }
  }
}

// Tile epilogue: I and Q of one output sit in registers i and i + 8 of the same lane; 8 stores
// per lane. FULL: the whole tile exists (straight-line stores).
template <int EPI, bool FULL>
__device__ __forceinline__ void tileEpilogue(const I8FirArgs& a, const v16f& acc, int64_t tileOut, int lane,
                                             float outScale) {
  const int64_t rowOut = tileOut + 4 * (lane >> 5) * 32 + (lane & 31);  // register i: + 32 mrow(i)
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int64_t k = rowOut + 32 * ((i & 3) + 8 * (i >> 2));
    if (FULL || k < a.nOut) {
      if (EPI == kEpiAm) {
        // |y| = sqrt(yi^2 + yq^2) * scale, hardware square root (<= 1 ulp)
        const float m2 = fmaf(acc[i], acc[i], acc[i + 8] * acc[i + 8]);
        reinterpret_cast<float*>(a.out)[k] = __builtin_amdgcn_sqrtf(m2) * outScale;
      } else {
        reinterpret_cast<f2*>(a.out)[k] = f2{acc[i], acc[i + 8]} * outScale;
      }
    }
  }
}

template <int S, int EPI>
__device__ __forceinline__ void computeTile(const I8FirArgs& a, const int8_t* planes, const h8 (&bf)[S][2][2],
                                            int64_t chunkOut, int tile, int lane, float outScale) {
  v16f acc;
  tileMfma<S>(planes, bf, tile, lane, acc);
  const int64_t tileOut = chunkOut + (int64_t)tile * kI8TileOut;
  if (tileOut + kI8TileOut <= a.nOut) tileEpilogue<EPI, true>(a, acc, tileOut, lane, outScale);
  else tileEpilogue<EPI, false>(a, acc, tileOut, lane, outScale);
}

template <int S, int EPI>
__global__ __launch_bounds__(kI8Threads, GSDR_I8_BLOCKS_PER_CU) void firI8MfmaKernel(I8FirArgs a) {
  using G = I8Geom<S>;
  __shared__ __attribute__((aligned(16))) int8_t ring[kRingPad + kRing * G::kSlot];
  __shared__ __attribute__((aligned(16))) int8_t planes[2 * G::kPlaneBytes];
  __shared__ __attribute__((aligned(16))) _Float16 limbTab[2 * kLimbRow];
  __shared__ float waveMax[kI8Waves];

  const int tid = threadIdx.x;
  const int lane = tid & (kWave - 1);
  const int wave = waveUniform(tid >> 6);
  const int T = a.T;

  // this block's contiguous tile range [T0, T0 + nt), walked in n chunks of up to 8 tiles
  // (q tiles each, one more for the first r blocks: with blocks b, b + 256, b + 512 sharing a CU
  // under round-robin dispatch, the surplus spreads one per CU first - a speed heuristic only)
  const int q = a.tiles / (int)gridDim.x, r = a.tiles % (int)gridDim.x;
  const int T0 = (int)blockIdx.x * q + min((int)blockIdx.x, r);
  const int nt = q + ((int)blockIdx.x < r ? 1 : 0);
  if (nt <= 0) return;  // block-uniform, before any barrier or DMA
  const int n = (nt + kI8ChunkTiles - 1) / kI8ChunkTiles;

  // ---- tap load, then the ring prologue (chunks 0 .. kRing-2 of the range) -------------------
  // The tap load is an asm load too, so no compiler-inserted vmcnt(0) drains the DMA: it is
  // retired below by a counted wait that leaves the prologue pieces in flight.
  float hv = loadF32Async(a.taps + min(tid, T - 1));
  const uintptr_t base = reinterpret_cast<uintptr_t>(a.iq);
  const int shift = (int)(base & 15u);
  const uintptr_t alignedBase = base - shift;
  // last byte any output of this block reads: sample (T0 + nt) 512 + 32 S - 32 - 1 (K = 32 S
  // covers the T - 1 history), capped at the input end
  const int64_t needEnd = min((int64_t)(T0 + nt) * kI8TileOut + 32 * S - 32, a.nIn);
  const uintptr_t lastBlock = (base + 2 * (uintptr_t)needEnd - 1) & ~(uintptr_t)15;
  // slot j's window starts at ring + kRingPad + j kSlot + (shift & 3): the DMA destination moves
  // down by the dword part of the misalignment (into the previous slot's unused tail / the pad)
  const uint32_t ringLds =
      (uint32_t)waveUniform((int)(uint32_t)reinterpret_cast<uintptr_t>(ring)) + kRingPad - (uint32_t)(shift & ~3);
  const int sub = shift & 3;
  // DMA instructions this wave issues per chunk
  const int perChunk = (G::kPieces - wave + kI8Waves - 1) / kI8Waves;
  constexpr int kMaxPerChunk = (G::kPieces + kI8Waves - 1) / kI8Waves;
#pragma unroll
  for (int j = 0; j < kRing - 1; ++j)
    if (j < n)
      issueChunk<S>(alignedBase, lastBlock, T0 + j * kI8ChunkTiles, ringLds + j * G::kSlot, wave, lane);
  reinterpret_cast<uint32_t*>(limbTab)[tid] = 0u;  // 2 rows x 256 f16 = one dword per thread
  vmWaitDyn<0, (kRing - 1) * kMaxPerChunk>(waveUniform(min(kRing - 1, n) * perChunk));
  asm volatile("" : "+v"(hv));  // hv is defined only after the wait
  hv = tid < T ? hv : 0.0f;

  // ---- taps -> block-uniform power-of-two scale, two f16 limbs --------------------------------
  float m = fabsf(hv);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off));
  if (lane == 0) waveMax[wave] = m;
  __syncthreads();
  const float maxAbs = fmaxf(fmaxf(waveMax[0], waveMax[1]), fmaxf(waveMax[2], waveMax[3]));
  const int sc = maxAbs > 0.0f ? 14 - ilogbf(maxAbs) : 0;  // max |h 2^sc| in [2^14, 2^15)
  if (tid < T) {
    const float hs = ldexpf(hv, sc);
    const _Float16 hi = (_Float16)hs;
    limbTab[kLimbPad + tid] = hi;
    limbTab[kLimbRow + kLimbPad + tid] = (_Float16)(hs - (float)hi);
  }
  __syncthreads();
  const float outScale = ldexpf(1.0f / 127.0f, -sc);

  // ---- B fragments: bf[s][u][l] = limb l of h[kappa - n], kappa = 32 s + 16 u + 8 half + j -----
  const int half = lane >> 5;
  const int col = lane & 31;
  h8 bf[S][2][2];
#pragma unroll
  for (int s = 0; s < S; ++s) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int e0 = kLimbPad + 32 * s + 16 * u + 8 * half - col;  // first f16 element
#pragma unroll
      for (int l = 0; l < 2; ++l) {
        const uint32_t* d = reinterpret_cast<const uint32_t*>(limbTab + l * kLimbRow + (e0 & ~1));
        uint32_t e[5];
#pragma unroll
        for (int q = 0; q < 5; ++q) e[q] = d[q];
        const int sh = 2 * (e0 & 1);
        const uint32_t w0 = __builtin_amdgcn_alignbyte(e[1], e[0], sh);
        const uint32_t w1 = __builtin_amdgcn_alignbyte(e[2], e[1], sh);
        const uint32_t w2 = __builtin_amdgcn_alignbyte(e[3], e[2], sh);
        const uint32_t w3 = __builtin_amdgcn_alignbyte(e[4], e[3], sh);
        bf[s][u][l] = __builtin_bit_cast(h8, uint4{w0, w1, w2, w3});
      }
    }
  }
  // from here on the only vector-memory operations are the DMA pieces and the epilogue stores

  constexpr int kSteady = (kRing - 2) * kMaxPerChunk + (kRing - 1) * kStoresPerChunk;
  for (int i = 0; i < n; ++i) {
    // Retire slot i: after its pieces this wave issued min(kRing-2, n-1-i) later chunks' pieces
    // and the stores of min(i, kRing-1) chunks (stores of chunk j follow the pieces of j+kRing-1).
    // (only the last chunk may be partial: its stores follow every wait but the final one)
    const int later = min(kRing - 2, n - 1 - i) * perChunk + min(i, kRing - 1) * kStoresPerChunk;
    if (later == kSteady) vmWait<kSteady>();  // the steady state of the widest waves
    else vmWaitDyn<0, kSteady>(waveUniform(later));
    ldsBarrier();  // every wave's pieces of slot i landed; compute(i-1) done with the planes
    const int slot = i % kRing;
    splitSlot<S>(ring + kRingPad + slot * G::kSlot + sub, planes, sub, tid);
    if (a.carryDst != nullptr && T0 == 0 && i == 0) {
      // streaming history: the only block that reads samples [0, T - 1) has them in LDS now,
      // so the carry may overwrite them in place (source [nOut, nIn) is disjoint: nOut >= T - 1)
      const uint16_t* src = reinterpret_cast<const uint16_t*>(a.iq) + (a.nIn - (T - 1));
      for (int t = tid; t < T - 1; t += kI8Threads) reinterpret_cast<uint16_t*>(a.carryDst)[t] = src[t];
    }
    // refill the slot chunk i-1 used (its split finished before the barrier above)
    if (i + kRing - 1 < n)
      issueChunk<S>(alignedBase, lastBlock, T0 + (i + kRing - 1) * kI8ChunkTiles,
                    ringLds + ((i + kRing - 1) % kRing) * G::kSlot, wave, lane);
    ldsBarrier();  // planes complete
    const int c0 = T0 + i * kI8ChunkTiles;
    const int ct = min(kI8ChunkTiles, T0 + nt - c0);  // tiles in this chunk (< 8 only for the last)
    const int64_t chunkOut = (int64_t)c0 * kI8TileOut;
#pragma unroll
    for (int t = 0; t < kI8TilesPerWave; ++t) {
      const int tile = wave + kI8Waves * t;  // a partial chunk spreads over the waves
      if (tile < ct) computeTile<S, EPI>(a, planes, bf, chunkOut, tile, lane, outScale);
    }
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
  // IQ samples are 2-byte pairs; any sample-aligned pointer works (the DMA re-aligns)
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
  const int64_t tiles = ((int64_t)nOut + kI8TileOut - 1) / kI8TileOut;
  if (tiles > 0x7fffffff) return hipErrorInvalidValue;
  a.tiles = (int32_t)tiles;
  // 3 resident blocks per CU (<= 168 VGPRs); each streams a contiguous tile range
  const int grid = (int)(tiles < 256 * GSDR_I8_BLOCKS_PER_CU ? tiles : 256 * GSDR_I8_BLOCKS_PER_CU);
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
