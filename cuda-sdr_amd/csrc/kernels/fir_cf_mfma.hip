// MFMA FIR for cf32 input and real taps (gsdrFirFC / gsdrFirFCAmDemod: the C3 / C4 chains, up to
// K = 31 D + T <= 1408, D <= 16), split-precision bf16 on v_mfma_f32_32x32x16_bf16.
//
// Arithmetic. Every fp32 value v (sample component or tap) is split EXACTLY into three bf16
// limbs by round-to-nearest: v0 = bf16(v), v1 = bf16(v - v0), v2 = v - v0 - v1 (<= 8 significant
// bits, exact in bf16), |v1| <= 2^-9 |v|, |v2| <= 2^-18 |v|. The kernel sums the six products
// x_i h_j with i + j <= 2; the dropped ones are below 2^-26 |x h|. The MFMA forms each bf16
// product exactly and accumulates in fp32, so the result carries the rounding of an fp32
// accumulation - the class of the reference's fp32 direct form (tests: 1e-6 of sum |h||x|).
//
// GEMM shape (decimating Toeplitz). Output k = 32 m + n of a 512-output tile (m < 16 rows,
// n < 32 columns):
//     C[m][n] = sum_kappa A[m][kappa] B[kappa][n],  A[m][kappa] = x[32 D m + kappa],
//     B[kappa][n] = h[kappa - n D] (0 <= kappa - n D < T, else 0),  kappa < K = 31 D + T.
// A rows 0-15 read the I planes, rows 16-31 the Q planes of the same 16 output rows, so a lane
// holds I and Q of one output in accumulator registers i and i + 8.
//
// Work split. One 512-thread block per CU walks a contiguous range of tiles. The tile's input
// window (W = 480 D + 128 KS samples) is loaded into registers one tile ahead, split into six
// bf16 planes (3 limbs x I/Q) in LDS, and the K range is split over the 8 waves (KS K-steps of 16
// each): a wave's B fragments (3 limbs x KS K-steps of the Toeplitz tap matrix) stay in VGPRs for
// the whole launch. Partial accumulators meet in LDS; each wave reduces and stores 64 outputs.
// Plane units (8 samples, 16 B) are padded (unit u at u + (u >> padShift)) and the I / Q planes
// offset so that every ds_read_b128 lane group of the A fragments is bank-conflict free; the host
// picks both per D (cfPlaneLayout).
//
// int8 IQ input (firI8DecMfmaKernel: gsdrInt8FirFC / gsdrInt8FirFCAmDemod with D > 1 or T > 129,
// the C5 RF stage; any sample-aligned input): the same Toeplitz tiles and work split, but
// x' = max(x, -127) is an integer,
// exact in f16, so the window becomes two f16 planes (I, Q) with one split pass of 3 VALU per
// sample pair, and the taps are scaled by a block-uniform 2^sc and split into two f16 limbs as in
// fir_i8_mfma.hip: 2 v_mfma_f32_32x32x16_f16 per K-step instead of 6 bf16 products.
#include <algorithm>
#include <atomic>
#include <cstddef>
#include <mutex>
#include <vector>

#include "kcommon.h"
#include "fir_launch.h"
#include "ws_common.h"

#include <gsdr/gsdr_amd.h>

namespace gsdr_amd {


struct CfFirArgs {
  const float* x;     // interleaved re, im
  const float* taps;
  void* out;
  int64_t nOut;
  int64_t nIn;        // complex samples readable: (nOut - 1) D + T
  int32_t T;
  int32_t D;
  int32_t KS;         // K-steps per wave
  int32_t tiles;
  int32_t Wu;         // window units (8 samples) per tile = 60 D + 16 KS
  int32_t padShift;   // plane unit u lives at u + (u >> padShift)
  int32_t planeStride;  // bytes between the six planes (limb l, component c at 2 l + c)
  int32_t dbp;          // wave-specialised kernels: two partial-sum buffers
  int32_t spinLimit;    // wave-specialised kernels: microseconds a hand-off wait may take before it gives up
  uint32_t* abortOut;   // wave-specialised kernels: host-visible abort counter (wsAbortWord)
};


// fp32 pair -> three bf16 limb pairs (exact).
__device__ __forceinline__ void split3(float a, float b, uint32_t& l0, uint32_t& l1, uint32_t& l2) {
  typedef float f2v __attribute__((ext_vector_type(2)));
  const f2v v = {a, b};
  const bf2 h0 = __builtin_convertvector(v, bf2);
  const f2v r1 = v - __builtin_convertvector(h0, f2v);
  const bf2 h1 = __builtin_convertvector(r1, bf2);
  const f2v r2 = r1 - __builtin_convertvector(h1, f2v);
  const bf2 h2 = __builtin_convertvector(r2, bf2);
  l0 = __builtin_bit_cast(uint32_t, h0);
  l1 = __builtin_bit_cast(uint32_t, h1);
  l2 = __builtin_bit_cast(uint32_t, h2);
}

// Window loads: G groups of 8 samples (64 B) per thread, group g = tid + 512 j.
template <int G>
struct CfWindow {
  f4 v[G][4];  // native vector type: HIP's float4 union defeats register promotion
};

// Branch-free, so the loads stay in flight until the split that consumes them: blocks past the
// input end re-read the last 16-byte block holding input bytes (never crossing a page); those
// samples feed only outputs >= nOut or meet zero taps. Surplus groups (g >= Wu) repeat the last.
template <int G>
__device__ __forceinline__ void loadWindow(const CfFirArgs& a, int tile, int tid, CfWindow<G>& w) {
  // f4 = 2 samples; index arithmetic on the kernel-argument pointer keeps these global_load
  // (a flat load would also count on lgkmcnt and stall every LDS wait of the MFMA loop)
  const f4* x4 = reinterpret_cast<const f4*>(a.x);
  const int64_t base = (int64_t)tile * kCfTileOut * a.D / 2;
  const int64_t last = (a.nIn - 1) >> 1;
#pragma unroll
  for (int j = 0; j < G; ++j) {
    const int g = min(tid + kCfThreads * j, a.Wu - 1);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int64_t i = base + 4 * (int64_t)g + q;
      w.v[j][q] = x4[i < last ? i : last];
    }
  }
}

// Split the window into the planes; a non-finite sample sets *nonFinite (0 * x is NaN exactly
// for x = +-inf or NaN), so the tile takes the direct path: the Toeplitz product would multiply
// the sample by the zero taps of outputs whose windows do not contain it (0 * inf = NaN).
template <int G>
__device__ __forceinline__ void splitWindow(const CfFirArgs& a, const CfWindow<G>& w, int8_t* planes, int tid,
                                            int* nonFinite) {
  f4 probe = f4{};
#pragma unroll
  for (int j = 0; j < G; ++j) {
    const int g = tid + kCfThreads * j;
    if (g < a.Wu) {
      uint32_t iL[3][4], qL[3][4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {  // samples 2q, 2q + 1: (re, im, re, im)
        split3(w.v[j][q].x, w.v[j][q].z, iL[0][q], iL[1][q], iL[2][q]);
        split3(w.v[j][q].y, w.v[j][q].w, qL[0][q], qL[1][q], qL[2][q]);
        probe += w.v[j][q] * 0.0f;
      }
      const int off = 16 * cfPhys(g, a.padShift);
#pragma unroll
      for (int l = 0; l < 3; ++l) {
        *reinterpret_cast<uint4*>(planes + (2 * l) * a.planeStride + off) = uint4{iL[l][0], iL[l][1], iL[l][2], iL[l][3]};
        *reinterpret_cast<uint4*>(planes + (2 * l + 1) * a.planeStride + off) =
            uint4{qL[l][0], qL[l][1], qL[l][2], qL[l][3]};
      }
    }
  }
  const float pr = (probe.x + probe.y) + (probe.z + probe.w);
  if (pr != pr) *nonFinite = 1;
}

// Direct fp32 form of one tile, one output per thread (the statistics' tiles: a non-finite sample, a quiet
// or exact-zero 64-sample block).
template <int EPI>
__device__ __forceinline__ void directTile(const CfFirArgs& a, int tile, int tid) {
  const int64_t k = (int64_t)tile * kCfTileOut + tid;
  if (k >= a.nOut) return;
  const f2* x = reinterpret_cast<const f2*>(a.x) + k * a.D;
  // accumulated in double (rare tiles: the sequential fp32 sum of ~1 000 products reached 1.2e-6 of
  // sum|h||x| - tests/test_mfma_guard.py), then the envelope in double too: the guard's tiles hold outputs
  // far below 1 (windows whose samples meet only tail taps), whose squares would be fp32 subnormals
  double yr = 0.0, yi = 0.0;
  for (int j = 0; j < a.T; ++j) {
    const double h = a.taps[j];
    const f2 v = x[j];
    yr = fma(h, (double)v.x, yr);
    yi = fma(h, (double)v.y, yi);
  }
  if (EPI == kEpiAm) reinterpret_cast<float*>(a.out)[k] = (float)__builtin_sqrt(fma(yr, yr, yi * yi));
  else reinterpret_cast<f2*>(a.out)[k] = f2{(float)yr, (float)yi};
}

template <int KS, int G, int EPI>
__global__ __launch_bounds__(kCfThreads, 1) void firCfMfmaKernel(CfFirArgs a) {
  extern __shared__ __attribute__((aligned(16))) int8_t smem[];
  int8_t* planes = smem;
  float* part = reinterpret_cast<float*>(smem + 6 * a.planeStride);
  __shared__ int nonFinite[2];  // per tile parity: the window holds an inf / NaN

  const int tid = threadIdx.x;
  const int lane = tid & (kWave - 1);
  const int wave = waveUniform(tid >> 6);
  const int D = a.D, T = a.T;

  // contiguous tile range of this block
  const int q = a.tiles / (int)gridDim.x, r = a.tiles % (int)gridDim.x;
  const int t0 = (int)blockIdx.x * q + min((int)blockIdx.x, r);
  const int n = q + ((int)blockIdx.x < r ? 1 : 0);
  if (n <= 0) return;

  // first window in flight while the taps are prepared
  CfWindow<G> win;
  loadWindow<G>(a, t0, tid, win);

  // ---- taps -> LDS (zero-padded to [-31 D, 128 KS)), then this wave's B fragments -------------
  if (tid < 2) nonFinite[tid] = 0;
  const int off0 = 31 * D;
  const int span = off0 + 128 * KS;
  for (int i = tid; i < span; i += kCfThreads) {
    const int j = i - off0;
    part[i] = (j >= 0 && j < T) ? a.taps[j] : 0.0f;
  }
  __syncthreads();
  const int half = lane >> 5;
  const int col = lane & 31;
  bf8 bf[kCfMaxKS][3];
#pragma unroll
  for (int s = 0; s < kCfMaxKS; ++s) {
    if (s < KS) {
      const int kap = 16 * (wave * KS + s) + 8 * half;  // first kappa of this lane's 8
      uint32_t l[3][4];
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const float h0 = part[off0 + kap + 2 * p - col * D];
        const float h1 = part[off0 + kap + 2 * p + 1 - col * D];
        split3(h0, h1, l[0][p], l[1][p], l[2][p]);
      }
#pragma unroll
      for (int i = 0; i < 3; ++i) bf[s][i] = __builtin_bit_cast(bf8, uint4{l[i][0], l[i][1], l[i][2], l[i][3]});
    } else {
#pragma unroll
      for (int i = 0; i < 3; ++i) bf[s][i] = bf8{};
    }
  }
  __syncthreads();  // the tap staging area becomes the partial-sum area

  // ---- prologue: tile t0's window into the planes, tile t0 + 1's loads in flight -------------
  splitWindow<G>(a, win, planes, tid, &nonFinite[t0 & 1]);
  if (n > 1) loadWindow<G>(a, t0 + 1, tid, win);
  __syncthreads();

  // A-fragment geometry: row r = lane & 15 of component c = (lane >> 4) & 1, K-half `half`
  const int arow = lane & 15;
  const int comp = (lane >> 4) & 1;
  const int uRow = 4 * D * arow + half;
  const int8_t* pI = planes + comp * a.planeStride;

  for (int i = 0; i < n; ++i) {
    const int tile = t0 + i;
    const bool direct = nonFinite[tile & 1] != 0;  // block-uniform (set before the last barrier)
    if (tid == 0) nonFinite[(tile + 1) & 1] = 0;    // last read in tile - 1's compute
    if (direct) {
      directTile<EPI>(a, tile, tid);
      __syncthreads();  // the flag reset above precedes the next split's writes
    } else {
    // ---- this wave's K range: KS K-steps x 6 split-precision MFMAs ---------------------------
    v16f acc = v16f{};
#pragma unroll
    for (int s = 0; s < kCfMaxKS; ++s) {
      if (s < KS) {
        const int u = uRow + 2 * (wave * KS + s);
        const int off = 16 * cfPhys(u, a.padShift);
        const bf8 x0 = *reinterpret_cast<const bf8*>(pI + off);
        const bf8 x1 = *reinterpret_cast<const bf8*>(pI + 2 * a.planeStride + off);
        const bf8 x2 = *reinterpret_cast<const bf8*>(pI + 4 * a.planeStride + off);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x0, bf[s][0], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x0, bf[s][1], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x1, bf[s][0], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x0, bf[s][2], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x1, bf[s][1], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x2, bf[s][0], acc, 0, 0, 0);
      }
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) part[(wave * 16 + k) * kWave + lane] = acc[k];
    __syncthreads();  // partials complete; every wave is done reading the planes

    // ---- reduction + epilogue: wave w finishes accumulator register w (I) / w + 8 (Q) --------
    float yi = 0.0f, yq = 0.0f;
#pragma unroll
    for (int v = 0; v < kCfWaves; ++v) {
      yi += part[(v * 16 + wave) * kWave + lane];
      yq += part[(v * 16 + wave + 8) * kWave + lane];
    }
    const int orow = (wave & 3) + 8 * (wave >> 2) + 4 * half;
    const int64_t k = (int64_t)tile * kCfTileOut + 32 * orow + col;
    if (k < a.nOut) {
      if (EPI == kEpiAm) reinterpret_cast<float*>(a.out)[k] = amEnvelope(f2{yi, yq});
      else reinterpret_cast<f2*>(a.out)[k] = f2{yi, yq};
    }
    }

    // ---- next tile's window into the planes, the one after into registers ------------------
    if (i + 1 < n) {
      splitWindow<G>(a, win, planes, tid, &nonFinite[(tile + 1) & 1]);
      if (i + 2 < n) loadWindow<G>(a, tile + 2, tid, win);
      __syncthreads();
    }
  }
}


// ---- cf32 input on f16 limbs with a per-tile scale (default cf32 MFMA path) ---------------------
//
// x = x0 + x1 (two f16 limbs, RNE, after scaling the tile by 2^sx so that its largest component
// lands in [2^14, 2^15)) and h = h0 + h1 (two f16 limbs, block scale 2^sh): the three products
// x0 h0, x0 h1, x1 h0 carry every term down to 2^-22 of |x h| (the dropped x1 h1 and the limb
// remainders are <= 2^-22 each), on v_mfma_f32_32x32x16_f16 - half the matrix work of the bf16 x 3
// split and four planes instead of six. A fixed scale per tile keeps 22 bits for samples down to
// 2^-16 of the tile's largest: a tile holding a non-finite sample, or a 64-sample block whose
// largest magnitude is below 2^-16 of the tile's (a quiet stretch next to a loud one), takes the
// direct fp32 path, so every output keeps its error relative to its OWN window
// (test_cf_mfma_dynamic_range).

// Window units (8 samples) of tile `tile` wholly inside the input, capped at the units loaded (`cap`).
__device__ __forceinline__ int cfUnitsInInput(const CfFirArgs& a, int tile, int cap) {
  const int64_t u = (a.nIn - (int64_t)tile * kCfTileOut * a.D) >> 3;
  return u < cap ? (int)(u > 0 ? u : 0) : cap;
}

// The exact-zero rule (r06): the taps are two f16 limbs under one block scale, so a
// tap below ~2^-17 of the largest keeps only an absolute 2^-39 of it (a Blackman filter's tails), and an
// output whose window has non-zero samples ONLY under such taps - after an exact-zero gap, at a
// zero-padded start, between sparse impulses - misses the 1e-6 sum|h||x| bound. Such a window holds
// long exact-zero runs, i.e. whole zero 64-sample blocks: a block wholly inside the input counts in the
// smallest-block statistic even when it is zero, which sends the tile to the direct path (B = 0 < M /
// 2^16). The blocks of the last tile past the input's end do not count. Unit g's block: lanes g & ~7 ..
// g | 7 (g = lane mod 8: the thread strides are multiples of 64).
__device__ __forceinline__ bool cfBlockInInput(int g, int inU) { return (g | 7) < inU; }

// Window statistics of one tile, in two halves around a barrier the caller provides:
// cfStatsLocal reduces the thread's units over the wave and leaves the wave's (max, smallest
// nonzero 64-sample-block max) in red[.][wave]; cfStatsFinish reads all waves' after the barrier
// and decides the tile's scale or the direct path.
template <int G>
__device__ __forceinline__ void cfStatsLocal(const CfFirArgs& a, const CfWindow<G>& w, int tile, int tid,
                                             float (*red)[kCfWaves]) {
  const int lane = tid & (kWave - 1);
  const int wave = tid >> 6;
  float m = 0.0f;         // largest |component| of this thread's units
  float bmin = INFINITY;  // smallest 64-sample-block maximum seen by this thread (see cfBlockInInput)
  f4 probe = f4{};
  const int inU = cfUnitsInInput(a, tile, a.Wu);
#pragma unroll
  for (int j = 0; j < G; ++j) {
    const int g = tid + kCfThreads * j;
    float um = 0.0f;
    if (g < a.Wu) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const f4 v = w.v[j][q];
        probe += v * 0.0f;
        um = fmaxf(um, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
      }
    }
    // 64-sample block = 8 consecutive units = 8 consecutive lanes
    float bm = um;
    bm = fmaxf(bm, __shfl_xor(bm, 1));
    bm = fmaxf(bm, __shfl_xor(bm, 2));
    bm = fmaxf(bm, __shfl_xor(bm, 4));
    m = fmaxf(m, um);
    if (bm > 0.0f || cfBlockInInput(g, inU)) bmin = fminf(bmin, bm);
  }
  const float pr = (probe.x + probe.y) + (probe.z + probe.w);
  if (pr != pr) m = INFINITY;  // non-finite sample: direct path
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    m = fmaxf(m, __shfl_xor(m, o));
    bmin = fminf(bmin, __shfl_xor(bmin, o));
  }
  if (lane == 0) {
    red[0][wave] = m;
    red[1][wave] = bmin;
  }
}

__device__ __forceinline__ bool cfStatsFinish(const float (*red)[kCfWaves], int* sxOut) {
  float M = red[0][0], B = red[1][0];
#pragma unroll
  for (int v = 1; v < kCfWaves; ++v) {
    M = fmaxf(M, red[0][v]);
    B = fminf(B, red[1][v]);
  }
  *sxOut = 0;
  if (!(M <= 3.0e38f)) return true;  // inf / NaN
  if (M == 0.0f) return false;
  if (M < 1.0e-30f || B < M * (1.0f / 65536.0f)) return true;  // would lose bits below 2^-22
  *sxOut = 14 - ilogbf(M);
  return false;
}

// Both halves with their own barriers (prologue and the single-set kernel).
template <int G>
__device__ __forceinline__ bool cfTileStats(const CfFirArgs& a, const CfWindow<G>& w, int tile, int tid,
                                            float (*red)[kCfWaves], int* sxOut) {
  cfStatsLocal<G>(a, w, tile, tid, red);
  __syncthreads();
  const bool d = cfStatsFinish(red, sxOut);
  __syncthreads();  // red[] is rewritten by the next tile's statistics
  return d;
}

// Split group j of the thread's window into the four f16 planes (limb l, component c at 2 l + c).
template <int G>
__device__ __forceinline__ void splitGroupF16(const CfFirArgs& a, const CfWindow<G>& w, int8_t* planes, int tid,
                                              float scale, int j) {
  const int g = tid + kCfThreads * j;
  if (g < a.Wu) {
    h8 i0, i1, q0, q1;
#pragma unroll
    for (int q = 0; q < 4; ++q) {  // samples 2q, 2q + 1: (re, im, re, im)
      const f4 v = w.v[j][q] * scale;
      const _Float16 a0 = (_Float16)v.x, b0 = (_Float16)v.y, c0 = (_Float16)v.z, d0 = (_Float16)v.w;
      i0[2 * q] = a0;
      i0[2 * q + 1] = c0;
      q0[2 * q] = b0;
      q0[2 * q + 1] = d0;
      i1[2 * q] = (_Float16)(v.x - (float)a0);
      i1[2 * q + 1] = (_Float16)(v.z - (float)c0);
      q1[2 * q] = (_Float16)(v.y - (float)b0);
      q1[2 * q + 1] = (_Float16)(v.w - (float)d0);
    }
    const int off = 16 * cfPhys(g, a.padShift);
    *reinterpret_cast<h8*>(planes + off) = i0;
    *reinterpret_cast<h8*>(planes + a.planeStride + off) = q0;
    *reinterpret_cast<h8*>(planes + 2 * a.planeStride + off) = i1;
    *reinterpret_cast<h8*>(planes + 3 * a.planeStride + off) = q1;
  }
}

template <int G>
__device__ __forceinline__ void splitWindowF16(const CfFirArgs& a, const CfWindow<G>& w, int8_t* planes, int tid,
                                               float scale) {
#pragma unroll
  for (int j = 0; j < G; ++j) splitGroupF16<G>(a, w, planes, tid, scale, j);
}

struct CfF16State {
  int sx;       // scale exponent of the tile
  bool direct;  // that tile takes the direct path
};

// One tile of the double-buffered f16 kernel. On entry the planes of tile i are in set i & 1, wCur
// holds tile i + 1's window and `nx` its statistics, wNext is free: it receives tile i + 2's loads
// right away. The split of tile i + 1 runs between the MFMAs of tile i; tile i + 2's statistics
// travel with tile i's partial sums through the same barrier. Two barriers per tile.
template <int KS, int G, int EPI>
__device__ __forceinline__ void cfF16Tile(const CfFirArgs& a, int8_t* smem, float* part, float (*red2)[2][kCfWaves],
                                          const h8 (&bh)[kCfMaxKS], const h8 (&bl)[kCfMaxKS], int sh, int i, int n,
                                          int t0, int tid, CfWindow<G>& wCur, CfWindow<G>& wNext, CfF16State& st,
                                          CfF16State& nx) {
  const int lane = tid & (kWave - 1);
  const int wave = waveUniform(tid >> 6);
  const int half = lane >> 5;
  const int col = lane & 31;
  const int tile = t0 + i;
  int8_t* cur = smem + (i & 1) * 4 * a.planeStride;
  int8_t* nxt = smem + ((i + 1) & 1) * 4 * a.planeStride;
  if (i + 2 < n) loadWindow<G>(a, tile + 2, tid, wNext);
  const bool splitNext = i + 1 < n && !nx.direct;
  const float scaleN = ldexpf(1.0f, nx.sx);
  if (st.direct) {
    directTile<EPI>(a, tile, tid);
    if (splitNext) splitWindowF16<G>(a, wCur, nxt, tid, scaleN);
  } else {
    const int arow = lane & 15;
    const int comp = (lane >> 4) & 1;
    const int uRow = 4 * a.D * arow + half;
    const int8_t* pI = cur + comp * a.planeStride;
    v16f acc = v16f{};
#pragma unroll
    for (int s = 0; s < kCfMaxKS; ++s) {
      if (s < KS) {
        const int u = uRow + 2 * (wave * KS + s);
        const int off = 16 * cfPhys(u, a.padShift);
        const h8 x0 = *reinterpret_cast<const h8*>(pI + off);
        const h8 x1 = *reinterpret_cast<const h8*>(pI + 2 * a.planeStride + off);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(x0, bh[s], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(x0, bl[s], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(x1, bh[s], acc, 0, 0, 0);
#pragma unroll
        for (int j = 0; j < G; ++j)
          if (s == (KS * (j + 1)) / (G + 1) && splitNext) splitGroupF16<G>(a, wCur, nxt, tid, scaleN, j);
      }
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) part[(wave * 16 + k) * kWave + lane] = acc[k];
  }
  // tile i + 2's statistics (its loads had the MFMA phase to land); red2 alternates by tile
  if (i + 2 < n) cfStatsLocal<G>(a, wNext, tile + 2, tid, red2[i & 1]);
  __syncthreads();  // partials and statistics published; `cur` read and `nxt` written by all waves
  CfF16State nn{0, true};
  if (i + 2 < n) nn.direct = cfStatsFinish(red2[i & 1], &nn.sx);
  if (!st.direct) {
    float yi = 0.0f, yq = 0.0f;
#pragma unroll
    for (int v = 0; v < kCfWaves; ++v) {
      yi += part[(v * 16 + wave) * kWave + lane];
      yq += part[(v * 16 + wave + 8) * kWave + lane];
    }
    const float outScale = ldexpf(1.0f, -(st.sx + sh));
    const int orow = (wave & 3) + 8 * (wave >> 2) + 4 * half;
    const int64_t k = (int64_t)tile * kCfTileOut + 32 * orow + col;
    if (k < a.nOut) {
      if (EPI == kEpiAm) {
        reinterpret_cast<float*>(a.out)[k] = amEnvelope(f2{yi, yq}) * outScale;
      } else {
        reinterpret_cast<f2*>(a.out)[k] = f2{yi, yq} * outScale;
      }
    }
  }
  __syncthreads();  // every wave has read `part` before the next tile rewrites it
  st = nx;
  nx = nn;
}

// DB: two plane sets and two register windows (cfF16Tile); else one of each, the split after the
// tile's reduction.
template <int KS, int G, int EPI, bool DB>
__global__ __launch_bounds__(kCfThreads, 1) void firCfF16MfmaKernel(CfFirArgs a) {
  extern __shared__ __attribute__((aligned(16))) int8_t smem[];
  constexpr int kSets = DB ? 2 : 1;
  float* part = reinterpret_cast<float*>(smem + 4 * kSets * a.planeStride);
  __shared__ float red[2][kCfWaves];
  __shared__ float red2[2][2][kCfWaves];  // DB: statistics of tiles i + 2, alternating
  __shared__ float waveMax[kCfWaves];

  const int tid = threadIdx.x;
  const int lane = tid & (kWave - 1);
  const int wave = waveUniform(tid >> 6);
  const int D = a.D, T = a.T;

  const int q = a.tiles / (int)gridDim.x, r = a.tiles % (int)gridDim.x;
  const int t0 = (int)blockIdx.x * q + min((int)blockIdx.x, r);
  const int n = q + ((int)blockIdx.x < r ? 1 : 0);
  if (n <= 0) return;

  CfWindow<G> winA, winB;
  loadWindow<G>(a, t0, tid, winB);

  // ---- taps -> LDS (zero-padded to [-31 D, 128 KS)), block max, two scaled f16 limbs ----------
  const int off0 = 31 * D;
  const int span = off0 + 128 * KS;
  float hm = 0.0f;
  for (int i = tid; i < span; i += kCfThreads) {
    const int j = i - off0;
    const float h = (j >= 0 && j < T) ? a.taps[j] : 0.0f;
    part[i] = h;
    hm = fmaxf(hm, fabsf(h));
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) hm = fmaxf(hm, __shfl_xor(hm, o));
  if (lane == 0) waveMax[wave] = hm;
  __syncthreads();
  float hMax = waveMax[0];
#pragma unroll
  for (int v = 1; v < kCfWaves; ++v) hMax = fmaxf(hMax, waveMax[v]);
  const int sh = hMax > 0.0f ? 14 - ilogbf(hMax) : 0;
  const int half = lane >> 5;
  const int col = lane & 31;
  h8 bh[kCfMaxKS], bl[kCfMaxKS];
#pragma unroll
  for (int s = 0; s < kCfMaxKS; ++s) {
    if (s < KS) {
      const int kap = 16 * (wave * KS + s) + 8 * half;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float hs = ldexpf(part[off0 + kap + e - col * D], sh);
        const _Float16 hi = (_Float16)hs;
        bh[s][e] = hi;
        bl[s][e] = (_Float16)(hs - (float)hi);
      }
    } else {
      bh[s] = h8{};
      bl[s] = h8{};
    }
  }
  __syncthreads();  // the tap staging area becomes the partial-sum area

  // ---- prologue: tile t0 into plane set 0; tile t0 + 1's window and statistics ---------------
  CfF16State st{0, true};
  st.direct = cfTileStats<G>(a, winB, t0, tid, red, &st.sx);
  if (!st.direct) splitWindowF16<G>(a, winB, smem, tid, ldexpf(1.0f, st.sx));
  if (n > 1) loadWindow<G>(a, t0 + 1, tid, winA);
  __syncthreads();

  if constexpr (DB) {
    CfF16State nx{0, true};
    if (n > 1) nx.direct = cfTileStats<G>(a, winA, t0 + 1, tid, red, &nx.sx);
    for (int i = 0; i < n; i += 2) {
      cfF16Tile<KS, G, EPI>(a, smem, part, red2, bh, bl, sh, i, n, t0, tid, winA, winB, st, nx);
      if (i + 1 < n)
        cfF16Tile<KS, G, EPI>(a, smem, part, red2, bh, bl, sh, i + 1, n, t0, tid, winB, winA, st, nx);
    }
  } else {
    CfWindow<G>& win = winA;
    const int arow = lane & 15;
    const int comp = (lane >> 4) & 1;
    const int uRow = 4 * D * arow + half;
    const int8_t* pI = smem + comp * a.planeStride;
    for (int i = 0; i < n; ++i) {
      const int tile = t0 + i;
      if (st.direct) {
        directTile<EPI>(a, tile, tid);
      } else {
        v16f acc = v16f{};
#pragma unroll
        for (int s = 0; s < kCfMaxKS; ++s) {
          if (s < KS) {
            const int u = uRow + 2 * (wave * KS + s);
            const int off = 16 * cfPhys(u, a.padShift);
            const h8 x0 = *reinterpret_cast<const h8*>(pI + off);
            const h8 x1 = *reinterpret_cast<const h8*>(pI + 2 * a.planeStride + off);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(x0, bh[s], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(x0, bl[s], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(x1, bh[s], acc, 0, 0, 0);
          }
        }
#pragma unroll
        for (int k = 0; k < 16; ++k) part[(wave * 16 + k) * kWave + lane] = acc[k];
      }
      __syncthreads();  // partials complete; every wave is done reading the planes
      if (!st.direct) {
        float yi = 0.0f, yq = 0.0f;
#pragma unroll
        for (int v = 0; v < kCfWaves; ++v) {
          yi += part[(v * 16 + wave) * kWave + lane];
          yq += part[(v * 16 + wave + 8) * kWave + lane];
        }
        const float outScale = ldexpf(1.0f, -(st.sx + sh));
        const int orow = (wave & 3) + 8 * (wave >> 2) + 4 * half;
        const int64_t k = (int64_t)tile * kCfTileOut + 32 * orow + col;
        if (k < a.nOut) {
          if (EPI == kEpiAm) {
            reinterpret_cast<float*>(a.out)[k] = amEnvelope(f2{yi, yq}) * outScale;
          } else {
            reinterpret_cast<f2*>(a.out)[k] = f2{yi, yq} * outScale;
          }
        }
      }
      if (i + 1 < n) {
        // the next tile's statistics (two barriers, which also fence this tile's partial reads),
        // its planes, then the loads of the one after
        st.direct = cfTileStats<G>(a, win, tile + 1, tid, red, &st.sx);
        if (!st.direct) splitWindowF16<G>(a, win, smem, tid, ldexpf(1.0f, st.sx));
        if (i + 2 < n) loadWindow<G>(a, tile + 2, tid, win);
        __syncthreads();
      }
    }
  }
}

// ---- wave-specialised f16 x 2 kernel (default cf32 MFMA path) ----------------------------------
//
// The barrier-synchronous kernels above keep all eight waves in the same phase, so the matrix
// cores idle while every wave splits, reduces or waits at a barrier (C3 attribution: MFMA alone
// 0.32 ms of 0.97). Here one 768-thread block per CU runs two roles that meet only through
// counters in LDS:
//   * 8 consumer waves (2 per SIMD): the split-K MFMA loop of the kernels above (tap fragments
//     resident in VGPRs), their 32x32 partial accumulators into LDS, and the reduction + epilogue
//     of 64 outputs each (the synchronous kernels' epilogue, same summation order);
//   * 4 producer waves (1 per SIMD): window loads (two register windows, each group refilled with
//     the tile two ahead right after it is split), the tile statistics (DPP reductions, no LDS
//     round trips) and the split into one of two plane sets.
// A producer's split of tile i + 1 runs on the vector ALUs while the consumers' MFMAs of tile i
// run on the matrix cores of the same SIMDs.
//
// Producer window: G units (8 samples, 64 B) per producer thread, unit g = ptid + 256 j; only the
// Wl units that hold window samples are loaded (the K padding beyond them stays zero in LDS).
// Buffer loads against a per-tile descriptor whose range ends at the input's last byte: past the
// end they return zeros (finite; those samples meet zero taps or feed outputs >= nOut), so no
// per-load clamping, one 32-bit offset per unit and the 64-bit base in SGPRs.
// The loads are inline asm with explicit vmcnt waits: the producer issues no other vector memory
// operations, every tile issues exactly 4 G loads (a window past the block's last tile gets an
// empty range, no traffic), and the only wait - before a window's statistics - is vmcnt(4 G): the
// window in question is then complete while the 4 G loads issued after it stay in flight. (The
// compiler's own counting merged both register windows at the loop header and waited for the
// newer window's loads before every split.)

__device__ __forceinline__ i4v wsTileRsrc(const CfFirArgs& a, int tile, bool valid = true) {
  const int64_t first = (int64_t)tile * kCfTileOut * a.D;  // first window sample
  const int64_t left = valid ? a.nIn - first : 0;          // >= 1 for every tile
  const int64_t bytes = left * 8 < 0x7fffffff ? left * 8 : 0x7fffffff;
  const uint64_t base = reinterpret_cast<uint64_t>(a.x + 2 * first);
  i4v r;
  r.x = waveUniform((int)(uint32_t)base);
  r.y = waveUniform((int)((base >> 32) & 0xffffu));  // stride 0
  r.z = waveUniform((int)bytes);                      // num_records (bytes)
  r.w = 0x00020000;                                   // gfx9 raw buffer: dword3
  return r;
}

template <int G>
__device__ __forceinline__ void wsLoadGroup(i4v rsrc, int Wl, int ptid, int j, CfWindow<G>& w) {
  const int g = ptid + kWsPThreads * j;
  const int voff = g < Wl ? 64 * g : 0x7ffffff0;  // unused unit: out of range, reads nothing
  asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen" : "=v"(w.v[j][0]) : "v"(voff), "s"(rsrc) : "memory");
  asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen offset:16" : "=v"(w.v[j][1]) : "v"(voff), "s"(rsrc) : "memory");
  asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen offset:32" : "=v"(w.v[j][2]) : "v"(voff), "s"(rsrc) : "memory");
  asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen offset:48" : "=v"(w.v[j][3]) : "v"(voff), "s"(rsrc) : "memory");
}

// Wait until at most N of this wave's loads are outstanding, then pin the window's registers
// behind the wait (the empty asm statements keep every use of them after it).
template <int N, int G>
__device__ __forceinline__ void wsWaitWindow(CfWindow<G>& w) {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
#pragma unroll
  for (int j = 0; j < G; ++j)
#pragma unroll
    for (int q = 0; q < 4; ++q) asm volatile("" : "+v"(w.v[j][q]));
}

// Branch-free (see wsTileRsrc): a unit past Wl holds zeros (its load was out of range) and is
// written to the spare unit Wu that no A fragment reads.
template <int G>
__device__ __forceinline__ void wsSplitGroup(const CfFirArgs& a, int Wl, const CfWindow<G>& w, int8_t* planes,
                                             int ptid, float scale, int j) {
  const int g = ptid + kWsPThreads * j;
  typedef float f2v __attribute__((ext_vector_type(2)));
  typedef _Float16 h2v __attribute__((ext_vector_type(2)));
  uint32_t i0[4], i1[4], q0[4], q1[4];
  const f2v sc = {scale, scale};
#pragma unroll
  for (int q = 0; q < 4; ++q) {  // samples 2q, 2q + 1: (re, im, re, im)
    // packed math on the natural (re, im) register pairs; the I / Q pairing happens in the
    // two-source f16 conversions, so no register moves: 12 VALU per two samples
    const f2v s0 = f2v{w.v[j][q].x, w.v[j][q].y} * sc;
    const f2v s1 = f2v{w.v[j][q].z, w.v[j][q].w} * sc;
    const h2v hi = __builtin_convertvector(f2v{s0.x, s1.x}, h2v);  // re0, re1
    const h2v hq = __builtin_convertvector(f2v{s0.y, s1.y}, h2v);  // im0, im1
    const f2v r0 = s0 - f2v{(float)hi.x, (float)hq.x};
    const f2v r1 = s1 - f2v{(float)hi.y, (float)hq.y};
    i0[q] = __builtin_bit_cast(uint32_t, hi);
    q0[q] = __builtin_bit_cast(uint32_t, hq);
    i1[q] = __builtin_bit_cast(uint32_t, __builtin_convertvector(f2v{r0.x, r1.x}, h2v));
    q1[q] = __builtin_bit_cast(uint32_t, __builtin_convertvector(f2v{r0.y, r1.y}, h2v));
  }
  const int off = 16 * cfPhys(g < Wl ? g : a.Wu, a.padShift);
  *reinterpret_cast<uint4*>(planes + off) = uint4{i0[0], i0[1], i0[2], i0[3]};
  *reinterpret_cast<uint4*>(planes + a.planeStride + off) = uint4{q0[0], q0[1], q0[2], q0[3]};
  *reinterpret_cast<uint4*>(planes + 2 * a.planeStride + off) = uint4{i1[0], i1[1], i1[2], i1[3]};
  *reinterpret_cast<uint4*>(planes + 3 * a.planeStride + off) = uint4{q1[0], q1[1], q1[2], q1[3]};
}

// Producer-local statistics of a window (as cfStatsLocal over the producer threads).
template <int G>
__device__ __forceinline__ void wsStatsLocal(const CfFirArgs& a, int Wl, int tile, const CfWindow<G>& w, int ptid,
                                             WsCtl* c, int parity) {
  const int lane = ptid & (kWave - 1);
  const int pw = ptid >> 6;
  const int inU = cfUnitsInInput(a, tile, Wl);  // units past Wl are not loaded (zeros)
  // on the bit patterns of |x|: a NaN pattern exceeds +inf's, so M > 3e38 (or NaN) sends a tile
  // holding a non-finite sample to the direct path without a separate probe
  uint32_t mu = 0, bminu = 0x7f800000u;
#pragma unroll
  for (int j = 0; j < G; ++j) {
    uint32_t um = 0;  // units past Wl read as zeros: no effect on either statistic
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      // the whole vector cast, then its lanes: this compiler's __builtin_bit_cast of an ext-vector ELEMENT
      // (v.y, v.z, v.w) reads element 0 - r06 found the statistics had seen only every other sample (a lone
      // impulse or NaN at an odd sample missed; tests/test_mfma_guard.py)
      const u4v b = __builtin_bit_cast(u4v, w.v[j][q]) & 0x7fffffffu;
      um = max(max(um, b.x), max(max(b.y, b.z), b.w));
    }
    const uint32_t bm = dppMax8u(um);  // 64-sample block = 8 consecutive units = 8 consecutive lanes
    mu = max(mu, um);
    if (bm > 0 || cfBlockInInput(ptid + kWsPThreads * j, inU)) bminu = min(bminu, bm);
  }
  const float m = __builtin_bit_cast(float, waveMaxU(mu));
  const float bmin = __builtin_bit_cast(float, waveMinU(bminu));
  if (lane == 0) {
    c->stat[parity][0][pw] = m;
    c->stat[parity][1][pw] = bmin;
  }
}

__device__ __forceinline__ bool wsStatsFinish(const WsCtl* c, int parity, int* sxOut) {
  // on the bit patterns (the statistics are |x| patterns): fmaxf would drop a NaN wave maximum
  uint32_t Mu = __builtin_bit_cast(uint32_t, c->stat[parity][0][0]);
  uint32_t Bu = __builtin_bit_cast(uint32_t, c->stat[parity][1][0]);
#pragma unroll
  for (int v = 1; v < kWsProducers; ++v) {
    Mu = max(Mu, __builtin_bit_cast(uint32_t, c->stat[parity][0][v]));
    Bu = min(Bu, __builtin_bit_cast(uint32_t, c->stat[parity][1][v]));
  }
  const float M = __builtin_bit_cast(float, Mu), B = __builtin_bit_cast(float, Bu);
  *sxOut = 0;
  if (!(M <= 3.0e38f)) return true;
  if (M == 0.0f) return false;
  if (M < 1.0e-30f || B < M * (1.0f / 65536.0f)) return true;
  *sxOut = 14 - ilogbf(M);
  return false;
}

// Producer, tile i: wCur holds tile i's window, wNext tile i + 1's (in flight).
template <int G>
__device__ __forceinline__ void wsProducerTile(const CfFirArgs& a, int Wl, int8_t* smem, WsCtl* c, int n, int tile,
                                               int i, int ptid, CfWindow<G>& wCur, CfWindow<G>& wNext) {
  const int lane = ptid & (kWave - 1);
  const int set = i & 1;
  wsWait(c, &c->pstat, kWsProducers * (i + 1));
  int sx = 0;
  const bool direct = wsStatsFinish(c, set, &sx);
  wsWait(c, &c->planesFree[set], kCfWaves * (i >> 1));
  int8_t* planes = smem + set * 4 * a.planeStride;
  const float scale = ldexpf(1.0f, sx);
  const i4v rsrc2 = wsTileRsrc(a, tile + 2, i + 2 < n);
#pragma unroll
  for (int j = 0; j < G; ++j) {
    if (!direct) wsSplitGroup<G>(a, Wl, wCur, planes, ptid, scale, j);
    wsLoadGroup<G>(rsrc2, Wl, ptid, j, wCur);
  }
  if (ptid == 0) c->mode[set] = direct ? kWsDirect : sx;
  wsSignal(&c->planesFull[set], lane);
  // unconditional (past the last tile: statistics of an empty window, never read), so that every
  // path waits for wNext's loads at the same point and the loop-carried wait counts stay exact
  wsWaitWindow<4 * G>(wNext);
  wsStatsLocal<G>(a, Wl, tile + 1, wNext, ptid, c, (i + 1) & 1);
  wsSignal(&c->pstat, lane);
}

// Consumer wave `wave` reduces accumulator register wave (I) / wave + 8 (Q) of one tile over the
// eight waves' partials (the synchronous kernels' order) and stores 64 outputs; j is the block-
// local tile index (its partials: buffer j & 1 when double-buffered, else the single buffer),
// waited for until every wave has written them. `mode`: the tile's scale exponent, or kWsDirect
// (outputs already stored).
template <int EPI, bool I8, bool AUD>
__device__ __forceinline__ void wsReduceFinish(const CfFirArgs& a, WsCtl* c, int sh, int tile, int j, int b, int mode,
                                               int tid, float yi, float yq, float* ring, bool lead);

template <int EPI, bool I8, bool AUD = false>
__device__ __forceinline__ void wsReduceTile(const CfFirArgs& a, const float* part, WsCtl* c, int sh, int tile, int j,
                                             bool dbp, int mode, int tid, float* ring = nullptr, bool lead = false) {
  const int lane = tid & (kWave - 1);
  const int wave = tid >> 6;
  const int b = dbp ? (j & 1) : 0;
  wsWait(c, &c->partsFull[b], kCfWaves * (dbp ? (j >> 1) + 1 : j + 1));
  if (I8 || mode != kWsDirect) {
    const float* pb = part + b * (kCfPartialBytes / 4);
    float yi = 0.0f, yq = 0.0f;
#pragma unroll
    for (int v = 0; v < kCfWaves; ++v) {
      yi += pb[(v * 16 + wave) * kWave + lane];
      yq += pb[(v * 16 + wave + 8) * kWave + lane];
    }
    wsReduceFinish<EPI, I8, AUD>(a, c, sh, tile, j, b, mode, tid, yi, yq, ring, lead);
  } else {
    wsSignal(&c->partsFree[b], lane);
  }
}

// The rest of a tile's reduction once its sums are formed: release the partial buffer, then the
// epilogue (AM ring + audio hand-off, or the output store).
template <int EPI, bool I8, bool AUD>
__device__ __forceinline__ void wsReduceFinish(const CfFirArgs& a, WsCtl* c, int sh, int tile, int j, int b, int mode,
                                               int tid, float yi, float yq, float* ring, bool lead) {
  const int lane = tid & (kWave - 1);
  const int wave = tid >> 6;
  {
    wsSignal(&c->partsFree[b], lane);
    const int orow = (wave & 3) + 8 * (wave >> 2) + 4 * (lane >> 5);
    const int64_t k = (int64_t)tile * kCfTileOut + 32 * orow + (lane & 31);
    // int8: the zero-window guard's tiles (mode bit 1, ws_common.h wsI8ZeroRun) in the direct fp32 form;
    // a.x carries the int8 input (iq4 + sub) on the int8 path
    if (I8 && (mode & 1) && k < a.nOut)
      wsI8DirectOutput(reinterpret_cast<const int8_t*>(a.x), a.taps, a.T, a.D, k, sh, yi, yq);
    if constexpr (AUD) {  // int8, AM: the tile's AM samples into the ring for the producers' audio FIR
      const float v = __builtin_amdgcn_sqrtf(fmaf(yi, yi, yq * yq)) * ldexpf(1.0f / 127.0f, -sh);
      // slot j mod kAmRing is free once the producers finished the audio outputs of tile j - kAmRing + 1
      if (j - kAmRing + 2 > 0) wsWait(c, &c->amFree, kWsProducers * (j - kAmRing + 2));
      const int pos = (j & (kAmRing - 1)) * kCfTileOut + 32 * orow + (lane & 31);
#if GSDR_WS_DIAG
      wsDiag(3, pos < 0 || pos >= kAmRing * kCfTileOut);
#endif
      const float rv = k < a.nOut ? v : 0.0f;
      ring[pos] = rv;
      if (pos < kAmRingMirror) ring[kAmRing * kCfTileOut + pos] = rv;
      wsSignal(&c->amSlot[j & (kAmRing - 1)], lane);
      // the lead tile belongs to the previous block (computed here only for the audio windows)
      if (a.out != nullptr && k < a.nOut && !(lead && j == 0)) reinterpret_cast<float*>(a.out)[k] = v;
    } else if (k < a.nOut) {
      if (I8) {  // the epilogue of firI8DecMfmaKernel: y = acc 2^-sc / 127
        const float outScale = ldexpf(1.0f / 127.0f, -sh);
        if (EPI == kEpiAm) reinterpret_cast<float*>(a.out)[k] = __builtin_amdgcn_sqrtf(fmaf(yi, yi, yq * yq)) * outScale;
        else reinterpret_cast<f2*>(a.out)[k] = f2{yi, yq} * outScale;
      } else {
        const float outScale = ldexpf(1.0f, -(mode + sh));
        if (EPI == kEpiAm) reinterpret_cast<float*>(a.out)[k] = amEnvelope(f2{yi, yq}) * outScale;
        else reinterpret_cast<f2*>(a.out)[k] = f2{yi, yq} * outScale;
      }
    }
  }
}

// Consumer waves of the wave-specialised kernels (cf32: 4 planes per set, 3 products; int8 IQ:
// 2 planes, 2 products, no direct tiles). `part` first holds the staged taps (consumers turn them
// into B fragments), then the partial accumulators.
template <int KS, int EPI, bool I8, bool AUD = false>
__device__ __forceinline__ void wsConsumers(const CfFirArgs& a, int8_t* smem, float* part, WsCtl* c, int sh, int t0,
                                            int n, int tid, bool dbp, float* ring = nullptr, bool lead = false) {
  constexpr int NP = I8 ? 2 : 4;
  const int lane = tid & (kWave - 1);
  const int wave = waveUniform(tid >> 6);
  const int D = a.D;
  const int off0 = 31 * D;
  const int half = lane >> 5;
  const int col = lane & 31;
  h8 bh[kCfMaxKS], bl[kCfMaxKS];
#pragma unroll
  for (int s = 0; s < kCfMaxKS; ++s) {
    if (s < KS) {
      const int kap = 16 * (wave * KS + s) + 8 * half;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float hs = ldexpf(part[off0 + kap + e - col * D], sh);
        const _Float16 hi = (_Float16)hs;
        bh[s][e] = hi;
        bl[s][e] = (_Float16)(hs - (float)hi);
      }
    } else {
      bh[s] = h8{};
      bl[s] = h8{};
    }
  }
  // no barrier past this point (the roles diverge): the tap staging area becomes the partial-sum
  // area once every consumer wave has its fragments (tapsRead, awaited before the first partials)
  wsSignal(&c->tapsRead, lane);

  const int arow = lane & 15;
  const int comp = (lane >> 4) & 1;
  const int uRow = 4 * D * arow + half;
  int prevMode = kWsDirect;
  for (int i = 0; i < n; ++i) {
    const int set = i & 1;
    const int tile = t0 + i;
    wsWait(c, &c->planesFull[set], kWsProducers * ((i >> 1) + 1));
    // int8: bit 0 = the zero-window guard's flag (the cf32 kernels: the tile's scale, or kWsDirect)
    const int mode = I8 ? (wsI8Zflag(c, set) ? 1 : 0) : waveUniform(c->mode[set]);
    if (!I8 && mode == kWsDirect) {
      wsSignal(&c->planesFree[set], lane);
      directTile<EPI>(a, tile, tid);
      // the partial hand-off counters advance as for any tile (the count-based waits rely on it)
      if (dbp) {
        wsSignal(&c->partsFull[i & 1], lane);
        if (i >= 1) wsReduceTile<EPI, I8, AUD>(a, part, c, sh, tile - 1, i - 1, true, prevMode, tid, ring, lead);
      } else {
        wsWait(c, &c->partsFree[0], kCfWaves * i);
        wsSignal(&c->partsFull[0], lane);
        wsReduceTile<EPI, I8, AUD>(a, part, c, sh, tile, i, false, mode, tid, ring, lead);
      }
      prevMode = mode;
      continue;
    }
    const int8_t* pI = smem + set * NP * a.planeStride + comp * a.planeStride;
    v16f acc = v16f{};
    // int8, two partial buffers: tile i - 1's sums are formed between this tile's MFMAs (the wave
    // would otherwise sit at each dependent MFMA's issue), in the same order as wsReduceTile
    constexpr bool IL = I8 && GSDR_WS_RED_IL;
    const bool red = IL && dbp && i >= 1;
    if (red) wsWait(c, &c->partsFull[(i - 1) & 1], kCfWaves * (((i - 1) >> 1) + 1));
    // (the reads are unconditional - no branch in the K loop; without a second buffer they stay in
    // the first, and their values are used only when `red`)
    const float* pr = part + (dbp ? ((i - 1) & 1) * (kCfPartialBytes / 4) : 0);
    float ri[kCfWaves], rq[kCfWaves];
    float yi = 0.0f, yq = 0.0f;
    auto readP = [&](int v) {
      ri[v] = pr[(v * 16 + wave) * kWave + lane];
      rq[v] = pr[(v * 16 + wave + 8) * kWave + lane];
    };
    // A fragments PF K-steps ahead; the empty asm keeps the scheduler from hoisting more reads
    // (the tap fragments already hold 88 VGPRs). int8 input: one plane per component (x' exact in
    // f16), cf32: two limbs. With one step ahead the compiler reuses the fragment's registers, so
    // each step's read is issued behind the previous step's two MFMAs and waited for in full
    // before the next pair: the LDS latency, not the matrix pipe, paced the step.
    constexpr int PF = I8 ? GSDR_WS_PF : 1;
    h8 xa[kCfMaxKS], xb[kCfMaxKS];
    auto readA = [&](int s) {
      const int off = 16 * cfPhys(uRow + 2 * (wave * KS + s), a.padShift);
      xa[s] = *reinterpret_cast<const h8*>(pI + off);
      if (!I8) xb[s] = *reinterpret_cast<const h8*>(pI + 2 * a.planeStride + off);
    };
#pragma unroll
    for (int s = 0; s < PF; ++s)
      if (s < KS) readA(s);
#pragma unroll
    for (int s = 0; s < kCfMaxKS; ++s) {
      if (s < KS) {
        if (s + PF < KS) readA(s + PF);
        if (IL && s < kCfWaves) readP(s);
        asm volatile("" ::: "memory");
        if (PF > 1) __builtin_amdgcn_sched_barrier(0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(xa[s], bh[s], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(xa[s], bl[s], acc, 0, 0, 0);
        if (!I8) acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(xb[s], bh[s], acc, 0, 0, 0);
        if (PF > 1) __builtin_amdgcn_sched_barrier(0);
        if (IL && s >= 1 && s - 1 < kCfWaves) {
          yi += ri[s - 1];
          yq += rq[s - 1];
        }
      }
    }
    if (IL) {  // shares the K loop did not reach (KS < 9)
#pragma unroll
      for (int v = 0; v < kCfWaves; ++v) {
        if (v >= KS) readP(v);
        if (v >= KS - 1) {
          yi += ri[v];
          yq += rq[v];
        }
      }
    }
    wsSignal(&c->planesFree[set], lane);  // this wave's A reads are complete
    if (dbp) {
      // two partial buffers: tile i's partials go to buffer i & 1 and tile i - 1 is reduced right
      // after, while the other waves may still be finishing tile i (no wait on the slowest wave
      // before the next tile's MFMAs)
      const int b = i & 1;
      wsWait(c, &c->partsFree[b], kCfWaves * (i >> 1));  // tile i - 2 reduced by every wave
      if (i < 2) wsWait(c, &c->tapsRead, kCfWaves);
      float* pb = part + b * (kCfPartialBytes / 4);
      if (red) wsReduceFinish<EPI, I8, AUD>(a, c, sh, tile - 1, i - 1, (i - 1) & 1, prevMode, tid, yi, yq, ring, lead);
#pragma unroll
      for (int k = 0; k < 16; ++k) pb[(wave * 16 + k) * kWave + lane] = acc[k];
      wsSignal(&c->partsFull[b], lane);
      if (!IL && i >= 1) wsReduceTile<EPI, I8, AUD>(a, part, c, sh, tile - 1, i - 1, true, prevMode, tid, ring, lead);
    } else {
      wsWait(c, &c->partsFree[0], kCfWaves * i);  // every wave has read tile i - 1's partials
      if (i == 0) wsWait(c, &c->tapsRead, kCfWaves);
#pragma unroll
      for (int k = 0; k < 16; ++k) part[(wave * 16 + k) * kWave + lane] = acc[k];
      wsSignal(&c->partsFull[0], lane);
      wsReduceTile<EPI, I8, AUD>(a, part, c, sh, tile, i, false, mode, tid, ring, lead);
    }
    prevMode = mode;
  }
  if (dbp && n >= 1) wsReduceTile<EPI, I8, AUD>(a, part, c, sh, t0 + n - 1, n - 1, true, prevMode, tid, ring, lead);
}

template <int KS, int G, int EPI>
__global__ __launch_bounds__(kWsThreads, 1) void firCfWsKernel(CfFirArgs a, int Wl) {
  extern __shared__ __attribute__((aligned(16))) int8_t smem[];
  float* part = reinterpret_cast<float*>(smem + 8 * a.planeStride);
  __shared__ WsCtl ctl;
  __shared__ float waveMax[kCfWaves + kWsProducers];
  WsCtl* c = &ctl;

  const int tid = threadIdx.x;
  const int lane = tid & (kWave - 1);
  const int wave = waveUniform(tid >> 6);
  const int D = a.D, T = a.T;

  const int q = a.tiles / (int)gridDim.x, r = a.tiles % (int)gridDim.x;
  const int t0 = (int)blockIdx.x * q + min((int)blockIdx.x, r);
  const int n = q + ((int)blockIdx.x < r ? 1 : 0);
  if (n <= 0) return;

  const int ptid = tid - kCfThreads;

  // ---- taps -> LDS (zero-padded to [-31 D, 128 KS)), block max; zero both plane sets --------
  if (tid < kWsCtlZeroWords) reinterpret_cast<int*>(c)[tid] = 0;
  if (tid == 0) {
    c->spinLimit = a.spinLimit;
    c->abortOut = a.abortOut;
  }
  const int off0 = 31 * D;
  const int span = off0 + 128 * KS;
  float hm = 0.0f;
  for (int i = tid; i < span; i += kWsThreads) {
    const int j = i - off0;
    const float h = (j >= 0 && j < T) ? a.taps[j] : 0.0f;
    part[i] = h;
    hm = fmaxf(hm, fabsf(h));
  }
  for (int i = tid; i < 8 * a.planeStride / 16; i += kWsThreads) reinterpret_cast<uint4*>(smem)[i] = uint4{0, 0, 0, 0};
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) hm = fmaxf(hm, __shfl_xor(hm, o));
  if (lane == 0) waveMax[wave] = hm;
  __syncthreads();
  float hMax = waveMax[0];
#pragma unroll
  for (int v = 1; v < kCfWaves + kWsProducers; ++v) hMax = fmaxf(hMax, waveMax[v]);
  const int sh = hMax > 0.0f ? 14 - ilogbf(hMax) : 0;

  if (wave >= kCfWaves) {
    // ================= producers =================
    CfWindow<G> wA, wB;
    const i4v r0 = wsTileRsrc(a, t0);
#pragma unroll
    for (int j = 0; j < G; ++j) wsLoadGroup<G>(r0, Wl, ptid, j, wA);
    const i4v r1 = wsTileRsrc(a, t0 + 1, n > 1);
#pragma unroll
    for (int j = 0; j < G; ++j) wsLoadGroup<G>(r1, Wl, ptid, j, wB);
    wsWaitWindow<4 * G>(wA);
    wsStatsLocal<G>(a, Wl, t0, wA, ptid, c, 0);
    wsSignal(&c->pstat, lane);
    // the back-edge only after the second tile: a path that skipped it would leave wA's loads as
    // the newest on entry and make the compiler's wait counts conservative for both windows
    for (int i = 0;; i += 2) {
      wsProducerTile<G>(a, Wl, smem, c, n, t0 + i, i, ptid, wA, wB);
      if (i + 1 >= n) break;
      wsProducerTile<G>(a, Wl, smem, c, n, t0 + i + 1, i + 1, ptid, wB, wA);
      if (i + 2 >= n) break;
    }
    wsWaitWindow<0>(wA);  // no load outlives the wave, and none lands in a register reused meanwhile
    wsWaitWindow<0>(wB);
    return;
  }

  wsConsumers<KS, EPI, false>(a, smem, part, c, sh, t0, n, tid, a.dbp != 0);
}

// ---- int8 IQ input -------------------------------------------------------------------------


template <int G>
struct I8DecWindow {
  uint32_t d[G][5];  // the dword holding the unit's first byte and the next four (a 2-byte-aligned
                     // unit straddles five)
};

// Branch-free window loads (kept in flight until the split), one dword each: indices are clamped
// to the last dword holding input bytes, which never crosses a page; clamped data only meets zero
// taps or feeds outputs >= nOut. (A dwordx4 clamped as a whole would shift the valid dwords of
// the input's last unit.)
template <int G>
__device__ __forceinline__ void loadWindowI8(const I8DecArgs& a, int tile, int tid, I8DecWindow<G>& w) {
  const uint32_t* d = reinterpret_cast<const uint32_t*>(a.iq4);
  const int64_t base = (int64_t)tile * kCfTileOut * a.D / 2;  // dwords (tile starts: multiples of 8 samples)
  const int64_t lastDw = (2 * a.nIn - 1 + a.sub) >> 2;
#pragma unroll
  for (int j = 0; j < G; ++j) {
    const int g = min(tid + kCfThreads * j, a.Wu - 1);
    const int64_t i = base + 4 * (int64_t)g;
#pragma unroll
    for (int q = 0; q < 5; ++q) w.d[j][q] = d[i + q < lastDw ? i + q : lastDw];
  }
}

template <int G>
__device__ __forceinline__ void splitWindowI8(const I8DecArgs& a, const I8DecWindow<G>& w, int8_t* planes, int tid) {
#pragma unroll
  for (int j = 0; j < G; ++j) {
    const int g = tid + kCfThreads * j;
    if (g < a.Wu) {
      uint32_t words[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) words[q] = __builtin_amdgcn_alignbyte(w.d[j][q + 1], w.d[j][q], a.sub);
      uint4 iu, qu;
      int8IqToF16Units(words, iu, qu);
      const int off = 16 * cfPhys(g, a.padShift);
      *reinterpret_cast<uint4*>(planes + off) = iu;
      *reinterpret_cast<uint4*>(planes + a.planeStride + off) = qu;
    }
  }
}

template <int KS, int G, int EPI>
__global__ __launch_bounds__(kCfThreads, 1) void firI8DecMfmaKernel(I8DecArgs a) {
  extern __shared__ __attribute__((aligned(16))) int8_t smem[];
  int8_t* planes = smem;
  float* part = reinterpret_cast<float*>(smem + 2 * a.planeStride);
  __shared__ float waveMax[kCfWaves];

  const int tid = threadIdx.x;
  const int lane = tid & (kWave - 1);
  const int wave = waveUniform(tid >> 6);
  const int D = a.D, T = a.T;

  const int q = a.tiles / (int)gridDim.x, r = a.tiles % (int)gridDim.x;
  const int t0 = (int)blockIdx.x * q + min((int)blockIdx.x, r);
  const int n = q + ((int)blockIdx.x < r ? 1 : 0);
  if (n <= 0) return;

  I8DecWindow<G> win;
  loadWindowI8<G>(a, t0, tid, win);

  // ---- taps -> LDS (zero-padded to [-31 D, 128 KS)), block max, two f16 limbs per tap ----------
  const int off0 = 31 * D;
  const int span = off0 + 128 * KS;
  float m = 0.0f;
  for (int i = tid; i < span; i += kCfThreads) {
    const int j = i - off0;
    const float h = (j >= 0 && j < T) ? a.taps[j] : 0.0f;
    part[i] = h;
    m = fmaxf(m, fabsf(h));
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  if (lane == 0) waveMax[wave] = m;
  __syncthreads();
  float maxAbs = waveMax[0];
#pragma unroll
  for (int v = 1; v < kCfWaves; ++v) maxAbs = fmaxf(maxAbs, waveMax[v]);
  const int sc = maxAbs > 0.0f ? 14 - ilogbf(maxAbs) : 0;  // max |h 2^sc| in [2^14, 2^15)
  const float outScale = ldexpf(1.0f / 127.0f, -sc);
  const int half = lane >> 5;
  const int col = lane & 31;
  h8 bh[kCfMaxKS], bl[kCfMaxKS];
#pragma unroll
  for (int s = 0; s < kCfMaxKS; ++s) {
    if (s < KS) {
      const int kap = 16 * (wave * KS + s) + 8 * half;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float hs = ldexpf(part[off0 + kap + e - col * D], sc);
        const _Float16 hi = (_Float16)hs;
        bh[s][e] = hi;
        bl[s][e] = (_Float16)(hs - (float)hi);
      }
    } else {
      bh[s] = h8{};
      bl[s] = h8{};
    }
  }
  __syncthreads();  // the tap staging area becomes the partial-sum area

  splitWindowI8<G>(a, win, planes, tid);
  if (n > 1) loadWindowI8<G>(a, t0 + 1, tid, win);
  __syncthreads();

  const int arow = lane & 15;
  const int comp = (lane >> 4) & 1;
  const int uRow = 4 * D * arow + half;
  const int8_t* pI = planes + comp * a.planeStride;

  for (int i = 0; i < n; ++i) {
    const int tile = t0 + i;
    v16f acc = v16f{};
#pragma unroll
    for (int s = 0; s < kCfMaxKS; ++s) {
      if (s < KS) {
        const int u = uRow + 2 * (wave * KS + s);
        const h8 x = *reinterpret_cast<const h8*>(pI + 16 * cfPhys(u, a.padShift));
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(x, bh[s], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(x, bl[s], acc, 0, 0, 0);
      }
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) part[(wave * 16 + k) * kWave + lane] = acc[k];
    __syncthreads();  // partials complete; every wave is done reading the planes

    float yi = 0.0f, yq = 0.0f;
#pragma unroll
    for (int v = 0; v < kCfWaves; ++v) {
      yi += part[(v * 16 + wave) * kWave + lane];
      yq += part[(v * 16 + wave + 8) * kWave + lane];
    }
    const int orow = (wave & 3) + 8 * (wave >> 2) + 4 * half;
    const int64_t k = (int64_t)tile * kCfTileOut + 32 * orow + col;
    if (k < a.nOut) {
      if (EPI == kEpiAm) {
        reinterpret_cast<float*>(a.out)[k] = __builtin_amdgcn_sqrtf(fmaf(yi, yi, yq * yq)) * outScale;
      } else {
        reinterpret_cast<f2*>(a.out)[k] = f2{yi, yq} * outScale;
      }
    }

    if (i + 1 < n) {
      splitWindowI8<G>(a, win, planes, tid);
      if (i + 2 < n) loadWindowI8<G>(a, tile + 2, tid, win);
      __syncthreads();
    }
  }
}

// ---- wave-specialised int8 IQ decimating kernel (default for firI8DecMfma) --------------------
//
// firCfWsKernel's roles and hand-offs with the int8 window: producers load 16-byte units (8 IQ
// samples) plus the following dword (a 2-byte-misaligned input straddles it), funnel-shift by the
// misalignment and convert to the exact f16 I / Q planes (no statistics, no direct tiles);
// consumers run two products per K-step and firI8DecMfmaKernel's epilogue (bit-identical).

template <int KS, int G, int EPI, bool AUD = false>
__global__ __launch_bounds__(kWsThreads, 1) void firI8WsKernel(I8DecArgs a8, int Wl) {
  extern __shared__ __attribute__((aligned(16))) int8_t smem[];
  float* part = reinterpret_cast<float*>(smem + 4 * a8.planeStride);
  __shared__ WsCtl ctl;
  __shared__ float waveMax[kCfWaves + kWsProducers];
  WsCtl* c = &ctl;

  const int tid = threadIdx.x;
  const int lane = tid & (kWave - 1);
  const int wave = waveUniform(tid >> 6);
  const int D = a8.D, T = a8.T;

  const int q = a8.tiles / (int)gridDim.x, r = a8.tiles % (int)gridDim.x;
  int t0 = (int)blockIdx.x * q + min((int)blockIdx.x, r);
  int n = q + ((int)blockIdx.x < r ? 1 : 0);
  if (n <= 0) return;
  // fused audio: every block but the first also computes the tile before its range (the lead) into
  // its AM ring, so each audio window it owns is complete on chip (+1 tile in ~100 at C5's size)
  bool lead = false;
  if (AUD && t0 > 0) {
    --t0;
    ++n;
    lead = true;
  }
  float* ring = AUD ? reinterpret_cast<float*>(smem + 4 * a8.planeStride + 2 * kCfPartialBytes) : nullptr;

  // ---- taps -> LDS (zero-padded to [-31 D, 128 KS)), block max; zero both plane sets --------
  if (tid < kWsCtlZeroWords) reinterpret_cast<int*>(c)[tid] = 0;
  if (tid == 0) {
    c->spinLimit = a8.spinLimit;
    c->abortOut = a8.abortOut;
  }
  const int off0 = 31 * D;
  const int span = off0 + 128 * KS;
  float hm = 0.0f;
  for (int i = tid; i < span; i += kWsThreads) {
    const int j = i - off0;
    const float h = (j >= 0 && j < T) ? a8.taps[j] : 0.0f;
    part[i] = h;
    hm = fmaxf(hm, fabsf(h));
  }
  for (int i = tid; i < 4 * a8.planeStride / 16; i += kWsThreads) reinterpret_cast<uint4*>(smem)[i] = uint4{0, 0, 0, 0};
  // the AM ring starts zeroed: an audio window reads 256 ring samples whatever the tap count, the
  // ones past its taps multiplied by zero - and 0 * NaN is NaN, so a slot this block never writes
  // (its tiles fill fewer than 8) must not hold whatever the LDS held before the launch (r04: NaN
  // audio outputs in short-filter steps on fresh boxes, 2 of 6 full-suite runs)
  if constexpr (AUD && GSDR_WS_RING_ZERO)
    for (int i = tid; i < (kAmRing * kCfTileOut + kAmRingMirror) / 4; i += kWsThreads)
      reinterpret_cast<uint4*>(ring)[i] = uint4{0, 0, 0, 0};
  hm = waveMaxNonNeg(hm);
  if (lane == 0) waveMax[wave] = hm;
  __syncthreads();
  float hMax = waveMax[0];
#pragma unroll
  for (int v = 1; v < kCfWaves + kWsProducers; ++v) hMax = fmaxf(hMax, waveMax[v]);
  const int sh = hMax > 0.0f ? 14 - ilogbf(hMax) : 0;  // max |h 2^sh| in [2^14, 2^15)
#if GSDR_WS_WAITS
  const unsigned long long span0 = __builtin_amdgcn_s_memtime();
#endif

  if (wave >= kCfWaves) {
    const int ptid = tid - kCfThreads;
    I8WsWindow<G> wA, wB;
    const i4v r0 = wsI8TileRsrc(a8, t0, true);
#pragma unroll
    for (int j = 0; j < G; ++j) wsI8LoadGroup<G>(r0, Wl, ptid, j, wA);
    const i4v r1 = wsI8TileRsrc(a8, t0 + 1, n > 1);
#pragma unroll
    for (int j = 0; j < G; ++j) wsI8LoadGroup<G>(r1, Wl, ptid, j, wB);
    float ht[kAudioTapsPerLane];  // audio taps (lane % 8) + 8 u
    AudioBounds ab = AUD ? audioBounds(a8, t0, n, lead) : AudioBounds{0, 0, 0};
#pragma unroll
    for (int u = 0; u < kAudioTapsPerLane; ++u) {
      const int tp = (lane & 7) + 8 * u;
      ht[u] = AUD && tp < a8.aT ? a8.aTaps[tp] : 0.0f;
    }
    for (int i = 0;; i += 2) {
      wsI8ProducerTile<G>(a8, Wl, smem, c, n, t0 + i, i, ptid, wA, [&] {
        if (AUD && i >= kAudioLag) wsAudioTile(a8, ring, c, t0, n, lead, i - kAudioLag, ptid, ht, ab);
      });
      if (i + 1 >= n) break;
      wsI8ProducerTile<G>(a8, Wl, smem, c, n, t0 + i + 1, i + 1, ptid, wB, [&] {
        if (AUD && i + 1 >= kAudioLag) wsAudioTile(a8, ring, c, t0, n, lead, i + 1 - kAudioLag, ptid, ht, ab);
      });
      if (i + 2 >= n) break;
    }
    wsI8DrainWindows<G>(wA, wB);  // ws_common.h: no register reuse under a landing load
    if constexpr (AUD)
      for (int t = n > kAudioLag ? n - kAudioLag : 0; t < n; ++t) wsAudioTile(a8, ring, c, t0, n, lead, t, ptid, ht, ab);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#if GSDR_WS_WAITS
    wsSpanStore(__builtin_amdgcn_s_memtime() - span0);
#endif
    return;
  }
  CfFirArgs a{};
  a.x = reinterpret_cast<const float*>(a8.iq4 + a8.sub);  // the int8 input (the zero-window guard's direct form)
  a.taps = a8.taps;
  a.out = a8.out;
  a.nOut = a8.nOut;
  a.nIn = a8.nIn;
  a.T = a8.T;
  a.D = a8.D;
  a.KS = a8.KS;
  a.tiles = a8.tiles;
  a.Wu = a8.Wu;
  a.padShift = a8.padShift;
  a.planeStride = a8.planeStride;
  a.dbp = a8.dbp;
  wsConsumers<KS, EPI, true, AUD>(a, smem, part, c, sh, t0, n, tid, a8.dbp != 0, ring, lead);
#if GSDR_WS_WAITS
  wsSpanStore(__builtin_amdgcn_s_memtime() - span0);
#endif
}

// ---- two-group int8 kernel (the fused C5 chain; built with -DGSDR_WS_GROUPS=1 only) ----------
// Measured r04 (profiles/r04/exp/c5_groups/): bit-identical to firI8WsKernel, all chain / fused /
// shard / abort tests green, but 263 us per C5 launch against 212 us: the B fragments read from LDS
// add 176 KB of ds_read_b128 traffic per tile, and while both groups issue MFMAs a CU asks its LDS for
// ~384 B/clk (peak 256) - the latency the groups hide is paid again as LDS bandwidth. Kept for the
// record, off.
#ifndef GSDR_WS_GROUPS
#define GSDR_WS_GROUPS 0
#endif
#define GSDR_POLICY_NO_WS_GROUPS 32u  // experimental builds: the 8-way kernel after all
// firI8WsKernel splits K over all 8 consumer waves: every tile is one round of hand-offs among 8
// waves for 22 MFMAs per wave, and the per-tile chain of one wave (waits, A reads, MFMAs, partial
// write / read, epilogue) is latency the matrix pipe sits idle behind (r04: MFMA pipe 34 % busy,
// LDS 43 %). Here the consumers form two groups of 4 (one wave of each group per SIMD): group g takes
// the block's tiles i = g, g + 2, ... (plane set g), each wave does TWO of the 8-way K shares (44
// MFMAs per tile, two accumulators), so a SIMD's two consumer waves work on different tiles and one
// wave's hand-offs and epilogue overlap the other's MFMAs. The B fragments (taps) come from LDS:
// 8 / gcd(D, 8) copies of the scaled hi / lo tap limbs, copy r shifted by r elements, so every lane's
// 8 taps h[kap - col D .. + 7] are one aligned ds_read_b128 (44 fragments per wave would not fit in
// VGPRs). The 8 partials of a tile are the 8-way kernel's, summed in its order: outputs are bit-
// identical to firI8WsKernel's.
template <int KS, bool AUD>
__device__ __forceinline__ void wsConsumersGroup(const I8DecArgs& a, int8_t* smem, float* part, const int8_t* tc, WsCtl* c,
                                                 int sh, int t0, int n, int tid, float* ring, bool lead) {
  constexpr int KW = 2 * KS;  // K-steps per wave
  constexpr int PF = GSDR_WS_PF;
  const int lane = tid & (kWave - 1);
  const int wave = waveUniform(tid >> 6);
  const int gr = wave >> 2, kq = wave & 3;
  const int D = a.D, off0 = 31 * D;
  const int half = lane >> 5, col = lane & 31;
  const int gd = (D & 1) ? 1 : (D & 2) ? 2 : (D & 4) ? 4 : 8;  // gcd(D, 8)
  // taps part[p .. p + 7], p = off0 + 16 gs + 8 half - col D, from the copy shifted by r = -p mod 8
  const int r = (8 - ((off0 - col * D) & 7)) & 7;
  const int bHi0 = 2 * (r / gd) * a.tcStride + 2 * (off0 - col * D + r + 8 * half);
  const int bLo0 = bHi0 + a.tcStride;
  const int kneed = waveUniform(a.kneed);
  const int arow = lane & 15;
  const int comp = (lane >> 4) & 1;
  const int uRow = 4 * D * arow + half;
  float* pg = part + gr * (kCfPartialBytes / 4);
  const float outScale = ldexpf(1.0f / 127.0f, -sh);
  for (int i = gr; i < n; i += 2) {
    const int set = i & 1;
    const int gi = i >> 1;  // the group's tile count
    const int tile = t0 + i;
    wsWait(c, &c->planesFull[set], kWsProducers * (gi + 1));
    const int8_t* pI = smem + set * 2 * a.planeStride + comp * a.planeStride;
    v16f acc0 = v16f{}, acc1 = v16f{};
    h8 xa[KW], bh[KW], bl[KW];
    auto readAB = [&](int s) {
      const int gs = kq * KW + s;
      xa[s] = *reinterpret_cast<const h8*>(pI + 16 * cfPhys(uRow + 2 * gs, a.padShift));
      // K-steps past the last nonzero tap read 8 zeros at a copy's start (part index < 8 <= off0)
      const bool live = gs < kneed;
      bh[s] = *reinterpret_cast<const h8*>(tc + (live ? bHi0 + 32 * gs : 0));
      bl[s] = *reinterpret_cast<const h8*>(tc + (live ? bLo0 + 32 * gs : 0));
    };
#pragma unroll
    for (int s = 0; s < PF; ++s)
      if (s < KW) readAB(s);
#pragma unroll
    for (int s = 0; s < KW; ++s) {
      if (s + PF < KW) readAB(s + PF);
      asm volatile("" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      if (s < KS) {
        acc0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(xa[s], bh[s], acc0, 0, 0, 0);
        acc0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(xa[s], bl[s], acc0, 0, 0, 0);
      } else {
        acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(xa[s], bh[s], acc1, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(xa[s], bl[s], acc1, 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    wsSignal(&c->planesFree[set], lane);  // this wave's A reads are complete
    // partials: accumulator a of wave kq is share v = 2 kq + a of the 8-way kernel
    wsWait(c, &c->partsFree[gr], kGWaves * gi);  // the group's previous tile reduced
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      pg[((2 * kq) * 16 + k) * kWave + lane] = acc0[k];
      pg[((2 * kq + 1) * 16 + k) * kWave + lane] = acc1[k];
    }
    wsSignal(&c->partsFull[gr], lane);
    wsWait(c, &c->partsFull[gr], kGWaves * (gi + 1));
    // wave kq reduces accumulator registers kq, kq + 4 (I) and kq + 8, kq + 12 (Q) in the 8-way
    // kernel's order (shares 0..7)
    float yi[2] = {0.0f, 0.0f}, yq[2] = {0.0f, 0.0f};
#pragma unroll
    for (int v = 0; v < kCfWaves; ++v)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        yi[h] += pg[(v * 16 + kq + 4 * h) * kWave + lane];
        yq[h] += pg[(v * 16 + kq + 4 * h + 8) * kWave + lane];
      }
    wsSignal(&c->partsFree[gr], lane);
    if (AUD && i - kAmRing + 2 > 0) wsWait(c, &c->amFree, kWsProducers * (i - kAmRing + 2));
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int orow = kq + 8 * h + 4 * half;
      const int64_t k = (int64_t)tile * kCfTileOut + 32 * orow + col;
      const float v = __builtin_amdgcn_sqrtf(fmaf(yi[h], yi[h], yq[h] * yq[h])) * outScale;
      if constexpr (AUD) {
        const int pos = (i & (kAmRing - 1)) * kCfTileOut + 32 * orow + col;
        const float rv = k < a.nOut ? v : 0.0f;
        ring[pos] = rv;
        if (pos < kAmRingMirror) ring[kAmRing * kCfTileOut + pos] = rv;
        if (a.out != nullptr && k < a.nOut && !(lead && i == 0)) reinterpret_cast<float*>(a.out)[k] = v;
      } else if (k < a.nOut) {
        reinterpret_cast<float*>(a.out)[k] = v;
      }
    }
    if constexpr (AUD) wsSignal(&c->amSlot[i & (kAmRing - 1)], lane);
  }
}

template <int KS, int G, bool AUD>
__global__ __launch_bounds__(kWsThreads, 1) void firI8WsGroupKernel(I8DecArgs a8, int Wl) {
  extern __shared__ __attribute__((aligned(16))) int8_t smem[];
  float* part = reinterpret_cast<float*>(smem + 4 * a8.planeStride);
  float* ring = reinterpret_cast<float*>(smem + 4 * a8.planeStride + 2 * kCfPartialBytes);
  int8_t* tc = smem + 4 * a8.planeStride + 2 * kCfPartialBytes + 4 * (kAmRing * kCfTileOut + kAmRingMirror);
  __shared__ WsCtl ctl;
  __shared__ float waveMax[kCfWaves + kWsProducers];
  WsCtl* c = &ctl;

  const int tid = threadIdx.x;
  const int lane = tid & (kWave - 1);
  const int wave = waveUniform(tid >> 6);
  const int D = a8.D, T = a8.T;

  const int q = a8.tiles / (int)gridDim.x, r = a8.tiles % (int)gridDim.x;
  int t0 = (int)blockIdx.x * q + min((int)blockIdx.x, r);
  int n = q + ((int)blockIdx.x < r ? 1 : 0);
  if (n <= 0) return;
  bool lead = false;  // as firI8WsKernel: the tile before the block's range, for the ring only
  if (AUD && t0 > 0) {
    --t0;
    ++n;
    lead = true;
  }

  if (tid < kWsCtlZeroWords) reinterpret_cast<int*>(c)[tid] = 0;
  if (tid == 0) {
    c->spinLimit = a8.spinLimit;
    c->abortOut = a8.abortOut;
  }
  const int off0 = 31 * D;
  float hm = 0.0f;
  for (int i = tid; i < T; i += kWsThreads) hm = fmaxf(hm, fabsf(a8.taps[i]));
  for (int i = tid; i < 4 * a8.planeStride / 16; i += kWsThreads) reinterpret_cast<uint4*>(smem)[i] = uint4{0, 0, 0, 0};
  // the AM ring starts zeroed: an audio window reads 256 ring samples whatever the tap count, the
  // ones past its taps multiplied by zero - and 0 * NaN is NaN, so a slot this block never writes
  // (its tiles fill fewer than 8) must not hold whatever the LDS held before the launch (r04: NaN
  // audio outputs in short-filter steps on fresh boxes, 2 of 6 full-suite runs)
  if constexpr (AUD && GSDR_WS_RING_ZERO)
    for (int i = tid; i < (kAmRing * kCfTileOut + kAmRingMirror) / 4; i += kWsThreads)
      reinterpret_cast<uint4*>(ring)[i] = uint4{0, 0, 0, 0};
  hm = waveMaxNonNeg(hm);
  if (lane == 0) waveMax[wave] = hm;
  __syncthreads();
  float hMax = waveMax[0];
#pragma unroll
  for (int v = 1; v < kCfWaves + kWsProducers; ++v) hMax = fmaxf(hMax, waveMax[v]);
  const int sh = hMax > 0.0f ? 14 - ilogbf(hMax) : 0;  // max |h 2^sh| in [2^14, 2^15)
  // tap copies: copy ci (shift ci gd) element j = part[j - ci gd] (part[i] = h[i - off0], zero
  // outside the taps), scaled by 2^sh and split into f16 hi + lo exactly as the 8-way kernel's
  // B fragments
  {
    const int gd = (D & 1) ? 1 : (D & 2) ? 2 : (D & 4) ? 4 : 8;
    const int nc = 8 / gd, L = a8.tcLen;
    for (int e = tid; e < nc * L; e += kWsThreads) {
      const int ci = e / L, j = e - ci * L;
      const int ti = j - ci * gd - off0;
      const float hs = ldexpf((ti >= 0 && ti < T) ? a8.taps[ti] : 0.0f, sh);
      const _Float16 hi = (_Float16)hs;
      reinterpret_cast<_Float16*>(tc + 2 * ci * a8.tcStride)[j] = hi;
      reinterpret_cast<_Float16*>(tc + (2 * ci + 1) * a8.tcStride)[j] = (_Float16)(hs - (float)hi);
    }
  }
  __syncthreads();

  if (wave >= kCfWaves) {
    const int ptid = tid - kCfThreads;
    I8WsWindow<G> wA, wB;
    const i4v r0 = wsI8TileRsrc(a8, t0, true);
#pragma unroll
    for (int j = 0; j < G; ++j) wsI8LoadGroup<G>(r0, Wl, ptid, j, wA);
    const i4v r1 = wsI8TileRsrc(a8, t0 + 1, n > 1);
#pragma unroll
    for (int j = 0; j < G; ++j) wsI8LoadGroup<G>(r1, Wl, ptid, j, wB);
    float ht[kAudioTapsPerLane];
    AudioBounds ab = AUD ? audioBounds(a8, t0, n, lead) : AudioBounds{0, 0, 0};
#pragma unroll
    for (int u = 0; u < kAudioTapsPerLane; ++u) {
      const int tp = (lane & 7) + 8 * u;
      ht[u] = AUD && tp < a8.aT ? a8.aTaps[tp] : 0.0f;
    }
    for (int i = 0;; i += 2) {
      wsI8ProducerTile<G, kGWaves>(a8, Wl, smem, c, n, t0 + i, i, ptid, wA, [&] {
        if (AUD && i >= kAudioLag) wsAudioTile<kGWaves>(a8, ring, c, t0, n, lead, i - kAudioLag, ptid, ht, ab);
      });
      if (i + 1 >= n) break;
      wsI8ProducerTile<G, kGWaves>(a8, Wl, smem, c, n, t0 + i + 1, i + 1, ptid, wB, [&] {
        if (AUD && i + 1 >= kAudioLag) wsAudioTile<kGWaves>(a8, ring, c, t0, n, lead, i + 1 - kAudioLag, ptid, ht, ab);
      });
      if (i + 2 >= n) break;
    }
    wsI8DrainWindows<G>(wA, wB);
    if constexpr (AUD)
      for (int t = n > kAudioLag ? n - kAudioLag : 0; t < n; ++t) wsAudioTile<kGWaves>(a8, ring, c, t0, n, lead, t, ptid, ht, ab);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    return;
  }
  wsConsumersGroup<KS, AUD>(a8, smem, part, tc, c, sh, t0, n, tid, ring, lead);
}

// ---- host side ------------------------------------------------------------------------------

namespace {


// F16: 0 = bf16 x 3, 1 = f16 x 2 single plane set, 2 = f16 x 2 double-buffered
template <int F16, int KS, int G, int EPI>
hipError_t launchCfG(const CfFirArgs& a, size_t lds, int grid, hipStream_t stream) {
  auto kernel = F16 == 2 ? &firCfF16MfmaKernel<KS, G, EPI, true>
                         : (F16 == 1 ? &firCfF16MfmaKernel<KS, G, EPI, false> : &firCfMfmaKernel<KS, G, EPI>);
  // per launch (cheap; per device, no process-wide once-flag)
  const hipError_t attrErr = hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                                  kCfDynLdsMax);
  if (attrErr != hipSuccess) return attrErr;
  hipLaunchKernelGGL(kernel, dim3(grid), dim3(kCfThreads), lds, stream, a);
  return hipGetLastError();
}

template <int F16, int KS>
hipError_t launchCfKS(const CfFirArgs& a, size_t lds, int grid, int epi, hipStream_t stream) {
  const int G = (a.Wu + kCfThreads - 1) / kCfThreads;
  switch (G) {
    case 1: return epi == kEpiAm ? launchCfG<F16, KS, 1, kEpiAm>(a, lds, grid, stream) : launchCfG<F16, KS, 1, kEpiComplex>(a, lds, grid, stream);
    case 2: return epi == kEpiAm ? launchCfG<F16, KS, 2, kEpiAm>(a, lds, grid, stream) : launchCfG<F16, KS, 2, kEpiComplex>(a, lds, grid, stream);
    // three window groups: two register windows would not fit beside the tap fragments
    default: {
      constexpr int F = F16 == 2 ? 1 : F16;
      return epi == kEpiAm ? launchCfG<F, KS, 3, kEpiAm>(a, lds, grid, stream) : launchCfG<F, KS, 3, kEpiComplex>(a, lds, grid, stream);
    }
  }
}

template <int F16>
hipError_t launchCfAny(const CfFirArgs& a, size_t lds, int grid, int epi, hipStream_t stream) {
  switch (a.KS) {
    case 1: return launchCfKS<F16, 1>(a, lds, grid, epi, stream);
    case 2: return launchCfKS<F16, 2>(a, lds, grid, epi, stream);
    case 3: return launchCfKS<F16, 3>(a, lds, grid, epi, stream);
    case 4: return launchCfKS<F16, 4>(a, lds, grid, epi, stream);
    case 5: return launchCfKS<F16, 5>(a, lds, grid, epi, stream);
    case 6: return launchCfKS<F16, 6>(a, lds, grid, epi, stream);
    case 7: return launchCfKS<F16, 7>(a, lds, grid, epi, stream);
    case 8: return launchCfKS<F16, 8>(a, lds, grid, epi, stream);
    case 9: return launchCfKS<F16, 9>(a, lds, grid, epi, stream);
    case 10: return launchCfKS<F16, 10>(a, lds, grid, epi, stream);
    default: return launchCfKS<F16, 11>(a, lds, grid, epi, stream);
  }
}


template <int KS, int G, int EPI>
hipError_t launchI8DecG(const I8DecArgs& a, size_t lds, int grid, hipStream_t stream) {
  // per launch (cheap; per device, no process-wide once-flag)
  const hipError_t attrErr = hipFuncSetAttribute(reinterpret_cast<const void*>(&firI8DecMfmaKernel<KS, G, EPI>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, kCfDynLdsMax);
  if (attrErr != hipSuccess) return attrErr;
  hipLaunchKernelGGL((firI8DecMfmaKernel<KS, G, EPI>), dim3(grid), dim3(kCfThreads), lds, stream, a);
  return hipGetLastError();
}

template <int KS, int G, int EPI>
hipError_t launchCfWsG(const CfFirArgs& a, int Wl, size_t lds, int grid, hipStream_t stream) {
  auto kernel = &firCfWsKernel<KS, G, EPI>;
  // per launch (cheap; per device, no process-wide once-flag)
  const hipError_t attrErr = hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                                  kCfDynLdsMax);
  if (attrErr != hipSuccess) return attrErr;
  hipLaunchKernelGGL(kernel, dim3(grid), dim3(kWsThreads), lds, stream, a, Wl);
  return hipGetLastError();
}

template <int KS>
hipError_t launchCfWsKS(const CfFirArgs& a, int Wl, size_t lds, int grid, int epi, hipStream_t stream) {
  const int G = (Wl + kWsPThreads - 1) / kWsPThreads;
  switch (G) {
    case 1: return epi == kEpiAm ? launchCfWsG<KS, 1, kEpiAm>(a, Wl, lds, grid, stream) : launchCfWsG<KS, 1, kEpiComplex>(a, Wl, lds, grid, stream);
    case 2: return epi == kEpiAm ? launchCfWsG<KS, 2, kEpiAm>(a, Wl, lds, grid, stream) : launchCfWsG<KS, 2, kEpiComplex>(a, Wl, lds, grid, stream);
    default: return epi == kEpiAm ? launchCfWsG<KS, 3, kEpiAm>(a, Wl, lds, grid, stream) : launchCfWsG<KS, 3, kEpiComplex>(a, Wl, lds, grid, stream);
  }
}

hipError_t launchCfWsAny(const CfFirArgs& a, int Wl, size_t lds, int grid, int epi, hipStream_t stream) {
  switch (a.KS) {
    case 1: return launchCfWsKS<1>(a, Wl, lds, grid, epi, stream);
    case 2: return launchCfWsKS<2>(a, Wl, lds, grid, epi, stream);
    case 3: return launchCfWsKS<3>(a, Wl, lds, grid, epi, stream);
    case 4: return launchCfWsKS<4>(a, Wl, lds, grid, epi, stream);
    case 5: return launchCfWsKS<5>(a, Wl, lds, grid, epi, stream);
    case 6: return launchCfWsKS<6>(a, Wl, lds, grid, epi, stream);
    case 7: return launchCfWsKS<7>(a, Wl, lds, grid, epi, stream);
    case 8: return launchCfWsKS<8>(a, Wl, lds, grid, epi, stream);
    case 9: return launchCfWsKS<9>(a, Wl, lds, grid, epi, stream);
    case 10: return launchCfWsKS<10>(a, Wl, lds, grid, epi, stream);
    default: return launchCfWsKS<11>(a, Wl, lds, grid, epi, stream);
  }
}

template <int KS, int G, int EPI>
hipError_t launchI8WsG(const I8DecArgs& a, int Wl, size_t lds, int grid, hipStream_t stream) {
  auto kernel = &firI8WsKernel<KS, G, EPI>;
  // per launch (cheap; per device, no process-wide once-flag)
  const hipError_t attrErr = hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                                  kCfDynLdsMax);
  if (attrErr != hipSuccess) return attrErr;
  hipLaunchKernelGGL(kernel, dim3(grid), dim3(kWsThreads), lds, stream, a, Wl);
  return hipGetLastError();
}

template <int KS, int G>
hipError_t launchI8WsAudioG(const I8DecArgs& a, int Wl, size_t lds, int grid, hipStream_t stream) {
  auto kernel = &firI8WsKernel<KS, G, kEpiAm, true>;
  const hipError_t attrErr = hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                                  kCfDynLdsMax);
  if (attrErr != hipSuccess) return attrErr;
  hipLaunchKernelGGL(kernel, dim3(grid), dim3(kWsThreads), lds, stream, a, Wl);
  return hipGetLastError();
}

template <int KS>
hipError_t launchI8WsAudioKS(const I8DecArgs& a, int Wl, size_t lds, int grid, hipStream_t stream) {
  switch ((Wl + kWsPThreads - 1) / kWsPThreads) {
    case 1: return launchI8WsAudioG<KS, 1>(a, Wl, lds, grid, stream);
    case 2: return launchI8WsAudioG<KS, 2>(a, Wl, lds, grid, stream);
    case 3: return launchI8WsAudioG<KS, 3>(a, Wl, lds, grid, stream);
    default: return launchI8WsAudioG<KS, 4>(a, Wl, lds, grid, stream);
  }
}

hipError_t launchI8WsAudioAny(const I8DecArgs& a, int Wl, size_t lds, int grid, hipStream_t stream) {
  switch (a.KS) {
    case 1: return launchI8WsAudioKS<1>(a, Wl, lds, grid, stream);
    case 2: return launchI8WsAudioKS<2>(a, Wl, lds, grid, stream);
    case 3: return launchI8WsAudioKS<3>(a, Wl, lds, grid, stream);
    case 4: return launchI8WsAudioKS<4>(a, Wl, lds, grid, stream);
    case 5: return launchI8WsAudioKS<5>(a, Wl, lds, grid, stream);
    case 6: return launchI8WsAudioKS<6>(a, Wl, lds, grid, stream);
    case 7: return launchI8WsAudioKS<7>(a, Wl, lds, grid, stream);
    case 8: return launchI8WsAudioKS<8>(a, Wl, lds, grid, stream);
    case 9: return launchI8WsAudioKS<9>(a, Wl, lds, grid, stream);
    case 10: return launchI8WsAudioKS<10>(a, Wl, lds, grid, stream);
    default: return launchI8WsAudioKS<11>(a, Wl, lds, grid, stream);
  }
}

#if GSDR_WS_GROUPS
template <int KS, int G>
hipError_t launchI8WsGroupG(const I8DecArgs& a, int Wl, size_t lds, int grid, hipStream_t stream) {
  auto kernel = &firI8WsGroupKernel<KS, G, true>;
  const hipError_t attrErr = hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                                  kCfDynLdsMax);
  if (attrErr != hipSuccess) return attrErr;
  hipLaunchKernelGGL(kernel, dim3(grid), dim3(kWsThreads), lds, stream, a, Wl);
  return hipGetLastError();
}

template <int KS>
hipError_t launchI8WsGroupKS(const I8DecArgs& a, int Wl, size_t lds, int grid, hipStream_t stream) {
  switch ((Wl + kWsPThreads - 1) / kWsPThreads) {
    case 1: return launchI8WsGroupG<KS, 1>(a, Wl, lds, grid, stream);
    case 2: return launchI8WsGroupG<KS, 2>(a, Wl, lds, grid, stream);
    case 3: return launchI8WsGroupG<KS, 3>(a, Wl, lds, grid, stream);
    default: return launchI8WsGroupG<KS, 4>(a, Wl, lds, grid, stream);
  }
}

// the two-group kernel is built for the long filters (8 - 11 K-steps per 8-way share)
constexpr int kGroupMinKS = 8;
hipError_t launchI8WsGroupAny(const I8DecArgs& a, int Wl, size_t lds, int grid, hipStream_t stream) {
  switch (a.KS) {
    case 8: return launchI8WsGroupKS<8>(a, Wl, lds, grid, stream);
    case 9: return launchI8WsGroupKS<9>(a, Wl, lds, grid, stream);
    case 10: return launchI8WsGroupKS<10>(a, Wl, lds, grid, stream);
    default: return launchI8WsGroupKS<11>(a, Wl, lds, grid, stream);
  }
}

// Tap-copy stride of the two-group kernel: 2 tcLen bytes + a pad (16-byte steps, within `room`)
// that minimises the B-fragment ds_read_b128 bank conflicts (every K-step shifts all lanes alike, so
// one step's pattern is every step's).
int groupTapStride(int D, int tcLen, size_t room) {
  const int off0 = 31 * D;
  const int gd = (D & 1) ? 1 : (D & 2) ? 2 : (D & 4) ? 4 : 8;
  const int nc = 8 / gd;
  int best = -1;
  int bestCost = 1 << 30;
  for (int pad = 0; pad <= 240; pad += 16) {
    const int stride = 2 * tcLen + pad;
    if ((size_t)2 * nc * stride > room) break;
    int cost = 0;
    for (const auto& grp : kB128Groups) {
      int units[16][16];
      int cnt[16] = {};
      int worst = 1;
      for (int li = 0; li < 16; ++li) {
        const int l = grp[li], col = l & 31, half = l >> 5;
        const int r = (8 - ((off0 - col * D) & 7)) & 7;
        const int unit = (2 * (r / gd) * stride + 2 * (off0 - col * D + r + 8 * half)) / 16;
        const int slot = unit & 15;
        bool dup = false;
        for (int k = 0; k < cnt[slot]; ++k) dup |= units[slot][k] == unit;
        if (!dup) units[slot][cnt[slot]++] = unit;
        worst = cnt[slot] > worst ? cnt[slot] : worst;
      }
      cost += worst;
    }
    if (cost < bestCost) {
      bestCost = cost;
      best = stride;
    }
  }
  return best;
}
#endif

template <int KS>
hipError_t launchI8WsKS(const I8DecArgs& a, int Wl, size_t lds, int grid, int epi, hipStream_t stream) {
  const int G = (Wl + kWsPThreads - 1) / kWsPThreads;
  switch (G) {
    case 1: return epi == kEpiAm ? launchI8WsG<KS, 1, kEpiAm>(a, Wl, lds, grid, stream) : launchI8WsG<KS, 1, kEpiComplex>(a, Wl, lds, grid, stream);
    case 2: return epi == kEpiAm ? launchI8WsG<KS, 2, kEpiAm>(a, Wl, lds, grid, stream) : launchI8WsG<KS, 2, kEpiComplex>(a, Wl, lds, grid, stream);
    case 3: return epi == kEpiAm ? launchI8WsG<KS, 3, kEpiAm>(a, Wl, lds, grid, stream) : launchI8WsG<KS, 3, kEpiComplex>(a, Wl, lds, grid, stream);
    default: return epi == kEpiAm ? launchI8WsG<KS, 4, kEpiAm>(a, Wl, lds, grid, stream) : launchI8WsG<KS, 4, kEpiComplex>(a, Wl, lds, grid, stream);
  }
}

hipError_t launchI8WsAny(const I8DecArgs& a, int Wl, size_t lds, int grid, int epi, hipStream_t stream) {
  switch (a.KS) {
    case 1: return launchI8WsKS<1>(a, Wl, lds, grid, epi, stream);
    case 2: return launchI8WsKS<2>(a, Wl, lds, grid, epi, stream);
    case 3: return launchI8WsKS<3>(a, Wl, lds, grid, epi, stream);
    case 4: return launchI8WsKS<4>(a, Wl, lds, grid, epi, stream);
    case 5: return launchI8WsKS<5>(a, Wl, lds, grid, epi, stream);
    case 6: return launchI8WsKS<6>(a, Wl, lds, grid, epi, stream);
    case 7: return launchI8WsKS<7>(a, Wl, lds, grid, epi, stream);
    case 8: return launchI8WsKS<8>(a, Wl, lds, grid, epi, stream);
    case 9: return launchI8WsKS<9>(a, Wl, lds, grid, epi, stream);
    case 10: return launchI8WsKS<10>(a, Wl, lds, grid, epi, stream);
    default: return launchI8WsKS<11>(a, Wl, lds, grid, epi, stream);
  }
}

template <int KS>
hipError_t launchI8DecKS(const I8DecArgs& a, size_t lds, int grid, int epi, hipStream_t stream) {
  const int G = (a.Wu + kCfThreads - 1) / kCfThreads;
  switch (G) {
    case 1: return epi == kEpiAm ? launchI8DecG<KS, 1, kEpiAm>(a, lds, grid, stream) : launchI8DecG<KS, 1, kEpiComplex>(a, lds, grid, stream);
    case 2: return epi == kEpiAm ? launchI8DecG<KS, 2, kEpiAm>(a, lds, grid, stream) : launchI8DecG<KS, 2, kEpiComplex>(a, lds, grid, stream);
    default: return epi == kEpiAm ? launchI8DecG<KS, 3, kEpiAm>(a, lds, grid, stream) : launchI8DecG<KS, 3, kEpiComplex>(a, lds, grid, stream);
  }
}

// Wave-specialised kernels: a wait that gives up (a hand-off that never completes) leaves that
// launch's outputs undefined. The aborting waves count it in a pinned, device-mapped host word per
// device; the next launch of a wave-specialised kernel on that device reports it as
// hipErrorLaunchTimeOut, and gsdrAmdWsAborts reads it after a device synchronisation.
constexpr int kMaxDevices = 64;
std::mutex gAbortMu;
uint32_t* gAbortHost[kMaxDevices];
uint32_t* gAbortDev[kMaxDevices];
std::atomic<int> gWsSpinLimit{kWsSpinLimit};

// Device view of this device's abort word (allocated on first use; nullptr if that fails).
uint32_t* wsAbortWord(int dev) {
  if (dev < 0 || dev >= kMaxDevices) return nullptr;
  std::lock_guard<std::mutex> lock(gAbortMu);
  if (gAbortDev[dev] == nullptr) {
    // not a stream operation: allowed even if the caller's stream is being captured
    hipStreamCaptureMode mode = hipStreamCaptureModeRelaxed;
    (void)hipThreadExchangeStreamCaptureMode(&mode);
    void* h = nullptr;
    void* d = nullptr;
    if (hipHostMalloc(&h, 64, hipHostMallocMapped | hipHostMallocCoherent) == hipSuccess) {
      *static_cast<volatile uint32_t*>(h) = 0;
      if (hipHostGetDevicePointer(&d, h, 0) == hipSuccess) {
        gAbortHost[dev] = static_cast<uint32_t*>(h);
        gAbortDev[dev] = static_cast<uint32_t*>(d);
      } else {
        (void)hipHostFree(h);
      }
    }
    (void)hipThreadExchangeStreamCaptureMode(&mode);
  }
  return gAbortDev[dev];
}

// Aborts counted on `dev` so far, without clearing them (a host read of the mapped word).
uint32_t peekWsAborts(int dev) {
  if (dev < 0 || dev >= kMaxDevices) return 0;
  uint32_t* h;
  {
    std::lock_guard<std::mutex> lock(gAbortMu);
    h = gAbortHost[dev];
  }
  return h == nullptr ? 0u : __atomic_load_n(h, __ATOMIC_SEQ_CST);
}

// Aborts counted since the last read on `dev` (host read of the mapped word; clears it).
uint32_t takeWsAborts(int dev) {
  if (dev < 0 || dev >= kMaxDevices) return 0;
  uint32_t* h;
  {
    std::lock_guard<std::mutex> lock(gAbortMu);
    h = gAbortHost[dev];
  }
  return h == nullptr ? 0u : __atomic_exchange_n(h, 0u, __ATOMIC_SEQ_CST);
}

// Before a wave-specialised launch: report an earlier launch's abort, and arm this one. The abort
// word is only peeked at (a host read); when it is set, the device is synchronised first, so the
// count is complete and no kernel is still writing it, then it is taken: a caller that
// synchronises after a launch gets the report from its next call, deterministically, and the
// common case (no abort) costs no API call. Under stream capture nothing is read (a graph
// executor checks before its next replay, gsdrAmdWsAbortsPending / gsdrAmdWsTakeAborts).
hipError_t wsPrepare(hipStream_t stream, int32_t& spinLimit, uint32_t*& abortOut) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if ((e = hipStreamIsCapturing(stream, &cs)) != hipSuccess) return e;
  if (cs == hipStreamCaptureStatusNone && peekWsAborts(dev) != 0) {
    if ((e = hipDeviceSynchronize()) != hipSuccess) return e;
    if (takeWsAborts(dev) != 0) return hipErrorLaunchTimeOut;
  }
  spinLimit = gWsSpinLimit.load(std::memory_order_relaxed);
  abortOut = wsAbortWord(dev);
  return hipSuccess;
}

}  // namespace

hipError_t wsPrepareLaunch(hipStream_t stream, int32_t& spinLimit, uint32_t*& abortOut) {
  return wsPrepare(stream, spinLimit, abortOut);
}

bool firCfMfmaEligible(size_t tapCount, size_t decimation, const void* in) {
  const size_t d = decimation < 1 ? 1 : decimation;
  return tapCount >= 64 && d <= (size_t)kCfMaxD && 31 * d + tapCount <= (size_t)(kCfWaves * kCfMaxKS * 16) &&
         (reinterpret_cast<uintptr_t>(in) & 15u) == 0;
}

hipError_t launchFirCfMfma(const float* x, const float* taps, size_t tapCount, size_t decimation, void* out,
                           size_t nOut, int epi, hipStream_t stream) {
  CfFirArgs a{};
  a.x = x;
  a.taps = taps;
  a.out = out;
  a.D = (int32_t)(decimation < 1 ? 1 : decimation);
  a.T = (int32_t)tapCount;
  a.nOut = (int64_t)nOut;
  a.nIn = (int64_t)(nOut - 1) * a.D + (int64_t)tapCount;
  const int ksteps = (31 * a.D + a.T + 15) / 16;
  a.KS = (ksteps + kCfWaves - 1) / kCfWaves;
  const int64_t tiles = ((int64_t)nOut + kCfTileOut - 1) / kCfTileOut;
  if (tiles > 0x7fffffff) return hipErrorInvalidValue;
  a.tiles = (int32_t)tiles;
  a.Wu = 60 * a.D + 16 * a.KS;
  // f16 x 2 with a per-tile scale by default: the wave-specialised kernel when two plane sets fit
  // and a producer thread holds at most 3 window units, else the barrier-synchronous one (double-
  // buffered when two plane sets fit); GSDR_POLICY_CF_BF16 selects bf16 x 3
#ifdef GSDR_FORCE_POLICY  // variant builds only (tools/exp)
  const uint32_t policy = GSDR_FORCE_POLICY;
#else
  const uint32_t policy = kernelPolicy();
#endif
  const bool f16 = (policy & GSDR_POLICY_CF_BF16) == 0;
  const int grid = (int)(tiles < 256 ? tiles : 256);
  const int Wl = std::min(a.Wu, (511 * a.D + a.T + 7) / 8);  // units holding window samples
  if (f16 && (policy & GSDR_POLICY_NO_WS) == 0 && Wl <= 3 * kWsPThreads) {
    static std::mutex wsMu;
    static int wsD = -1, wsKS = -1;
    static CfLayout wsLayout{};
    CfLayout lay;
    {
      std::lock_guard<std::mutex> lock(wsMu);
      if (wsD != a.D || wsKS != a.KS) {
        wsLayout = cfPlaneLayout(a.D, a.KS, a.Wu, 8);
        wsD = a.D;
        wsKS = a.KS;
      }
      lay = wsLayout;
    }
    if (lay.planeStride != 0) {
      a.padShift = lay.padShift;
      a.planeStride = lay.planeStride;
      size_t lds = 8 * (size_t)a.planeStride + 2 * kCfPartialBytes;
      a.dbp = lds <= (size_t)kCfDynLdsMax;  // double-buffered partials when they fit
      if (!a.dbp) lds -= kCfPartialBytes;
      if (lds <= (size_t)kCfDynLdsMax) {
        if (hipError_t e = wsPrepare(stream, a.spinLimit, a.abortOut); e != hipSuccess) return e;
        return launchCfWsAny(a, Wl, lds, grid, epi, stream);
      }
    }
  }
  static std::mutex mu;
  static int cachedD = -1, cachedKS = -1, cachedMode = -1;
  static CfLayout cached{};
  static int cachedPlanes = 0;
  {
    std::lock_guard<std::mutex> lock(mu);
    const int mode = f16 ? 1 : 0;
    if (cachedD != a.D || cachedKS != a.KS || cachedMode != mode) {
      cachedPlanes = f16 ? 8 : 6;
      cached = cfPlaneLayout(a.D, a.KS, a.Wu, cachedPlanes);
      if (f16 && cached.planeStride == 0) {  // two sets do not fit: one set
        cachedPlanes = 4;
        cached = cfPlaneLayout(a.D, a.KS, a.Wu, cachedPlanes);
      }
      cachedD = a.D;
      cachedKS = a.KS;
      cachedMode = mode;
    }
    a.padShift = cached.padShift;
    a.planeStride = cached.planeStride;
  }
  const int nPlanes = cachedPlanes;
  const size_t lds = nPlanes * (size_t)a.planeStride + kCfPartialBytes;
  if (a.planeStride == 0 || lds > (size_t)kCfDynLdsMax) return hipErrorInvalidValue;
  if (!f16) return launchCfAny<0>(a, lds, grid, epi, stream);
  return nPlanes == 8 ? launchCfAny<2>(a, lds, grid, epi, stream) : launchCfAny<1>(a, lds, grid, epi, stream);
}

bool firI8DecMfmaEligible(size_t tapCount, size_t decimation, const void* in) {
  const size_t d = decimation < 1 ? 1 : decimation;
  // the Toeplitz K = 31 D + T beats the fp32 direct form once T >= 5 D (16x the FLOP rate, 2 limbs)
  return tapCount >= 32 && tapCount >= 5 * d && d <= (size_t)kCfMaxD &&
         31 * d + tapCount <= (size_t)(kCfWaves * kCfMaxKS * 16) && (reinterpret_cast<uintptr_t>(in) & 1u) == 0;
}

hipError_t launchFirI8DecMfma(const int8_t* iq, const float* taps, size_t tapCount, size_t decimation, void* out,
                              size_t nOut, int epi, hipStream_t stream) {
  I8DecArgs a{};
  a.sub = (int32_t)(reinterpret_cast<uintptr_t>(iq) & 3u);
  a.iq4 = iq - a.sub;
  a.taps = taps;
  a.out = out;
  a.D = (int32_t)(decimation < 1 ? 1 : decimation);
  a.T = (int32_t)tapCount;
  a.nOut = (int64_t)nOut;
  a.nIn = (int64_t)(nOut - 1) * a.D + (int64_t)tapCount;
  const int ksteps = (31 * a.D + a.T + 15) / 16;
  a.KS = (ksteps + kCfWaves - 1) / kCfWaves;
  const int64_t tiles = ((int64_t)nOut + kCfTileOut - 1) / kCfTileOut;
  if (tiles > 0x7fffffff) return hipErrorInvalidValue;
  a.tiles = (int32_t)tiles;
  a.Wu = 60 * a.D + 16 * a.KS;
#ifdef GSDR_FORCE_POLICY
  const uint32_t policy = GSDR_FORCE_POLICY;
#else
  const uint32_t policy = kernelPolicy();
#endif
  const int grid = (int)(tiles < 256 ? tiles : 256);
  // the 4-way split-K kernel (r05) unless GSDR_POLICY_NO_WS / GSDR_POLICY_I8_WS8
  if ((policy & (GSDR_POLICY_NO_WS | GSDR_POLICY_I8_WS8)) == 0) {
    const hipError_t e = launchFirI8Ws4(a, ksteps, epi, false, stream);
    if (e != hipErrorNotSupported) return e;
  }
  // wave-specialised unless GSDR_POLICY_NO_WS (two plane sets of the int8 window always fit)
  const int Wl = std::min(a.Wu, (511 * a.D + a.T + 7) / 8);
  if ((policy & GSDR_POLICY_NO_WS) == 0 && Wl <= 4 * kWsPThreads) {
    static std::mutex wsMu;
    static int wsD = -1, wsKS = -1;
    static CfLayout wsLayout{};
    CfLayout lay;
    {
      std::lock_guard<std::mutex> lock(wsMu);
      if (wsD != a.D || wsKS != a.KS) {
        wsLayout = cfPlaneLayout(a.D, a.KS, a.Wu, 4);
        wsD = a.D;
        wsKS = a.KS;
      }
      lay = wsLayout;
    }
    if (lay.planeStride != 0) {
      a.padShift = lay.padShift;
      a.planeStride = lay.planeStride;
      size_t lds = 4 * (size_t)a.planeStride + 2 * kCfPartialBytes;
      a.dbp = lds <= (size_t)kCfDynLdsMax;
      if (!a.dbp) lds -= kCfPartialBytes;
      if (lds <= (size_t)kCfDynLdsMax) {
        if (hipError_t e = wsPrepare(stream, a.spinLimit, a.abortOut); e != hipSuccess) return e;
        return launchI8WsAny(a, Wl, lds, grid, epi, stream);
      }
    }
  }
  static std::mutex mu;
  static int cachedD = -1, cachedKS = -1;
  static CfLayout cached{};
  {
    std::lock_guard<std::mutex> lock(mu);
    if (cachedD != a.D || cachedKS != a.KS) {
      cached = cfPlaneLayout(a.D, a.KS, a.Wu, 2);
      cachedD = a.D;
      cachedKS = a.KS;
    }
    a.padShift = cached.padShift;
    a.planeStride = cached.planeStride;
  }
  const size_t lds = 2 * (size_t)a.planeStride + kCfPartialBytes;
  if (a.planeStride == 0 || lds > (size_t)kCfDynLdsMax) return hipErrorInvalidValue;
  switch (a.KS) {
    case 1: return launchI8DecKS<1>(a, lds, grid, epi, stream);
    case 2: return launchI8DecKS<2>(a, lds, grid, epi, stream);
    case 3: return launchI8DecKS<3>(a, lds, grid, epi, stream);
    case 4: return launchI8DecKS<4>(a, lds, grid, epi, stream);
    case 5: return launchI8DecKS<5>(a, lds, grid, epi, stream);
    case 6: return launchI8DecKS<6>(a, lds, grid, epi, stream);
    case 7: return launchI8DecKS<7>(a, lds, grid, epi, stream);
    case 8: return launchI8DecKS<8>(a, lds, grid, epi, stream);
    case 9: return launchI8DecKS<9>(a, lds, grid, epi, stream);
    case 10: return launchI8DecKS<10>(a, lds, grid, epi, stream);
    default: return launchI8DecKS<11>(a, lds, grid, epi, stream);
  }
}

// int8 IQ -> FC FIR -> AM -> FF FIR in ONE launch of the wave-specialised kernel (firI8WsKernel<..,
// true>): the consumers keep each tile's AM samples in an LDS ring, the producers run the audio FIR
// from it. Returns hipErrorNotSupported when the shape or the policy does not take that kernel (the
// caller then runs the two stages). amOut (nullable: AM not stored) = AM output 0; amHist[0, amH)
// the AM samples before it.
hipError_t launchFirI8DecMfmaAudio(const int8_t* iq, const float* taps, size_t tapCount, size_t decimation,
                                   float* amOut, size_t nOut, const float* amHist, size_t amH, const float* aTaps,
                                   size_t aT, size_t aD, float* aOut, size_t aN, hipStream_t stream) {
  static_assert(kCfTileOut == 512, "the audio ring indexes AM samples by k >> 9");
#ifdef GSDR_FORCE_POLICY
  const uint32_t policy = GSDR_FORCE_POLICY;
#else
  const uint32_t policy = kernelPolicy();
#endif
  if ((policy & (GSDR_POLICY_NO_MFMA | GSDR_POLICY_NO_WS | GSDR_POLICY_PREFER_FFT)) != 0) return hipErrorNotSupported;
  if (!firI8DecMfmaEligible(tapCount, decimation, iq) || aT == 0 || aT > (size_t)kAudioMaxTaps || aD == 0 ||
      aD > 0x7fffffff || amH > 0x1fffffff || nOut == 0 || aN == 0)  // history: one 32-bit buffer range
    return hipErrorNotSupported;
  I8DecArgs a{};
  a.sub = (int32_t)(reinterpret_cast<uintptr_t>(iq) & 3u);
  a.iq4 = iq - a.sub;
  a.taps = taps;
  a.out = amOut;
  a.D = (int32_t)(decimation < 1 ? 1 : decimation);
  a.T = (int32_t)tapCount;
  a.nOut = (int64_t)nOut;
  a.nIn = (int64_t)(nOut - 1) * a.D + (int64_t)tapCount;
  const int ksteps = (31 * a.D + a.T + 15) / 16;
  a.KS = (ksteps + kCfWaves - 1) / kCfWaves;
  const int64_t tiles = ((int64_t)nOut + kCfTileOut - 1) / kCfTileOut;
  if (tiles > 0x7fffffff) return hipErrorNotSupported;
  a.tiles = (int32_t)tiles;
  a.Wu = 60 * a.D + 16 * a.KS;
  const int Wl = std::min(a.Wu, (511 * a.D + a.T + 7) / 8);
  if (Wl > 4 * kWsPThreads) return hipErrorNotSupported;
  if (!audioIndexFits(tiles, (int64_t)amH, (int64_t)aN, (int64_t)aD, (int64_t)aT)) return hipErrorNotSupported;
  // the layout search costs ~1 ms of host time: cached per (D, KS) like the other launchers' (an
  // uncached search per call starved the GPU between eager launches: 0.70 ms per C5 step); a small
  // map, so chains with different RF decimations / tap counts stepped alternately stay cached
  static std::mutex layMu;
  static std::vector<std::pair<uint64_t, CfLayout>> layCache;
  auto cachedLayout = [&](int tag, size_t extra) {
    const uint64_t key = ((uint64_t)(uint32_t)a.D << 32) | ((uint64_t)(uint32_t)a.KS << 8) | (uint32_t)tag;
    std::lock_guard<std::mutex> lock(layMu);
    for (const auto& [k, v] : layCache)
      if (k == key) return v;
    const CfLayout l = cfPlaneLayout(a.D, a.KS, a.Wu, 4, extra);
    if (layCache.size() >= 16) layCache.erase(layCache.begin());
    layCache.emplace_back(key, l);
    return l;
  };
  a.audioPerm = cachedAudioSlotPerm((int)aD);
  if ((policy & GSDR_POLICY_I8_WS8) == 0) {  // the 4-way split-K kernel (r05)
    I8DecArgs w = a;
    w.aTaps = aTaps;
    w.aOut = aOut;
    w.amHist = amHist;
    w.aN = (int64_t)aN;
    w.aT = (int32_t)aT;
    w.aD = (int32_t)aD;
    w.amH = (int32_t)amH;
    const hipError_t e = launchFirI8Ws4(w, ksteps, kEpiAm, true, stream);
    if (e != hipErrorNotSupported) return e;
  }
  const size_t ringBytes = sizeof(float) * (kAmRing * kCfTileOut + kAmRingMirror);
#if GSDR_WS_GROUPS
  // the two-group kernel (bit-identical outputs; GSDR_POLICY_NO_WS_GROUPS keeps the 8-way one)
  if ((policy & GSDR_POLICY_NO_WS_GROUPS) == 0 && a.KS >= kGroupMinKS) {
    const int gd = (a.D & 1) ? 1 : (a.D & 2) ? 2 : (a.D & 4) ? 4 : 8;
    const int nc = 8 / gd;
    const int tcLen = (31 * a.D + 16 * ksteps + 8 + 7) / 8 * 8;
    const size_t fixed = 2 * (size_t)kCfPartialBytes + ringBytes;
    const CfLayout gl = cachedLayout(1, fixed + (size_t)2 * nc * 2 * tcLen);
    if (gl.planeStride != 0) {
      const size_t used = 4 * (size_t)gl.planeStride + fixed;
      const int stride = used < (size_t)kCfDynLdsMax ? groupTapStride(a.D, tcLen, kCfDynLdsMax - used) : -1;
      if (stride > 0) {
        I8DecArgs g = a;
        g.padShift = gl.padShift;
        g.planeStride = gl.planeStride;
        g.dbp = 0;
        g.aTaps = aTaps;
        g.aOut = aOut;
        g.amHist = amHist;
        g.aN = (int64_t)aN;
        g.aT = (int32_t)aT;
        g.aD = (int32_t)aD;
        g.amH = (int32_t)amH;
        g.kneed = ksteps;
        g.tcLen = tcLen;
        g.tcStride = stride;
        const size_t glds = used + (size_t)2 * nc * stride;
        const int grid = (int)(tiles < 256 ? tiles : 256);
        if (hipError_t e = wsPrepare(stream, g.spinLimit, g.abortOut); e != hipSuccess) return e;
        return launchI8WsGroupAny(g, Wl, glds, grid, stream);
      }
    }
  }
#endif
  const CfLayout lay = cachedLayout(0, kCfPartialBytes);
  if (lay.planeStride == 0) return hipErrorNotSupported;
  a.padShift = lay.padShift;
  a.planeStride = lay.planeStride;
  const size_t lds = 4 * (size_t)a.planeStride + 2 * kCfPartialBytes + ringBytes;
  if (lds > (size_t)kCfDynLdsMax) return hipErrorNotSupported;
  a.dbp = 1;
  a.aTaps = aTaps;
  a.aOut = aOut;
  a.amHist = amHist;
  a.aN = (int64_t)aN;
  a.aT = (int32_t)aT;
  a.aD = (int32_t)aD;
  a.amH = (int32_t)amH;
  const int grid = (int)(tiles < 256 ? tiles : 256);
  if (hipError_t e = wsPrepare(stream, a.spinLimit, a.abortOut); e != hipSuccess) return e;
  return launchI8WsAudioAny(a, Wl, lds, grid, stream);
}

}  // namespace gsdr_amd

#if GSDR_WS_WAITS
namespace gsdr_amd {
hipError_t w4WaitsRead(unsigned long long* out, size_t n, int reset);
}
extern "C" __attribute__((visibility("default"))) hipError_t gsdrAmdWsWaits(unsigned long long* out, size_t count,
                                                                             int reset) {
  hipError_t e = hipDeviceSynchronize();
  const size_t n = count < (size_t)256 * 12 * gsdr_amd::kWaitSlots ? count : (size_t)256 * 12 * gsdr_amd::kWaitSlots;
  if (e == hipSuccess) e = hipMemcpyFromSymbol(out, HIP_SYMBOL(gsdr_amd::gWsWaits), n * sizeof(unsigned long long));
  if (e == hipSuccess && reset) {
    void* p = nullptr;
    e = hipGetSymbolAddress(&p, HIP_SYMBOL(gsdr_amd::gWsWaits));
    if (e == hipSuccess) e = hipMemset(p, 0, sizeof(unsigned long long) * 256 * 12 * gsdr_amd::kWaitSlots);
  }
  if (e == hipSuccess) e = gsdr_amd::w4WaitsRead(out, n, reset);  // the 4-way kernel's unit
  return e;
}
#endif

#if GSDR_WS_DIAG
namespace gsdr_amd {
hipError_t w4DiagRead(unsigned long long* out8, int reset);
}
extern "C" __attribute__((visibility("default"))) hipError_t gsdrAmdWsDiag(unsigned long long* out8, int reset) {
  hipError_t e = hipDeviceSynchronize();
  if (e == hipSuccess) e = hipMemcpyFromSymbol(out8, HIP_SYMBOL(gsdr_amd::gWsDiag), 8 * sizeof(unsigned long long));
  if (e == hipSuccess && reset) {
    const unsigned long long z[8] = {};
    e = hipMemcpyToSymbol(HIP_SYMBOL(gsdr_amd::gWsDiag), z, sizeof z);
  }
  if (e == hipSuccess) e = gsdr_amd::w4DiagRead(out8, reset);  // the 4-way kernel's unit
  return e;
}
#endif

extern "C" {
// include/gsdr/gsdr_amd.h: wave-specialised kernel hand-off limit and abort diagnostics.
void gsdrAmdSetWsSpinLimit(int32_t microseconds) {
  gsdr_amd::gWsSpinLimit.store(microseconds < 0 ? 0 : microseconds, std::memory_order_relaxed);
}
int32_t gsdrAmdGetWsSpinLimit(void) { return gsdr_amd::gWsSpinLimit.load(std::memory_order_relaxed); }

// Graph executors (am_chain, the stepping driver): aborts counted on `device` so far, cleared; no
// synchronisation - call it once the replays of interest are known to have completed.
uint32_t gsdrAmdWsTakeAborts(int32_t device) { return gsdr_amd::takeWsAborts(device); }
uint32_t gsdrAmdWsAbortsPending(int32_t device) { return gsdr_amd::peekWsAborts(device); }

hipError_t gsdrAmdWsAborts(int32_t device, uint64_t* count, int reset) {
  int prev = 0;
  hipError_t e = hipGetDevice(&prev);
  if (e != hipSuccess) return e;
  if ((e = hipSetDevice(device)) != hipSuccess) return e;
  e = hipDeviceSynchronize();
  uint64_t v = 0;
  if (e == hipSuccess) {
    if (reset) {
      v = gsdr_amd::takeWsAborts(device);
    } else {
      std::lock_guard<std::mutex> lock(gsdr_amd::gAbortMu);
      const uint32_t* h = device >= 0 && device < gsdr_amd::kMaxDevices ? gsdr_amd::gAbortHost[device] : nullptr;
      v = h ? __atomic_load_n(h, __ATOMIC_SEQ_CST) : 0;
    }
  }
  if (count) *count = v;
  (void)hipSetDevice(prev);
  return e;
}
}
