// Does a SIMD overlap one wave's MFMA chain with another wave's VALU work? (r05 C5 analysis)
// 512-thread blocks, one per CU: waves 0-3 (one per SIMD) run a dependent chain of NM MFMAs
// (32x32x16 f16 or 32x32x32 i8), waves 4-7 run NV independent-FMA VALU instructions. Times the
// kernel for MFMA only, VALU only and both: both ~ max = overlap, ~ sum = the SIMD serialises them.
// Build: hipcc --offload-arch=gfx950 -O3 tools/exp/mfma_valu_overlap.hip -o tools/exp/_build_w4/mvo
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));
typedef int i4v __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

template <int MODE, int NACC = 1>  // bit 0: MFMA waves work, bit 1: VALU waves work, bit 2: i8 MFMA; NACC accumulators round robin
__global__ __launch_bounds__(512, 1) void k(float* out, int nm, int nv, float seed) {
  const int wave = threadIdx.x >> 6;
  float r = 0.0f;
  if (wave < 4) {
    if (MODE & 1) {
      if (MODE & 4) {
        i4v a = i4v{(int)threadIdx.x, 3, 5, 7}, b = i4v{1, 2, (int)seed, 4};
        v16i acc[NACC];
        for (int q = 0; q < NACC; ++q) acc[q] = v16i{};
        for (int i = 0; i < nm; i += NACC)
#pragma unroll
          for (int q = 0; q < NACC; ++q) acc[q] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, acc[q], 0, 0, 0);
        for (int q = 0; q < NACC; ++q)
          for (int i = 0; i < 16; ++i) r += (float)acc[q][i];
      } else {
        h8 a, b;
        for (int e = 0; e < 8; ++e) { a[e] = (_Float16)(seed * e); b[e] = (_Float16)(seed + e); }
        v16f acc[NACC];
        for (int q = 0; q < NACC; ++q) acc[q] = v16f{};
        for (int i = 0; i < nm; i += NACC)
#pragma unroll
          for (int q = 0; q < NACC; ++q) acc[q] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc[q], 0, 0, 0);
        for (int q = 0; q < NACC; ++q)
          for (int i = 0; i < 16; ++i) r += acc[q][i];
      }
    }
  } else if (MODE & 2) {
    float x0 = seed + threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;
    for (int i = 0; i < nv; i += 8) {
      x0 = fmaf(x0, 1.0001f, 0.5f); x1 = fmaf(x1, 1.0001f, 0.5f); x2 = fmaf(x2, 1.0001f, 0.5f); x3 = fmaf(x3, 1.0001f, 0.5f);
      x4 = fmaf(x4, 1.0001f, 0.5f); x5 = fmaf(x5, 1.0001f, 0.5f); x6 = fmaf(x6, 1.0001f, 0.5f); x7 = fmaf(x7, 1.0001f, 0.5f);
    }
    r = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;
  }
  if (r == 12345.678f) out[threadIdx.x] = r;
}

template <int MODE, int NACC = 1>
float timeIt(float* out, int nm, int nv) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  for (int w = 0; w < 20; ++w) hipLaunchKernelGGL((k<MODE, NACC>), dim3(256), dim3(512), 0, 0, out, nm, nv, 1.0f);
  std::vector<float> t;
  for (int r = 0; r < 15; ++r) {
    hipEventRecord(e0);
    hipLaunchKernelGGL((k<MODE, NACC>), dim3(256), dim3(512), 0, 0, out, nm, nv, 1.0f);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1); t.push_back(ms * 1000.0f);
  }
  std::sort(t.begin(), t.end());
  return t[t.size() / 2];
}

float timeIt1(float* out, int nm) {  // one block: no chip-wide power load
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  for (int w = 0; w < 5; ++w) hipLaunchKernelGGL((k<1, 1>), dim3(1), dim3(512), 0, 0, out, nm, 0, 1.0f);
  hipEventRecord(e0);
  hipLaunchKernelGGL((k<1, 1>), dim3(1), dim3(512), 0, 0, out, nm, 0, 1.0f);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  return ms * 1000.0f;
}

int main() {
  float* out; hipMalloc(&out, 4096 * 4);
  const int nm = 20000, nv = 40000;
  // nm MFMAs x 32 cycles; nv VALU x 4 cycles (wave64 on a 16-lane SIMD) -> ~comparable
  printf("f16 MFMA chain (%d) only      %8.1f us\n", nm, timeIt<1>(out, nm, nv));
  printf("VALU (%d fma) only            %8.1f us\n", nv, timeIt<2>(out, nm, nv));
  printf("both                          %8.1f us\n", timeIt<3>(out, nm, nv));
  printf("i8 MFMA chain (%d) only       %8.1f us\n", nm, timeIt<5>(out, nm, nv));
  printf("i8 MFMA + VALU                %8.1f us\n", timeIt<7>(out, nm, nv));
  printf("VALU (%d fma) only, 2x        %8.1f us\n", 2 * nv, timeIt<2>(out, nm, 2 * nv));
  printf("f16 MFMA + VALU 2x            %8.1f us\n", timeIt<3>(out, nm, 2 * nv));
  printf("f16 MFMA 2 accumulators       %8.1f us\n", timeIt<1, 2>(out, nm, nv));
  printf("f16 MFMA 4 accumulators       %8.1f us\n", timeIt<1, 4>(out, nm, nv));
  printf("i8 MFMA 3 accumulators        %8.1f us\n", timeIt<5, 3>(out, nm, nv));
  printf("f16 MFMA, 1 block (clock ref) %8.1f us\n", timeIt1(out, nm));
  return 0;
}
