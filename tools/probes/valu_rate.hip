// Probe: issue cost per wave-instruction of the VALU forms a register-resident FFT uses
// (v_pk_fma_f32, v_fma_f32, v_pk_add_f32, v_permlane32/16_swap, DPP row_ror moves, DPP + cndmask)
// at 1 and 2 waves per SIMD. Each wave runs 16 independent chains; cycles from s_memtime.
//   hipcc --offload-arch=gfx950 -O3 -std=c++20 tools/probes/valu_rate.hip -o tools/probes/valu_rate
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int kIters = 4096;

template <int OP>
__global__ void probe(float* out, unsigned long long* cyc, float seed) {
  const int l = threadIdx.x & 63;
  f2 a[16], b = {seed, 1.0f - seed}, c = {0.5f * seed, 0.25f};
  unsigned u[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    a[i] = f2{seed + i + l, seed - i};
    u[i] = __float_as_uint(seed + i * l);
  }
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < kIters; ++it) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      if (OP == 0) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
      if (OP == 1) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[i].x) : "v"(b.x), "v"(c.x));
      if (OP == 2) asm volatile("v_pk_add_f32 %0, %0, %1 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]" : "+v"(a[i]) : "v"(b));
      if (OP == 3 && (i & 1) == 0) {
        auto r = __builtin_amdgcn_permlane32_swap(u[i], u[i + 1], false, false);
        u[i] = r[0];
        u[i + 1] = r[1];
      }
      if (OP == 4 && (i & 1) == 0) {
        auto r = __builtin_amdgcn_permlane16_swap(u[i], u[i + 1], false, false);
        u[i] = r[0];
        u[i + 1] = r[1];
      }
      if (OP == 5) u[i] = __builtin_amdgcn_update_dpp(u[i], u[(i + 1) & 15], 0x128, 0xf, 0xc, false);  // row_ror:8, banks 2-3
      if (OP == 6) {  // 2x2 transpose of lane bit 3 with a register pair: select(dpp) both ways
        if ((i & 1) == 0) {
          const unsigned x = u[i], y = u[i + 1];
          const unsigned xs = __builtin_amdgcn_mov_dpp(x, 0x128, 0xf, 0xf, false);
          const unsigned ys = __builtin_amdgcn_mov_dpp(y, 0x128, 0xf, 0xf, false);
          u[i] = (l & 8) ? ys : x;
          u[i + 1] = (l & 8) ? y : xs;
        }
      }
      if (OP == 7) asm volatile("v_pk_mul_f32 %0, %0, %1 op_sel_hi:[1,0]" : "+v"(a[i]) : "v"(b));
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0.0f;
#pragma unroll
  for (int i = 0; i < 16; ++i) s += a[i].x + a[i].y + __uint_as_float(u[i]);
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (l == 0) cyc[blockIdx.x * 16 + (threadIdx.x >> 6)] = t1 - t0;
}

template <int OP>
void run(const char* name, int insnsPerIter, float* out, unsigned long long* cyc) {
  for (int waves : {4, 8}) {
    hipLaunchKernelGGL(probe<OP>, dim3(256), dim3(64 * waves), 0, 0, out, cyc, 0.5f);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(probe<OP>, dim3(256), dim3(64 * waves), 0, 0, out, cyc, 0.5f);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    unsigned long long h[256 * 16];
    hipMemcpy(h, cyc, sizeof h, hipMemcpyDeviceToHost);
    double sum = 0;
    for (int bk = 0; bk < 256; ++bk)
      for (int w = 0; w < waves; ++w) sum += (double)h[bk * 16 + w];
    const double perWave = sum / (256.0 * waves);
    const double insns = (double)kIters * insnsPerIter;
    printf("%-34s waves/SIMD %d: %6.2f cycles per wave-instruction (per SIMD %5.2f), clock %.2f GHz\n", name,
           waves / 4, perWave / insns, perWave / insns / (waves / 4), perWave / (ms * 1e-3) / 1e9);
  }
}

int main() {
  float* out;
  unsigned long long* cyc;
  hipMalloc(&out, 256 * 512 * sizeof(float));
  hipMalloc(&cyc, 256 * 16 * sizeof(unsigned long long));
  run<0>("v_pk_fma_f32", 16, out, cyc);
  run<1>("v_fma_f32", 16, out, cyc);
  run<2>("v_pk_add_f32 (op_sel/neg)", 16, out, cyc);
  run<7>("v_pk_mul_f32", 16, out, cyc);
  run<3>("v_permlane32_swap (builtin)", 8, out, cyc);
  run<4>("v_permlane16_swap (builtin)", 8, out, cyc);
  run<5>("update_dpp row_ror:8 bank-masked", 16, out, cyc);
  run<6>("bit-3 transpose (per dword pair)", 8, out, cyc);
  return 0;
}
