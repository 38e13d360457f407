// Lane-permutation probe: prints, for each cross-lane primitive the register-exchange FFT
// transposes use, which (register, lane) each output lane received.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void probe(unsigned* out) {
  const unsigned l = threadIdx.x;
  const unsigned a = 1000 + l, b = 2000 + l;
  auto p16 = __builtin_amdgcn_permlane16_swap(a, b, false, false);
  auto p32 = __builtin_amdgcn_permlane32_swap(a, b, false, false);
  out[0 * 64 + l] = p16[0];
  out[1 * 64 + l] = p16[1];
  out[2 * 64 + l] = p32[0];
  out[3 * 64 + l] = p32[1];
  out[4 * 64 + l] = __builtin_amdgcn_update_dpp(a, b, 0x128, 0xF, 0xC, false);  // row_ror:8, banks 2,3
  out[5 * 64 + l] = __builtin_amdgcn_update_dpp(a, b, 0x114, 0xF, 0xA, false);  // row_shr:4, banks 1,3
  out[6 * 64 + l] = __builtin_amdgcn_update_dpp(a, b, 0x104, 0xF, 0x5, false);  // row_shl:4, banks 0,2
  out[7 * 64 + l] = __builtin_amdgcn_update_dpp(a, b, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
}

int mainXA();
int main() {
  mainXA();
  unsigned* d;
  unsigned h[8 * 64];
  if (hipMalloc(&d, sizeof h) != hipSuccess) return 1;
  probe<<<1, 64>>>(d);
  if (hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) return 1;
  const char* names[8] = {"p16[0]", "p16[1]", "p32[0]", "p32[1]", "ror8 b3:2", "shr4 b3,1", "shl4 b2,0", "qp1032"};
  for (int k = 0; k < 8; ++k) {
    printf("%-10s", names[k]);
    for (int l = 0; l < 64; ++l) printf(" %c%02u", h[k * 64 + l] >= 2000 ? 'b' : 'a', h[k * 64 + l] % 1000);
    printf("\n");
  }
  return 0;
}

// exchangeA (LDS, the shipped layout) against the register version, on one column
typedef float f2v __attribute__((ext_vector_type(2)));
template <int BANKS>
__device__ __forceinline__ float dppRor8(float old, float src) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, old), __builtin_bit_cast(int, src), 0x128, 0xF, BANKS, false));
}
// the swaps as inline asm; s_nop 1 covers the VALU-write -> v_permlane read hazard (2 wait states)
__device__ __forceinline__ void swap16(float& a, float& b) {
  asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(a), "+v"(b));
}
__device__ __forceinline__ void swap32(float& a, float& b) {
  asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(a), "+v"(b));
}
__device__ __forceinline__ void swap16v(f2v& a, f2v& b) {
  float ax = a.x, ay = a.y, bx = b.x, by = b.y;
  swap16(ax, bx);
  swap16(ay, by);
  a = f2v{ax, ay};
  b = f2v{bx, by};
}
__device__ __forceinline__ void swap32v(f2v& a, f2v& b) {
  float ax = a.x, ay = a.y, bx = b.x, by = b.y;
  swap32(ax, bx);
  swap32(ay, by);
  a = f2v{ax, ay};
  b = f2v{bx, by};
}
__global__ void probeXA(float* out) {
  __shared__ f2v s[64 * 10];
  const int l = threadIdx.x, a = l & 7, hi = l >> 3;
  f2v z[8], y[8];
  for (int r = 0; r < 8; ++r) z[r] = y[r] = f2v{(float)(l * 8 + r), -(float)(l * 8 + r)};
  for (int r = 0; r < 8; ++r) s[(a + 8 * r) * 10 + hi] = z[r];
  __syncthreads();
  for (int c = 0; c < 8; ++c) z[c] = s[l * 10 + c];
  for (int r = 0; r < 8; r += 2) {
    const f2v p = y[r], q = y[r + 1];
    y[r] = f2v{dppRor8<0xC>(p.x, q.x), dppRor8<0xC>(p.y, q.y)};
    y[r + 1] = f2v{dppRor8<0x3>(q.x, p.x), dppRor8<0x3>(q.y, p.y)};
  }
  for (int r : {0, 1, 4, 5}) {
    swap16v(y[r], y[r + 2]);
  }
  for (int r = 0; r < 4; ++r) {
    swap32v(y[r], y[r + 4]);
  }
  for (int r = 0; r < 8; ++r) {
    out[(l * 8 + r) * 4 + 0] = z[r].x;
    out[(l * 8 + r) * 4 + 1] = y[r].x;
    out[(l * 8 + r) * 4 + 2] = z[r].y;
    out[(l * 8 + r) * 4 + 3] = y[r].y;
  }
}

int mainXA() {
  float* d;
  float h[64 * 8 * 4];
  if (hipMalloc(&d, sizeof h) != hipSuccess) return 1;
  probeXA<<<1, 64>>>(d);
  if (hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) return 1;
  int bad = 0;
  for (int i = 0; i < 64 * 8; ++i)
    if (h[4 * i] != h[4 * i + 1] || h[4 * i + 2] != h[4 * i + 3]) {
      if (bad < 16) printf("lane %d reg %d: lds %g/%g reg %g/%g\n", i / 8, i % 8, h[4 * i], h[4 * i + 2], h[4 * i + 1], h[4 * i + 3]);
      ++bad;
    }
  printf("exchangeA lds vs registers: %d mismatches\n", bad);
  return 0;
}
