// Probe: confirm the lane -> (row, k) operand maps of v_mfma_i32_32x32x32_i8 on gfx950 with exact
// integer data (cdna_hip_programming.md §3: "check the map with exact integer data").
// Hypothesis H1: lane l holds A[l&31][16*(l>>5) + j] and B[16*(l>>5) + j][l&31], j < 16 (byte j);
// H2: two K halves: j < 8 -> k = 8*(l>>5) + j, j >= 8 -> k = 16 + 8*(l>>5) + (j-8).
// C/D: lane l, reg i -> C[(i&3) + 8*(i>>2) + 4*(l>>5)][l&31].
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

__device__ int kOf(int hyp, int lane, int j) {
  const int h = lane >> 5;
  if (hyp == 1) return 16 * h + j;
  return j < 8 ? 8 * h + j : 16 + 8 * h + (j - 8);
}

__global__ void probe(const signed char* A, const signed char* B, int* C, int hyp) {
  const int l = threadIdx.x;
  signed char a[16], b[16];
  for (int j = 0; j < 16; ++j) {
    const int k = kOf(hyp, l, j);
    a[j] = A[(l & 31) * 32 + k];
    b[j] = B[k * 32 + (l & 31)];
  }
  v4i av, bv;
  __builtin_memcpy(&av, a, 16);
  __builtin_memcpy(&bv, b, 16);
  v16i c = {};
  c = __builtin_amdgcn_mfma_i32_32x32x32_i8(av, bv, c, 0, 0, 0);
  for (int i = 0; i < 16; ++i) {
    const int row = (i & 3) + 8 * (i >> 2) + 4 * (l >> 5);
    C[row * 32 + (l & 31)] = c[i];
  }
}

int main() {
  signed char hA[1024], hB[1024];
  int ref[1024], hC[1024];
  srand(7);
  for (int i = 0; i < 1024; ++i) { hA[i] = (signed char)(rand() % 255 - 127); hB[i] = (signed char)(rand() % 255 - 127); }
  for (int i = 0; i < 32; ++i)
    for (int j = 0; j < 32; ++j) {
      int s = 0;
      for (int k = 0; k < 32; ++k) s += hA[i * 32 + k] * hB[k * 32 + j];
      ref[i * 32 + j] = s;
    }
  signed char *dA, *dB; int* dC;
  hipMalloc(&dA, 1024); hipMalloc(&dB, 1024); hipMalloc(&dC, 4096);
  hipMemcpy(dA, hA, 1024, hipMemcpyHostToDevice); hipMemcpy(dB, hB, 1024, hipMemcpyHostToDevice);
  int ok = -1;
  for (int hyp = 1; hyp <= 2; ++hyp) {
    hipMemset(dC, 0, 4096);
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, dA, dB, dC, hyp);
    hipMemcpy(hC, dC, 4096, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 1024; ++i) bad += hC[i] != ref[i];
    printf("hypothesis H%d: %d / 1024 mismatches\n", hyp, bad);
    if (bad == 0 && ok < 0) ok = hyp;
  }
  printf("RESULT %s\n", ok > 0 ? (ok == 1 ? "H1" : "H2") : "NONE");
  return ok > 0 ? 0 : 1;
}
