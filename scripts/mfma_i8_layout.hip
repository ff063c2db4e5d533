// Checks the operand / accumulator lane maps of v_mfma_i32_32x32x32_i8 with exact integer data
// (asymmetric A and B), as used by the openings kernel (fri.hip: k_open_mfma):
//   lane l holds A[row l&31][k = 16 (l>>5) + j] and B[k = 16 (l>>5) + j][col l&31], j = 0..15
//   C/D: col = l&31, row = (r&3) + 8 (r>>2) + 4 (l>>5), r = 0..15
// hipcc --offload-arch=gfx950 -O2 scripts/mfma_i8_layout.hip -o /tmp/mfma_i8 && /tmp/mfma_i8
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

__global__ void k(const int8_t* A, const int8_t* B, int* C) {  // A 32x32 row-major, B 32x32 [k][n]
  const int l = threadIdx.x, r = l & 31, h = l >> 5;
  union { v4i v; int8_t b[16]; } a, b;
  for (int j = 0; j < 16; j++) {
    a.b[j] = A[r * 32 + 16 * h + j];
    b.b[j] = B[(16 * h + j) * 32 + r];
  }
  v16i acc = {};
  acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(a.v, b.v, acc, 0, 0, 0);
  for (int q = 0; q < 16; q++) C[((q & 3) + 8 * (q >> 2) + 4 * h) * 32 + r] = acc[q];
}

int main() {
  int8_t A[1024], B[1024];
  int C[1024], R[1024];
  for (int i = 0; i < 1024; i++) {
    A[i] = (int8_t)((i * 37 + 11) % 251 - 125);
    B[i] = (int8_t)((i * 91 + 5) % 253 - 126);
  }
  for (int m = 0; m < 32; m++)
    for (int n = 0; n < 32; n++) {
      int s = 0;
      for (int kk = 0; kk < 32; kk++) s += A[m * 32 + kk] * B[kk * 32 + n];
      R[m * 32 + n] = s;
    }
  int8_t *dA, *dB;
  int* dC;
  hipMalloc(&dA, 1024); hipMalloc(&dB, 1024); hipMalloc(&dC, 4096);
  hipMemcpy(dA, A, 1024, hipMemcpyHostToDevice);
  hipMemcpy(dB, B, 1024, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dC);
  hipMemcpy(C, dC, 4096, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < 1024; i++) bad += C[i] != R[i];
  printf("mfma_i32_32x32x32_i8 layout check: %d of 1024 wrong (C[0]=%d ref %d, C[33]=%d ref %d)\n",
         bad, C[0], R[0], C[33], R[33]);
  return bad != 0;
}
