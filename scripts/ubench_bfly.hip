// Radix-2 butterfly issue rate with no memory at all: every thread keeps 16 elements and 8
// twiddles in registers and runs K windows of 4 DIT (or DIF) stages -- the arithmetic of
// ntt.hip's r16_window -- to find the VALU ceiling of the NTT's instruction stream.
// Build: hipcc --offload-arch=gfx950 -O3 -I zkvm-brainfuck_amd/csrc scripts/ubench_bfly.hip -o /tmp/ubench_bfly
#include <hip/hip_runtime.h>
#include <cstdio>

#include "kb.h"

using namespace kb;

template <bool DIF>
__device__ __forceinline__ void window(uint32_t (&x)[16], const uint32_t (&tw)[8]) {
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const int kk = DIF ? 3 - q : q;
#pragma unroll
    for (int i = 0; i < 16; i++) {
      if (i & (1 << kk)) continue;
      const int j = i | (1 << kk);
      const uint32_t w = tw[i & 7];
      const uint32_t u = x[i], v = x[j];
      if (DIF) {
        x[i] = madd(u, v);
        x[j] = mmul_s((int32_t)(u - v), w);
      } else {
        const uint32_t vw = mmul(v, w);
        const uint32_t s_ = u + vw, d = u - vw;
        x[i] = umin(s_, s_ - P);
        x[j] = umin(d, d + P);
      }
    }
  }
}

template <bool DIF, int TPB>
__global__ __launch_bounds__(TPB) void k_bfly(uint32_t* buf, int iters) {
  const size_t t = (size_t)blockIdx.x * TPB + threadIdx.x;
  uint32_t x[16], tw[8];
#pragma unroll
  for (int i = 0; i < 16; i++) x[i] = (uint32_t)((t * 16 + i) * 2654435761u) % P;
#pragma unroll
  for (int i = 0; i < 8; i++) tw[i] = (uint32_t)((t + i) * 40503u) % P;
  for (int it = 0; it < iters; it++) window<DIF>(x, tw);
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < 16; i++) acc ^= x[i];
  buf[t] = acc;
}

template <bool DIF, int TPB>
static void run(uint32_t* buf, int blocks, int iters) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL((k_bfly<DIF, TPB>), dim3(blocks), dim3(TPB), 0, 0, buf, iters);
  hipDeviceSynchronize();
  hipEventRecord(e0, 0);
  const int reps = 5;
  for (int r = 0; r < reps; r++) hipLaunchKernelGGL((k_bfly<DIF, TPB>), dim3(blocks), dim3(TPB), 0, 0, buf, iters);
  hipEventRecord(e1, 0);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double s = ms * 1e-3 / reps;
  const double es = (double)blocks * TPB * 16.0 * 4 * iters;  // element-stages
  printf("%s TPB=%4d blocks=%6d: %.3f ms  %.2f T element-stages/s\n", DIF ? "DIF" : "DIT", TPB, blocks,
         s * 1e3, es / s / 1e12);
}

int main() {
  uint32_t* buf;
  hipMalloc(&buf, (size_t)1 << 28);
  for (int bpc : {1, 2, 4, 8}) {  // 256-thread blocks per CU
    run<false, 256>(buf, 256 * bpc, 200);
    run<true, 256>(buf, 256 * bpc, 200);
  }
  run<false, 1024>(buf, 512, 200);
  run<true, 1024>(buf, 512, 200);
  return 0;
}
