// Poseidon2-16 compute throughput on gfx950: permutations chained in registers (no memory),
// to compare the Merkle kernels' achieved rate against the pure VALU ceiling.
// Build: hipcc --offload-arch=gfx950 -O3 -I zkvm-brainfuck_amd/csrc scripts/ubench_p2.hip
#include <cstdio>

#include "poseidon2.h"

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s\n", hipGetErrorString(e)); return 1; } } while (0)

template <int BS>
__global__ __launch_bounds__(BS) void k_chain(uint32_t* out, int iters) {
  uint32_t s[16];
  const uint32_t t = blockIdx.x * BS + threadIdx.x;
#pragma unroll
  for (int i = 0; i < 16; i++) s[i] = (t * 16 + i) % kb::P;
  for (int it = 0; it < iters; it++) kb::poseidon2_permute(s);
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < 16; i++) acc ^= s[i];
  out[t] = acc;
}

int main() {
  const int iters = 64;
  uint32_t* out;
  const int threads = 1 << 20;
  CHK(hipMalloc(&out, threads * 4));
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  for (int bs : {256, 512}) {
    for (int rep = 0; rep < 2; rep++) {
      CHK(hipEventRecord(e0));
      if (bs == 256)
        hipLaunchKernelGGL(k_chain<256>, dim3(threads / 256), dim3(256), 0, 0, out, iters);
      else
        hipLaunchKernelGGL(k_chain<512>, dim3(threads / 512), dim3(512), 0, 0, out, iters);
      CHK(hipEventRecord(e1));
      CHK(hipEventSynchronize(e1));
      float ms;
      CHK(hipEventElapsedTime(&ms, e0, e1));
      printf("block %d: %.3f ms, %.2f G perms/s\n", bs, ms, (double)threads * iters / (ms * 1e-3) / 1e9);
    }
  }
  return 0;
}
