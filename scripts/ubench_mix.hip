// Does the VALU cost of a mixed instruction stream add up from the per-op rates
// (full rate = 1, half rate = 2)?  Interleaved full/half-rate mixes plus the NTT's radix-2
// butterflies (kb.h arithmetic) run in registers only, no memory, 8 waves/SIMD.
// Build: hipcc --offload-arch=gfx950 -O3 -I zkvm-brainfuck_amd/csrc scripts/ubench_mix.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#include "kb.h"

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s\n", hipGetErrorString(e)); return 1; } } while (0)

constexpr int ITERS = 1024;
#define A8(ASM) asm volatile(ASM : "+v"(a0) : "v"(k)); asm volatile(ASM : "+v"(a1) : "v"(k)); \
  asm volatile(ASM : "+v"(a2) : "v"(k)); asm volatile(ASM : "+v"(a3) : "v"(k));               \
  asm volatile(ASM : "+v"(a4) : "v"(k)); asm volatile(ASM : "+v"(a5) : "v"(k));               \
  asm volatile(ASM : "+v"(a6) : "v"(k)); asm volatile(ASM : "+v"(a7) : "v"(k));
#define MIXK(NAME, BODY)                                                                   \
  __global__ __launch_bounds__(256) void NAME(uint32_t* out, uint32_t seed) {              \
    uint32_t k = seed ^ threadIdx.x;                                                       \
    uint32_t a0 = k, a1 = k + 1, a2 = k + 2, a3 = k + 3, a4 = k + 4, a5 = k + 5, a6 = k + 6, \
             a7 = k + 7;                                                                   \
    for (int i = 0; i < ITERS; i++) { BODY BODY BODY BODY }                                \
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;     \
  }
#define ADD A8("v_add_u32 %0, %0, %1")
#define MIN A8("v_min_u32 %0, %0, %1")
#define MUL A8("v_mul_lo_u32 %0, %0, %1")
MIXK(k_full, ADD ADD)                 // 16 ops, expect 16 units
MIXK(k_half, MIN MIN)                 // 16 ops, expect 32 units
MIXK(k_f_h, ADD MIN)                  // expect 24 units if additive, 32 if every op costs 2
MIXK(k_ff_h, ADD ADD MIN)             // 24 ops: 32 units additive
MIXK(k_f_mul, ADD MUL)                // 24 units additive

// radix-2 DIT butterflies on 16 registers (4 stages per iteration), canonical outputs
__global__ __launch_bounds__(256) void k_bfly(uint32_t* out, uint32_t seed, uint32_t w0) {
  uint32_t x[16];
  for (int i = 0; i < 16; i++) x[i] = (seed * 2654435761u + threadIdx.x * 16 + i) % kb::P;
  const uint32_t w = w0 ^ (threadIdx.x & 1);
  for (int it = 0; it < ITERS / 4; it++) {
#pragma unroll
    for (int kk = 0; kk < 4; kk++)
#pragma unroll
      for (int i = 0; i < 16; i++) {
        if (i & (1 << kk)) continue;
        const int j = i | (1 << kk);
        const uint32_t vw = kb::mmul(x[j], w), u = x[i];
        const uint32_t s = u + vw, d = u - vw;
        x[i] = kb::umin(s, s - kb::P);
        x[j] = kb::umin(d, d + kb::P);
      }
  }
  uint32_t acc = 0;
  for (int i = 0; i < 16; i++) acc ^= x[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <typename F>
static double run(F launch, int blocks) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  launch();
  hipDeviceSynchronize();
  hipEventRecord(e0);
  launch();
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  return ms;
}

int main() {
  const int blocks = 256 * 8 * 4;  // 8 waves per SIMD, 4 rounds
  uint32_t* out;
  CHK(hipMalloc(&out, (size_t)blocks * 256 * 4));
  const double lanes = (double)blocks * 256;
  struct { const char* name; void (*k)(uint32_t*, uint32_t); int ops; int units; } ks[] = {
      {"add,add (16 F)", k_full, 16, 16}, {"min,min (16 H)", k_half, 16, 32},
      {"add,min (8F+8H)", k_f_h, 16, 24}, {"add,add,min (16F+8H)", k_ff_h, 24, 32},
      {"add,mul_lo (8F+8H)", k_f_mul, 16, 24}};
  for (auto& k : ks) {
    const double ms = run([&] { hipLaunchKernelGGL(k.k, dim3(blocks), dim3(256), 0, 0, out, 7u); }, blocks);
    const double n = lanes * ITERS * 4;  // BODY repetitions per lane
    printf("%-22s %7.3f ms  %6.2f T instr-lanes/s  %6.2f T units/s (additive model)\n", k.name, ms,
           n * k.ops / (ms * 1e-3) / 1e12, n * k.units / (ms * 1e-3) / 1e12);
  }
  const double ms = run([&] { hipLaunchKernelGGL(k_bfly, dim3(blocks), dim3(256), 0, 0, out, 7u, 12345u); }, blocks);
  const double bfl = lanes * (ITERS / 4) * 4 * 8;
  printf("DIT butterfly          %7.3f ms  %6.2f G butterflies/s = %6.2f T element-stages/s\n", ms,
         bfl / (ms * 1e-3) / 1e9, 2 * bfl / (ms * 1e-3) / 1e12);
  return 0;
}
