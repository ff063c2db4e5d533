// VALU throughput microbenchmark for the integer ops the field arithmetic uses (gfx950).
// Each thread runs 8 independent chains of one instruction; reports lane-ops/s per op.
// Build: hipcc --offload-arch=gfx950 -O3 scripts/ubench_valu.hip -o /tmp/ubench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s\n", hipGetErrorString(e)); return 1; } } while (0)

constexpr int ITERS = 2048;

#define OP8(ASM)                                                                        \
  asm volatile(ASM : "+v"(a0) : "v"(k)); asm volatile(ASM : "+v"(a1) : "v"(k));         \
  asm volatile(ASM : "+v"(a2) : "v"(k)); asm volatile(ASM : "+v"(a3) : "v"(k));         \
  asm volatile(ASM : "+v"(a4) : "v"(k)); asm volatile(ASM : "+v"(a5) : "v"(k));         \
  asm volatile(ASM : "+v"(a6) : "v"(k)); asm volatile(ASM : "+v"(a7) : "v"(k));

#define KERNEL(NAME, ASM)                                                               \
  __global__ __launch_bounds__(256) void NAME(uint32_t* out, uint32_t seed) {           \
    uint32_t k = seed ^ threadIdx.x;                                                    \
    uint32_t a0 = k, a1 = k + 1, a2 = k + 2, a3 = k + 3, a4 = k + 4, a5 = k + 5,        \
             a6 = k + 6, a7 = k + 7;                                                    \
    for (int i = 0; i < ITERS; i++) { OP8(ASM) OP8(ASM) OP8(ASM) OP8(ASM) }             \
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;  \
  }

KERNEL(k_add, "v_add_u32 %0, %0, %1")
KERNEL(k_add_e64, "v_add_u32_e64 %0, %0, %1")
KERNEL(k_sub, "v_sub_u32 %0, %0, %1")
KERNEL(k_add_lit, "v_add_u32 %0, 0x80ffffff, %0")
KERNEL(k_add_sgpr, "v_add_u32 %0, s4, %0")
KERNEL(k_min_lit, "v_min_u32 %0, 0x7f000001, %0")
KERNEL(k_mul_hi_sgpr, "v_mul_hi_u32 %0, %0, s4")
KERNEL(k_add_co, "v_add_co_u32 %0, vcc, %0, %1")
KERNEL(k_addc, "v_addc_co_u32 %0, vcc, %0, %1, vcc")
KERNEL(k_min, "v_min_u32 %0, %0, %1")
KERNEL(k_min_i32, "v_min_i32 %0, %0, %1")
KERNEL(k_max, "v_max_u32 %0, %0, %1")
KERNEL(k_med3, "v_med3_u32 %0, %0, %1, %0")
KERNEL(k_min3, "v_min3_u32 %0, %0, %1, %0")
KERNEL(k_and, "v_and_b32 %0, %0, %1")
KERNEL(k_xor, "v_xor_b32 %0, %0, %1")
KERNEL(k_lshl, "v_lshlrev_b32 %0, 3, %0")
KERNEL(k_ashr, "v_ashrrev_i32 %0, 31, %0")
KERNEL(k_bfi, "v_bfi_b32 %0, %0, %1, %0")
KERNEL(k_cndmask, "v_cndmask_b32 %0, %0, %1, vcc")
KERNEL(k_cmp, "v_cmp_gt_u32 vcc, %0, %1")
KERNEL(k_add3, "v_add3_u32 %0, %0, %1, %0")
KERNEL(k_lshl_add, "v_lshl_add_u32 %0, %0, 3, %1")
KERNEL(k_mul_lo, "v_mul_lo_u32 %0, %0, %1")
KERNEL(k_mul_hi, "v_mul_hi_u32 %0, %0, %1")
KERNEL(k_mul_u24, "v_mul_u32_u24 %0, %0, %1")
KERNEL(k_mad_u24, "v_mad_u32_u24 %0, %0, %1, %0")
KERNEL(k_pk_add_u16, "v_pk_add_u16 %0, %0, %1")
KERNEL(k_mul_f32, "v_mul_f32 %0, %0, %1")
KERNEL(k_fma_f32, "v_fma_f32 %0, %0, %1, %0")
KERNEL(k_cvt_f32, "v_cvt_f32_u32 %0, %0")

// 64-bit ops need register pairs
#define KERNEL64(NAME, ASM)                                                             \
  __global__ __launch_bounds__(256) void NAME(uint32_t* out, uint32_t seed) {           \
    uint32_t k = seed ^ threadIdx.x;                                                    \
    uint64_t a0 = k, a1 = k + 1, a2 = k + 2, a3 = k + 3, a4 = k + 4, a5 = k + 5,        \
             a6 = k + 6, a7 = k + 7;                                                    \
    for (int i = 0; i < ITERS; i++) { OP8(ASM) OP8(ASM) OP8(ASM) OP8(ASM) }             \
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7); \
  }
KERNEL64(k_mad_u64, "v_mad_u64_u32 %0, vcc, %1, %1, %0")
KERNEL64(k_lshl_add_u64, "v_lshl_add_u64 %0, %0, 1, %0")

typedef void (*kfn)(uint32_t*, uint32_t);

int main() {
  const int blocks = 256 * 8 * 4;  // 8 waves/SIMD worth of 256-thread blocks
  uint32_t* out;
  CHK(hipMalloc(&out, (size_t)blocks * 256 * 4));
  struct { const char* name; kfn f; } ks[] = {
      {"v_add_u32", k_add},
      {"v_add_u32_e64", k_add_e64},
      {"v_sub_u32", k_sub},
      {"v_add_u32 literal", k_add_lit},
      {"v_add_u32 sgpr", k_add_sgpr},
      {"v_min_u32 literal", k_min_lit},
      {"v_mul_hi sgpr", k_mul_hi_sgpr},
      {"v_add_co_u32", k_add_co},
      {"v_addc_co_u32", k_addc},
      {"v_min_u32", k_min},
      {"v_min_i32", k_min_i32},
      {"v_max_u32", k_max},
      {"v_med3_u32", k_med3},
      {"v_min3_u32", k_min3},
      {"v_and_b32", k_and},
      {"v_xor_b32", k_xor},
      {"v_lshlrev_b32", k_lshl},
      {"v_ashrrev_i32", k_ashr},
      {"v_bfi_b32", k_bfi},
      {"v_cndmask_b32", k_cndmask},
      {"v_cmp_gt_u32", k_cmp},
      {"v_add3_u32", k_add3},
      {"v_lshl_add_u32", k_lshl_add},
      {"v_mul_lo_u32", k_mul_lo},
      {"v_mul_hi_u32", k_mul_hi},
      {"v_mul_u32_u24", k_mul_u24},
      {"v_mad_u32_u24", k_mad_u24},
      {"v_pk_add_u16", k_pk_add_u16},
      {"v_mul_f32", k_mul_f32},
      {"v_fma_f32", k_fma_f32},
      {"v_cvt_f32_u32", k_cvt_f32},
      {"v_mad_u64_u32", k_mad_u64},
      {"v_lshl_add_u64", k_lshl_add_u64}};
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  for (auto& k : ks) {
    hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out, 1);
    CHK(hipDeviceSynchronize());
    CHK(hipEventRecord(e0));
    for (int r = 0; r < 5; r++) hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out, r);
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    float ms;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    const double ops = 5.0 * blocks * 256.0 * ITERS * 32;
    printf("%-16s %8.2f T lane-ops/s  (%.3f ms)\n", k.name, ops / (ms * 1e-3) / 1e12, ms);
  }
  return 0;
}
