// Issue cost of the integer instructions the field arithmetic compiles to (gfx950): each kernel
// runs 8 independent chains of one instruction per thread, 2048 threads per CU (8 waves per SIMD)
// on every CU; cycles per wave-instruction per SIMD = wall x clock x SIMDs / wave-instructions.
//   hipcc --offload-arch=gfx950 -O3 -o scripts/ubench_intops scripts/ubench_intops.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::printf("HIP %s\n", hipGetErrorString(e)); return 1; } } while (0)

constexpr int ITERS = 4096, CH = 8;

#define KERNEL(NAME, ASM)                                                                         \
  __global__ __launch_bounds__(256) void NAME(uint32_t* out, uint32_t seed) {                    \
    uint32_t a[CH], b = seed ^ threadIdx.x;                                                       \
    for (int c = 0; c < CH; c++) a[c] = seed + c * 7919u + threadIdx.x;                           \
    for (int it = 0; it < ITERS; it++) {                                                          \
      _Pragma("unroll") for (int c = 0; c < CH; c++) { ASM; }                                     \
    }                                                                                             \
    uint32_t s = 0;                                                                               \
    for (int c = 0; c < CH; c++) s ^= a[c];                                                       \
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;                                               \
  }

KERNEL(k_add, asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[c]) : "v"(b)))
KERNEL(k_min, asm volatile("v_min_u32 %0, %0, %1" : "+v"(a[c]) : "v"(b)))
KERNEL(k_mul_lo, asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[c]) : "v"(b)))
KERNEL(k_mul_hi, asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a[c]) : "v"(b)))
KERNEL(k_mul_u24, asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a[c]) : "v"(b)))
KERNEL(k_mad_u64, {
  uint64_t t;
  asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, 0" : "=v"(t) : "v"(a[c]), "v"(b) : "vcc");
  a[c] = (uint32_t)(t >> 32);
})
KERNEL(k_lshl_add, asm volatile("v_lshl_add_u32 %0, %0, 24, %1" : "+v"(a[c]) : "v"(b)))

int main() {
  int dev = 0, cus = 0, clk_khz = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  CHECK(hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, dev));
  const int blocks = cus * 8;  // 8 x 256 threads = 2048 per CU
  uint32_t* out;
  CHECK(hipMalloc(&out, (size_t)blocks * 256 * 4));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  struct K { const char* name; void (*f)(uint32_t*, uint32_t); };
  const K ks[] = {{"v_add_u32", k_add}, {"v_min_u32", k_min}, {"v_lshl_add_u32", k_lshl_add},
                  {"v_mul_u32_u24", k_mul_u24}, {"v_mul_lo_u32", k_mul_lo}, {"v_mul_hi_u32", k_mul_hi},
                  {"v_mad_u64_u32", k_mad_u64}};
  for (const K& k : ks) {
    hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out, 1u);  // warm
    CHECK(hipEventRecord(e0));
    for (int r = 0; r < 5; r++) hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out, 1u + r);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    const double wave_instr = 5.0 * blocks * 4 * (double)ITERS * CH;  // 4 waves per block
    const double simd_cycles = ms * 1e-3 * clk_khz * 1e3 * cus * 4;
    std::printf("%-16s %8.3f ms  %.2f cycles per wave-instruction per SIMD (at the %d MHz nominal clock)\n",
                k.name, ms, simd_cycles / wave_instr, clk_khz / 1000);
  }
  return 0;
}
