// NTT tile-pass rate with the data L2/MALL-resident vs streamed from HBM, to separate the
// kernel's compute ceiling from its memory overlap.  Links against libbfz.so (bfz::ntt_passes).
// Build: hipcc --offload-arch=gfx950 -O2 -I zkvm-brainfuck_amd/csrc scripts/ubench_ntt.cpp \
//          -L zkvm-brainfuck_amd -lbfz -Wl,-rpath,'$ORIGIN/../zkvm-brainfuck_amd' -o scripts/ubench_ntt
//   ubench_ntt            the 2^14 tile passes at several widths (time + output hash)
//   ubench_ntt lde L W R  R coset LDEs of a 2^L x W matrix (bfz::coset_lde: DIT tile, k_lde_mid<L>,
//                         DIF tile), for per-kernel PMC counts at a known element-stage count
//                         (scripts/gpu_ntt_counters.sh)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "ntt.h"

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s\n", hipGetErrorString(e)); return 1; } } while (0)

static int lde_mode(int L, int w, int reps) {
  const size_t n = (size_t)1 << L, words = n * (size_t)w;
  hipStream_t st = bfz::stream();
  uint32_t *a, *b;
  CHK(hipMalloc(&a, words * 4));
  CHK(hipMalloc(&b, 2 * words * 4));
  std::vector<uint32_t> h(words);
  for (size_t i = 0; i < words; i++) h[i] = (uint32_t)((i * 2654435761u) % 0x7f000001u);
  CHK(hipMemcpy(a, h.data(), words * 4, hipMemcpyHostToDevice));
  const uint32_t shift = (uint32_t)(((uint64_t)3 << 32) % 0x7f000001u);  // 3, Montgomery
  bfz::coset_lde(a, n, w, shift, b, st);
  CHK(hipStreamSynchronize(st));
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  CHK(hipEventRecord(e0, st));
  for (int r = 0; r < reps; r++) bfz::coset_lde(a, n, w, shift, b, st);
  CHK(hipEventRecord(e1, st));
  CHK(hipEventSynchronize(e1));
  float ms;
  CHK(hipEventElapsedTime(&ms, e0, e1));
  const double s = ms * 1e-3 / reps;
  std::vector<uint32_t> o(2 * words);
  CHK(hipMemcpy(o.data(), b, 2 * words * 4, hipMemcpyDeviceToHost));
  uint64_t hsh = 1469598103934665603ull;
  for (uint32_t v : o) hsh = (hsh ^ v) * 1099511628211ull;
  printf("coset LDE 2^%d x %d: %8.1f us  %7.0f GB/s (12 B/input elem)  %6.2f T elem-stages/s  out %016llx\n",
         L, w, s * 1e6, 12.0 * words / s / 1e9, 3.0 * L * words / s / 1e12, (unsigned long long)hsh);
  return 0;
}

int main(int argc, char** argv) {
  if (argc > 1 && std::string(argv[1]) == "lde")
    return lde_mode(argc > 2 ? atoi(argv[2]) : 22, argc > 3 ? atoi(argv[3]) : 8,
                    argc > 4 ? atoi(argv[4]) : 5);
  const int L = 14;  // the 2^14 tile pass alone
  const size_t n = (size_t)1 << L;
  hipStream_t st = bfz::stream();
  for (int w : {16, 64, 256, 4096}) {
    const size_t words = n * (size_t)w;
    uint32_t *a, *b;
    CHK(hipMalloc(&a, words * 4));
    CHK(hipMalloc(&b, words * 4));
    std::vector<uint32_t> h(words);
    for (size_t i = 0; i < words; i++) h[i] = (uint32_t)((i * 2654435761u) % 0x7f000001u);
    CHK(hipMemcpy(a, h.data(), words * 4, hipMemcpyHostToDevice));
    for (int dif = 0; dif < 2; dif++) {
      bfz::ntt_passes(a, b, n, n, w, L, dif, st);
      CHK(hipStreamSynchronize(st));
      hipEvent_t e0, e1;
      CHK(hipEventCreate(&e0));
      CHK(hipEventCreate(&e1));
      const int reps = w >= 4096 ? 20 : 400;
      CHK(hipEventRecord(e0, st));
      for (int r = 0; r < reps; r++) bfz::ntt_passes(a, b, n, n, w, L, dif, st);
      CHK(hipEventRecord(e1, st));
      CHK(hipEventSynchronize(e1));
      float ms;
      CHK(hipEventElapsedTime(&ms, e0, e1));
      const double s = ms * 1e-3 / reps;
      std::vector<uint32_t> o(words);
      CHK(hipMemcpy(o.data(), b, words * 4, hipMemcpyDeviceToHost));
      uint64_t hsh = 1469598103934665603ull;
      for (uint32_t v : o) hsh = (hsh ^ v) * 1099511628211ull;
      printf("L=%d w=%5d (%7.1f MB) %s: %8.2f us/pass  %7.1f G elem/s  %7.0f GB/s (8 B/elem)  out %016llx\n", L, w,
             words * 4 / 1e6, dif ? "DIF" : "DIT", s * 1e6, words / s / 1e9, 8.0 * words / s / 1e9,
             (unsigned long long)hsh);
    }
    CHK(hipFree(a));
    CHK(hipFree(b));
  }
  return 0;
}
