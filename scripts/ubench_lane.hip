// Latency of one lane-mode Poseidon2 permutation on gfx950 (the tree tops and the FRI tail are
// chains of them): one 64-thread block (4 states of 16 lanes) runs ITERS dependent
// permutations, v <- P(v), timed with HIP events; then the two lane forms and the thread form
// are compared on 2^16 random states.
// Build: hipcc --offload-arch=gfx950 -O3 -I zkvm-brainfuck_amd/csrc scripts/ubench_lane.hip -o /tmp/ubench_lane
#include <cstdio>
#include <cstdlib>

#include "poseidon2.h"

// The 64-bit lazy lane form measured here (not shipped: 11% lower latency per permutation,
// ~0.06 ms per proof across the tree tops -- profiles/r03/ubench_lane.txt).
namespace kb {
// ---- lane mode in the signed 64-bit lazy form ----------------------------------------------
// The same permutation, one element per lane, with the thread-mode arithmetic of
// poseidon2_permute: every cross-lane sum is a 64-bit add of unreduced values (two DPP moves
// per 64-bit operand, issued back to back), so a modular correction (add, sub, min) no longer
// sits behind each DPP step, and the round constants ride on the S-box's multiply-add
// (P2PRE).  The dependent chain per external round drops from ~36 to ~17 instructions, per
// internal round from ~32 to ~22: the top layers of a Merkle tree are chains of these
// permutations, one per layer.
struct LaneConsts64 {
  int32_t init0, ki[4], kt[3], d, rt0;
};
__device__ __forceinline__ LaneConsts64 lane_consts64(int lane) {
  LaneConsts64 k;
  k.init0 = P2PRE.init0[lane];
#pragma unroll
  for (int r = 0; r < 4; r++) k.ki[r] = P2PRE.init[r][lane];
#pragma unroll
  for (int r = 0; r < 3; r++) k.kt[r] = P2PRE.term[r][lane];
  k.d = P2S.d[lane];
  k.rt0 = P2S.rc_term[0][lane];
  return k;
}
template <int CTRL>
__device__ __forceinline__ int64_t dpp64(int64_t v) {
  const uint64_t u = (uint64_t)v;
  const uint32_t lo = dpp<CTRL>((uint32_t)u), hi = dpp<CTRL>((uint32_t)(u >> 32));
  return (int64_t)(((uint64_t)hi << 32) | lo);
}
// MDS-light on 64-bit values, one element per lane (rows sum to 35: |out| < 35 max|in|)
__device__ __forceinline__ int64_t mds_light_lane64(int64_t x) {
  const int64_t a1 = dpp64<DPP_QROT1>(x), a2 = dpp64<DPP_QROT2>(x), a3 = dpp64<DPP_QROT3>(x);
  const int64_t s4 = (x + a1) + (a2 + a3);
  const int64_t y = s4 + lshl_add64<1>(a1, x);  // 2x_j + 3x_{j+1} + x_{j+2} + x_{j+3}
  const int64_t t = y + dpp64<DPP_ROR8>(y);
  return y + (t + dpp64<DPP_ROR4>(t));
}
__device__ __forceinline__ int64_t sum_lanes16_64(int64_t v) {
  v += dpp64<DPP_ROR1>(v);
  v += dpp64<DPP_ROR2>(v);
  v += dpp64<DPP_ROR4>(v);
  return v + dpp64<DPP_ROR8>(v);
}
// External rounds from the S-box inputs x (R-form, constant included); leaves the last MDS
// output (64-bit R^2-form) -- external_rounds_pre, one element per lane.
template <bool TERM>
__device__ __forceinline__ int64_t external_rounds_lane64(int32_t x, const LaneConsts64& k) {
  int64_t y = 0;
#pragma unroll
  for (int r = 0; r < 4; r++) {
    if (r) x = mred_s(y);
    const int32_t K = TERM ? (r < 3 ? k.kt[r] : 0) : k.ki[r];
    y = mds_light_lane64(fold_s((int64_t)mred_s((int64_t)x * x) * x + K));
  }
  return y;
}
__device__ __forceinline__ uint32_t poseidon2_permute_lane64(uint32_t s, int lane,
                                                             const LaneConsts64& k) {
  int64_t y = mds_light_lane64((int64_t)((uint64_t)s * C32) + k.init0);
  y = external_rounds_lane64<false>(mred_s(y), k);
  int32_t t = mred_s(y);  // rc_int[0] already in element 0
#pragma unroll
  for (int r = 0; r < 13; r++) {
    const int32_t c = mred_s(cube_s(t));
    const int32_t v = lane == 0 ? c : t;
    const int32_t sp = mred_s(sum_lanes16_64(v));  // plain sum of the 16 elements
    const int64_t q = (int64_t)P2S.k * sp;           // sum x R^2
    // the next round's constant: internal (element 0) or the first terminal round's (all)
    const int32_t rc = r < 12 ? (lane == 0 ? P2S.rc_int[r + 1] : 0) : k.rt0;
    t = mred_s((int64_t)k.d * v + (q + rc));
  }
  y = external_rounds_lane64<true>(t, k);
  const uint32_t r = (uint32_t)mred_s(y);
  return umin(r, r + P);
}

}  // namespace kb

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s\n", hipGetErrorString(e)); return 1; } } while (0)

template <int V>
__global__ __launch_bounds__(64) void k_chain(uint32_t* io, int iters) {
  const int lane = threadIdx.x & 15;
  uint32_t v = io[threadIdx.x];
  if (V == 0) {
    const kb::LaneConsts kc = kb::lane_consts(lane);
    for (int it = 0; it < iters; it++) v = kb::poseidon2_permute_lane(v, lane, kc);
  } else {
    const kb::LaneConsts64 kc = kb::lane_consts64(lane);
    for (int it = 0; it < iters; it++) v = kb::poseidon2_permute_lane64(v, lane, kc);
  }
  io[threadIdx.x] = v;
}

__global__ __launch_bounds__(256) void k_check(const uint32_t* in, uint32_t* bad, int n) {
  const int st = (blockIdx.x * blockDim.x + threadIdx.x) >> 4, lane = threadIdx.x & 15;
  if (st >= n) return;
  const uint32_t x = in[16 * st + lane];
  const uint32_t a = kb::poseidon2_permute_lane(x, lane);
  const uint32_t b = kb::poseidon2_permute_lane64(x, lane, kb::lane_consts64(lane));
  uint32_t s[16] = {};
  if (lane == 0) {
    for (int i = 0; i < 16; i++) s[i] = in[16 * st + i];
    kb::poseidon2_permute(s);
  }
  uint32_t t = 0;
  for (int i = 0; i < 16; i++) {
    const uint32_t si = __shfl(s[i], threadIdx.x & ~15, 64);
    if (i == lane) t = si;
  }
  if (a != b || a != t) atomicAdd(bad, 1u);
}

int main() {
  const int n = 1 << 16;
  uint32_t *in, *bad, *io;
  CHK(hipMalloc(&in, (size_t)16 * n * 4));
  CHK(hipMalloc(&bad, 4));
  CHK(hipMalloc(&io, 64 * 4));
  uint32_t* h = (uint32_t*)malloc((size_t)16 * n * 4);
  uint64_t z = 0x5EED;
  for (int i = 0; i < 16 * n; i++) {
    z = z * 6364136223846793005ull + 1442695040888963407ull;
    uint32_t w = (uint32_t)(z >> 33) % kb::P;
    if (i < 64) w = i % 3 == 0 ? 0 : (i % 3 == 1 ? kb::P - 1 : w);  // extreme words
    h[i] = w;
  }
  CHK(hipMemcpy(in, h, (size_t)16 * n * 4, hipMemcpyHostToDevice));
  CHK(hipMemset(bad, 0, 4));
  hipLaunchKernelGGL(k_check, dim3(n * 16 / 256), dim3(256), 0, 0, in, bad, n);
  uint32_t nb = 0;
  CHK(hipMemcpy(&nb, bad, 4, hipMemcpyDeviceToHost));
  printf("mismatching lanes (lane32 vs lane64 vs thread form) over %d states: %u\n", n, nb);
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  const int iters = 4096;
  for (int rep = 0; rep < 3; rep++)
    for (int v = 0; v < 2; v++) {
      CHK(hipMemcpy(io, h, 64 * 4, hipMemcpyHostToDevice));
      CHK(hipEventRecord(e0));
      if (v == 0) hipLaunchKernelGGL(k_chain<0>, dim3(1), dim3(64), 0, 0, io, iters);
      else hipLaunchKernelGGL(k_chain<1>, dim3(1), dim3(64), 0, 0, io, iters);
      CHK(hipEventRecord(e1));
      CHK(hipEventSynchronize(e1));
      float ms;
      CHK(hipEventElapsedTime(&ms, e0, e1));
      printf("%s: %.3f us per dependent permutation\n", v ? "lane64 (64-bit lazy)" : "lane32 (shipped)",
             ms * 1e3 / iters);
    }
  return nb ? 2 : 0;
}
