// Register-window NTT building blocks shared by the coset-LDE kernels (ntt.hip) and the NTT
// microbenchmarks under scripts/ (ubench_ntt_mfma.hip): the compile-time small roots, the
// radix-16 register window and its twiddle prefetch.  Device code only; include after kb.h.
#pragma once
#include "kb.h"

namespace bfz {

using namespace kb;

// Register-resident radix-16 pass.  A tile is 2^(b+c) elements: 2^b points of a butterfly
// group (stride 2^s0) x 2^c adjacent groups (coalesced runs).  Every thread holds 16
// elements; each "window" of 4 index bits is done in registers (4 stages, butterfly
// twiddle = one table value x a compile-time root of order <= 16), and windows exchange
// through LDS.  The first window loads straight from HBM and the last stores straight
// back, so a pass is one read + one write of the data.


constexpr uint32_t G24 = cpow(3, 127);
constexpr uint32_t root_pow2(int k) {  // w_(2^k), canonical
  uint32_t g = G24;
  for (int i = k; i < 24; i++) g = cmul(g, g);
  return g;
}
struct SmallRoots {
  uint32_t f[32], i[32];  // [2^k + l] = w_(2^(k+1))^(+-l), k = 0..4 (Montgomery)
};
constexpr SmallRoots make_small_roots() {
  SmallRoots r{};
  for (int k = 0; k < 5; k++) {
    const uint32_t w = root_pow2(k + 1), wi = cpow(w, P - 2);
    uint32_t a = 1, b = 1;
    for (int l = 0; l < (1 << k); l++) {
      r.f[(1 << k) + l] = to_mont_c(a);
      r.i[(1 << k) + l] = to_mont_c(b);
      a = cmul(a, w);
      b = cmul(b, wi);
    }
  }
  return r;
}
constexpr SmallRoots SMALL = make_small_roots();

// One 4-stage window on a thread's 16 elements.  Lazy reduction: a Montgomery product only
// needs its multiplicand < 2^32, so
//   DIT: an output of stage kk < 3 whose index has bit kk+1 set is the multiplied operand of
//        the next stage and stays in [0, 2p) (saves the min() of its add/sub);
//   DIF: u - v + p feeds the twiddle product directly.
// CONST_TW: the tile's base twiddle is 1 (first DIT / last DIF window of a pass starting at
// stage 0), so the twiddles are the compile-time small roots and w = 1 products vanish.
// TW_LOAD: read every twiddle of the stage from the table (tile kernels: s0 = lo_g = 0, the
// table slice below 2^14 is L2-resident) instead of multiplying one loaded base by the small
// roots -- a load replaces a Montgomery product.
// R is the window size in stages (2^R elements per thread); every launch uses R = 4.
// PRE: the stage twiddles were loaded ahead into pre[(1 << kk) - 1 + l] (load_window_tw, issued
// one window earlier so their latency hides behind that window's butterflies).
template <bool DIF, bool CONST_TW, bool TW_LOAD = false, int R = 4, bool PRE = false>
__device__ __forceinline__ void r16_window(uint32_t (&x)[1 << R], int g0, int kk_lo, int kk_hi, int s0,
                                           uint32_t m_low, uint32_t lo_g, const uint32_t* __restrict__ tw,
                                           const uint32_t* pre = nullptr) {
  // performs stages t = g0 + kk for kk in [kk_lo, kk_hi), ascending (DIT) or descending (DIF)
  constexpr int E = 1 << R, H = E / 2;
#pragma unroll
  for (int q = 0; q < R; q++) {
    const int kk = DIF ? R - 1 - q : q;
    if (kk < kk_lo || kk >= kk_hi) continue;
    uint32_t tws[H];
    if (CONST_TW) {
#pragma unroll
      for (int l = 0; l < H; l++)
        if (l < (1 << kk)) tws[l] = DIF ? SMALL.f[(1 << kk) + l] : SMALL.i[(1 << kk) + l];
    } else if (PRE) {
#pragma unroll
      for (int l = 0; l < H; l++)
        if (l < (1 << kk)) tws[l] = pre[(1 << kk) - 1 + l];
    } else if (TW_LOAD) {  // one table load per twiddle instead of a load and a multiply
      const __amdgpu_buffer_rsrc_t rt = rsrc_of(tw);
      const uint32_t off = ((m_low << s0) + lo_g) * 4u;  // the per-thread part of the index
#pragma unroll
      for (int l = 0; l < H; l++)
        if (l < (1 << kk))
          tws[l] = ld_b(rt, off, ((1u << (s0 + g0 + kk)) + ((uint32_t)l << (g0 + s0))) * 4u);
    } else {
      const int t = g0 + kk;
      const uint32_t wb = tw[(1u << (s0 + t)) + (m_low << s0) + lo_g];
#pragma unroll
      for (int l = 0; l < H; l++)
        if (l < (1 << kk))
          tws[l] = l == 0 ? wb : mmul(wb, DIF ? SMALL.f[(1 << kk) + l] : SMALL.i[(1 << kk) + l]);
    }
#pragma unroll
    for (int i = 0; i < E; i++) {
      if (i & (1 << kk)) continue;
      const int j = i | (1 << kk);
      const int l = i & ((1 << kk) - 1);
      const bool unit = CONST_TW && l == 0;  // twiddle known to be 1
      const uint32_t w = tws[l];
      const uint32_t u = x[i], v = x[j];
      if (DIF) {
        x[i] = madd(u, v);
        x[j] = unit ? msub(u, v) : mmul_s((int32_t)(u - v), w);
      } else {
        const uint32_t vw = unit ? umin(v, v - P) : mmul(v, w);
        const bool lazy = kk < R - 1 && ((i >> (kk + 1)) & 1);
        const uint32_t s_ = u + vw, d = u - vw;
        x[i] = lazy ? s_ : umin(s_, s_ - P);
        x[j] = lazy ? d + P : umin(d, d + P);
      }
    }
  }
}

// The table twiddles of one tile window (s0 = lo_g = 0): pre[(1 << kk) - 1 + l] = the twiddle of
// stage g0 + kk at position m_low + l 2^g0, for kk in [kk_lo, kk_hi).
template <int R>
__device__ __forceinline__ void load_window_tw(uint32_t (&pre)[(1 << R) - 1], int g0, int kk_lo,
                                               int kk_hi, uint32_t m_low,
                                               const uint32_t* __restrict__ tw) {
#pragma unroll
  for (int kk = 0; kk < R; kk++) {
    if (kk < kk_lo || kk >= kk_hi) continue;
#pragma unroll
    for (int l = 0; l < (1 << kk); l++)
      pre[(1 << kk) - 1 + l] = ld_b(rsrc_of(tw), m_low * 4u, ((1u << (g0 + kk)) + ((uint32_t)l << g0)) * 4u);
  }
}

// The same for a strided window (stage s0 + g0 + kk, positions (m_low + l 2^g0) << s0 + lo_g).
template <int R>
__device__ __forceinline__ void load_window_tw_s(uint32_t (&pre)[(1 << R) - 1], int g0, int kk_lo,
                                                 int kk_hi, int s0, uint32_t m_low, uint32_t lo_g,
                                                 const uint32_t* __restrict__ tw) {
  const __amdgpu_buffer_rsrc_t rt = rsrc_of(tw);
  const uint32_t off = ((m_low << s0) + lo_g) * 4u;
#pragma unroll
  for (int kk = 0; kk < R; kk++) {
    if (kk < kk_lo || kk >= kk_hi) continue;
#pragma unroll
    for (int l = 0; l < (1 << kk); l++)
      pre[(1 << kk) - 1 + l] = ld_b(rt, off, ((1u << (s0 + g0 + kk)) + ((uint32_t)l << (g0 + s0))) * 4u);
  }
}

}  // namespace bfz
