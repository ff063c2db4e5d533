// Coset low-degree extension on the device (the p3 `Radix2DitParallel::coset_lde_batch` +
// `bit_reverse_rows` step of TwoAdicFriPcs::commit, called from crates/stark/src/
// prover.rs:227,334,411 and machine.rs:196).
//
//   evals (bit-reversed rows, n per column)
//     --iDFT, DIT (bit-reversed in -> natural out)-->  coefficients c_k
//     --scale-split--> lo_k = c_k s^k / n,  hi_k = c_k (s w_2n)^k / n
//     --DFT, DIF on each half (natural in -> bit-reversed out)-->  LDE
// The first DIF stage of a size-2n transform on a zero-padded input is exactly the
// scale-split (upper half = lower half times w_2n^k), so [DIF_n(lo); DIF_n(hi)] is the
// bit-reversed LDE on s*H_2n.  Passes are LDS-tiled radix-2^b with coalesced 2^c-element
// runs; all columns of a matrix go in one launch (grid.y).
#include "ntt.h"

#include <cstdlib>
#include <cstring>

namespace bfz {

using namespace kb;

constexpr int TILE_LOG = 12;  // 4096 u32 per tile (16 KiB LDS)
constexpr int CMAX = 5;       // coalesced runs of 32 elements for strided passes

template <bool DIF>
__global__ __launch_bounds__(256) void k_ntt_pass(const uint32_t* __restrict__ src,
                                                  uint32_t* __restrict__ dst, size_t src_stride,
                                                  size_t dst_stride, int s0, int b, int c,
                                                  const uint32_t* __restrict__ tw) {
  __shared__ uint32_t tile[1 << TILE_LOG];
  const uint32_t* s = src + (size_t)blockIdx.y * src_stride;
  uint32_t* d = dst + (size_t)blockIdx.y * dst_stride;
  const int nlo_log = s0 - c;
  const size_t lo_blk = blockIdx.x & ((1u << nlo_log) - 1);
  const size_t hi = (size_t)blockIdx.x >> nlo_log;
  const size_t base = (hi << (s0 + b)) + (lo_blk << c);
  const int nelem = 1 << (b + c);
  const int cmask = (1 << c) - 1;
  for (int e = threadIdx.x; e < nelem; e += blockDim.x) {
    const int lo = e & cmask, m = e >> c;
    tile[e] = s[base + ((size_t)m << s0) + lo];
  }
  __syncthreads();
  const int nbf = nelem >> 1;
  for (int tt = 0; tt < b; tt++) {
    const int t = DIF ? (b - 1 - tt) : tt;
    const uint32_t* twt = tw + ((size_t)1 << (s0 + t)) + (lo_blk << c);
    for (int q = threadIdx.x; q < nbf; q += blockDim.x) {
      const int lo = q & cmask, qq = q >> c;
      const int mlow = qq & ((1 << t) - 1);
      const int m1 = ((qq >> t) << (t + 1)) | mlow;
      const int i1 = (m1 << c) | lo, i2 = i1 + (1 << (t + c));
      const uint32_t w = twt[((size_t)mlow << s0) + lo];
      const uint32_t u = tile[i1], v = tile[i2];
      if (DIF) {
        tile[i1] = madd(u, v);
        tile[i2] = mmul_s((int32_t)(u - v), w);
      } else {
        const uint32_t vw = mmul(v, w);
        tile[i1] = madd(u, vw);
        tile[i2] = msub(u, vw);
      }
    }
    __syncthreads();
  }
  for (int e = threadIdx.x; e < nelem; e += blockDim.x) {
    const int lo = e & cmask, m = e >> c;
    d[base + ((size_t)m << s0) + lo] = tile[e];
  }
}

// ---------------------------------------------------------------------------------------
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

// 2^14 elements per tile: 1024 threads x 16 (2^13 tiles measured +7%)
constexpr int R16_TILE_LOG = 14;
// Second-pass tiles take 2^c adjacent columns (2^c * 4 B coalesced runs); c <= MID_CMAX
// (16- or 64-column runs measured +8% / +2%).
constexpr int MID_CMAX = 5;
// k_lde_mid reads every twiddle of a stage from the table instead of multiplying one loaded
// base by the small roots (a load replaces a Montgomery product).
#ifndef BFZ_MID_TW_LOAD
#define BFZ_MID_TW_LOAD 1
#endif
constexpr bool MID_TW_LOAD = BFZ_MID_TW_LOAD;

__device__ __forceinline__ int lds_pad(int idx, int c) { return c < 5 ? idx + (idx >> 4) : idx; }

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
      const uint32_t* tt = tw + (1u << (s0 + g0 + kk)) + ((size_t)m_low << s0) + lo_g;
#pragma unroll
      for (int l = 0; l < H; l++)
        if (l < (1 << kk)) tws[l] = tt[(size_t)l << (g0 + s0)];
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
      pre[(1 << kk) - 1 + l] = tw[(1u << (g0 + kk)) + m_low + ((uint32_t)l << g0)];
  }
}

template <bool DIF>
__global__ __launch_bounds__(1024) void k_ntt_r16(const uint32_t* __restrict__ src,
                                                  uint32_t* __restrict__ dst, size_t src_stride,
                                                  size_t dst_stride, int s0, int b, int c,
                                                  const uint32_t* __restrict__ tw) {
  extern __shared__ uint32_t lds[];
  const int tid = threadIdx.x;
  const int nlo_log = s0 - c;
  const size_t lo_blk = blockIdx.x & ((1u << nlo_log) - 1);
  const size_t hi = (size_t)blockIdx.x >> nlo_log;
  const size_t base = (hi << (s0 + b)) + (lo_blk << c);
  const uint32_t* S = src + (size_t)blockIdx.y * src_stride + base;
  uint32_t* D = dst + (size_t)blockIdx.y * dst_stride + base;
  const int lo = tid & ((1 << c) - 1);
  const uint32_t lo_g = (uint32_t)(lo_blk << c) + lo;
  const int rest = tid >> c;
  const int nwin = (b + 3) >> 2;
  // A contiguous tile (c == 0) is moved between HBM and LDS with thread t touching elements
  // t, t + T, t + 2T, ... so every wave instruction is one 256-byte segment; the window
  // pattern (16 adjacent elements per thread in the first DIT window) would otherwise
  // stride 64 bytes across the lanes of a wave.
  const bool stage = (c == 0);
  const int T = (int)blockDim.x;
  uint32_t x[16];
  if (stage) {
#pragma unroll
    for (int i = 0; i < 16; i++) lds[lds_pad(i * T + tid, 0)] = S[(uint32_t)(i * T + tid)];
  }
  int done_lo = 0, done_hi = b;  // DIT: stages < done_lo done; DIF: stages >= done_hi done
  for (int w = 0; w < nwin; w++) {
    const int g0 = DIF ? max(b - 4 - 4 * w, 0) : min(4 * w, b - 4);
    const uint32_t m_low = rest & ((1 << g0) - 1);
    const uint32_t m_base = m_low | ((uint32_t)(rest >> g0) << (g0 + 4));
    if (w == 0 && !stage) {
#pragma unroll
      for (int i = 0; i < 16; i++) x[i] = S[(uint32_t)((m_base | ((uint32_t)i << g0)) << s0) + lo];
    } else {
      __syncthreads();
#pragma unroll
      for (int i = 0; i < 16; i++)
        x[i] = lds[lds_pad((int)(((m_base | ((uint32_t)i << g0)) << c) | lo), c)];
    }
    int kk_lo, kk_hi;
    if (DIF) {
      kk_lo = 0;
      kk_hi = min(4, done_hi - g0);
      done_hi = g0;
    } else {
      kk_lo = max(0, done_lo - g0);
      kk_hi = 4;
      done_lo = g0 + 4;
    }
    if (s0 == 0 && g0 == 0)
      r16_window<DIF, true>(x, g0, kk_lo, kk_hi, s0, m_low, lo_g, tw);
    else
      r16_window<DIF, false>(x, g0, kk_lo, kk_hi, s0, m_low, lo_g, tw);
    if (w == nwin - 1 && !stage) {
#pragma unroll
      for (int i = 0; i < 16; i++) D[(uint32_t)((m_base | ((uint32_t)i << g0)) << s0) + lo] = x[i];
    } else {
      // each thread rewrites exactly the slots it read for this window: no barrier needed
#pragma unroll
      for (int i = 0; i < 16; i++)
        lds[lds_pad((int)(((m_base | ((uint32_t)i << g0)) << c) | lo), c)] = x[i];
    }
  }
  if (stage) {
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 16; i++) D[(uint32_t)(i * T + tid)] = lds[lds_pad(i * T + tid, 0)];
  }
}

// Contiguous pass (stages 0..B-1 of 2^B-element tiles, s0 = c = 0) with B a compile-time
// constant: the window loop unrolls, every window's g0 is a constant, and the LDS address of
// element i is pad(m_base) + (i << g0) + ((i << g0) >> 4) (the bits [g0, g0+4) of m_base are
// zero, so the padding never carries) -- all offsets fold into ds_read/ds_write immediates.
template <int G0>
__device__ __forceinline__ constexpr int tile_off(int i) { return (i << G0) + ((i << G0) >> 4); }

// DIN (DIT only): the first window (g0 = 0) holds the 16 consecutive words tid*16 + i, read
// straight from HBM as four 16-byte loads (no LDS staging, one barrier fewer); the launch picks
// it when the source rows are 16-byte aligned.
// R: 2^R elements per thread and R stages per register window (R = 5, three windows of a 2^14
// tile at 512 threads, measured DIT neutral / DIF +2%: R = 4 everywhere).
// PERSIST: a grid of a few blocks per CU walks the launch's tiles (column-major order), and each
// block issues the HBM loads of its NEXT tile into registers before working on the current one,
// so the load latency of a tile hides behind the previous tile's windows instead of stalling
// all of a block's waves at its start (tiles_per_col / ntiles describe the launch).
// TWPF: each window's table twiddles are loaded one window ahead (into registers, double
// buffered) instead of at the window's start, where every wave of the block would wait for the
// L2 round trip at the same time (the waves run in lockstep between the LDS exchanges).
// WS (B >= 13, R = 4): windows g0 = 0, 4, 6, B-4 (DIT; the DIF the reverse).  The threads of a
// wave hold the same 1024 consecutive elements (bits [10, B) = the wave index) in every window
// with g0 <= 6, so the exchanges between such windows go through the wave's own LDS region with
// a wave-level fence instead of a block barrier: one block barrier per DIT tile instead of three.
template <bool DIF, int B, bool DIN = false, int R = 4, bool PERSIST = false, bool TWPF = false,
          bool WS = false>
__global__ __launch_bounds__(1 << (B - R)) void k_ntt_tile(const uint32_t* __restrict__ src,
                                                           uint32_t* __restrict__ dst,
                                                           size_t src_stride, size_t dst_stride,
                                                           const uint32_t* __restrict__ tw,
                                                           uint32_t tiles_per_col = 0,
                                                           uint32_t ntiles = 0) {
  static_assert(B >= 8 && B <= R16_TILE_LOG, "tile");
  constexpr int E = 1 << R;  // elements per thread
  constexpr int T = 1 << (B - R);
  constexpr int NW = (B + R - 1) / R;
  extern __shared__ uint32_t lds[];
  const int tid = threadIdx.x;
  const int tpad = tid + (tid >> R);
  // A DIT's last window (g0 = B - R) holds elements tid + i T: those go straight from registers
  // to HBM (one coalesced 256-byte segment per wave instruction; -2.4% per pass).  The DIF's
  // first window would read the same way, but measured slower than LDS staging (+4.5%,
  // profiles/r02/ntt_lab_variants.txt), so a DIF pass keeps it.
  // BFZ_NTT_REPS (diagnostic builds only, scripts/ubench_ntt.cpp): 0 = data movement alone,
  // 2 = the stages twice, to split a pass's time into its memory and compute parts.
#ifndef BFZ_NTT_REPS
#define BFZ_NTT_REPS 1
#endif
  constexpr bool DIRECT = BFZ_NTT_REPS == 1;
  // (The WS DIF's last window, 16 consecutive words per thread, stored straight to HBM as four
  // 16-byte stores instead of through LDS: DIF pass 173-179 -> 192-199 us, profiles/r04/
  // ab_tile_dout.txt.)
  static_assert(!DIN || (!DIF && BFZ_NTT_REPS == 1), "direct first window: DIT passes only");
  constexpr bool DINL = DIN;
  static_assert(!PERSIST || BFZ_NTT_REPS == 1, "persistent tiles: production builds only");
  static_assert(!WS || (R == 4 && B >= 13), "wave-local windows: 2^13 / 2^14 tiles");
  uint32_t tile = PERSIST ? blockIdx.x : 0;
  auto src_of = [&](uint32_t t) {
    const size_t col = PERSIST ? t / tiles_per_col : blockIdx.y;
    const size_t tx = PERSIST ? t % tiles_per_col : blockIdx.x;
    return src + col * src_stride + (tx << B);
  };
  auto dst_of = [&](uint32_t t) {
    const size_t col = PERSIST ? t / tiles_per_col : blockIdx.y;
    const size_t tx = PERSIST ? t % tiles_per_col : blockIdx.x;
    return dst + col * dst_stride + (tx << B);
  };
  // the tile's words as the first window wants them: DIN 16 consecutive words per thread, else
  // words tid + i T (staged through LDS)
  uint32_t pf[E];
  auto load = [&](uint32_t t) {
    const uint32_t* S = src_of(t);
    if constexpr (DINL) {
      const uint4* s4 = reinterpret_cast<const uint4*>(S + (tid << R));
#pragma unroll
      for (int q = 0; q < E / 4; q++) {
        const uint4 v = s4[q];
        pf[4 * q] = v.x; pf[4 * q + 1] = v.y; pf[4 * q + 2] = v.z; pf[4 * q + 3] = v.w;
      }
    } else {
#pragma unroll
      for (int i = 0; i < E; i++) pf[i] = S[i * T + tid];
    }
  };
  load(tile);
  for (;;) {
    uint32_t* D = dst_of(tile);
    // the stage twiddles are the same for every tile: re-read per tile (an opaque offset) rather
    // than hoisted out of the tile loop into ~70 registers (which halves the occupancy)
    const uint32_t* twl = tw;
    if constexpr (PERSIST) {
      uint32_t z = 0;
      asm volatile("" : "+v"(z));
      twl = tw + z;
    }
    uint32_t x[E];
    if constexpr (DINL) {
#pragma unroll
      for (int i = 0; i < E; i++) x[i] = pf[i];
    } else {
#pragma unroll
      for (int i = 0; i < E; i++) lds[i * (T + T / E) + tpad] = pf[i];
    }
    const uint32_t next = tile + gridDim.x;
    if (PERSIST && next < ntiles) load(next);  // in flight while this tile's windows run
    // window w: first stage g0(w) and its stage range [kk_lo, kk_hi) (compile-time after unrolling)
    auto win_g0 = [](int w) {
      if (WS) {
        constexpr int g[4] = {0, 4, 6, B - 4};
        return DIF ? g[3 - w] : g[w];
      }
      return DIF ? (B - R - R * w > 0 ? B - R - R * w : 0) : (R * w < B - R ? R * w : B - R);
    };
    auto win_range = [&](int w, int& lo, int& hi) {
      int done_lo = 0, done_hi = B;
      for (int v = 0; v <= w; v++) {
        const int g = win_g0(v);
        lo = 0;
        hi = R;
        if (DIF) {
          hi = done_hi - g < R ? done_hi - g : R;
          done_hi = g;
        } else {
          lo = done_lo - g > 0 ? done_lo - g : 0;
          done_lo = g + R;
        }
      }
    };
    uint32_t pre[2][(1 << R) - 1];
    if constexpr (TWPF) {
      if (win_g0(0) != 0) {
        int lo, hi;
        win_range(0, lo, hi);
        load_window_tw<R>(pre[0], win_g0(0), lo, hi, tid & ((1 << win_g0(0)) - 1), twl);
      }
    }
#pragma nounroll
    for (int rep = 0; rep < BFZ_NTT_REPS; rep++) {
#pragma unroll
    for (int w = 0; w < NW; w++) {
      const int g0 = win_g0(w);
      const uint32_t m_low = tid & ((1 << g0) - 1);
      const uint32_t m_base = m_low | ((uint32_t)(tid >> g0) << (g0 + R));
      const uint32_t pb = m_base + (m_base >> R);
      const bool direct_out = DIRECT && !DIF && w == NW - 1;
      if (!DINL || w > 0) {
        if (WS && w > 0 && win_g0(w - 1) <= 6 && g0 <= 6) {  // the wave's own 1024 elements
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        } else {
          __syncthreads();
        }
#pragma unroll
        for (int i = 0; i < E; i++) x[i] = lds[pb + (i << g0) + ((i << g0) >> R)];
      }
      int kk_lo, kk_hi;
      win_range(w, kk_lo, kk_hi);
      if constexpr (TWPF) {  // the next window's twiddles, in flight during this window
        if (w + 1 < NW && win_g0(w + 1) != 0) {
          int lo, hi;
          win_range(w + 1, lo, hi);
          load_window_tw<R>(pre[(w + 1) & 1], win_g0(w + 1), lo, hi,
                            tid & ((1 << win_g0(w + 1)) - 1), twl);
        }
      }
      if (g0 == 0)
        r16_window<DIF, true, false, R>(x, g0, kk_lo, kk_hi, 0, m_low, 0, twl);
      else if (TWPF)
        r16_window<DIF, false, true, R, true>(x, g0, kk_lo, kk_hi, 0, m_low, 0, twl, pre[w & 1]);
      else
        r16_window<DIF, false, true, R>(x, g0, kk_lo, kk_hi, 0, m_low, 0, twl);
      if (direct_out) {
#pragma unroll
        for (int i = 0; i < E; i++) D[i * T + tid] = x[i];
      } else {
#pragma unroll
        for (int i = 0; i < E; i++) lds[pb + (i << g0) + ((i << g0) >> R)] = x[i];
      }
    }
    }
    if (DIF || !DIRECT) {
      __syncthreads();
#pragma unroll
      for (int i = 0; i < E; i++) D[i * T + tid] = lds[i * (T + T / E) + tpad];
    }
    if (!PERSIST || next >= ntiles) break;
    tile = next;
    __syncthreads();  // every wave is done with this tile's LDS before the next one's writes
  }
}

// ---------------------------------------------------------------------------------------
// 2^14-point tile passes with ten of the fourteen stages on the matrix cores (gfx950
// v_mfma_i32_32x32x32_i8).  A 1024-point DFT with a root w of order 1024 is two 32-point
// DFTs and a twiddle (j = jl + 32 jh, k = kl + 32 kh:  w^(jk) = w^(jl kl) w32^(jl kh) w32^(jh kl)),
// and a 32-point DFT of 32 rows is a 32 x 32 matrix product.  A 31-bit product is 16 int8
// products: each data word is split into 4 signed digits (x = sum_d x_d 2^(8d), K = 32 words
// x 4 digits = 4 MFMA K-steps) and the constant matrix entry into the 4 signed digit planes of
// V_d = M 2^(8d) R mod p (4 accumulators e); sum_e 2^(8e) acc_e = sum_j M_j x_j R (mod p) as an
// exact 64-bit integer (|acc_e| < 2^21), and one signed Montgomery reduction gives the
// Montgomery product.  Per element that is ~36 VALU units for ten stages against ~75 for ten
// radix-2 stages (the 32 MFMAs per 1024 elements run on the matrix pipe beside them).
//   DIT tile (bit-reversed in, natural out):  wave b transforms block b (positions
//     [1024 b, 1024 b + 1024) hold the bit-reversed 1024-point subsequence: stages 0..9 are its
//     DFT), results to LDS; then the radix-16 window g0 = 10 (stages 10..13) as k_ntt_tile's
//     and straight to HBM.
//   DIF tile (natural in, bit-reversed out): the radix-16 window g0 = 10 (stages 13..10) on
//     elements tid + 1024 i straight from HBM, to LDS; then wave b runs stages 9..0 = the
//     1024-point DFT of block b, natural in, bit-reversed out, straight to HBM.
// The MFMA layouts (v_mfma_i32_32x32x32_i8, wave64): A operand lane l = row l & 31, K bytes
// [16 (l >> 5), +16); B operand lane l = column l & 31, same K split; accumulator element q of
// lane l = row (q & 3) + 8 (q >> 2) + 4 (l >> 5), column l & 31.  Pass A's accumulator is
// therefore pass B's B operand with no lane exchange (scripts/ubench_mfma_dft.hip checks both
// directions against an O(n^2) DFT).
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

__device__ __forceinline__ uint32_t i8_digits(uint32_t x) {  // x < 0x7f7f7f7f
  return (x + 0x80808080u) ^ 0x80808080u;
}
// sum_e 2^(8e) acc_e, Montgomery-reduced: result in (-p, p) as int32
__device__ __forceinline__ int32_t mfma_combine(int32_t a0, int32_t a1, int32_t a2, int32_t a3) {
  const int32_t lo = a0 + a1 * 256, hi = a2 + a3 * 256;
  const int64_t y = (int64_t)hi * 65536 + (int64_t)lo;
  const int32_t m = (int32_t)((uint32_t)y * MU_NEG);
  return (int32_t)(((int64_t)m * (int64_t)P + y) >> 32);
}

constexpr int MF_DATA = 1 << 14;  // LDS words of tile data (64 KiB: two tiles per CU)
constexpr int MF_THREADS = 512;   // 8 waves, two 1024-point blocks each
// DIT: the 16 KiB table staged in LDS per block (64 + 16 KiB: still two tiles per CU; -24% against
// reading it through L1/L2); the DIF's two tables (32 KiB) are read from L1/L2.
constexpr bool MF_LDSW = true;
#ifndef BFZ_MF_DIAG
#define BFZ_MF_DIAG 0  // diagnostic builds: 1 = no 1024-point transforms, 2 = no radix-16 window
#endif

// The constant tables live in global memory (L1/L2-resident, 16 or 32 KiB) in [reg][lane]
// order: one register of the table is 64 consecutive v4i, one coalesced 1 KiB wave load.
typedef const __attribute__((address_space(1))) v4i gv4i;
typedef const __attribute__((address_space(1))) uint32_t gu32;
// a zero the compiler cannot see through or merge with another (volatile: never CSE'd), so
// each use of a table is a fresh load instead of registers held across the kernel
__device__ __forceinline__ uint32_t fresh_zero() {
  uint32_t z = 0;
  asm volatile("" : "+v"(z));
  return z;
}

// 16 MFMAs: acc_e = sum_s X[s] x W[e][s] (data as the A operand) or W[e][s] x X[s] (as B);
// out[q] = Montgomery(sum_e 2^(8e) acc_e) in (-p, p).  The table registers of each K-step are
// read afresh (4 in flight, not the whole 16-register table held across the kernel).
// (Two accumulator groups of two planes each, 32 registers instead of 64, measured slower.)
template <bool DATA_IS_A, class TW>
__device__ __forceinline__ void mf_pass(int32_t (&out)[16], const v4i (&X)[4], TW* __restrict__ W) {
  v16i acc[4];
#pragma unroll
  for (int e = 0; e < 4; e++) acc[e] = v16i{};
#pragma unroll
  for (int s = 0; s < 4; s++) {
    TW* WL = W + fresh_zero();
#pragma unroll
    for (int e = 0; e < 4; e++) {
      const v4i w = WL[64 * (4 * e + s)];
      acc[e] = DATA_IS_A ? __builtin_amdgcn_mfma_i32_32x32x32_i8(X[s], w, acc[e], 0, 0, 0)
                         : __builtin_amdgcn_mfma_i32_32x32x32_i8(w, X[s], acc[e], 0, 0, 0);
    }
  }
#pragma unroll
  for (int q = 0; q < 16; q++) out[q] = mfma_combine(acc[0][q], acc[1][q], acc[2][q], acc[3][q]);
}
// pass A -> twiddle -> pass B on one 1024-point block; X: the block's digits (A operand);
// out: the transform in (-p, p), element q of lane l at pass B's accumulator position
template <class TW>
__device__ __forceinline__ void mf_dft1024(int32_t (&out)[16], v4i (&X)[4], TW* __restrict__ WA,
                                           TW* __restrict__ WB, gu32* __restrict__ TL) {
#if BFZ_MF_DIAG == 1  // diagnostic: no transform (data movement + the radix-16 window)
#pragma unroll
  for (int q = 0; q < 16; q++) out[q] = X[q >> 2][q & 3] & 0x3fffffff;
  return;
#endif
  mf_pass<true>(out, X, WA);
#pragma unroll
  for (int q = 0; q < 16; q++) X[q >> 2][q & 3] = (int)i8_digits(mmul_s(out[q], TL[64 * q]));
  mf_pass<false>(out, X, WB);
}

template <bool DIF>
__global__ __launch_bounds__(MF_THREADS) __attribute__((amdgpu_waves_per_eu(4, 4))) void k_tile14_mfma(
    const uint32_t* __restrict__ src, uint32_t* __restrict__ dst, size_t src_stride, size_t dst_stride,
    const uint32_t* __restrict__ tw, const v4i* __restrict__ wtab, const uint32_t* __restrict__ ttab) {
  extern __shared__ uint32_t lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = lane & 31, h = lane >> 5;
  const size_t base = (size_t)blockIdx.x << 14;
  const uint32_t* S = src + (size_t)blockIdx.y * src_stride + base;
  uint32_t* D = dst + (size_t)blockIdx.y * dst_stride + base;
  gv4i* WA = (gv4i*)wtab + lane;
  gv4i* WB = WA + (DIF ? 64 * 16 : 0);
  gu32* TL = (gu32*)ttab + lane;
  v4i* wl = reinterpret_cast<v4i*>(lds + MF_DATA);
  if constexpr (!DIF && MF_LDSW) {
    for (int i = tid; i < 16 * 64; i += MF_THREADS) wl[i] = ((gv4i*)wtab)[i];
    __syncthreads();
  }
  int32_t y[16];
  if constexpr (!DIF) {
#pragma nounroll
    for (int k = 0; k < 2; k++) {  // (unrolled: neutral)
      const uint32_t* Xg = S + (wave + 8 * k) * 1024;
      v4i X[4];
#pragma unroll
      for (int s = 0; s < 4; s++) {
        const uint4 v = *reinterpret_cast<const uint4*>(Xg + 32 * r + 8 * s + 4 * h);
        X[s] = v4i{(int)i8_digits(v.x), (int)i8_digits(v.y), (int)i8_digits(v.z), (int)i8_digits(v.w)};
      }
      if constexpr (MF_LDSW)
        mf_dft1024(y, X, (const v4i*)wl + lane, (const v4i*)wl + lane, TL);
      else
        mf_dft1024(y, X, WA, WB, TL);
      uint32_t* blk = lds + (wave + 8 * k) * 1024;
#pragma unroll
      for (int q = 0; q < 16; q++)
        blk[r + 32 * ((q & 3) + 8 * (q >> 2) + 4 * h)] = umin((uint32_t)y[q], (uint32_t)y[q] + P);
    }
    __syncthreads();
#pragma nounroll
    for (int k = 0; k < 2; k++) {
      const int c = tid + MF_THREADS * k;
      uint32_t x[16];
#pragma unroll
      for (int i = 0; i < 16; i++) x[i] = lds[c + 1024 * i];
#if BFZ_MF_DIAG != 2
      r16_window<false, false, true, 4>(x, 10, 0, 4, 0, (uint32_t)c, 0, tw);
#endif
#pragma unroll
      for (int i = 0; i < 16; i++) D[c + 1024 * i] = x[i];
    }
  } else {
#pragma unroll
    for (int k = 0; k < 2; k++) {
      const int c = tid + MF_THREADS * k;
      uint32_t x[16];
#pragma unroll
      for (int i = 0; i < 16; i++) x[i] = S[c + 1024 * i];
#if BFZ_MF_DIAG != 2
      r16_window<true, false, true, 4>(x, 10, 0, 4, 0, (uint32_t)c, 0, tw);
#endif
#pragma unroll
      for (int i = 0; i < 16; i++) lds[c + 1024 * i] = x[i];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 2; k++) {
      const uint32_t* blk = lds + (wave + 8 * k) * 1024;
      v4i X[4];
#pragma unroll
      for (int s = 0; s < 4; s++)
#pragma unroll
        for (int t = 0; t < 4; t++) X[s][t] = (int)i8_digits(blk[r + 32 * (8 * s + 4 * h + t)]);
      mf_dft1024(y, X, WA, WB, TL);
      uint32_t* Y = D + (wave + 8 * k) * 1024 + 32 * (__builtin_bitreverse32((uint32_t)r) >> 27);
#pragma unroll
      for (int g = 0; g < 4; g++) {
        uint32_t o[4];
#pragma unroll
        for (int t = 0; t < 4; t++) o[t] = umin((uint32_t)y[4 * g + t], (uint32_t)y[4 * g + t] + P);
        *reinterpret_cast<uint4*>(Y + 8 * g + 4 * h) = uint4{o[0], o[1], o[2], o[3]};
      }
    }
  }
}

// Host tables of the 1024-point DFTs (root w of order 1024, Montgomery):
//   DIT: [pass A = pass B] M[i][j] = w32^(bitrev5(j) i);  twiddle lane (i, h), q: w^(bitrev5(a) i)
//   DIF: pass A F[i][j] = w32^(j i), pass B M2[i][j] = w32^(j bitrev5(i));  twiddle w^(a i)
// with a = (q & 3) + 8 (q >> 2) + 4 h.  Table entry [16 pass + 4 e + s][lane] holds, for K byte
// kb (j = 8 s + 4 h + kb / 4, d = kb % 4), digit e of V = M[lane & 31][j] 2^(8d) R mod p.
struct MfmaTables {
  DBuf<v4i> w_dit, w_dif;
  DBuf<uint32_t> t_dit, t_dif;
  bool ready = false;
};
static int brev(int x, int bits) {
  int r = 0;
  for (int i = 0; i < bits; i++) r |= ((x >> i) & 1) << (bits - 1 - i);
  return r;
}
static MfmaTables& mfma_tables() {
  static MfmaTables T;
  if (T.ready) return T;
  for (int dif = 0; dif < 2; dif++) {
    const uint32_t w = dif ? two_adic_gen(10) : minv(two_adic_gen(10));
    const uint32_t w32 = mpow(w, 32);
    const int NT = dif ? 2 : 1;
    std::vector<v4i> wt(64 * 16 * NT);
    std::vector<uint32_t> tt(64 * 16);
    for (int lane = 0; lane < 64; lane++) {
      const int i = lane & 31, h = lane >> 5;
      for (int pass = 0; pass < NT; pass++)
        for (int e = 0; e < 4; e++)
          for (int s = 0; s < 4; s++) {
            int8_t bytes[16];
            for (int kb = 0; kb < 16; kb++) {
              const int j = 8 * s + 4 * h + kb / 4, d = kb % 4;
              const uint64_t ex = !dif ? (uint64_t)brev(j, 5) * i
                                       : (pass == 0 ? (uint64_t)j * i : (uint64_t)j * brev(i, 5));
              const uint32_t m = mpow(w32, ex);
              const uint32_t V = from_mont(mmul(mmul(m, to_mont(1u << (8 * d))), R2));
              bytes[kb] = (int8_t)(((V + 0x80808080u) ^ 0x80808080u) >> (8 * e));
            }
            std::memcpy(&wt[(16 * pass + 4 * e + s) * 64 + lane], bytes, 16);
          }
      for (int q = 0; q < 16; q++) {
        const int a = (q & 3) + 8 * (q >> 2) + 4 * h;
        tt[q * 64 + lane] = mpow(w, (uint64_t)(dif ? a : brev(a, 5)) * i);
      }
    }
    DBuf<v4i>& dw = dif ? T.w_dif : T.w_dit;
    DBuf<uint32_t>& dt = dif ? T.t_dif : T.t_dit;
    dw.reset(wt.size());
    dt.reset(tt.size());
    HIP_CHECK(hipMemcpyAsync(dw.p, wt.data(), wt.size() * sizeof(v4i), hipMemcpyHostToDevice, stream()));
    HIP_CHECK(hipMemcpyAsync(dt.p, tt.data(), tt.size() * 4, hipMemcpyHostToDevice, stream()));
  }
  HIP_CHECK(hipStreamSynchronize(stream()));
  HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_tile14_mfma<false>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, MF_DATA * 4 + (MF_LDSW ? 16384 : 0)));
  HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_tile14_mfma<true>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, MF_DATA * 4));
  T.ready = true;
  return T;
}
// BFZ_NTT_MFMA=1 selects the matrix-core 2^14 tiles (A/B switch).  Default: the all-VALU
// k_ntt_tile -- the MFMA tiles are bit-exact but measured slower (DIT 205 vs
// 176 us, DIF 232 vs 189 us per 2^26-element pass): the ten MFMA stages alone cost ~200 us
// (the data movement and radix-16 window alone 108 us), well above their 10/14 share.
static bool use_mfma_tiles() {
  static const bool on = [] {
    const char* e = std::getenv("BFZ_NTT_MFMA");
    return e && *e == '1';
  }();
  return on;
}

// Fused middle of a two-pass coset LDE (L > 14).  One tile = 2^b points at stride 2^s0 x 2^c
// adjacent groups, as the second k_ntt_r16 pass:
//   iDFT stages [s0, s0+b) (DIT)  ->  coefficients c_k in registers
//   lo_k = c_k s^k / n, hi_k = c_k t^k / n  (t = s w_2n)
//   DFT stages [s0+b-1 .. s0] (DIF) of each half  ->  lde[col][0..n) and lde[col][n..2n)
// The DIT's last window and the DIF's first window hold the same 16 elements per thread, so
// the coefficients never leave registers.  A thread's coefficient indices step by
// D = 2^(s0+b-4): its powers are one table lookup times the launch constants (s^D)^i, (t^D)^i.
struct MidPowers {
  uint32_t lo[16], hi[16];
};

// Plan of an L-stage transform: pass 1 = stages [0, b1) contiguous, pass 2 = [b1, L) with
// 2^c2-element coalesced runs (see r16_plan); everything is a compile-time function of L.
template <int L>
struct MidPlan {
  static constexpr int b1 = L - 4 < R16_TILE_LOG ? L - 4 : R16_TILE_LOG;
  static constexpr int b2 = L - b1;
  static constexpr int c2 = b1 < R16_TILE_LOG - b2 ? (b1 < MID_CMAX ? b1 : MID_CMAX)
                                                  : (R16_TILE_LOG - b2 < MID_CMAX ? R16_TILE_LOG - b2 : MID_CMAX);
};

template <int L>
__global__ __launch_bounds__(1 << (MidPlan<L>::b2 + MidPlan<L>::c2 - 4)) void k_lde_mid(
    const uint32_t* __restrict__ src, size_t src_stride, uint32_t* __restrict__ lde, size_t n,
    const uint32_t* __restrict__ tw_inv, const uint32_t* __restrict__ tw_fwd,
    const uint32_t* __restrict__ pw, int B, MidPowers mp, int only_half) {
  constexpr int s0 = MidPlan<L>::b1, b = MidPlan<L>::b2, c = MidPlan<L>::c2;
  extern __shared__ uint32_t lds[];
  const int tid = threadIdx.x;
  const int nlo_log = s0 - c;
  const size_t lo_blk = blockIdx.x & ((1u << nlo_log) - 1);
  const size_t hi = (size_t)blockIdx.x >> nlo_log;
  const size_t base = (hi << (s0 + b)) + (lo_blk << c);
  const uint32_t* S = src + (size_t)blockIdx.y * src_stride + base;
  uint32_t* D = lde + (size_t)blockIdx.y * 2 * n + base;
  const int lo = tid & ((1 << c) - 1);
  const uint32_t lo_g = (uint32_t)(lo_blk << c) + lo;
  const int rest = tid >> c;
  const int nwin = (b + 3) >> 2;
  uint32_t x[16];
  int done_lo = 0;
#pragma unroll
  for (int w = 0; w < nwin; w++) {  // iDFT
    const int g0 = min(4 * w, b - 4);
    const uint32_t m_low = rest & ((1 << g0) - 1);
    const uint32_t m_base = m_low | ((uint32_t)(rest >> g0) << (g0 + 4));
    if (w == 0) {
#pragma unroll
      for (int i = 0; i < 16; i++) x[i] = S[(uint32_t)((m_base | ((uint32_t)i << g0)) << s0) + lo];
    } else {
      __syncthreads();
#pragma unroll
      for (int i = 0; i < 16; i++)
        x[i] = lds[lds_pad((int)(((m_base | ((uint32_t)i << g0)) << c) | lo), c)];
    }
    const int kk_lo = max(0, done_lo - g0);
    done_lo = g0 + 4;
    r16_window<false, false, MID_TW_LOAD>(x, g0, kk_lo, 4, s0, m_low, lo_g, tw_inv);
    if (w < nwin - 1) {
#pragma unroll
      for (int i = 0; i < 16; i++)
        lds[lds_pad((int)(((m_base | ((uint32_t)i << g0)) << c) | lo), c)] = x[i];
    }
  }
  uint32_t coef[16];
#pragma unroll
  for (int i = 0; i < 16; i++) coef[i] = x[i];
  {
    const int g0 = b - 4;
    const uint32_t m_base = (rest & ((1 << g0) - 1)) | ((uint32_t)(rest >> g0) << (g0 + 4));
    const size_t k0 = base + ((size_t)m_base << s0) + lo;
    const size_t mask = ((size_t)1 << B) - 1, nb = mask + 1;
    const uint32_t S0 = mmul(pw[k0 & mask], pw[nb + (k0 >> B)]);
    const uint32_t T0 = mmul(pw[2 * nb + (k0 & mask)], pw[3 * nb + (k0 >> B)]);
    for (int half = 0; half < 2; half++) {
      if (only_half >= 0 && half != only_half) continue;  // uniform across the block
      const uint32_t P0 = half ? T0 : S0;
#pragma unroll
      for (int i = 0; i < 16; i++) x[i] = mmul(coef[i], mmul(P0, half ? mp.hi[i] : mp.lo[i]));
      if (half && nwin > 1) __syncthreads();  // the lo half's last LDS reads are done
      uint32_t* Dh = D + (size_t)half * n;
      int done_hi = b;
#pragma unroll
      for (int w = 0; w < nwin; w++) {  // DFT of this half
        const int gg = max(b - 4 - 4 * w, 0);
        const uint32_t m_low = rest & ((1 << gg) - 1);
        const uint32_t mb = m_low | ((uint32_t)(rest >> gg) << (gg + 4));
        if (w > 0) {
          __syncthreads();
#pragma unroll
          for (int i = 0; i < 16; i++)
            x[i] = lds[lds_pad((int)(((mb | ((uint32_t)i << gg)) << c) | lo), c)];
        }
        const int kk_hi = min(4, done_hi - gg);
        done_hi = gg;
        r16_window<true, false, MID_TW_LOAD>(x, gg, 0, kk_hi, s0, m_low, lo_g, tw_fwd);
        if (w == nwin - 1) {
#pragma unroll
          for (int i = 0; i < 16; i++) Dh[(uint32_t)((mb | ((uint32_t)i << gg)) << s0) + lo] = x[i];
        } else {
#pragma unroll
          for (int i = 0; i < 16; i++)
            lds[lds_pad((int)(((mb | ((uint32_t)i << gg)) << c) | lo), c)] = x[i];
        }
      }
    }
  }
}

// lo_k = c_k * s^k / n ; hi_k = c_k * t^k / n  with s^k = SL[k & m] * SH[k >> B] (1/n in SH)
__global__ __launch_bounds__(256) void k_scale_split(const uint32_t* __restrict__ coef,
                                                     uint32_t* __restrict__ lde, size_t n, int B,
                                                     const uint32_t* __restrict__ pw,
                                                     int only_half) {
  const uint32_t* c = coef + (size_t)blockIdx.y * n;
  uint32_t* o = lde + (size_t)blockIdx.y * 2 * n;
  const size_t mask = ((size_t)1 << B) - 1;
  const size_t nb = mask + 1;
  const uint32_t* SL = pw;
  const uint32_t* SH = pw + nb;
  const uint32_t* TL = pw + 2 * nb;
  const uint32_t* TH = pw + 3 * nb;
  for (size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x; k < n;
       k += (size_t)gridDim.x * blockDim.x) {
    const uint32_t v = c[k];
    const size_t kl = k & mask, kh = k >> B;
    if (only_half != 1) o[k] = mmul(v, mmul(SL[kl], SH[kh]));
    if (only_half != 0) o[n + k] = mmul(v, mmul(TL[kl], TH[kh]));
  }
}

// out[c][t] = in[bitrev(t)][c]: row-major natural -> column-major bit-reversed.
__global__ __launch_bounds__(256) void k_transpose_bitrev(const uint32_t* __restrict__ in,
                                                          uint32_t* __restrict__ out, size_t n,
                                                          int w, int logn) {
  __shared__ uint32_t tile[64 * 65];
  const size_t t0 = (size_t)blockIdx.x * 64;
  const int total = 64 * w;
  for (int cb = 0; cb < w; cb += 65) {
    const int cw = min(65, w - cb);
    for (int e = threadIdx.x; e < 64 * cw; e += blockDim.x) {
      const int r = e / cw, cc = e % cw;
      const size_t t = t0 + r;
      if (t < n) tile[r * 65 + cc] = in[(size_t)dbitrev((uint32_t)t, logn) * w + cb + cc];
    }
    __syncthreads();
    for (int e = threadIdx.x; e < 64 * cw; e += blockDim.x) {
      const int cc = e / 64, r = e % 64;
      const size_t t = t0 + r;
      if (t < n) out[(size_t)(cb + cc) * n + t] = tile[r * 65 + cc];
    }
    __syncthreads();
  }
  (void)total;
}

// row-major out[r*w + c] = column-major in[c*H + r]
__global__ __launch_bounds__(256) void k_transpose_rowmajor(const uint32_t* __restrict__ in,
                                                            uint32_t* __restrict__ out, size_t H,
                                                            int w) {
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= H * (size_t)w) return;
  const size_t r = e / w, c = e % w;
  out[e] = in[c * H + r];
}

// -------------------------------------------------------------------------- host side
std::vector<std::pair<int, int>> ntt_plan(int L) {
  std::vector<std::pair<int, int>> p;
  int s0 = 0;
  while (s0 < L) {
    const int c = std::min(s0, CMAX);
    const int b = std::min(L - s0, TILE_LOG - c);
    p.push_back({s0, b});
    s0 += b;
  }
  return p;
}

struct R16Pass {
  int s0, b, c;
};
// L <= 14: one pass; otherwise two: a fully contiguous first pass of up to 14 stages and a
// strided second pass with 2^c-element coalesced runs (c <= 6).
static std::vector<R16Pass> r16_plan(int L) {
  if (L <= R16_TILE_LOG) return {{0, L, 0}};
  const int b1 = std::min(R16_TILE_LOG, L - 4), b2 = L - b1;
  const int c2 = std::min({b1, R16_TILE_LOG - b2, MID_CMAX});
  return {{0, b1, 0}, {b1, b2, c2}};
}

static void r16_attrs() {
  static bool done = false;
  if (done) return;
  const int bytes = ((1 << R16_TILE_LOG) + (1 << (R16_TILE_LOG - 4))) * 4;
  HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_ntt_r16<true>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, bytes));
  HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_ntt_r16<false>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, bytes));
  const void* mids[] = {(const void*)&k_lde_mid<14>, (const void*)&k_lde_mid<15>, (const void*)&k_lde_mid<16>,
                        (const void*)&k_lde_mid<17>, (const void*)&k_lde_mid<18>,
                        (const void*)&k_lde_mid<19>, (const void*)&k_lde_mid<20>,
                        (const void*)&k_lde_mid<21>, (const void*)&k_lde_mid<22>,
                        (const void*)&k_lde_mid<23>};
  for (const void* f : mids)
    HIP_CHECK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, bytes));
  HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_ntt_tile<true, R16_TILE_LOG, false>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, bytes));
  HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_ntt_tile<false, R16_TILE_LOG, false>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, bytes));
  HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_ntt_tile<false, R16_TILE_LOG, true>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, bytes));
  HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_ntt_tile<true, R16_TILE_LOG, false, 4, false, true>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, bytes));
  HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_ntt_tile<false, R16_TILE_LOG, true, 4, false, true>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, bytes));
  HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_ntt_tile<true, R16_TILE_LOG, false, 4, true>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, bytes));
  HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_ntt_tile<false, R16_TILE_LOG, true, 4, true>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, bytes));
  const void* ws[] = {(const void*)&k_ntt_tile<true, R16_TILE_LOG, false, 4, false, false, true>,
                      (const void*)&k_ntt_tile<true, R16_TILE_LOG, false, 4, false, true, true>,
                      (const void*)&k_ntt_tile<false, R16_TILE_LOG, false, 4, false, false, true>,
                      (const void*)&k_ntt_tile<false, R16_TILE_LOG, false, 4, false, true, true>,
                      (const void*)&k_ntt_tile<false, R16_TILE_LOG, true, 4, false, false, true>,
                      (const void*)&k_ntt_tile<false, R16_TILE_LOG, true, 4, false, true, true>};
  for (const void* f : ws)
    HIP_CHECK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, bytes));
  done = true;
}

// BFZ_TILE_PERSIST=1: the 2^14 tiles run persistent with a prefetched next tile (A/B switch)
static bool tile_persist() {
  static const bool on = [] {
    const char* e = std::getenv("BFZ_TILE_PERSIST");
    return e && *e == '1';
  }();
  return on;
}
// Table twiddles loaded one window ahead in the 2^14 DIF tiles (profiles/r04/ab_twiddle_prefetch.txt:
// DIF pass 198 -> 185 us per 2^26 elements, DIT neutral, so DIF only); BFZ_TW_PREFETCH=0 / 1
// forces it off / on for both directions (A/B switch).
static int tw_prefetch() {
  static const int mode = [] {
    const char* e = std::getenv("BFZ_TW_PREFETCH");
    return e ? (*e == '1' ? 1 : 0) : 2;  // 2: DIF only
  }();
  return mode;
}
// 2^14 tiles with wave-local LDS exchanges (k_ntt_tile WS): default since
// profiles/r04/ab_tile_ws.txt (DIT pass 180 -> 167-172 us per 2^26 elements, DIF neutral, coset
// LDE 2^22 x 8 471 -> 466 us, bit-exact); BFZ_TILE_WS=0 turns it off (A/B switch)
static bool tile_ws() {
  static const bool on = [] {
    const char* e = std::getenv("BFZ_TILE_WS");
    return !(e && *e == '0');
  }();
  return on;
}
template <bool DIF, int B>
static void tile_launch(dim3 grid, const uint32_t* in, size_t is, uint32_t* dst, size_t ds,
                        const uint32_t* tw, hipStream_t st) {
  constexpr int R = 4;
  const size_t lds = ((size_t)1 << B) + ((size_t)1 << (B - R));
  const dim3 block(1 << (B - R));
  const bool din = !DIF && BFZ_NTT_REPS == 1 && ((uintptr_t)in & 15) == 0 && (is & 3) == 0;
  if constexpr (B == R16_TILE_LOG && BFZ_NTT_REPS == 1) {
    if (tile_ws()) {
      const bool pf = tw_prefetch() == 1 || (DIF && tw_prefetch() == 2);
      if (din) {
        if (pf)
          hipLaunchKernelGGL((k_ntt_tile<false, B, true, R, false, true, true>), grid, block, lds * 4,
                             st, in, dst, is, ds, tw, 0u, 0u);
        else
          hipLaunchKernelGGL((k_ntt_tile<false, B, true, R, false, false, true>), grid, block, lds * 4,
                             st, in, dst, is, ds, tw, 0u, 0u);
      } else if (pf) {
        hipLaunchKernelGGL((k_ntt_tile<DIF, B, false, R, false, true, true>), grid, block, lds * 4, st,
                           in, dst, is, ds, tw, 0u, 0u);
      } else {
        hipLaunchKernelGGL((k_ntt_tile<DIF, B, false, R, false, false, true>), grid, block, lds * 4, st,
                           in, dst, is, ds, tw, 0u, 0u);
      }
      return;
    }
    if (tw_prefetch() == 1 || (DIF && tw_prefetch() == 2)) {
      if (din)
        hipLaunchKernelGGL((k_ntt_tile<false, B, true, R, false, true>), grid, block, lds * 4, st, in,
                           dst, is, ds, tw, 0u, 0u);
      else
        hipLaunchKernelGGL((k_ntt_tile<DIF, B, false, R, false, true>), grid, block, lds * 4, st, in,
                           dst, is, ds, tw, 0u, 0u);
      return;
    }
  }
  if constexpr (B == R16_TILE_LOG && BFZ_NTT_REPS == 1) {
    const uint32_t ntiles = grid.x * grid.y;
    if (tile_persist() && ntiles > 512) {  // 2 blocks per CU (LDS-bound) x 256 CUs
      const dim3 pgrid(512);
      if (din)
        hipLaunchKernelGGL((k_ntt_tile<false, B, true, R, true>), pgrid, block, lds * 4, st, in, dst,
                           is, ds, tw, grid.x, ntiles);
      else
        hipLaunchKernelGGL((k_ntt_tile<DIF, B, false, R, true>), pgrid, block, lds * 4, st, in, dst,
                           is, ds, tw, grid.x, ntiles);
      return;
    }
  }
  if constexpr (!DIF && BFZ_NTT_REPS == 1) {
    if (din) {
      hipLaunchKernelGGL((k_ntt_tile<false, B, true, R>), grid, block, lds * 4, st, in, dst, is,
                         ds, tw, 0u, 0u);
      return;
    }
  }
  hipLaunchKernelGGL((k_ntt_tile<DIF, B, false, R>), grid, block, lds * 4, st, in, dst, is, ds,
                     tw, 0u, 0u);
}

template <bool DIF>
static bool tile_dispatch(int b, dim3 grid, const uint32_t* in, size_t is, uint32_t* dst,
                          size_t ds, const uint32_t* tw, hipStream_t st) {
  switch (b) {
    case 8: tile_launch<DIF, 8>(grid, in, is, dst, ds, tw, st); return true;
    case 9: tile_launch<DIF, 9>(grid, in, is, dst, ds, tw, st); return true;
    case 10: tile_launch<DIF, 10>(grid, in, is, dst, ds, tw, st); return true;
    case 11: tile_launch<DIF, 11>(grid, in, is, dst, ds, tw, st); return true;
    case 12: tile_launch<DIF, 12>(grid, in, is, dst, ds, tw, st); return true;
    case 13: tile_launch<DIF, 13>(grid, in, is, dst, ds, tw, st); return true;
    case 14:
      // 16-byte loads (DIT input) / stores (DIF output) need aligned rows
      if (use_mfma_tiles() && (DIF ? ((uintptr_t)dst & 15) == 0 && (ds & 3) == 0
                                   : ((uintptr_t)in & 15) == 0 && (is & 3) == 0)) {
        MfmaTables& M = mfma_tables();
        hipLaunchKernelGGL(k_tile14_mfma<DIF>, grid, dim3(MF_THREADS), MF_DATA * 4 + (DIF || !MF_LDSW ? 0 : 16384), st, in, dst, is,
                           ds, tw, (const v4i*)(DIF ? M.w_dif.p : M.w_dit.p),
                           (const uint32_t*)(DIF ? M.t_dif.p : M.t_dit.p));
        return true;
      }
      if constexpr (R16_TILE_LOG >= 14) {
        tile_launch<DIF, 14>(grid, in, is, dst, ds, tw, st);
        return true;
      }
      return false;
  }
  return false;
}

static void r16_launch(const R16Pass& p, const uint32_t* in, size_t is, uint32_t* dst, size_t ds,
                       int ncols, int L, bool dif, hipStream_t st) {
  Twiddles& T = twiddles();
  const int threads = 1 << (p.b + p.c - 4);
  const size_t lds = ((size_t)1 << (p.b + p.c)) + ((size_t)1 << (p.b + p.c - 4));
  dim3 grid(1u << (L - p.b - p.c), ncols);
  KernelProbe& probe = ntt_probe();
  hipEvent_t ev0 = probe.on ? probe.begin(st) : nullptr;
  if (p.s0 == 0 && p.c == 0 &&
      (dif ? tile_dispatch<true>(p.b, grid, in, is, dst, ds, (const uint32_t*)T.fwd.p, st)
           : tile_dispatch<false>(p.b, grid, in, is, dst, ds, (const uint32_t*)T.inv.p, st))) {
    // specialised contiguous pass
  } else if (dif)
    hipLaunchKernelGGL(k_ntt_r16<true>, grid, dim3(threads), lds * 4, st, in, dst, is, ds, p.s0,
                       p.b, p.c, (const uint32_t*)T.fwd.p);
  else
    hipLaunchKernelGGL(k_ntt_r16<false>, grid, dim3(threads), lds * 4, st, in, dst, is, ds, p.s0,
                       p.b, p.c, (const uint32_t*)T.inv.p);
  KCHECK();
  if (probe.on) probe.end(ev0, st, 8.0 * (double)((size_t)1 << L) * ncols);
}

void ntt_passes(const uint32_t* src, uint32_t* dst, size_t src_stride, size_t dst_stride, int ncols,
                int L, bool dif, hipStream_t st) {
  Twiddles& T = twiddles();
  T.ensure(std::max(L, 1));
  if (L >= 4) {
    r16_attrs();
    auto plan = r16_plan(L);
    if (dif) std::reverse(plan.begin(), plan.end());
    bool first = true;
    for (const R16Pass& p : plan) {
      r16_launch(p, first ? src : dst, first ? src_stride : dst_stride, dst, dst_stride, ncols, L,
                 dif, st);
      first = false;
    }
    return;
  }
  auto plan = ntt_plan(L);
  if (dif) std::reverse(plan.begin(), plan.end());
  bool first = true;
  for (auto [s0, b] : plan) {
    const int c = std::min(s0, CMAX);
    dim3 grid(1u << (L - b - c), ncols);
    const uint32_t* in = first ? src : dst;
    const size_t is = first ? src_stride : dst_stride;
    if (dif)
      hipLaunchKernelGGL(k_ntt_pass<true>, grid, dim3(256), 0, st, in, dst, is, dst_stride, s0, b,
                         c, T.fwd.p);
    else
      hipLaunchKernelGGL(k_ntt_pass<false>, grid, dim3(256), 0, st, in, dst, is, dst_stride, s0, b,
                         c, T.inv.p);
    KCHECK();
    first = false;
  }
  if (plan.empty() && src != dst)
    HIP_CHECK(hipMemcpy2DAsync(dst, dst_stride * 4, src, src_stride * 4, 4, ncols,
                               hipMemcpyDeviceToDevice, st));
}

namespace {
struct PowKey {
  uint32_t s;
  int L;
  bool operator<(const PowKey& o) const { return s != o.s ? s < o.s : L < o.L; }
};
std::map<PowKey, DBuf<uint32_t>>& pow_cache() {
  static auto* m = new std::map<PowKey, DBuf<uint32_t>>();
  return *m;
}
const uint32_t* scale_tables(uint32_t shift, int L, int B) {
  auto& cache = pow_cache();
  auto it = cache.find({shift, L});
  if (it != cache.end()) return it->second.p;
  const size_t nb = (size_t)1 << B;
  std::vector<uint32_t> h(4 * nb);
  const uint32_t ninv = minv(to_mont((uint32_t)(((uint64_t)1 << L) % P)));
  const uint32_t t = mmul(shift, two_adic_gen(L + 1));
  for (int which = 0; which < 2; which++) {
    const uint32_t base = which ? t : shift;
    uint32_t* lo = &h[2 * which * nb];
    uint32_t* hi = &h[(2 * which + 1) * nb];
    uint32_t a = ONE;
    for (size_t k = 0; k < nb; k++) { lo[k] = a; a = mmul(a, base); }
    const uint32_t step = a;  // base^(2^B)
    uint32_t b = ninv;
    for (size_t k = 0; k < nb; k++) { hi[k] = b; b = mmul(b, step); }
  }
  DBuf<uint32_t> d(4 * nb);
  // stream-ordered: a pooled buffer may still be read by kernels queued on stream()
  HIP_CHECK(hipMemcpyAsync(d.p, h.data(), h.size() * 4, hipMemcpyHostToDevice, stream()));
  HIP_CHECK(hipStreamSynchronize(stream()));
  const uint32_t* p = d.p;
  cache.emplace(PowKey{shift, L}, std::move(d));
  return p;
}
}  // namespace

void coset_lde(const uint32_t* evals, size_t n, int w, uint32_t shift, uint32_t* lde,
               hipStream_t st) {
  coset_lde_ex(evals, n, n, w, shift, lde, -1, st);
}

void coset_lde_ex(const uint32_t* evals, size_t src_stride, size_t n, int w, uint32_t shift,
                  uint32_t* lde, int only_half, hipStream_t st) {
  const int L = log2i(n);
  // the DFT of one half: its w columns of n at stride 2n; both halves: 2w columns at stride n
  uint32_t* dft_base = only_half >= 0 ? lde + (size_t)only_half * n : lde;
  const size_t dft_stride = only_half >= 0 ? 2 * n : n;
  const int dft_cols = only_half >= 0 ? w : 2 * w;
  if (L > R16_TILE_LOG) {  // iDFT pass 1 -> fused middle -> DFT last pass (3 HBM passes)
    Twiddles& T = twiddles();
    T.ensure(L);
    r16_attrs();
    const auto plan = r16_plan(L);  // {(0, b1, 0), (b1, b2, c2)}
    const R16Pass& p1 = plan[0];
    const R16Pass& p2 = plan[1];
    DBuf<uint32_t> coef(n * (size_t)w);
    r16_launch(p1, evals, src_stride, coef.p, n, w, L, false, st);
    const int B = (L + 1) / 2;
    const uint32_t* pw = scale_tables(shift, L, B);
    MidPowers mp;
    const uint64_t D = (uint64_t)1 << (p2.s0 + p2.b - 4);
    const uint32_t gs = mpow(shift, D), gt = mpow(mmul(shift, two_adic_gen(L + 1)), D);
    uint32_t a = ONE, c = ONE;
    for (int i = 0; i < 16; i++) {
      mp.lo[i] = a;
      mp.hi[i] = c;
      a = mmul(a, gs);
      c = mmul(c, gt);
    }
    const int threads = 1 << (p2.b + p2.c - 4);
    const size_t ldsz = ((size_t)1 << (p2.b + p2.c)) + ((size_t)1 << (p2.b + p2.c - 4));
    KernelProbe& probe = ntt_probe();
    hipEvent_t ev0 = probe.on ? probe.begin(st) : nullptr;
    const dim3 grid(1u << (L - p2.b - p2.c), w);
#define BFZ_MID(LL)                                                                              \
  case LL:                                                                                       \
    static_assert(MidPlan<LL>::b2 >= 4, "plan");                                                 \
    hipLaunchKernelGGL(k_lde_mid<LL>, grid, dim3(threads), ldsz * 4, st, (const uint32_t*)coef.p, \
                       n, lde, n, (const uint32_t*)T.inv.p, (const uint32_t*)T.fwd.p, pw, B, mp, \
                       only_half);                                                               \
    break;
    switch (L) {
      BFZ_MID(14) BFZ_MID(15) BFZ_MID(16) BFZ_MID(17) BFZ_MID(18) BFZ_MID(19) BFZ_MID(20) BFZ_MID(21)
      BFZ_MID(22) BFZ_MID(23)
      default: throw std::runtime_error("coset_lde: log height above 23");
    }
#undef BFZ_MID
    KCHECK();
    if (probe.on) probe.end(ev0, st, (only_half >= 0 ? 8.0 : 12.0) * (double)n * w);
    r16_launch(p1, dft_base, dft_stride, dft_base, dft_stride, dft_cols, L, true, st);
    return;
  }
  DBuf<uint32_t> coef(n * (size_t)w);
  ntt_passes(evals, coef.p, src_stride, n, w, L, /*dif=*/false, st);
  const int B = (L + 1) / 2;
  const uint32_t* pw = scale_tables(shift, L, B);
  dim3 grid(std::min<unsigned>(ceil_div(n, 256), 4096), w);
  hipLaunchKernelGGL(k_scale_split, grid, dim3(256), 0, st, coef.p, lde, n, B, pw, only_half);
  KCHECK();
  ntt_passes(dft_base, dft_base, dft_stride, dft_stride, dft_cols, L, /*dif=*/true, st);
  // coef goes back to the pool here; every consumer is ordered on the same stream.
}

// ---------------------------------------------------------------- residue-class shards
// A row shard of a sharded proof: rank k holds bit-reversed LDE positions
// [k m, (k+1) m), m = 2n / G, i.e. the natural points i = G t + r (r = bitrev_G(k)), which
// form the coset a <w_m> with a = shift w_2n^r.  With the coefficients c_j of the trace
// interpolant,  p(a w_m^t) = sum_(u < m) w_m^(u t) d_u,  d_u = sum_l c_(u + l m) a^(u + l m),
// so the shard is a size-m forward DIF of d (natural in -> bit-reversed out, exactly the shard's
// position order): no exchange between ranks, the iDFT is the only full-size transform.

// d[u] = sum_(l < n/m) coef[u + l m] a^(u + l m) / n  (coef = n c: the iDFT leaves 1/n out;
// a^j / n = A[j & mask] * AH[j >> B] with the 1/n folded into AH)
struct ColMap {  // output column y reads input column col[y]
  uint8_t col[64];
};
__global__ __launch_bounds__(256) void k_fold_residue(const uint32_t* __restrict__ coef, size_t n,
                                                      uint32_t* __restrict__ out, size_t m, int B,
                                                      const uint32_t* __restrict__ pw, ColMap cm) {
  const uint32_t* c = coef + (size_t)cm.col[blockIdx.y] * n;
  uint32_t* o = out + (size_t)blockIdx.y * m;
  const size_t mask = ((size_t)1 << B) - 1, nb = mask + 1;
  for (size_t u = (size_t)blockIdx.x * blockDim.x + threadIdx.x; u < m;
       u += (size_t)gridDim.x * blockDim.x) {
    uint32_t acc = 0;
    for (size_t j = u; j < n; j += m) acc = madd(acc, mmul(c[j], mmul(pw[j & mask], pw[nb + (j >> B)])));
    o[u] = acc;
  }
}

// Two-level power table of a (with 1/2^L folded into the high half), cached per (a, L).
static const uint32_t* residue_powers(uint32_t a, int L, int B) {
  static auto* cache = new std::map<std::pair<uint32_t, int>, DBuf<uint32_t>>();
  auto it = cache->find({a, L});
  if (it != cache->end()) return it->second.p;
  const size_t nb = (size_t)1 << B;
  std::vector<uint32_t> h(2 * nb);
  uint32_t x = ONE;
  for (size_t k = 0; k < nb; k++) { h[k] = x; x = mmul(x, a); }
  const uint32_t step = x;  // a^(2^B)
  uint32_t y = minv(to_mont((uint32_t)(((uint64_t)1 << L) % P)));
  for (size_t k = 0; k < nb; k++) { h[nb + k] = y; y = mmul(y, step); }
  DBuf<uint32_t> d(2 * nb);
  HIP_CHECK(hipMemcpyAsync(d.p, h.data(), h.size() * 4, hipMemcpyHostToDevice, stream()));
  HIP_CHECK(hipStreamSynchronize(stream()));
  const uint32_t* p = d.p;
  cache->emplace(std::make_pair(a, L), std::move(d));
  return p;
}

void lde_coefficients(const uint32_t* evals, size_t n, int w, uint32_t* coef, hipStream_t st) {
  ntt_passes(evals, coef, n, n, w, log2i(n), /*dif=*/false, st);
}

void coset_residue(const uint32_t* coef, size_t n, int w, uint32_t shift, int logG, int r,
                   uint32_t* out, hipStream_t st) {
  std::vector<int> all(w);
  for (int c = 0; c < w; c++) all[c] = c;
  coset_residue_cols(coef, n, all, shift, logG, r, out, st);
}

void coset_residue_cols(const uint32_t* coef, size_t n, const std::vector<int>& cols,
                        uint32_t shift, int logG, int r, uint32_t* out, hipStream_t st) {
  const int w = (int)cols.size();
  if (w < 1 || w > 64) throw std::runtime_error("coset_residue: 1..64 columns");
  ColMap map{};
  for (int y = 0; y < w; y++) map.col[y] = (uint8_t)cols[y];
  const int L = log2i(n);
  if (logG < 1 || logG > L + 1) throw std::runtime_error("coset_residue: bad shard count");
  const size_t m = (2 * n) >> logG;
  const uint32_t a = mmul(shift, mpow(two_adic_gen(L + 1), (uint64_t)r));
  const int B = (L + 1) / 2;
  const uint32_t* pw = residue_powers(a, L, B);
  const dim3 grid(std::min<unsigned>(ceil_div(m, 256), 2048), w);
  hipLaunchKernelGGL(k_fold_residue, grid, dim3(256), 0, st, coef, n, out, m, B, pw, map);
  KCHECK();
  ntt_passes(out, out, m, m, w, log2i(m), /*dif=*/true, st);
}

void transpose_to_rowmajor(const uint32_t* colmajor, size_t H, int w, uint32_t* rowmajor,
                           hipStream_t st) {
  hipLaunchKernelGGL(k_transpose_rowmajor, dim3(ceil_div(H * (size_t)w, 256)), dim3(256), 0, st,
                     colmajor, rowmajor, H, w);
  KCHECK();
}

// Counts words >= p (non-canonical Montgomery words) into *count (atomic, wave-aggregated).
__global__ __launch_bounds__(256) void k_count_noncanonical(const uint32_t* __restrict__ a,
                                                            size_t n, unsigned* count) {
  unsigned bad = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x)
    bad += a[i] >= kb::P;
  const unsigned long long any = __ballot(bad != 0);
  if (any && (threadIdx.x & 63) == 0) atomicAdd(count, 1u);
}

size_t count_noncanonical(const uint32_t* d, size_t n, hipStream_t st) {
  DBuf<unsigned> c(1);
  HIP_CHECK(hipMemsetAsync(c.p, 0, sizeof(unsigned), st));
  hipLaunchKernelGGL(k_count_noncanonical, dim3(std::min<size_t>(ceil_div(n, 256), 4096)),
                     dim3(256), 0, st, d, n, c.p);
  KCHECK();
  unsigned h = 0;
  HIP_CHECK(hipMemcpyAsync(&h, c.p, sizeof(unsigned), hipMemcpyDeviceToHost, st));
  HIP_CHECK(hipStreamSynchronize(st));
  return h;
}

void transpose_bitrev(const uint32_t* rowmajor, size_t n, int w, uint32_t* colmajor,
                      hipStream_t st) {
  hipLaunchKernelGGL(k_transpose_bitrev, dim3(ceil_div(n, 64)), dim3(256), 0, st, rowmajor,
                     colmajor, n, w, log2i(n));
  KCHECK();
}

}  // namespace bfz
