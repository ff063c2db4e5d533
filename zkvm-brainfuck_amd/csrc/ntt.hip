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
#include "ntt_dev.h"

#include <cstdlib>
#include <mutex>
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


// 2^14 elements per tile: 1024 threads x 16 (2^13 tiles measured +7%)
constexpr int R16_TILE_LOG = 14;
// Second-pass tiles take 2^c adjacent columns (2^c * 4 B coalesced runs); c <= MID_CMAX
// (16- or 64-column runs measured +8% / +2%).
constexpr int MID_CMAX = 5;

__device__ __forceinline__ int lds_pad(int idx, int c) { return c < 5 ? idx + (idx >> 4) : idx; }

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
// DIN (DIT only): the first window (g0 = 0) holds the 16 consecutive words tid*16 + i, read
// straight from HBM as four 16-byte loads (no LDS staging, one barrier fewer); the launch picks
// it when the source rows are 16-byte aligned.  The DIT's last window (g0 = B - 4) holds elements
// tid + i T: those go straight from registers to HBM (one coalesced 256-byte segment per wave
// instruction; -2.4% per pass).  The DIF's first window would read the same way, but measured
// slower than LDS staging (+4.5%, profiles/r02/ntt_lab_variants.txt), so a DIF pass keeps it.
// TWPF: each window's table twiddles are loaded one window ahead (into registers, double
// buffered) instead of at the window's start, where every wave of the block would wait for the
// L2 round trip at the same time (the waves run in lockstep between the LDS exchanges).  Shipped
// for the 2^14 tiles: DIF pass 198 -> 185 us per 2^26 elements (profiles/r04/
// ab_twiddle_prefetch.txt); the DIT pass, neutral with flat loads, 86.5 -> 79 us per 2^25 once the
// loads were buffer loads with scalar offsets (profiles/r05/ab_ntt_variants.txt).
// WS (B = 14): windows g0 = 0, 4, 6, 10 (DIT; the DIF the reverse).  The threads of a wave hold
// the same 1024 consecutive elements (bits [10, 14) = the wave index) in every window with
// g0 <= 6, so the exchanges between such windows go through the wave's own LDS region with a
// wave-level fence instead of a block barrier: one block barrier per DIT tile instead of three
// (profiles/r04/ab_tile_ws.txt: DIT pass 180 -> 167-172 us per 2^26 elements).
// (Measured and dropped, DESIGN.md §7: persistent tiles with the next tile's loads prefetched,
// radix-32 windows, matrix-core tiles -- scripts/ubench_ntt_mfma.hip.)
template <bool DIF, int B, bool DIN = false, bool TWPF = false, bool WS = false>
__global__ __launch_bounds__(1 << (B - 4)) void k_ntt_tile(const uint32_t* __restrict__ src,
                                                           uint32_t* __restrict__ dst,
                                                           size_t src_stride, size_t dst_stride,
                                                           const uint32_t* __restrict__ tw) {
  static_assert(B >= 8 && B <= R16_TILE_LOG, "tile");
  static_assert(!DIN || !DIF, "direct first window: DIT passes only");
  static_assert(!WS || B >= 13, "wave-local windows: 2^13 / 2^14 tiles");
  constexpr int R = 4, E = 1 << R, T = 1 << (B - R), NW = (B + R - 1) / R;
  // WS DIF: the first window (g0 = B - 4) holds elements tid + i T, a coalesced HBM order, so
  // it is read straight from HBM (no LDS staging, one block barrier fewer), and the last window
  // leaves each wave its own 1024 consecutive outputs, which the wave stores itself: one block
  // barrier per DIF tile (DIF pass 162 -> 153-156 us per 2^26 elements, profiles/r05/
  // ab_ntt_variants.txt; in round 2, before the wave-local windows, direct reads measured +4.5%)
  constexpr bool DIFIN = DIF && WS;
  extern __shared__ uint32_t lds[];
  const int tid = threadIdx.x;
  const int tpad = tid + (tid >> R);
  const uint32_t* S = src + (size_t)blockIdx.y * src_stride + ((size_t)blockIdx.x << B);
  uint32_t* D = dst + (size_t)blockIdx.y * dst_stride + ((size_t)blockIdx.x << B);
  uint32_t x[E];
  if constexpr (DIN) {
    const uint4* s4 = reinterpret_cast<const uint4*>(S + (tid << R));
#pragma unroll
    for (int q = 0; q < E / 4; q++) {
      const uint4 v = s4[q];
      x[4 * q] = v.x; x[4 * q + 1] = v.y; x[4 * q + 2] = v.z; x[4 * q + 3] = v.w;
    }
  } else if constexpr (DIFIN) {
    const __amdgpu_buffer_rsrc_t rs = rsrc_of(S);
#pragma unroll
    for (int i = 0; i < E; i++) x[i] = ld_b(rs, tid * 4u, (uint32_t)(i * T) * 4u);
  } else {
    const __amdgpu_buffer_rsrc_t rs = rsrc_of(S);
#pragma unroll
    for (int i = 0; i < E; i++) lds[i * (T + T / E) + tpad] = ld_b(rs, tid * 4u, (uint32_t)(i * T) * 4u);
  }
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
      load_window_tw<R>(pre[0], win_g0(0), lo, hi, tid & ((1 << win_g0(0)) - 1), tw);
    }
  }
#pragma unroll
  for (int w = 0; w < NW; w++) {
    const int g0 = win_g0(w);
    const uint32_t m_low = tid & ((1 << g0) - 1);
    const uint32_t m_base = m_low | ((uint32_t)(tid >> g0) << (g0 + R));
    const uint32_t pb = m_base + (m_base >> R);
    const bool direct_out = !DIF && w == NW - 1;
    if (!(DIN || DIFIN) || w > 0) {
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
                          tid & ((1 << win_g0(w + 1)) - 1), tw);
      }
    }
    if (g0 == 0)
      r16_window<DIF, true, false, R>(x, g0, kk_lo, kk_hi, 0, m_low, 0, tw);
    else if (TWPF)
      r16_window<DIF, false, true, R, true>(x, g0, kk_lo, kk_hi, 0, m_low, 0, tw, pre[w & 1]);
    else
      r16_window<DIF, false, true, R>(x, g0, kk_lo, kk_hi, 0, m_low, 0, tw);
    if (direct_out) {
      const __amdgpu_buffer_rsrc_t rd = rsrc_of(D);
#pragma unroll
      for (int i = 0; i < E; i++) st_b(rd, tid * 4u, (uint32_t)(i * T) * 4u, x[i]);
    } else {
#pragma unroll
      for (int i = 0; i < E; i++) lds[pb + (i << g0) + ((i << g0) >> R)] = x[i];
    }
  }
  if constexpr (DIFIN) {
    // the last window (g0 = 0) left each wave's own 1024 consecutive elements in its own LDS
    // region: the wave stores them itself, 64 consecutive words per instruction (no block barrier)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const __amdgpu_buffer_rsrc_t rd = rsrc_of(D);
    const uint32_t e0 = (uint32_t)(tid >> 6) * 1024u + (tid & 63);
#pragma unroll
    for (int j = 0; j < E; j++) {
      const uint32_t e = e0 + 64u * j;
      st_b(rd, e0 * 4u, 256u * j, lds[e + (e >> R)]);
    }
  } else if constexpr (DIF) {
    __syncthreads();
    const __amdgpu_buffer_rsrc_t rd = rsrc_of(D);
#pragma unroll
    for (int i = 0; i < E; i++) st_b(rd, tid * 4u, (uint32_t)(i * T) * 4u, lds[i * (T + T / E) + tpad]);
  }
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

#ifndef BFZ_MID_CPB
#define BFZ_MID_CPB 1
#endif
// Columns per block (one tile position, its stage twiddles reused from the first column): 2 and 4
// cut k_lde_mid<22>'s FETCH_SIZE 221 -> 205 / 194 MB per launch but not its time, and cost
// +0.08 ms of NTT kernel time per proof at 2 (profiles/r06/ab_mid_cpb.txt): 1.
constexpr int MID_CPB = BFZ_MID_CPB;

// Where k_lde_mid writes: column y's half h at lde + y dstride + h hoff (the coset LDE: 2n, n;
// a 2-GPU shard, one half per rank: n, 0), plus -- coef != nullptr -- the coefficients k in
// [j0, j0 + len) of column y at coef + y n (the sharded proof's opening range).
struct MidOut {
  size_t dstride, hoff;
  uint32_t* coef;
  size_t j0, len;
};

template <int L>
__device__ __forceinline__ void lde_mid_col(
    const uint32_t* __restrict__ src, size_t src_stride, uint32_t* __restrict__ lde, size_t n,
    const uint32_t* __restrict__ tw_inv, const uint32_t* __restrict__ tw_fwd,
    const uint32_t* __restrict__ pw, int B, const MidPowers& mp, int only_half, uint32_t by,
    const MidOut& mo) {
  constexpr int s0 = MidPlan<L>::b1, b = MidPlan<L>::b2, c = MidPlan<L>::c2;
  extern __shared__ uint32_t lds[];
  const int tid = threadIdx.x;
  const int nlo_log = s0 - c;
  const uint32_t bx = blockIdx.x;
  const size_t lo_blk = bx & ((1u << nlo_log) - 1);
  const size_t hi = (size_t)bx >> nlo_log;
  const size_t base = (hi << (s0 + b)) + (lo_blk << c);
  const uint32_t* S = src + (size_t)by * src_stride + base;
  uint32_t* D = lde + (size_t)by * mo.dstride + base;
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
      const __amdgpu_buffer_rsrc_t rs = rsrc_of(S);
      const uint32_t off = ((m_base << s0) + lo) * 4u;  // i's part of the index is uniform
#pragma unroll
      for (int i = 0; i < 16; i++) x[i] = ld_b(rs, off, ((uint32_t)i << (g0 + s0)) * 4u);
    } else {
      __syncthreads();
#pragma unroll
      for (int i = 0; i < 16; i++)
        x[i] = lds[lds_pad((int)(((m_base | ((uint32_t)i << g0)) << c) | lo), c)];
    }
    const int kk_lo = max(0, done_lo - g0);
    done_lo = g0 + 4;
    r16_window<false, false, true>(x, g0, kk_lo, 4, s0, m_low, lo_g, tw_inv);
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
    if (mo.coef) {  // the sharded proof's opening range of the coefficients (see k_coef_fold)
      uint32_t* C = mo.coef + (size_t)by * n;
#pragma unroll
      for (int i = 0; i < 16; i++) {
        const size_t k = k0 + ((size_t)i << (L - 4));
        if (k - mo.j0 < mo.len) C[k] = coef[i];
      }
    }
    const size_t mask = ((size_t)1 << B) - 1, nb = mask + 1;
    const uint32_t S0 = mmul(pw[k0 & mask], pw[nb + (k0 >> B)]);
    const uint32_t T0 = mmul(pw[2 * nb + (k0 & mask)], pw[3 * nb + (k0 >> B)]);
    for (int half = 0; half < 2; half++) {
      if (only_half >= 0 && half != only_half) continue;  // uniform across the block
      const uint32_t P0 = half ? T0 : S0;
#pragma unroll
      for (int i = 0; i < 16; i++) x[i] = mmul(coef[i], mmul(P0, half ? mp.hi[i] : mp.lo[i]));
      if (half && nwin > 1) __syncthreads();  // the lo half's last LDS reads are done
      uint32_t* Dh = D + (size_t)half * mo.hoff;
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
        r16_window<true, false, true>(x, gg, 0, kk_hi, s0, m_low, lo_g, tw_fwd);
        if (w == nwin - 1) {
          const __amdgpu_buffer_rsrc_t rd = rsrc_of(Dh);
          const uint32_t off = ((mb << s0) + lo) * 4u;
#pragma unroll
          for (int i = 0; i < 16; i++) st_b(rd, off, ((uint32_t)i << (gg + s0)) * 4u, x[i]);
        } else {
#pragma unroll
          for (int i = 0; i < 16; i++)
            lds[lds_pad((int)(((mb | ((uint32_t)i << gg)) << c) | lo), c)] = x[i];
        }
      }
    }
  }
}

// Sharded LDE, fused: the second iDFT pass of a column (stages s0.., as the
// middle pass above) leaves each thread 16 coefficients n c_k at k = k0 + i D (D = 2^(L-4));
// instead of a coset DFT the thread stores the coefficients of the rank's opening range and
// folds them onto the rank's residue coset in registers -- d_u = a^u/n sum_l c_(u + l m) (a^m)^l
// with u = k0 + i0 D, i0 < m / D (the terms of an output are i0 + l m/D of the same thread) --
// plus the next-row residue for the columns the quotient reads there.  The coefficients are
// never read back for the folds (round 5 read them twice from HBM, once per residue).
struct ResidueFold {
  uint32_t A[4];       // halving stage j (h = 8 >> j): (a^m)^(h / S)
  uint32_t Q[16];      // (a^D)^i
  const uint32_t* pw;  // a^j / n two-level table (residue_powers)
  uint32_t* out;       // m x w
};
struct CoefFold {
  uint32_t* coef;   // coefficients (column stride n), written for k in [j0, j0 + len)
  size_t j0, len, m;
  int B, S;          // table split; S = m / D outputs per thread
  ResidueFold r[2];  // r[1]: the next-row residue (out == nullptr: none)
  uint8_t nidx[64];  // input column -> r[1] output column (0xff: not read at the next row)
};

// R > 0 (S = 2^R outputs per thread, G = 2^(5 - R) ranks): the thread's S outputs d_u are the
// first radix-S window of the residue's size-m DIF (stride D = m / S), and the block's outputs
// are a whole tile of its strided stages [s0, log m): those run here too (radix-S windows through
// LDS), so only the contiguous tile pass of stages [0, s0) is left (residue_dft).  R = 0: the
// folds alone, S at run time.
template <int L, int R>
__device__ __forceinline__ void coef_fold_col(const uint32_t* __restrict__ src, size_t n,
                                              const uint32_t* __restrict__ tw_inv,
                                              const uint32_t* __restrict__ tw_fwd,
                                              const CoefFold& cf, uint32_t by) {
  constexpr int s0 = MidPlan<L>::b1, b = MidPlan<L>::b2, c = MidPlan<L>::c2;
  extern __shared__ uint32_t lds[];
  const int tid = threadIdx.x;
  const int nlo_log = s0 - c;
  const uint32_t bx = blockIdx.x;
  const size_t lo_blk = bx & ((1u << nlo_log) - 1);
  const size_t hi = (size_t)bx >> nlo_log;
  const size_t base = (hi << (s0 + b)) + (lo_blk << c);
  const uint32_t* S = src + (size_t)by * n + base;
  const int lo = tid & ((1 << c) - 1);
  const uint32_t lo_g = (uint32_t)(lo_blk << c) + lo;
  const int rest = tid >> c;
  const int nwin = (b + 3) >> 2;
  uint32_t x[16];
  int done_lo = 0;
#pragma unroll
  for (int w = 0; w < nwin; w++) {  // iDFT, as lde_mid_col
    const int g0 = min(4 * w, b - 4);
    const uint32_t m_low = rest & ((1 << g0) - 1);
    const uint32_t m_base = m_low | ((uint32_t)(rest >> g0) << (g0 + 4));
    if (w == 0) {
      const __amdgpu_buffer_rsrc_t rs = rsrc_of(S);
      const uint32_t off = ((m_base << s0) + lo) * 4u;
#pragma unroll
      for (int i = 0; i < 16; i++) x[i] = ld_b(rs, off, ((uint32_t)i << (g0 + s0)) * 4u);
    } else {
      __syncthreads();
#pragma unroll
      for (int i = 0; i < 16; i++)
        x[i] = lds[lds_pad((int)(((m_base | ((uint32_t)i << g0)) << c) | lo), c)];
    }
    const int kk_lo = max(0, done_lo - g0);
    done_lo = g0 + 4;
    r16_window<false, false, true>(x, g0, kk_lo, 4, s0, m_low, lo_g, tw_inv);
    if (w < nwin - 1) {
#pragma unroll
      for (int i = 0; i < 16; i++)
        lds[lds_pad((int)(((m_base | ((uint32_t)i << g0)) << c) | lo), c)] = x[i];
    }
  }
  const int g0 = b - 4;
  const uint32_t m_base = (rest & ((1 << g0) - 1)) | ((uint32_t)(rest >> g0) << (g0 + 4));
  const size_t k0 = base + ((size_t)m_base << s0) + lo;
  constexpr size_t D = (size_t)1 << (L - 4);
  uint32_t* C = cf.coef + (size_t)by * n;
#pragma unroll
  for (int i = 0; i < 16; i++) {
    const size_t k = k0 + (size_t)i * D;
    if (k - cf.j0 < cf.len) C[k] = x[i];  // the rank's opening range only
  }
  const size_t mask = ((size_t)1 << cf.B) - 1, nb = mask + 1;
  const int SS = R ? 1 << R : cf.S;
#pragma unroll
  for (int q = 0; q < 2; q++) {
    const ResidueFold& rf = cf.r[q];
    if (!rf.out) break;  // uniform
    const int oc = q ? cf.nidx[by] : (int)by;
    if (oc == 0xff) break;  // uniform: the whole block is one column
    // y[i0] = sum_l x[i0 + l S] (a^m)^l by halving stages y[i] += y[i + h] (a^m)^(h/S), h = 8..S
    uint32_t y[16];
#pragma unroll
    for (int i = 0; i < 16; i++) y[i] = x[i];
#pragma unroll
    for (int st = 0; st < 4; st++) {
      const int h = 8 >> st;
      if (h < SS) break;
#pragma unroll
      for (int i = 0; i < h; i++) y[i] = madd(y[i], mmul(y[i + h], rf.A[st]));
    }
    const uint32_t ak0 = mmul(rf.pw[k0 & mask], rf.pw[nb + (k0 >> cf.B)]);  // a^k0 / n
    if constexpr (R == 0) {
      uint32_t* O = rf.out + (size_t)oc * cf.m + k0;
#pragma unroll
      for (int i = 0; i < 16; i++)
        if (i < SS) O[(size_t)i * D] = mmul(y[i], mmul(ak0, rf.Q[i]));
    } else {
      constexpr int E = 1 << R, bp = b - 4 + R, nw = (bp + R - 1) / R;
      uint32_t z[E];
#pragma unroll
      for (int i = 0; i < E; i++) z[i] = mmul(y[i], mmul(ak0, rf.Q[i]));
      uint32_t* O = rf.out + (size_t)oc * cf.m + base;
      __syncthreads();  // the previous phase's LDS reads are done
      int done_hi = bp;
#pragma unroll
      for (int w = 0; w < nw; w++) {  // DIF stages [s0, s0 + bp) of the size-m transform
        const int gg = max(bp - R - R * w, 0);
        const uint32_t m_low = rest & ((1 << gg) - 1);
        const uint32_t mb = m_low | ((uint32_t)(rest >> gg) << (gg + R));
        if (w > 0) {
          __syncthreads();
#pragma unroll
          for (int i = 0; i < E; i++)
            z[i] = lds[lds_pad((int)(((mb | ((uint32_t)i << gg)) << c) | lo), c)];
        }
        const int kk_hi = min(R, done_hi - gg);
        done_hi = gg;
        r16_window<true, false, true, R>(z, gg, 0, kk_hi, s0, m_low, lo_g, tw_fwd);
        if (w == nw - 1) {
#pragma unroll
          for (int i = 0; i < E; i++)
            O[((size_t)mb << s0) + lo + ((size_t)i << (gg + s0))] = z[i];
        } else {
#pragma unroll
          for (int i = 0; i < E; i++)
            lds[lds_pad((int)(((mb | ((uint32_t)i << gg)) << c) | lo), c)] = z[i];
        }
      }
    }
  }
}

template <int L, int R>
__global__ __launch_bounds__(1 << (MidPlan<L>::b2 + MidPlan<L>::c2 - 4)) void k_coef_fold(
    const uint32_t* __restrict__ src, size_t n, const uint32_t* __restrict__ tw_inv,
    const uint32_t* __restrict__ tw_fwd, CoefFold cf) {
  coef_fold_col<L, R>(src, n, tw_inv, tw_fwd, cf, blockIdx.y);
}

template <int L>
__global__ __launch_bounds__(1 << (MidPlan<L>::b2 + MidPlan<L>::c2 - 4)) void k_lde_mid(
    const uint32_t* __restrict__ src, size_t src_stride, uint32_t* __restrict__ lde, size_t n,
    const uint32_t* __restrict__ tw_inv, const uint32_t* __restrict__ tw_fwd,
    const uint32_t* __restrict__ pw, int B, MidPowers mp, int only_half, int w, MidOut mo) {
  for (int cc = 0; cc < MID_CPB; cc++) {
    const uint32_t by = blockIdx.y * MID_CPB + cc;
    if (by >= (uint32_t)w) break;  // uniform across the block
    if (cc) __syncthreads();       // the previous column's last LDS reads are done
    lde_mid_col<L>(src, src_stride, lde, n, tw_inv, tw_fwd, pw, B, mp, only_half, by, mo);
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

// Coset LDE of a column of n <= 2^TINY_LOG_MAX rows in one block, through LDS: iDFT (DIT,
// bit-reversed in -> natural coefficients, no 1/n), the coset scale of both halves (as
// k_scale_split), the DIF of each half.  At these sizes the general path's three launches
// (iDFT, k_scale_split, DFT) cost more than their work.
constexpr int TINY_LOG_MAX = 8;
__global__ __launch_bounds__(256) void k_lde_tiny(const uint32_t* __restrict__ evals,
                                                  size_t src_stride, uint32_t* __restrict__ lde,
                                                  int L, const uint32_t* __restrict__ tw_inv,
                                                  const uint32_t* __restrict__ tw_fwd,
                                                  const uint32_t* __restrict__ pw, int B,
                                                  int only_half) {
  __shared__ uint32_t a[1 << TINY_LOG_MAX], h[2][1 << TINY_LOG_MAX];
  const int n = 1 << L, tid = threadIdx.x;
  const uint32_t* S = evals + (size_t)blockIdx.x * src_stride;
  if (tid < n) a[tid] = S[tid];
  __syncthreads();
  for (int s = 0; s < L; s++) {
    const int hh = 1 << s;
    if (tid < n / 2) {
      const int j = tid & (hh - 1), i0 = ((tid >> s) << (s + 1)) + j, i1 = i0 + hh;
      const uint32_t u = a[i0], v = mmul(a[i1], tw_inv[hh + j]);
      a[i0] = madd(u, v);
      a[i1] = msub(u, v);
    }
    __syncthreads();
  }
  const int mask = (1 << B) - 1, nb = mask + 1;
  if (tid < n) {
    const uint32_t c = a[tid];
    const int kl = tid & mask, kh = tid >> B;
    h[0][tid] = mmul(c, mmul(pw[kl], pw[nb + kh]));
    h[1][tid] = mmul(c, mmul(pw[2 * nb + kl], pw[3 * nb + kh]));
  }
  __syncthreads();
  for (int s = L - 1; s >= 0; s--) {
    const int hh = 1 << s;
    if (tid < n / 2) {
      const int j = tid & (hh - 1), i0 = ((tid >> s) << (s + 1)) + j, i1 = i0 + hh;
      const uint32_t w = tw_fwd[hh + j];
#pragma unroll
      for (int q = 0; q < 2; q++) {
        const uint32_t u = h[q][i0], v = h[q][i1];
        h[q][i0] = madd(u, v);
        h[q][i1] = mmul(msub(u, v), w);
      }
    }
    __syncthreads();
  }
  uint32_t* D = lde + (size_t)blockIdx.x * 2 * n;
  if (tid < n) {
    if (only_half != 1) D[tid] = h[0][tid];
    if (only_half != 0) D[n + tid] = h[1][tid];
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

// The 2^14 tiles and the middle passes use more than the default 64 KiB of dynamic LDS.
static void r16_attrs() {
  static std::once_flag once;
  std::call_once(once, [] {
  const int bytes = ((1 << R16_TILE_LOG) + (1 << (R16_TILE_LOG - 4))) * 4;
  const void* fs[] = {(const void*)&k_ntt_r16<true>, (const void*)&k_ntt_r16<false>,
                      (const void*)&k_lde_mid<14>, (const void*)&k_lde_mid<15>,
                      (const void*)&k_lde_mid<16>, (const void*)&k_lde_mid<17>,
                      (const void*)&k_lde_mid<18>, (const void*)&k_lde_mid<19>,
                      (const void*)&k_lde_mid<20>, (const void*)&k_lde_mid<21>,
                      (const void*)&k_lde_mid<22>, (const void*)&k_lde_mid<23>,
                      (const void*)&k_ntt_tile<true, R16_TILE_LOG, false, true, true>,
                      (const void*)&k_ntt_tile<false, R16_TILE_LOG, true, true, true>,
                      (const void*)&k_ntt_tile<false, R16_TILE_LOG, false, true, true>};
  for (const void* f : fs)
    HIP_CHECK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, bytes));
#define BFZ_CF_ATTR(LL)                                                                        \
  for (const void* f : {(const void*)&k_coef_fold<LL, 0>, (const void*)&k_coef_fold<LL, 2>,   \
                        (const void*)&k_coef_fold<LL, 3>})                                     \
    HIP_CHECK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, bytes));
  BFZ_CF_ATTR(15) BFZ_CF_ATTR(16) BFZ_CF_ATTR(17) BFZ_CF_ATTR(18) BFZ_CF_ATTR(19) BFZ_CF_ATTR(20)
  BFZ_CF_ATTR(21) BFZ_CF_ATTR(22) BFZ_CF_ATTR(23)
#undef BFZ_CF_ATTR
  });
}

// One contiguous tile pass: the 2^14 tiles run wave-local (WS) with their twiddles one window
// ahead (TWPF); a DIT reads its first window straight from HBM when the rows are 16-byte aligned
// (DIN).
template <bool DIF, int B>
static void tile_launch(dim3 grid, const uint32_t* in, size_t is, uint32_t* dst, size_t ds,
                        const uint32_t* tw, hipStream_t st) {
  const size_t lds = ((size_t)1 << B) + ((size_t)1 << (B - 4));
  const dim3 block(1 << (B - 4));
  const bool din = !DIF && ((uintptr_t)in & 15) == 0 && (is & 3) == 0;
  constexpr bool WS = B == R16_TILE_LOG;
  if constexpr (DIF)
    hipLaunchKernelGGL((k_ntt_tile<true, B, false, WS, WS>), grid, block, lds * 4, st, in, dst, is,
                       ds, tw);
  else if (din)
    hipLaunchKernelGGL((k_ntt_tile<false, B, true, WS, WS>), grid, block, lds * 4, st, in, dst,
                       is, ds, tw);
  else
    hipLaunchKernelGGL((k_ntt_tile<false, B, false, WS, WS>), grid, block, lds * 4, st, in, dst,
                       is, ds, tw);
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
    case 14: tile_launch<DIF, 14>(grid, in, is, dst, ds, tw, st); return true;
  }
  return false;
}


static void r16_launch(const R16Pass& p, const uint32_t* in, size_t is, uint32_t* dst, size_t ds,
                       int ncols, int L, bool dif, hipStream_t st) {
  Twiddles& T = twiddles();
  // a pass reads table entries below 2^L: a caller that skipped ensure() must not reach the GPU
  if (T.logmax.load(std::memory_order_acquire) < L || !T.fwd())
    throw std::logic_error("r16_launch: twiddle table not built for this height");
  r16_attrs();  // the 2^14 tiles need more than the default dynamic LDS (once per process)
  const int threads = 1 << (p.b + p.c - 4);
  const size_t lds = ((size_t)1 << (p.b + p.c)) + ((size_t)1 << (p.b + p.c - 4));
  dim3 grid(1u << (L - p.b - p.c), ncols);
  KernelProbe& probe = ntt_probe();
  hipEvent_t ev0 = probe.on ? probe.begin(st) : nullptr;
  if (p.s0 == 0 && p.c == 0 &&
      (dif ? tile_dispatch<true>(p.b, grid, in, is, dst, ds, (const uint32_t*)T.fwd(), st)
           : tile_dispatch<false>(p.b, grid, in, is, dst, ds, (const uint32_t*)T.inv(), st))) {
    // specialised contiguous pass
  } else if (dif)
    hipLaunchKernelGGL(k_ntt_r16<true>, grid, dim3(threads), lds * 4, st, in, dst, is, ds, p.s0,
                       p.b, p.c, (const uint32_t*)T.fwd());
  else
    hipLaunchKernelGGL(k_ntt_r16<false>, grid, dim3(threads), lds * 4, st, in, dst, is, ds, p.s0,
                       p.b, p.c, (const uint32_t*)T.inv());
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
                         c, T.fwd());
    else
      hipLaunchKernelGGL(k_ntt_pass<false>, grid, dim3(256), 0, st, in, dst, is, dst_stride, s0, b,
                         c, T.inv());
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
std::mutex& cache_mu() {  // the device table caches below are shared by the proof lanes
  static std::mutex m;
  return m;
}
const uint32_t* scale_tables(uint32_t shift, int L, int B) {
  std::lock_guard<std::mutex> lk(cache_mu());
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
  ResidentScope rs;  // cached for the process, not part of the lane's working set
  DBuf<uint32_t> d(4 * nb);
  // stream-ordered: a pooled buffer may still be read by kernels queued on stream()
  HIP_CHECK(hipMemcpyAsync(d.p, h.data(), h.size() * 4, hipMemcpyHostToDevice, stream()));
  HIP_CHECK(hipStreamSynchronize(stream()));
  const uint32_t* p = d.p;
  cache.emplace(PowKey{shift, L}, std::move(d));
  return p;
}
}  // namespace

void prepare_lde_tables(int L) {
  // the coset shifts a proof's LDEs use at height 2^L: GENERATOR / 1 for the traces (prover.hip
  // lde_into), 1 and w_2n^-1 for the two quotient chunks' other halves
  const int B = (L + 1) / 2;
  twiddles().ensure(std::max(L + 1, 1));
  (void)scale_tables(to_mont(3), L, B);
  (void)scale_tables(ONE, L, B);
  (void)scale_tables(minv(two_adic_gen(L + 1)), L, B);
}

static bool lde_tiny_on() {  // BFZ_LDE_TINY=0: the three-launch path for n <= 2^8 too (A/B)
  static const bool on = [] {
    const char* e = getenv("BFZ_LDE_TINY");
    return !(e && e[0] == '0');
  }();
  return on;
}

// The fused middle pass (k_lde_mid) of an L > 14 coset LDE over the iDFT's first-pass output
// `coef` (w columns of n): coefficients, scaled by the coset powers, DIF stages of pass 2.
static void mid_launch(const uint32_t* coef, size_t n, int w, uint32_t shift, uint32_t* lde,
                       int only_half, const MidOut& mo, hipStream_t st) {
  const int L = log2i(n);
  Twiddles& T = twiddles();
  T.ensure(L);
  r16_attrs();
  const R16Pass p2 = r16_plan(L)[1];
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
  const dim3 grid(1u << (L - p2.b - p2.c), ceil_div(w, MID_CPB));
#define BFZ_MID(LL)                                                                              \
  case LL:                                                                                       \
    static_assert(MidPlan<LL>::b2 >= 4, "plan");                                                 \
    hipLaunchKernelGGL(k_lde_mid<LL>, grid, dim3(threads), ldsz * 4, st, coef, n, lde, n,        \
                       (const uint32_t*)T.inv(), (const uint32_t*)T.fwd(), pw, B, mp, only_half, \
                       w, mo);                                                                   \
    break;
  switch (L) {
    BFZ_MID(14) BFZ_MID(15) BFZ_MID(16) BFZ_MID(17) BFZ_MID(18) BFZ_MID(19) BFZ_MID(20) BFZ_MID(21)
    BFZ_MID(22) BFZ_MID(23)
    default: throw std::runtime_error("coset_lde: log height above 23");
  }
#undef BFZ_MID
  KCHECK();
  if (probe.on) probe.end(ev0, st, (only_half >= 0 ? 8.0 : 12.0) * (double)n * w);
}

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
    twiddles().ensure(L);  // before the first pass (a process's first LDE may be this one)
    r16_attrs();
    const auto plan = r16_plan(L);  // {(0, b1, 0), (b1, b2, c2)}
    DBuf<uint32_t> coef(n * (size_t)w);
    r16_launch(plan[0], evals, src_stride, coef.p, n, w, L, false, st);
    mid_launch(coef.p, n, w, shift, lde, only_half, MidOut{2 * n, n, nullptr, 0, 0}, st);
    r16_launch(plan[0], dft_base, dft_stride, dft_base, dft_stride, dft_cols, L, true, st);
    return;
  }
  if (L >= 1 && L <= TINY_LOG_MAX && lde_tiny_on()) {  // one launch, one block per column
    Twiddles& T = twiddles();
    T.ensure(L);
    const int B = (L + 1) / 2;
    const uint32_t* pw = scale_tables(shift, L, B);
    hipLaunchKernelGGL(k_lde_tiny, dim3(w), dim3(256), 0, st, evals, src_stride, lde, L,
                       (const uint32_t*)T.inv(), (const uint32_t*)T.fwd(), pw, B, only_half);
    KCHECK();
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
// a^(u + l m) = a^u (a^m)^l: one table power per output and the launch constants (a^m)^l, so a
// term is one product, summed lazily in 64 bits (four products < 2^64 between folds).
constexpr int FOLD_MAX_TERMS = 64;
struct FoldPowers {
  uint32_t p[FOLD_MAX_TERMS];  // (a^m)^l, l < n / m
};
__global__ __launch_bounds__(256) void k_fold_residue(const uint32_t* __restrict__ coef, size_t n,
                                                      uint32_t* __restrict__ out, size_t m, int B,
                                                      const uint32_t* __restrict__ pw, ColMap cm,
                                                      FoldPowers fp) {
  const uint32_t* c = coef + (size_t)cm.col[blockIdx.y] * n;
  uint32_t* o = out + (size_t)blockIdx.y * m;
  const size_t mask = ((size_t)1 << B) - 1, nb = mask + 1;
  const int terms = (int)(n / m);
  for (size_t u = (size_t)blockIdx.x * blockDim.x + threadIdx.x; u < m;
       u += (size_t)gridDim.x * blockDim.x) {
    uint64_t acc = 0;
    for (int l = 0; l < terms; l++) {
      acc += (uint64_t)c[u + (size_t)l * m] * fp.p[l];
      if ((l & 3) == 3) acc = fold32(acc);
    }
    o[u] = mmul(mreduce(acc), mmul(pw[u & mask], pw[nb + (u >> B)]));
  }
}

// Two-level power table of a (with 1/2^L folded into the high half), cached per (a, L).
static const uint32_t* residue_powers(uint32_t a, int L, int B) {
  std::lock_guard<std::mutex> lk(cache_mu());
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
  ResidentScope rs;
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
  const size_t terms = n >= m ? n / m : 1;
  if (terms > (size_t)FOLD_MAX_TERMS) throw std::runtime_error("coset_residue: more than 64 folds");
  FoldPowers fp{};
  const uint32_t am = mpow(a, (uint64_t)m);
  fp.p[0] = ONE;
  for (size_t l = 1; l < terms; l++) fp.p[l] = mmul(fp.p[l - 1], am);
  const dim3 grid(std::min<unsigned>(ceil_div(m, 256), 2048), w);
  hipLaunchKernelGGL(k_fold_residue, grid, dim3(256), 0, st, coef, n, out, m, B, pw, map, fp);
  KCHECK();
  ntt_passes(out, out, m, m, w, log2i(m), /*dif=*/true, st);
}

// The launch constants of one residue's fold in k_coef_fold: a = shift w_2n^r, S = m / D.
static ResidueFold residue_fold(uint32_t shift, int L, int logG, int r, int S, uint32_t* out) {
  ResidueFold f{};
  const size_t m = ((size_t)2 << L) >> logG;
  const uint32_t a = mmul(shift, mpow(two_adic_gen(L + 1), (uint64_t)r));
  f.pw = residue_powers(a, L, (L + 1) / 2);
  f.out = out;
  const uint32_t am = mpow(a, (uint64_t)m);
  for (int j = 0; j < 4; j++) f.A[j] = (8 >> j) >= S ? mpow(am, (uint64_t)((8 >> j) / S)) : ONE;
  const uint32_t aD = mpow(a, (uint64_t)1 << (L - 4));
  uint32_t q = ONE;
  for (int i = 0; i < 16; i++) { f.Q[i] = q; q = mmul(q, aD); }
  return f;
}

static bool env_on(const char* name) {
  const char* e = getenv(name);
  return !(e && e[0] == '0');
}
static bool fused_residues_on() {  // BFZ_FUSED_RESIDUE=0: the unfused round-5 path (A/B)
  static const bool on = env_on("BFZ_FUSED_RESIDUE");
  return on;
}
static bool mid_half_on() {  // BFZ_MID_HALF=0: two ranks use k_coef_fold too (A/B)
  static const bool on = env_on("BFZ_MID_HALF");
  return on;
}
static bool fused_dif_on() {  // BFZ_FUSED_DIF=0: k_coef_fold leaves the whole DFT (A/B)
  static const bool on = env_on("BFZ_FUSED_DIF");
  return on;
}

bool coef_fold_residues(const uint32_t* evals, size_t n, int w, uint32_t* coef, size_t j0,
                        size_t len, uint32_t shift, int logG, int r, uint32_t* out,
                        const std::vector<int>* next_cols, int r2, uint32_t* nxt, int* dft_low,
                        hipStream_t st) {
  const int L = log2i(n);
  if (!fused_residues_on() || L <= R16_TILE_LOG || L > 23 || logG < 1 || logG > 5 || w < 1 ||
      w > 64)
    return false;
  Twiddles& T = twiddles();
  T.ensure(L);
  r16_attrs();
  const auto plan = r16_plan(L);
  const R16Pass& p1 = plan[0];
  const R16Pass& p2 = plan[1];
  r16_launch(p1, evals, n, coef, n, w, L, false, st);
  if (logG == 1 && !(next_cols && !next_cols->empty()) && mid_half_on()) {
    // two ranks: the residue coset is one half of the coset LDE -- k_lde_mid's half r, written
    // at stride n, with the coefficient range on the side; only the DIF tile pass is left
    mid_launch(coef, n, w, shift, out, r, MidOut{n, 0, coef, j0, len}, st);
    *dft_low = p2.s0;
    return true;
  }
  CoefFold cf{};
  cf.coef = coef;
  cf.j0 = j0;
  cf.len = len;
  cf.m = ((size_t)2 << L) >> logG;
  cf.B = (L + 1) / 2;
  cf.S = 1 << (5 - logG);
  cf.r[0] = residue_fold(shift, L, logG, r, cf.S, out);
  std::fill(std::begin(cf.nidx), std::end(cf.nidx), (uint8_t)0xff);
  if (next_cols && !next_cols->empty()) {
    cf.r[1] = residue_fold(shift, L, logG, r2, cf.S, nxt);
    for (size_t y = 0; y < next_cols->size(); y++) cf.nidx[(*next_cols)[y]] = (uint8_t)y;
  }
  const int threads = 1 << (p2.b + p2.c - 4);
  const size_t ldsz = ((size_t)1 << (p2.b + p2.c)) + ((size_t)1 << (p2.b + p2.c - 4));
  const dim3 grid(1u << (L - p2.b - p2.c), w);
  // the strided DIF stages run in the kernel for 4 and 8 ranks (R = 3, 2)
  const int R = fused_dif_on() && (logG == 2 || logG == 3) ? 5 - logG : 0;
  const uint32_t* ti = (const uint32_t*)T.inv();
  const uint32_t* tf = (const uint32_t*)T.fwd();
#define BFZ_CF(LL)                                                                             \
  case LL:                                                                                     \
    if (R == 3)                                                                                \
      hipLaunchKernelGGL((k_coef_fold<LL, 3>), grid, dim3(threads), ldsz * 4, st,              \
                         (const uint32_t*)coef, n, ti, tf, cf);                                \
    else if (R == 2)                                                                           \
      hipLaunchKernelGGL((k_coef_fold<LL, 2>), grid, dim3(threads), ldsz * 4, st,              \
                         (const uint32_t*)coef, n, ti, tf, cf);                                \
    else                                                                                       \
      hipLaunchKernelGGL((k_coef_fold<LL, 0>), grid, dim3(threads), ldsz * 4, st,              \
                         (const uint32_t*)coef, n, ti, tf, cf);                                \
    break;
  switch (L) {
    BFZ_CF(15) BFZ_CF(16) BFZ_CF(17) BFZ_CF(18) BFZ_CF(19) BFZ_CF(20) BFZ_CF(21) BFZ_CF(22)
    BFZ_CF(23)
  }
#undef BFZ_CF
  KCHECK();
  *dft_low = R ? p2.s0 : -1;
  return true;
}

void residue_dft(uint32_t* out, size_t m, int w, int dft_low, hipStream_t st) {
  const int Lm = log2i(m);
  if (dft_low >= 0) {  // stages [dft_low, log m) ran in the fold kernel: the contiguous tile pass
    r16_launch(R16Pass{0, dft_low, 0}, out, m, out, m, w, Lm, true, st);
    return;
  }
  ntt_passes(out, out, m, m, w, Lm, /*dif=*/true, st);
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

// kernels a proof launches (gpu.h PreloadKernels)
static PreloadKernels preload_ntt{
    (const void*)&k_lde_tiny,
    (const void*)&k_transpose_bitrev,
    (const void*)&k_lde_mid<14>,
    (const void*)&k_lde_mid<15>,
    (const void*)&k_lde_mid<16>,
    (const void*)&k_lde_mid<17>,
    (const void*)&k_lde_mid<18>,
    (const void*)&k_lde_mid<19>,
    (const void*)&k_lde_mid<20>,
    (const void*)&k_lde_mid<21>,
    (const void*)&k_lde_mid<22>,
    (const void*)&k_lde_mid<23>,
    (const void*)&k_ntt_tile<true, 8, false, false, false>,
    (const void*)&k_ntt_tile<false, 8, true, false, false>,
    (const void*)&k_ntt_tile<false, 8, false, false, false>,
    (const void*)&k_ntt_tile<true, 9, false, false, false>,
    (const void*)&k_ntt_tile<false, 9, true, false, false>,
    (const void*)&k_ntt_tile<false, 9, false, false, false>,
    (const void*)&k_ntt_tile<true, 10, false, false, false>,
    (const void*)&k_ntt_tile<false, 10, true, false, false>,
    (const void*)&k_ntt_tile<false, 10, false, false, false>,
    (const void*)&k_ntt_tile<true, 11, false, false, false>,
    (const void*)&k_ntt_tile<false, 11, true, false, false>,
    (const void*)&k_ntt_tile<false, 11, false, false, false>,
    (const void*)&k_ntt_tile<true, 12, false, false, false>,
    (const void*)&k_ntt_tile<false, 12, true, false, false>,
    (const void*)&k_ntt_tile<false, 12, false, false, false>,
    (const void*)&k_ntt_tile<true, 13, false, false, false>,
    (const void*)&k_ntt_tile<false, 13, true, false, false>,
    (const void*)&k_ntt_tile<false, 13, false, false, false>,
    (const void*)&k_ntt_tile<true, 14, false, true, true>,
    (const void*)&k_ntt_tile<false, 14, true, true, true>,
    (const void*)&k_ntt_tile<false, 14, false, true, true>};

}  // namespace bfz
