// PCS opening on the device: TwoAdicFriPcs::open + fri::prover::prove [p3-recalled],
// called from crates/stark/src/prover.rs:460-470.
//
//  * inverse denominators 1/(x_t - z) over the largest coset, bit-reversed order
//    (compute_inverse_denominators); smaller heights use prefixes.
//  * opened values p(z) by barycentric interpolation over the low coset 3*H_n, which is the
//    first n rows of the bit-reversed LDE:  p(z) = (z^n - 3^n)/(n 3^n) * sum_t p_t x_t/(z-x_t)
//  * reduced openings per height:  ro[t] = sum_(mat,point) alpha^off sum_k alpha^k
//    (p_k(x_t) - y_k) / (x_t - z)
//  * FRI commit-phase fold: (1/2 + beta/2 g^-rev(i)) lo + (1/2 - beta/2 g^-rev(i)) hi
//  * proof-of-work grind over the challenger state (smallest witness = normal form)
#include "fri.h"
#include "ntt_dev.h"

#include "poseidon2.h"

#include <algorithm>

namespace bfz {

using namespace kb;

__device__ __forceinline__ uint32_t coset_point(uint32_t t, int logH, const uint32_t* twf) {
  // x_t = 3 * w_H^bitrev(t); w_H^j = twf[H/2 + j] for j < H/2, -twf[j] otherwise
  if (logH == 0) return to_mont_c(3);
  const uint32_t j = dbitrev(t, logH), half = 1u << (logH - 1);
  const uint32_t w = j < half ? twf[half + j] : mneg(twf[j]);
  return mmul(to_mont_c(3), w);
}

// Position of natural index bitrev(t) - 2 in a bit-reversed vector of 2^logH values.
__device__ __forceinline__ size_t prev2_pos(size_t t, int logH) {
  const uint32_t mask = (uint32_t)(((size_t)1 << logH) - 1);
  return dbitrev((dbitrev((uint32_t)t, logH) - 2u) & mask, logH);
}

constexpr int INV_CHUNK = 8;

// out[t - t0] = 1 / (x_t - z) for t in [t0, t0 + count)
// zp != nullptr: the point is read from device memory (sampled on the device)
// wout != nullptr: also the barycentric weights wout[t - t0] = x_t / (x_t - z) for t < wcount
// (the openings' weight table, see open_tile_body)
__global__ __launch_bounds__(256) void k_inv_denoms(EF z, const EF* __restrict__ zp, int logH,
                                                    size_t t0, size_t count,
                                                    const uint32_t* __restrict__ twf,
                                                    EF* __restrict__ out, EF* __restrict__ wout,
                                                    size_t wcount) {
  const size_t base = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) * INV_CHUNK;
  if (base >= count) return;
  if (zp) z = *zp;
  EF d[INV_CHUNK], pre[INV_CHUNK];
  uint32_t xs[INV_CHUNK];
  const int cnt = (int)min((size_t)INV_CHUNK, count - base);
  EF run = ef_one();
#pragma unroll
  for (int k = 0; k < INV_CHUNK; k++) {
    if (k < cnt) {
      xs[k] = coset_point((uint32_t)(t0 + base + k), logH, twf);
      d[k] = ef_sub(ef_base(xs[k]), z);
      run = ef_mul(run, d[k]);
    }
    pre[k] = run;
  }
  EF inv = ef_inv(run);
#pragma unroll
  for (int k = INV_CHUNK - 1; k >= 0; k--) {
    if (k < cnt) {
      const EF r = k ? ef_mul(inv, pre[k - 1]) : inv;
      out[base + k] = r;
      if (wout && base + k < wcount) wout[base + k] = ef_mul_base(r, xs[k]);
      inv = ef_mul(inv, d[k]);
    }
  }
}

// ------------------------------------------------------------------ openings
// Rows per thread: 8 at two points (6 and 4 measured 0.08-0.15 ms per proof slower,
// profiles/r05/ab_open_rows.txt); 16 at one point, where a row's weights take 4 registers
// instead of 8 and the per-column lane reduction is paid once per 16 rows.
#ifndef BFZ_OPEN_R1
#define BFZ_OPEN_R1 16
#endif
#ifndef BFZ_OPEN_R2
#define BFZ_OPEN_R2 8
#endif
constexpr int OPEN_T = 256, OPEN_R2 = BFZ_OPEN_R2;
template <int NP>
constexpr int open_rows() { return NP == 1 ? BFZ_OPEN_R1 : OPEN_R2; }
template <int NP>
constexpr int open_ch() { return OPEN_T * open_rows<NP>(); }

__device__ __forceinline__ EF wave_sum(EF v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1)
#pragma unroll
    for (int e = 0; e < 4; e++) v.c[e] = madd(v.c[e], __shfl_xor(v.c[e], off, 64));
  return v;
}

// Barycentric opening of one matrix at one or two points (NP):
// partial[(chunk * w + c) * NP + k] = sum_{t in chunk} W_k,t col_c[t],  W_k,t = x_t invd_k[t]
// (the barycentric weight is -x_t invd_k[t]: k_open_final_batch negates the scale instead).
// A thread owns OPEN_R rows and keeps their weights for both points in registers, so every
// matrix element is read once for both points.  Four column buffers form a ring (three columns
// in flight while one is consumed).  Each thread's reduced partial of a column goes to LDS and
// the block adds up every 4-column group cooperatively (PER threads per sum, one shuffle tree)
// instead of a DPP row-sum chain per column and coefficient (same-box A/B: the per-column DPP
// sums and a 2-deep prefetch were slower; so was a 4-deep prefetch with the DPP sums).
// TAB = false: barycentric weights W_k,t = -x_t invd_k[t] over the low coset (mat = the LDE).
// TAB = true: W_k,t = invd_k[t] read as a weight table (coefficient form: mat = a range of
// coefficients, the table = powers of the point), logH/twf unused.
// FULL: every thread of the chunk has all OPEN_R rows (every chunk of a matrix of >= OPEN_CH
// low-coset rows): no per-row bounds selects.  Column words come through a buffer descriptor per
// column with the row step in the scalar offset (no 64-bit VALU address arithmetic per load).
// The block's reduction buffer, one per kernel: declared in the FULL and the partial-chunk
// bodies separately it was allocated twice (67.5 KB at two points), which left room for two
// blocks per CU where the registers allow three.
template <int NP>
__device__ __forceinline__ uint32_t* open_lds() {
  constexpr int NSUM = NP * 16, PER = OPEN_T / NSUM, RS = OPEN_T + PER;
  __shared__ uint32_t red[NSUM * RS];
  return red;
}

template <int NP, bool TAB, bool FULL>
__device__ __forceinline__ void open_tile_body(const uint32_t* __restrict__ mat,
                                               const uint32_t* __restrict__ mat2, int w1,
                                               size_t height, int w,
                                               size_t n, int logH, const EF* __restrict__ invd_a,
                                               const EF* __restrict__ invd_b,
                                               const uint32_t* __restrict__ twf,
                                               EF* __restrict__ partial, unsigned chunk, int cb,
                                               int ce, const EF* __restrict__ wtab) {
  constexpr int OPEN_R = open_rows<NP>(), OPEN_CH = open_ch<NP>();
  const size_t c0 = (size_t)chunk * OPEN_CH + threadIdx.x;
  const int nr = FULL ? OPEN_R : c0 >= n ? 0 : (int)min((size_t)OPEN_R, (n - c0 + OPEN_T - 1) / OPEN_T);
  EF W[NP][OPEN_R];
#pragma unroll
  for (int r = 0; r < OPEN_R; r++) {
    const size_t t = c0 + (size_t)r * OPEN_T;
    if (TAB) {
#pragma unroll
      for (int k = 0; k < NP; k++) W[k][r] = r < nr ? ld_global(k ? invd_b : invd_a, t) : ef_zero();
      continue;
    }
    if (wtab) {  // weights x_t / (x_t - z) from k_inv_denoms; the second point z w_n reads the
                 // first's at t' (natural index i - 2): x_t / (x_t - z w_n) = x_t' / (x_t' - z)
#pragma unroll
      for (int k = 0; k < NP; k++)
        W[k][r] = r < nr ? ld_global(wtab, k ? prev2_pos(t, logH) : t) : ef_zero();
      continue;
    }
    const uint32_t x = r < nr ? coset_point((uint32_t)t, logH, twf) : 0u;
#pragma unroll
    for (int k = 0; k < NP; k++) {
      // invd_b == nullptr: the second point is z w_n and 1 / (x_t - z w_n) =
      // w_n^-1 / (x_t' - z) with t' the position of natural index i - 2 (the caller folds
      // w_n^-1 into scale_b), so the zeta table serves both points
      const size_t tk = k && !invd_b ? prev2_pos(t, logH) : t;
      const EF* tab = k && invd_b ? invd_b : invd_a;
      // + x_t invd: the minus sign of W is applied once per column, to the scale (k_open_final_batch)
      W[k][r] = r < nr ? ef_mul_base(ld_global(tab, tk), x) : ef_zero();
    }
  }
  auto colp = [&](int c) {  // column c of the descriptor (a second matrix from column w1 on)
    return c < w1 ? mat + (size_t)c * height : mat2 + (size_t)(c - w1) * height;
  };
  auto load = [&](int c, uint32_t (&v)[OPEN_R]) {
    if constexpr (FULL) {
      const __amdgpu_buffer_rsrc_t rc = rsrc_of(colp(c) + (size_t)chunk * OPEN_CH);
#pragma unroll
      for (int r = 0; r < OPEN_R; r++) v[r] = ld_b(rc, threadIdx.x * 4u, (uint32_t)(r * OPEN_T) * 4u);
    } else {
      const uint32_t* col = colp(c) + c0;
#pragma unroll
      for (int r = 0; r < OPEN_R; r++) v[r] = r < nr ? ld_global(col, (size_t)r * OPEN_T) : 0u;
    }
  };
  // column buffers in a ring: RING - 1 columns stay in flight while one is consumed (four of 8
  // rows; two of 16 rows hold as many loads in flight in half the registers)
  constexpr int RING = OPEN_R > 8 ? 2 : 4;
  uint32_t vr[RING][OPEN_R];
#pragma unroll
  for (int j = 0; j < RING; j++)
    if (cb + j < ce) load(cb + j, vr[j]);
  constexpr int NSUM = NP * 16, PER = OPEN_T / NSUM;  // sums per group, threads per sum
  // row stride OPEN_T + PER: the PER-strided reads of the 32 / PER sums a half-wave adds up
  // land in distinct banks (stride OPEN_T put 32 / PER of them in each bank; kernel -1.6%)
  constexpr int RS = OPEN_T + PER;
  uint32_t* red = open_lds<NP>();  // [(k * 4 + col) * 4 + coef][thread]
  for (int c = cb; c < ce; c += 4) {
#pragma unroll
    for (int j = 0; j < 4; j++) {
      if (c + j < ce) {
#pragma unroll
        for (int k = 0; k < NP; k++) {
          LazyEF lz;
          lz.init();
#pragma unroll
          for (int r = 0; r < OPEN_R; r++) lz.add(W[k][r], vr[j % RING][r]);
          const EF acc = lz.get();
#pragma unroll
          for (int e = 0; e < 4; e++) red[((k * 4 + j) * 4 + e) * RS + threadIdx.x] = acc.c[e];
        }
        if (c + j + RING < ce) load(c + j + RING, vr[j % RING]);
      }
    }
    __syncthreads();
    {  // sum q = (k * 4 + j) * 4 + e is added up by the PER threads q * PER .. q * PER + PER - 1
      const int q = threadIdx.x / PER, part = threadIdx.x % PER;
      const uint32_t* src = red + q * RS;
      uint64_t a64 = 0;
#pragma unroll 8
      for (int i = part; i < OPEN_T; i += PER) a64 += src[i];  // < 32 p < 2^36
      constexpr uint64_t C32 = (1u << 25) - 2;  // 2^32 mod p
      a64 = (a64 >> 32) * C32 + (uint32_t)a64;  // < 2^32 + 2^30
      a64 = (a64 >> 32) * C32 + (uint32_t)a64;  // < 2^32 + 2^25
      uint32_t v = (uint32_t)(a64 >= 2ull * P ? a64 - 2ull * P : a64 >= P ? a64 - P : a64);
#pragma unroll
      for (int off = 1; off < PER; off <<= 1) v = madd(v, __shfl_xor(v, off, 64));
      const int k = q / 16, j = (q / 4) % 4, e = q % 4;
      if (part == 0 && c + j < ce) partial[((size_t)chunk * w + c + j) * NP + k].c[e] = v;
    }
    __syncthreads();
  }
}

template <int NP, bool TAB>
__device__ __forceinline__ void open_tile(const uint32_t* __restrict__ mat,
                                          const uint32_t* __restrict__ mat2, int w1, size_t height,
                                          int w, size_t n, int logH, const EF* __restrict__ invd_a,
                                          const EF* __restrict__ invd_b,
                                          const uint32_t* __restrict__ twf,
                                          EF* __restrict__ partial, unsigned chunk, int cb, int ce,
                                          const EF* __restrict__ wtab = nullptr) {
  if ((size_t)(chunk + 1) * open_ch<NP>() <= n)  // uniform across the block
    open_tile_body<NP, TAB, true>(mat, mat2, w1, height, w, n, logH, invd_a, invd_b, twf, partial,
                                  chunk, cb, ce, wtab);
  else
    open_tile_body<NP, TAB, false>(mat, mat2, w1, height, w, n, logH, invd_a, invd_b, twf, partial,
                                   chunk, cb, ce, wtab);
}

template <int NP, bool TAB = false>
__global__ __launch_bounds__(OPEN_T) void k_open_partial(const uint32_t* __restrict__ mat,
                                                         size_t height, int w, size_t n, int logH,
                                                         const EF* __restrict__ invd_a,
                                                         const EF* __restrict__ invd_b,
                                                         const uint32_t* __restrict__ twf,
                                                         EF* __restrict__ partial) {
  open_tile<NP, TAB>(mat, mat, w, height, w, n, logH, invd_a, invd_b, twf, partial, blockIdx.x, 0, w);
}

// Batched barycentric openings: block b works on chunk (b - chunk0) of the matrix whose block
// range holds b; every matrix of a proof opened at NP points goes in one launch.
template <int NP>
__global__ __launch_bounds__(OPEN_T) void k_open_partial_batch(const OpenDesc* __restrict__ d,
                                                               int nd,
                                                               const uint32_t* __restrict__ twf,
                                                               EF* __restrict__ partial) {
  int m = 0;
  while (m + 1 < nd && d[m + 1].chunk0 <= blockIdx.x) m++;
  const OpenDesc& o = d[m];
  // the matrix's blocks: chunk-major, o.nslab column slabs of o.slab_w columns per row chunk
  const unsigned b = blockIdx.x - o.chunk0, slab = b % o.nslab;
  const int cb = (int)slab * o.slab_w, ce = min(o.w, cb + o.slab_w);
  if (o.tab)  // uniform: a sharded matrix's coefficient range against the power tables
    open_tile<NP, true>(o.mat, o.mat2, o.w1, o.height, o.w, o.rows, o.logH, o.invd_a, o.invd_b,
                        twf, partial + o.part_off, b / o.nslab, cb, ce);
  else
    open_tile<NP, false>(o.mat, o.mat2, o.w1, o.height, o.w, o.rows, o.logH, o.invd_a, o.invd_b,
                         twf, partial + o.part_off, b / o.nslab, cb, ce, o.wtab);
}

// out_k[c] = scale_k * sum_chunks partial[(chunk * w + c) * NP + k]   (one block per column)
template <int NP>
__device__ __forceinline__ void open_final(const EF* __restrict__ partial, int nchunks, int w,
                                           int c, EF scale_a, EF scale_b, EF* __restrict__ out_a,
                                           EF* __restrict__ out_b) {
  __shared__ EF sh[NP][4];
  EF s[NP];
#pragma unroll
  for (int k = 0; k < NP; k++) s[k] = ef_zero();
  for (int q = threadIdx.x; q < nchunks; q += blockDim.x)
#pragma unroll
    for (int k = 0; k < NP; k++) s[k] = ef_add(s[k], partial[((size_t)q * w + c) * NP + k]);
#pragma unroll
  for (int k = 0; k < NP; k++) {
    s[k] = wave_sum(s[k]);
    if ((threadIdx.x & 63) == 0) sh[k][threadIdx.x >> 6] = s[k];
  }
  __syncthreads();
  if (threadIdx.x < NP) {
    const int k = threadIdx.x;
    EF tot = sh[k][0];
    for (int q = 1; q < (int)(blockDim.x / 64); q++) tot = ef_add(tot, sh[k][q]);
    (k ? out_b : out_a)[c] = ef_mul(tot, k ? scale_b : scale_a);
  }
}

template <int NP>
__global__ __launch_bounds__(256) void k_open_final(const EF* __restrict__ partial, int nchunks,
                                                    int w, EF scale_a, EF scale_b,
                                                    EF* __restrict__ out_a, EF* __restrict__ out_b) {
  open_final<NP>(partial, nchunks, w, blockIdx.x, scale_a, scale_b, out_a, out_b);
}

// Batched final sums: block b is column (b - col0) of the matrix whose column range holds b.
template <int NP>
__global__ __launch_bounds__(256) void k_open_final_batch(const OpenDesc* __restrict__ d, int nd,
                                                          const EF* __restrict__ partial) {
  int m = 0;
  while (m + 1 < nd && d[m + 1].col0 <= blockIdx.x) m++;
  const OpenDesc& o = d[m];
  EF sa = o.scale_a, sb = o.scale_b;
  if (o.zeta) {  // the point was sampled on the device: (zeta^n - 3^n) / (3^n n), n = 2^zlog
    EF zn = *o.zeta;
    for (int i = 0; i < o.zlog; i++) zn = ef_mul(zn, zn);
    sa = ef_mul_base(ef_sub(zn, ef_base(o.z3n)), o.zc);
    sb = ef_mul_base(sa, o.zb);
  }
  // the partial sums are of x_t invd_k[t] col[t]: the weight's sign goes into the scale (the
  // coefficient form's weights are the powers themselves)
  if (!o.tab) {
    sa = ef_neg(sa);
    sb = ef_neg(sb);
  }
  const int c = (int)(blockIdx.x - o.col0);
  const bool second = c >= o.w1;  // a merged descriptor's second matrix: its own outputs
  open_final<NP>(partial + o.part_off, (int)o.nchunks, o.w, c, sa, sb,
                 second ? o.out_a2 - o.w1 : o.out_a, second ? o.out_b2 - o.w1 : o.out_b);
}

// ------------------------------------------------------------------ reduced openings
constexpr int RED_STEP = 16;  // column loads per step (8: neutral)
// Positions [t0, t1) (a shard's range; every pointer indexed by the global position).
// invd_b == nullptr (has_b): the second point's denominators come from the zeta table at the
// position of natural index i - 2 (see open_tile); the caller folds w_n^-1 into kb and yb.
__global__ __launch_bounds__(256) void k_reduce(const RedCol* __restrict__ cols,
                                                const RedMat* __restrict__ mats, int nmats,
                                                size_t t0, size_t t1, const EF* __restrict__ invd_a,
                                                const EF* __restrict__ invd_b,
                                                const EF* __restrict__ yab, int has_b, int logH,
                                                EF* __restrict__ ro) {
  const EF ya = yab[0], yb = yab[1];
  for (size_t t = t0 + (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < t1;
       t += (size_t)gridDim.x * blockDim.x) {
    EF sa = ef_zero(), sb = ef_zero();
    for (int m = 0; m < nmats; m++) {
      const RedMat rm = mats[m];
      LazyEF acc;
      acc.init();
      const int end = rm.first + rm.count;
      int c = rm.first;
      for (; c + RED_STEP <= end; c += RED_STEP) {  // RED_STEP column loads in flight per step
        uint32_t v[RED_STEP];
#pragma unroll
        for (int k = 0; k < RED_STEP; k++) v[k] = ld_global(cols[c + k].col, t);
#pragma unroll
        for (int k = 0; k < RED_STEP; k++) acc.add(cols[c + k].ca, v[k]);
      }
      if (RED_STEP > 8 && c + 8 <= end) {
        uint32_t v[8];
#pragma unroll
        for (int k = 0; k < 8; k++) v[k] = ld_global(cols[c + k].col, t);
#pragma unroll
        for (int k = 0; k < 8; k++) acc.add(cols[c + k].ca, v[k]);
        c += 8;
      }
      if (c + 4 <= end) {
        uint32_t v[4];
#pragma unroll
        for (int k = 0; k < 4; k++) v[k] = ld_global(cols[c + k].col, t);
#pragma unroll
        for (int k = 0; k < 4; k++) acc.add(cols[c + k].ca, v[k]);
        c += 4;
      }
      for (; c < end; c++) acc.add(cols[c].ca, ld_global(cols[c].col, t));
      const EF s = acc.get();
      sa = ef_add(sa, s);
      if (rm.has_b) sb = ef_add(sb, ef_mul(s, rm.kb));
    }
    EF r = ef_mul(ef_sub(sa, ya), invd_a[t]);
    if (has_b)
      r = ef_add(r, ef_mul(ef_sub(sb, yb), invd_b ? invd_b[t] : invd_a[prev2_pos(t, logH)]));
    ro[t] = r;  // one launch covers every matrix of the height
  }
}

// out[t] = z^(j0 + t), t < count.  A block writes POW_RUN x 256 consecutive powers, lane-
// interleaved (thread tid: t = block start + tid + 256 k, stepping by z^256); a thread's first
// power is the uniform z^(j0 + block start) times z^tid, products of the launch's squares
// z^(2^k) (no squaring chain).
constexpr int POW_RUN = 16;
struct PowSquares {
  EF sq[32];  // z^(2^k)
};
__global__ __launch_bounds__(256) void k_pow_table(PowSquares ps, size_t j0, size_t count,
                                                   EF* __restrict__ out) {
  const size_t b0 = (size_t)blockIdx.x * 256 * POW_RUN;
  const uint64_t eb = j0 + b0;
  EF p = ef_base(ONE);
#pragma unroll
  for (int k = 0; k < 32; k++)
    if ((eb >> k) & 1) p = ef_mul(p, ps.sq[k]);
#pragma unroll
  for (int k = 0; k < 8; k++)
    if ((threadIdx.x >> k) & 1) p = ef_mul(p, ps.sq[k]);
#pragma unroll 4
  for (int k = 0; k < POW_RUN; k++) {
    const size_t t = b0 + threadIdx.x + 256 * (size_t)k;
    if (t >= count) break;
    out[t] = p;
    p = ef_mul(p, ps.sq[8]);
  }
}

// pow_tables / inv_denoms_ranges: block b works for the job whose block range holds b
struct PowJobDev {
  EF sq[32];
  size_t j0, count;
  EF* out;
  uint32_t block0;
};
__global__ __launch_bounds__(256) void k_pow_tables(const PowJobDev* __restrict__ jobs, int nj) {
  int m = 0;
  while (m + 1 < nj && jobs[m + 1].block0 <= blockIdx.x) m++;
  const PowJobDev& jb = jobs[m];
  const size_t b0 = (size_t)(blockIdx.x - jb.block0) * 256 * POW_RUN;
  const uint64_t eb = jb.j0 + b0;
  EF p = ef_base(ONE);
  for (int k = 0; k < 32; k++)
    if ((eb >> k) & 1) p = ef_mul(p, jb.sq[k]);
#pragma unroll
  for (int k = 0; k < 8; k++)
    if ((threadIdx.x >> k) & 1) p = ef_mul(p, jb.sq[k]);
  const EF step = jb.sq[8];
#pragma unroll 4
  for (int k = 0; k < POW_RUN; k++) {
    const size_t t = b0 + threadIdx.x + 256 * (size_t)k;
    if (t >= jb.count) break;
    jb.out[t] = p;
    p = ef_mul(p, step);
  }
}

struct InvJobDev {
  EF z;
  int logH;
  size_t t0, count;
  EF* out;
  uint32_t block0;
};
__global__ __launch_bounds__(256) void k_inv_denoms_jobs(const InvJobDev* __restrict__ jobs, int nj,
                                                         const uint32_t* __restrict__ twf) {
  int m = 0;
  while (m + 1 < nj && jobs[m + 1].block0 <= blockIdx.x) m++;
  const InvJobDev& jb = jobs[m];
  const size_t base = ((size_t)(blockIdx.x - jb.block0) * blockDim.x + threadIdx.x) * INV_CHUNK;
  if (base >= jb.count) return;
  const EF z = jb.z;
  EF d[INV_CHUNK], pre[INV_CHUNK];
  const int cnt = (int)min((size_t)INV_CHUNK, jb.count - base);
  EF run = ef_one();
#pragma unroll
  for (int k = 0; k < INV_CHUNK; k++) {
    if (k < cnt) {
      d[k] = ef_sub(ef_base(coset_point((uint32_t)(jb.t0 + base + k), jb.logH, twf)), z);
      run = ef_mul(run, d[k]);
    }
    pre[k] = run;
  }
  EF inv = ef_inv(run);
#pragma unroll
  for (int k = INV_CHUNK - 1; k >= 0; k--) {
    if (k < cnt) {
      jb.out[base + k] = k ? ef_mul(inv, pre[k - 1]) : inv;
      inv = ef_mul(inv, d[k]);
    }
  }
}

// ------------------------------------------------------------------ FRI fold
// Outputs [i0, i0 + count) of a fold of 2h values to h; in/out/add hold that range only
// (in: 2 count values, from 2 i0).
__global__ __launch_bounds__(256) void k_fri_fold_dev(const EF* __restrict__ in,
                                                      EF* __restrict__ out, size_t h, int logh,
                                                      size_t i0, size_t count,
                                                      const EF* __restrict__ beta,
                                                      const uint32_t* __restrict__ twi,
                                                      const EF* __restrict__ add) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  const uint32_t halfv = to_mont_c((P + 1) / 2);
  const EF half_beta = ef_mul_base(*beta, halfv);
  const uint32_t g = twi[h + dbitrev((uint32_t)(i0 + i), logh)];
  const EF p = ef_mul_base(half_beta, g);
  const EF lo = in[2 * i], hi = in[2 * i + 1];
  EF r = ef_add(ef_mul(ef_add_base(p, halfv), lo), ef_mul(ef_sub(ef_base(halfv), p), hi));
  if (add) r = ef_add(r, add[i]);
  out[i] = r;
}

// Fold output k of a layer folded to n = 2^logn values (k_fri_fold_dev's formula).
__device__ __forceinline__ EF fold_one(const EF* __restrict__ in, size_t k, size_t n, int logn,
                                       const EF& half_beta, uint32_t halfv,
                                       const uint32_t* __restrict__ twi, const EF* __restrict__ add) {
  const EF p = ef_mul_base(half_beta, ld_global(twi, n + dbitrev((uint32_t)k, logn)));
  EF r = ef_add(ef_mul(ef_add_base(p, halfv), ld_global(in, 2 * k)),
                ef_mul(ef_sub(ef_base(halfv), p), ld_global(in, 2 * k + 1)));
  if (add) r = ef_add(r, ld_global(add, k));
  return r;
}

// Thread mode: thread i folds outputs 2i, 2i+1 and hashes them as leaf i.
__global__ __launch_bounds__(256) void k_fold_leaves(
    const EF* __restrict__ in, EF* __restrict__ out, size_t h, int logn,
    const EF* __restrict__ beta, const uint32_t* __restrict__ twi, const EF* __restrict__ add,
    uint32_t* __restrict__ digests) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= h) return;
  const uint32_t halfv = to_mont_c((P + 1) / 2);
  const EF half_beta = ef_mul_base(*beta, halfv);
  const EF a = fold_one(in, 2 * i, 2 * h, logn, half_beta, halfv, twi, add);
  const EF b = fold_one(in, 2 * i + 1, 2 * h, logn, half_beta, halfv, twi, add);
  out[2 * i] = a;
  out[2 * i + 1] = b;
  uint32_t st[16];
#pragma unroll
  for (int e = 0; e < 4; e++) {
    st[e] = a.c[e];
    st[4 + e] = b.c[e];
    st[8 + e] = 0;
    st[12 + e] = 0;
  }
  poseidon2_permute(st);
  uint4* o = reinterpret_cast<uint4*>(digests + 8 * i);
  o[0] = make_uint4(st[0], st[1], st[2], st[3]);
  o[1] = make_uint4(st[4], st[5], st[6], st[7]);
}

// One 16-lane row: lane l holds state word l (lane-mode permutation).
__global__ __launch_bounds__(64) void k_fri_challenge(uint32_t* __restrict__ state,
                                                      const uint32_t* __restrict__ root,
                                                      EF* __restrict__ beta) {
  const int lane = threadIdx.x & 15;
  const bool row0 = threadIdx.x < 16;
  uint32_t v = lane < 8 ? root[lane] : state[lane];
  v = poseidon2_permute_lane(v, lane);
  if (row0) {
    state[lane] = v;
    if (lane >= 4 && lane < 8) beta->c[7 - lane] = v;
  }
}

// The commit-phase tail (FriTailRounds, fri.h): one 1024-thread block, 16 lanes per
// permutation (lane-mode Poseidon2), 64 permutations per pass.
__global__ __launch_bounds__(1024) void k_fri_tail(FriTailRounds a, const uint32_t* __restrict__ twi) {
  __shared__ EF cur[2 * FRI_TAIL_MAXH];          // the round's input layer
  __shared__ uint32_t dig[2][FRI_TAIL_MAXH * 8];  // digests of the layer being built / below it
  __shared__ EF sbeta;
  const int lane = threadIdx.x & 15, row = threadIdx.x >> 4;
  constexpr int ROWS = 1024 / 16;
  const LaneConsts kc = lane_consts(lane);
  uint32_t stv = threadIdx.x < 16 ? ld_global(a.state, threadIdx.x) : 0u;  // lane l: state[l]
  for (int i = threadIdx.x; i < (2 << a.logh0); i += blockDim.x) cur[i] = ld_global(a.in, i);
  __syncthreads();
  const uint32_t halfv = to_mont_c((P + 1) / 2);
  for (int r = 0; r < a.nr; r++) {
    const int logh = a.logh0 - r, h = 1 << logh;
    uint32_t* out = a.tree[r];
    // leaves: row i = cur[2i] || cur[2i+1] (8 words), one permutation.  Waves with no row below
    // h skip the pass (a permutation costs its latency only while few waves share a SIMD); in
    // the others whole 16-lane rows permute (DPP) and rows < h store.
    for (int b = 0; b < h; b += ROWS) {
      if (b + (row & ~3) >= h) break;
      const int i = b + row;
      const uint32_t x = i < h && lane < 8 ? cur[2 * i + (lane >> 2)].c[lane & 3] : 0u;
      const uint32_t v = poseidon2_permute_lane(x, lane, kc);
      if (i < h && lane < 8) {
        out[8 * i + lane] = v;
        dig[0][8 * i + lane] = v;
      }
    }
    __syncthreads();
    out += 8 * h;
    int pp = 0;
    for (int m = h >> 1; m >= 1; m >>= 1) {  // node j = P(child 2j || child 2j+1)[0..8]
      for (int b = 0; b < m; b += ROWS) {
        if (b + (row & ~3) >= m) break;
        const int j = b + row;
        const uint32_t v = poseidon2_permute_lane(j < m ? dig[pp][16 * j + lane] : 0u, lane, kc);
        if (j < m && lane < 8) {
          out[8 * j + lane] = v;
          dig[pp ^ 1][8 * j + lane] = v;
        }
      }
      __syncthreads();
      pp ^= 1;
      out += 8 * m;
    }
    if (threadIdx.x < 64) {  // observe the root (input buffer empty), duplex, pop 4 outputs
      const uint32_t v = poseidon2_permute_lane(lane < 8 ? dig[pp][lane] : stv, lane, kc);
      if (threadIdx.x < 16) {
        stv = v;
        if (lane >= 4 && lane < 8) {
          sbeta.c[7 - lane] = v;
          a.beta[r].c[7 - lane] = v;
        }
      }
    }
    __syncthreads();
    EF f = ef_zero();  // fold (k_fri_fold_dev)
    const int i = threadIdx.x;
    if (i < h) {
      const EF half_beta = ef_mul_base(sbeta, halfv);
      const EF p = ef_mul_base(half_beta, ld_global(twi, (size_t)h + dbitrev((uint32_t)i, logh)));
      f = ef_add(ef_mul(ef_add_base(p, halfv), cur[2 * i]), ef_mul(ef_sub(ef_base(halfv), p), cur[2 * i + 1]));
      if (a.add[r]) f = ef_add(f, ld_global(a.add[r], i));
      a.layer[r][i] = f;
    }
    __syncthreads();
    if (i < h) cur[i] = f;
    __syncthreads();
  }
  if (threadIdx.x < 16) a.state[threadIdx.x] = stv;
}

// ------------------------------------------------------------------ transcript tail
// The challenger after the commit phase, then observe(final constant).  Also arms the grind's
// result word (no candidate yet).
__global__ __launch_bounds__(64) void k_fri_finish(DevChallenger* __restrict__ c,
                                                   const uint32_t* __restrict__ fri_state,
                                                   const EF* __restrict__ fin,
                                                   uint32_t* __restrict__ res) {
  LaneSponge sp;
  if (fri_state) {  // after the last round's duplex and its beta (4 pops): out = st[0..8), 4 left
    sp.lane = threadIdx.x & 15;
    sp.kc = lane_consts(sp.lane);
    sp.stv = fri_state[sp.lane];
    sp.inv = 0;
    sp.outv = sp.lane < 8 ? sp.stv : 0u;
    sp.nin = 0;
    sp.nout = 4;
  } else {
    sp.load(c);
  }
  const EF f = *fin;
  for (int e = 0; e < 4; e++) sp.observe(f.c[e]);
  sp.store(c);
  if (threadIdx.x == 0) {
    res[0] = 0xffffffffu;
    res[1] = 0;
  }
}

// Proof-of-work grind: observe(w) then sample_bits(bits) == 0  <=>  perm(st with in[0..nin),
// w at nin)[7] has its low bits clear.  The grid scans the candidates chunk by chunk (chunk =
// the grid's thread count) in order; a thread leaves once the best witness lies in a chunk it
// has finished, so every thread has covered every chunk up to the smallest witness's and the
// atomicMin result is that witness (the normal form).  Every thread reaches the exit: a witness
// turns up with probability 1 - e^-2 per 2^(bits+1)-candidate chunk, and the scan ends at P.
__global__ __launch_bounds__(256) void k_grind(const DevChallenger* __restrict__ c, uint32_t bits,
                                               uint32_t* __restrict__ best) {
  uint32_t s0[16];
  const int nin = c->nin;
#pragma unroll
  for (int i = 0; i < 16; i++) s0[i] = c->st[i];
#pragma unroll
  for (int i = 0; i < 8; i++)
    if (i < nin) s0[i] = c->in[i];
  const uint32_t stride = gridDim.x * blockDim.x;
  const uint32_t mask = (1u << bits) - 1;
  for (uint32_t base = 0; base < P; base += stride) {
    const uint32_t w = base + blockIdx.x * blockDim.x + threadIdx.x;
    if (w < P) {
      uint32_t s[16];
#pragma unroll
      for (int i = 0; i < 16; i++) s[i] = s0[i];
      const uint32_t wm = to_mont(w);
#pragma unroll
      for (int i = 0; i < 8; i++)
        if (i == nin) s[i] = wm;
      poseidon2_permute(s);
      if ((from_mont(s[7]) & mask) == 0) atomicMin(best, w);
    }
    const uint32_t b = __hip_atomic_load(best, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((uint64_t)b < (uint64_t)base + stride) break;
  }
}

// observe(witness), the witness check, then the query indices; the challenger is stored back.
__global__ __launch_bounds__(64) void k_sample_queries(DevChallenger* __restrict__ c, int bits,
                                                       int nq, int log_max,
                                                       uint32_t* __restrict__ qidx,
                                                       uint32_t* __restrict__ res) {
  LaneSponge sp;
  sp.load(c);
  const uint32_t w = res[0];
  sp.observe(to_mont(w));
  const uint32_t v = from_mont(sp.sample()) & ((1u << bits) - 1);
  const uint32_t qmask = (uint32_t)(((uint64_t)1 << log_max) - 1);
  for (int q = 0; q < nq; q++) {
    const uint32_t x = from_mont(sp.sample()) & qmask;
    if (threadIdx.x == 0) qidx[q] = x;
  }
  sp.store(c);
  if (threadIdx.x == 0) res[1] = (w < P && v == 0) ? 1u : 0u;
}

// ------------------------------------------------------------------ query gather
__global__ __launch_bounds__(256) void k_gather_segs(const GatherSeg* __restrict__ segs, int nseg,
                                                     const uint32_t* __restrict__ seg_off,
                                                     uint32_t words_per_q,
                                                     const uint32_t* __restrict__ qidx, int nq,
                                                     int rank, uint32_t* __restrict__ out) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (size_t)nseg * nq) return;
  const int q = (int)(t / nseg), s = (int)(t % nseg);
  const GatherSeg g = segs[s];
  uint32_t* o = out + (size_t)q * words_per_q + seg_off[s];
  if (!g.base) {  // literal words (the serialized length fields): rank 0 writes them
    for (uint32_t k = 0; k < g.count; k++) o[k] = rank == 0 ? g.xr : 0u;
    return;
  }
  const uint32_t e = (qidx[q] >> g.shift) ^ g.xr;
  const int owner = g.own_shift >= 0 ? (int)(e >> g.own_shift) : 0;
  const uint64_t pos = (uint64_t)e * g.unit;
  // canonical form here, so the host copies the words straight into the proof
  for (uint32_t k = 0; k < g.count; k++)
    o[k] = owner == rank ? from_mont(ld_global(g.base, pos + k * g.stride)) : 0u;
}

// ================================================================== host wrappers
void inv_denoms(const EF& z, int logH, EF* out, hipStream_t st) {
  inv_denoms_range(z, logH, 0, (size_t)1 << logH, out, st);
}

void inv_denoms_range(const EF& z, int logH, size_t t0, size_t count, EF* out, hipStream_t st) {
  twiddles().ensure(std::max(logH, 1));
  const size_t nthreads = (count + INV_CHUNK - 1) / INV_CHUNK;
  hipLaunchKernelGGL(k_inv_denoms, dim3(ceil_div(nthreads, 256)), dim3(256), 0, st, z,
                     (const EF*)nullptr, logH, t0, count, (const uint32_t*)twiddles().fwd(), out,
                     (EF*)nullptr, (size_t)0);
  KCHECK();
}

void inv_denoms_dev(const EF* z, int logH, EF* out, hipStream_t st, EF* wout) {
  twiddles().ensure(std::max(logH, 1));
  const size_t count = (size_t)1 << logH;
  const size_t nthreads = (count + INV_CHUNK - 1) / INV_CHUNK;
  hipLaunchKernelGGL(k_inv_denoms, dim3(ceil_div(nthreads, 256)), dim3(256), 0, st, ef_zero(), z,
                     logH, (size_t)0, count, (const uint32_t*)twiddles().fwd(), out, wout,
                     count / 2);
  KCHECK();
}

void pow_table(const EF& z, size_t j0, size_t count, EF* out, hipStream_t st) {
  if ((j0 + count) >> 32) throw std::runtime_error("pow_table: exponent above 2^32");
  PowSquares ps;
  ps.sq[0] = z;
  for (int k = 1; k < 32; k++) ps.sq[k] = ef_mul(ps.sq[k - 1], ps.sq[k - 1]);
  hipLaunchKernelGGL(k_pow_table, dim3(ceil_div(count, (size_t)256 * POW_RUN)), dim3(256), 0, st,
                     ps, j0, count, out);
  KCHECK();
}

void pow_tables(const std::vector<PowJob>& jobs, hipStream_t st) {
  if (jobs.empty()) return;
  std::vector<PowJobDev> jd(jobs.size());
  uint32_t blocks = 0;
  for (size_t i = 0; i < jobs.size(); i++) {
    const PowJob& j = jobs[i];
    if ((j.j0 + j.count) >> 32) throw std::runtime_error("pow_tables: exponent above 2^32");
    jd[i].sq[0] = j.z;
    for (int k = 1; k < 32; k++) jd[i].sq[k] = ef_mul(jd[i].sq[k - 1], jd[i].sq[k - 1]);
    jd[i].j0 = j.j0;
    jd[i].count = j.count;
    jd[i].out = j.out;
    jd[i].block0 = blocks;
    blocks += ceil_div(j.count, (size_t)256 * POW_RUN);
  }
  if (!blocks) return;
  DBuf<PowJobDev> dj(jd.size());
  upload_async(dj.p, jd.data(), jd.size() * sizeof(PowJobDev), st);
  hipLaunchKernelGGL(k_pow_tables, dim3(blocks), dim3(256), 0, st, (const PowJobDev*)dj.p,
                     (int)jd.size());
  KCHECK();
}

void inv_denoms_ranges(const std::vector<InvJob>& jobs, hipStream_t st) {
  if (jobs.empty()) return;
  std::vector<InvJobDev> jd(jobs.size());
  uint32_t blocks = 0;
  int logmax = 1;
  for (size_t i = 0; i < jobs.size(); i++) {
    const InvJob& j = jobs[i];
    jd[i].z = j.z;
    jd[i].logH = j.logH;
    jd[i].t0 = j.t0;
    jd[i].count = j.count;
    jd[i].out = j.out;
    jd[i].block0 = blocks;
    blocks += ceil_div(ceil_div(j.count, (size_t)INV_CHUNK), (size_t)256);
    logmax = std::max(logmax, j.logH);
  }
  if (!blocks) return;
  twiddles().ensure(logmax);
  DBuf<InvJobDev> dj(jd.size());
  upload_async(dj.p, jd.data(), jd.size() * sizeof(InvJobDev), st);
  hipLaunchKernelGGL(k_inv_denoms_jobs, dim3(blocks), dim3(256), 0, st, (const InvJobDev*)dj.p,
                     (int)jd.size(), (const uint32_t*)twiddles().fwd());
  KCHECK();
}

void open_coefficients(const uint32_t* coef, size_t col_stride, int w, size_t count,
                       const EF* tab_a, const EF& scale_a, EF* out_a, const EF* tab_b,
                       const EF& scale_b, EF* out_b, hipStream_t st) {
  const int np = tab_b ? 2 : 1;
  const int nchunks = (int)ceil_div(count, np == 2 ? open_ch<2>() : open_ch<1>());
  DBuf<EF> partial((size_t)nchunks * w * np);
  if (np == 2) {
    hipLaunchKernelGGL((k_open_partial<2, true>), dim3(nchunks), dim3(OPEN_T), 0, st, coef,
                       col_stride, w, count, 0, tab_a, tab_b, nullptr, partial.p);
    KCHECK();
    hipLaunchKernelGGL(k_open_final<2>, dim3(w), dim3(256), 0, st, (const EF*)partial.p,
                       nchunks, w, scale_a, scale_b, out_a, out_b);
  } else {
    hipLaunchKernelGGL((k_open_partial<1, true>), dim3(nchunks), dim3(OPEN_T), 0, st, coef,
                       col_stride, w, count, 0, tab_a, tab_a, nullptr, partial.p);
    KCHECK();
    hipLaunchKernelGGL(k_open_final<1>, dim3(w), dim3(256), 0, st, (const EF*)partial.p,
                       nchunks, w, scale_a, scale_a, out_a, out_a);
  }
  KCHECK();
}

// Two descriptors of one LDE height opened at the same points read the same weights: one
// descriptor for both (each keeps its own outputs).
static bool mergeable(const OpenDesc& a, const OpenDesc& b) {
  return !a.mat2 && !b.mat2 && a.tab == b.tab && a.rows == b.rows && a.height == b.height &&
         a.logH == b.logH && a.invd_a == b.invd_a &&
         a.invd_b == b.invd_b && a.zeta == b.zeta && a.zlog == b.zlog && a.z3n == b.z3n &&
         a.zc == b.zc && a.zb == b.zb && a.wtab == b.wtab && ef_eq(a.scale_a, b.scale_a) &&
         ef_eq(a.scale_b, b.scale_b);
}

void open_batch(std::vector<OpenDesc>& in, int np, hipStream_t st) {
  if (in.empty()) return;
  static const bool merge = [] {  // BFZ_OPEN_MERGE=0: one descriptor per matrix (A/B)
    const char* e = std::getenv("BFZ_OPEN_MERGE");
    return !(e && *e == '0');
  }();
  std::vector<OpenDesc> ds;
  for (OpenDesc& o : in)
    if (!o.rows) o.rows = o.height / 2;  // barycentric: the low coset
  for (const OpenDesc& o : in) {
    if (merge && !ds.empty() && mergeable(ds.back(), o)) {
      OpenDesc& m = ds.back();
      m.mat2 = o.mat;
      m.w1 = m.w;
      m.w += o.w;
      m.out_a2 = o.out_a;
      m.out_b2 = o.out_b;
      continue;
    }
    ds.push_back(o);
    ds.back().mat2 = nullptr;
    ds.back().w1 = o.w;
  }
  const uint32_t och = np == 2 ? open_ch<2>() : open_ch<1>();
  // A launch of few row chunks (short or merged matrices, 16 rows per thread at one point) splits
  // the columns of each chunk over several blocks, so it still fills the GPU; each slab of a
  // chunk computes the chunk's weights itself.
  uint64_t nch = 0;
  for (const OpenDesc& o : ds) nch += ceil_div(o.rows, och);
  static const uint64_t FILL = [] {  // blocks: 8 per CU (BFZ_OPEN_FILL=0: no slabs, A/B)
    const char* e = std::getenv("BFZ_OPEN_FILL");
    return e ? (uint64_t)std::strtoull(e, nullptr, 10) : (uint64_t)2048;
  }();
  const uint32_t want = nch >= FILL ? 1u : (uint32_t)((FILL + nch - 1) / nch);
  uint32_t chunks = 0, cols = 0;
  uint64_t part = 0;
  for (OpenDesc& o : ds) {
    o.nchunks = ceil_div(o.rows, och);
    const uint32_t groups = ceil_div(o.w, 4);  // 4-column reduction groups
    o.nslab = std::min(groups, want);
    o.slab_w = 4 * (int)ceil_div(groups, o.nslab);
    o.nslab = ceil_div(o.w, o.slab_w);
    o.chunk0 = chunks;
    o.col0 = cols;
    o.part_off = part;
    chunks += o.nchunks * o.nslab;
    cols += (uint32_t)o.w;
    part += (uint64_t)o.nchunks * o.w * np;
  }
  DBuf<OpenDesc> dd(ds.size());
  upload_async(dd.p, ds.data(), ds.size() * sizeof(OpenDesc), st);
  // algorithmic bytes: every matrix's low-coset words + one weight table (16 B per row and
  // point) per LDE height (matrices of one height share it)
  double obytes = 0;
  std::vector<uint64_t> heights;
  for (const OpenDesc& o : ds) {
    obytes += (double)o.rows * 4.0 * o.w;
    if (std::find(heights.begin(), heights.end(), o.height) == heights.end()) {
      heights.push_back(o.height);
      obytes += (double)o.rows * 16.0 * np;
    }
  }
  KernelProbe& probe = open_probe();
  DBuf<EF> partial(std::max<uint64_t>(part, 1));
  const uint32_t* twf = (const uint32_t*)twiddles().fwd();
  const int nd = (int)ds.size();
  hipEvent_t ev0 = probe.on ? probe.begin(st) : nullptr;
  if (np == 2)
    hipLaunchKernelGGL(k_open_partial_batch<2>, dim3(chunks), dim3(OPEN_T), 0, st, dd.p, nd, twf,
                       partial.p);
  else
    hipLaunchKernelGGL(k_open_partial_batch<1>, dim3(chunks), dim3(OPEN_T), 0, st, dd.p, nd, twf,
                       partial.p);
  KCHECK();
  if (probe.on) probe.end(ev0, st, obytes, np == 2 ? "k_open_partial_batch<2>" : "k_open_partial_batch<1>");
  if (np == 2)
    hipLaunchKernelGGL(k_open_final_batch<2>, dim3(cols), dim3(256), 0, st, dd.p, nd, partial.p);
  else
    hipLaunchKernelGGL(k_open_final_batch<1>, dim3(cols), dim3(256), 0, st, dd.p, nd, partial.p);
  KCHECK();
}

// One block per reduction job (LDE height): the columns' alpha powers and the job's ya / yb
// (block sum), and its matrices' kb.
__device__ __forceinline__ EF ef_pow_u32(EF a, uint32_t e) {
  EF r = ef_one();
  while (e) {
    if (e & 1) r = ef_mul(r, a);
    a = ef_mul(a, a);
    e >>= 1;
  }
  return r;
}
__global__ __launch_bounds__(256) void k_reduce_prep(RedCol* __restrict__ cols,
                                                     const RedColPrep* __restrict__ cp,
                                                     RedMat* __restrict__ mats,
                                                     const RedMatPrep* __restrict__ mp,
                                                     const RedJobPrep* __restrict__ jp,
                                                     const EF* __restrict__ opened,
                                                     const EF* __restrict__ alpha_p,
                                                     EF* __restrict__ yab) {
  const RedJobPrep j = jp[blockIdx.x];
  const EF alpha = *alpha_p;
  EF ya = ef_zero(), yb = ef_zero();
  for (uint32_t i = threadIdx.x; i < j.ncols; i += blockDim.x) {
    const RedColPrep p = cp[j.col0 + i];
    const EF ca = ef_pow_u32(alpha, p.e0);
    cols[j.col0 + i].ca = ca;
    ya = ef_add(ya, ef_mul(ca, opened[p.ia]));
    if (p.ib != 0xffffffffu) yb = ef_add(yb, ef_mul(ef_mul(ca, ef_pow_u32(alpha, p.w)), opened[p.ib]));
  }
  for (uint32_t i = threadIdx.x; i < j.nmats; i += blockDim.x) {
    const RedMatPrep m = mp[j.mat0 + i];
    mats[j.mat0 + i].kb = ef_mul_base(ef_pow_u32(alpha, m.w), m.fold);
  }
  __shared__ EF sh[2][4];
  ya = wave_sum(ya);
  yb = wave_sum(yb);
  if ((threadIdx.x & 63) == 0) {
    sh[0][threadIdx.x >> 6] = ya;
    sh[1][threadIdx.x >> 6] = yb;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    EF a = sh[0][0], b = sh[1][0];
    for (int q = 1; q < (int)(blockDim.x >> 6); q++) {
      a = ef_add(a, sh[0][q]);
      b = ef_add(b, sh[1][q]);
    }
    yab[2 * blockIdx.x] = a;
    yab[2 * blockIdx.x + 1] = ef_mul_base(b, j.yb_fold);
  }
}

void reduce_prep(RedCol* cols, const RedColPrep* cp, RedMat* mats, const RedMatPrep* mp,
                 const RedJobPrep* jp, int njobs, const EF* opened, const EF* alpha, EF* yab,
                 hipStream_t st) {
  if (njobs <= 0) return;
  hipLaunchKernelGGL(k_reduce_prep, dim3(njobs), dim3(256), 0, st, cols, cp, mats, mp, jp, opened,
                     alpha, yab);
  KCHECK();
}

// k_reduce's grid-stride cap in workgroups (8k: 0.02-0.04 ms slower, profiles/r02/ab_reduce_grid.txt)
constexpr unsigned RED_GRID = 32768;
void reduce_range(const RedCol* cols, const RedMat* mats, int nmats, size_t height, size_t t0,
                  size_t count, const EF* invd_a, const EF* invd_b, const EF* yab,
                  bool has_b, EF* ro, hipStream_t st, int ncols) {
  const unsigned grid = std::min<unsigned>(ceil_div(count, 256), RED_GRID);
  KernelProbe& probe = reduce_probe();
  hipEvent_t ev0 = probe.on ? probe.begin(st) : nullptr;
  hipLaunchKernelGGL(k_reduce, dim3(grid), dim3(256), 0, st, cols, mats, nmats, t0, t0 + count,
                     invd_a, invd_b, yab, has_b ? 1 : 0, log2i(height), ro);
  KCHECK();
  // the columns' words, the denominator tables read (one or two points) and ro written
  if (probe.on) probe.end(ev0, st, (double)count * (4.0 * ncols + 16.0 * (has_b ? 3 : 2)));
}

void fri_challenge(uint32_t* state, const uint32_t* root, EF* beta, hipStream_t st) {
  hipLaunchKernelGGL(k_fri_challenge, dim3(1), dim3(64), 0, st, state, root, beta);
  KCHECK();
}

void fri_fold_dev(const EF* in, EF* out, size_t h, const EF* beta, const EF* add, hipStream_t st) {
  fri_fold_range(in, out, h, 0, h, beta, add, st);
}

void fri_fold_range(const EF* in, EF* out, size_t h, size_t i0, size_t count, const EF* beta,
                    const EF* add, hipStream_t st) {
  const int logh = log2i(h);
  twiddles().ensure(logh + 1);
  hipLaunchKernelGGL(k_fri_fold_dev, dim3(ceil_div(count, 256)), dim3(256), 0, st, in, out, h,
                     logh, i0, count, beta, (const uint32_t*)twiddles().inv(), add);
  KCHECK();
}

void fri_fold_leaves(const EF* in, EF* out, size_t h, const EF* beta, const EF* add,
                     uint32_t* digests, hipStream_t st) {
  const int logn = log2i(2 * h);
  twiddles().ensure(logn + 1);
  const uint32_t* twi = (const uint32_t*)twiddles().inv();
  KernelProbe& probe = p2_probe();
  hipEvent_t ev0 = probe.on ? probe.begin(st) : nullptr;
  hipLaunchKernelGGL(k_fold_leaves, dim3(ceil_div(h, 256)), dim3(256), 0, st, in, out, h, logn,
                     beta, twi, add, digests);
  if (probe.on) probe.end(ev0, st, (double)h);
  KCHECK();
}

void fri_tail_rounds(const FriTailRounds& a, hipStream_t st) {
  if (a.nr < 1 || a.nr > FRI_TAIL_MAXR || a.logh0 < a.nr || (1 << a.logh0) > FRI_TAIL_MAXH)
    throw std::runtime_error("fri_tail_rounds: bad round count");
  twiddles().ensure(a.logh0 + 1);
  hipLaunchKernelGGL(k_fri_tail, dim3(1), dim3(1024), 0, st, a, (const uint32_t*)twiddles().inv());
  KCHECK();
}

void fri_transcript_tail(DevChallenger* c, const uint32_t* fri_state, const EF* fin, int bits,
                         int nq, int log_max, uint32_t* qidx, uint32_t* res, hipStream_t st) {
  if (bits < 0 || bits > 30 || log_max < 0 || log_max > 31 || nq < 0)
    throw std::runtime_error("fri_transcript_tail: bad parameters");
  hipLaunchKernelGGL(k_fri_finish, dim3(1), dim3(64), 0, st, c, fri_state, fin, res);
  KCHECK();
  // 2^(bits+1) candidates per chunk (2^17 at 16 bits: the first chunk holds a witness with
  // probability 1 - e^-2; a further chunk costs ~10 us and no round trip, where 2^18 per chunk
  // took 31 us)
  const uint32_t chunk = 1u << std::min(22, std::max(16, bits + 1));
  hipLaunchKernelGGL(k_grind, dim3(chunk / 256), dim3(256), 0, st, (const DevChallenger*)c,
                     (uint32_t)bits, res);
  KCHECK();
  hipLaunchKernelGGL(k_sample_queries, dim3(1), dim3(64), 0, st, c, bits, nq, log_max, qidx, res);
  KCHECK();
}

size_t query_words(const std::vector<GatherSeg>& segs) {
  size_t w = 0;
  for (const GatherSeg& g : segs) w += g.count;
  return w;
}

void gather_queries(const std::vector<GatherSeg>& segs, const uint32_t* qidx, int nq, uint32_t* out,
                    const ShardCtx* shard, hipStream_t st) {
  const int rank = shard ? shard->rank : 0;
  std::vector<uint32_t> off(segs.size());
  uint32_t wpq = 0;
  for (size_t s = 0; s < segs.size(); s++) {
    off[s] = wpq;
    wpq += segs[s].count;
  }
  const size_t nwords = (size_t)wpq * nq;
  if (!nwords) return;
  DBuf<GatherSeg> dseg(segs.size());
  DBuf<uint32_t> doff(off.size());
  upload_async(dseg.p, segs.data(), segs.size() * sizeof(GatherSeg), st);
  upload_async(doff.p, off.data(), off.size() * 4, st);
  const size_t nthreads = segs.size() * (size_t)nq;
  hipLaunchKernelGGL(k_gather_segs, dim3(ceil_div(nthreads, 256)), dim3(256), 0, st,
                     (const GatherSeg*)dseg.p, (int)segs.size(), (const uint32_t*)doff.p, wpq,
                     qidx, nq, rank, out);
  KCHECK();
  if (shard && shard->world > 1) {  // owner-masked words: one sum all-reduce, device to device
    coll_sync(st);
    shard->allreduce_sum_u32(out, nwords);
  }
}

// kernels a proof launches (gpu.h PreloadKernels)
static PreloadKernels preload_fri{
    (const void*)&k_inv_denoms,
    (const void*)&k_open_partial_batch<1>,
    (const void*)&k_open_partial_batch<2>,
    (const void*)&k_open_final_batch<1>,
    (const void*)&k_open_final_batch<2>,
    (const void*)&k_reduce,
    (const void*)&k_reduce_prep,
    (const void*)&k_fri_fold_dev,
    (const void*)&k_fold_leaves,
    (const void*)&k_fri_challenge,
    (const void*)&k_fri_tail,
    (const void*)&k_fri_finish,
    (const void*)&k_grind,
    (const void*)&k_sample_queries,
    (const void*)&k_gather_segs};

}  // namespace bfz
