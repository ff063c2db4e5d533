// LogUp permutation trace on the device: generate_permutation_trace
// (crates/stark/src/permutation.rs:75-148, row fn populate_permutation_row :27-69).
//
// Row r, batch b (interactions 2b, 2b+1 of the chain sends++receives):
//     perm[r][b] = sum_j  (+-m_j) / (alpha + kind_j + sum_k beta^(k+1) v_jk)
// last column = inclusive prefix sum over rows of sum_b perm[r][b]; cumulative_sum = last.
// One thread per storage position (bit-reversed row); per row the batch denominators are
// inverted together (Montgomery trick: one EF inversion per row).  The running sum is a
// natural-order scan, so row sums are gathered into natural order, scanned, and scattered
// back into the bit-reversed last column.
#include "logup.h"

#include <type_traits>

#include "poseidon2.h"

namespace bfz {

using namespace kb;

constexpr int MAIN_W[NUM_CHIPS] = {31, 1, 7, 45, 12, 2, 41, 5};
constexpr int PREP_W[NUM_CHIPS] = {0, 6, 0, 0, 0, 2, 0, 0};

template <int I, int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<I + 1, N>(f);
  }
}

// denominator alpha + kind + sum_k beta^(k+1) v_k and signed multiplicity of interaction J
template <int CHIP, int J, int MW, int PWD>
__device__ __forceinline__ void interaction(const uint32_t (&pr)[PWD], const uint32_t (&m)[MW],
                                            const PermChallenges& ch, EF& den, uint32_t& mult) {
  constexpr Lookup lk = LookupsOf<CHIP>::v.l[J];
  // the products accumulate unreduced in 64 bits (LazyEF): one reduction per component
  LazyEF lz;
  lz.init();
#pragma unroll
  for (int v = 0; v < lk.nvals; v++) lz.add(ch.beta_pows[v + 1], vcol_eval<BaseOps>(lk.vals[v], pr, m));
  den = ef_add(lz.get(), ef_add(ch.alpha, ef_base(to_mont_c(lk.kind))));
  const uint32_t mu = vcol_eval<BaseOps>(lk.mult, pr, m);
  mult = lk.send ? mu : mneg(mu);
}

// batch b: numerator / denominator of m_0/d_0 + m_1/d_1 (or m_0/d_0 for a trailing single)
template <int CHIP, int B, int MW, int PWD>
__device__ __forceinline__ void batch_frac(const uint32_t (&pr)[PWD], const uint32_t (&m)[MW],
                                           const PermChallenges& ch, EF& num, EF& den) {
  constexpr int N = LookupsOf<CHIP>::v.n;
  EF d0;
  uint32_t m0;
  interaction<CHIP, 2 * B>(pr, m, ch, d0, m0);
  if constexpr (2 * B + 1 < N) {
    EF d1;
    uint32_t m1;
    interaction<CHIP, 2 * B + 1>(pr, m, ch, d1, m1);
    num = ef_add(ef_mul_base(d1, m0), ef_mul_base(d0, m1));
    den = ef_mul(d0, d1);
  } else {
    num = ef_base(m0);
    den = d0;
  }
}

// The Cpu instance holds ~246 VGPRs (2 waves/SIMD); forcing 3 waves spilled and was slower
// (profiles/r02/ab_perm_occupancy.txt).
template <int CHIP>
__global__ __launch_bounds__(256) void k_perm_rows(const uint32_t* __restrict__ mainc,
                                                   const uint32_t* __restrict__ prepc, size_t n,
                                                   const PermChallenges* __restrict__ chp,
                                                   uint32_t* __restrict__ perm,
                                                   EF* __restrict__ rowsum) {
  const PermChallenges ch = *chp;  // uniform: scalar loads
  constexpr int MW = MAIN_W[CHIP];
  constexpr int PWD = PREP_W[CHIP] > 0 ? PREP_W[CHIP] : 1;
  constexpr int NB = (LookupsOf<CHIP>::v.n + 1) / 2;
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  uint32_t m[MW], pr[PWD];
#pragma unroll
  for (int c = 0; c < MW; c++) m[c] = mainc[(size_t)c * n + t];
#pragma unroll
  for (int c = 0; c < PWD; c++) pr[c] = PREP_W[CHIP] > 0 ? prepc[(size_t)c * n + t] : 0;
  // Batches are paired: pair q has denominator D_q = d_a d_b (or d_a alone).  1/D_q =
  // conj(D_q) / N(D_q), where conj = frob1 frob2 frob3 and the norm N is a base-field value,
  // and the norms of all pairs share one base-field inversion (Montgomery's trick): one
  // Fermat exponentiation per row instead of one per pair.
  constexpr int NP = (NB + 1) / 2;
  EF xa[NP], xb[NP], cj[NP];  // xa = n_a d_b, xb = n_b d_a: v_a = xa / D, v_b = xb / D
  uint32_t nrm[NP], pre[NP];
  static_for<0, NP>([&](auto P) {
    constexpr int q = decltype(P)::value, BA = 2 * q, BB = BA + 1;
    EF na, da;
    batch_frac<CHIP, BA>(pr, m, ch, na, da);
    EF D = da;
    if constexpr (BB < NB) {
      EF nb, db;
      batch_frac<CHIP, BB>(pr, m, ch, nb, db);
      D = ef_mul(da, db);
      xa[q] = ef_mul(na, db);
      xb[q] = ef_mul(nb, da);
    } else {
      xa[q] = na;
    }
    cj[q] = ef_mul(ef_mul(ef_frob1(D), ef_frob2(D)), ef_frob3(D));
    const uint64_t w0 = (uint64_t)D.c[1] * cj[q].c[3] + (uint64_t)D.c[2] * cj[q].c[2] +
                        (uint64_t)D.c[3] * cj[q].c[1];
    nrm[q] = madd(mreduce((uint64_t)D.c[0] * cj[q].c[0]), mul3(mreduce(w0)));
    pre[q] = q ? mmul(pre[q ? q - 1 : 0], nrm[q]) : nrm[q];
  });
  uint32_t inv = minv(pre[NP - 1]);
  EF sum = ef_zero();
  static_for<0, NP>([&](auto P) {
    constexpr int q = NP - 1 - decltype(P)::value, BA = 2 * q, BB = BA + 1;
    const uint32_t inv_n = q ? mmul(inv, pre[q ? q - 1 : 0]) : inv;  // 1 / N(D_q)
    if (q) inv = mmul(inv, nrm[q]);
    const EF invD = ef_mul_base(cj[q], inv_n);
    const EF va = ef_mul(xa[q], invD);
#pragma unroll
    for (int e = 0; e < 4; e++) perm[(size_t)(4 * BA + e) * n + t] = va.c[e];
    sum = ef_add(sum, va);
    if constexpr (BB < NB) {
      const EF vb = ef_mul(xb[q], invD);
#pragma unroll
      for (int e = 0; e < 4; e++) perm[(size_t)(4 * BB + e) * n + t] = vb.c[e];
      sum = ef_add(sum, vb);
    }
  });
  rowsum[t] = sum;
}

// perm last EF column (4 base columns from col0) at storage position t <- phi(i), i = bitrev(t):
// phi(i) = block-local inclusive sum + the prefix of the blocks before (scan of block sums).
// The row t = n - 1 (= bitrev(n - 1)) also holds the cumulative sum.
__global__ __launch_bounds__(256) void k_write_phi(const EF* __restrict__ local, size_t n, int logn,
                                                   const EF* __restrict__ block_prefix,
                                                   uint32_t* __restrict__ perm, int col0,
                                                   EF* __restrict__ cumsum);

// --------------------------------------------------------------------- EF prefix scan
constexpr int SCAN_T = 256, SCAN_PER = 8, SCAN_BLOCK = SCAN_T * SCAN_PER;

// Block-local inclusive scan of natural-order blocks of SCAN_BLOCK values.  With logn >= 0 the
// input is read from bit-reversed storage (in[bitrev(i)]: the LogUp row sums), else in place.
__global__ __launch_bounds__(SCAN_T) void k_scan_block(const EF* __restrict__ in, int logn,
                                                       EF* __restrict__ data, size_t n,
                                                       EF* __restrict__ block_sums) {
  __shared__ EF sh[SCAN_T];
  const size_t base = (size_t)blockIdx.x * SCAN_BLOCK + (size_t)threadIdx.x * SCAN_PER;
  EF v[SCAN_PER];
  EF run = ef_zero();
#pragma unroll
  for (int k = 0; k < SCAN_PER; k++) {
    const size_t i = base + k;
    v[k] = i < n ? in[logn >= 0 ? dbitrev((uint32_t)i, logn) : i] : ef_zero();
    run = ef_add(run, v[k]);
    v[k] = run;
  }
  sh[threadIdx.x] = run;
  __syncthreads();
  for (int off = 1; off < SCAN_T; off <<= 1) {
    EF o = threadIdx.x >= (unsigned)off ? sh[threadIdx.x - off] : ef_zero();
    __syncthreads();
    sh[threadIdx.x] = ef_add(sh[threadIdx.x], o);
    __syncthreads();
  }
  const EF prefix = threadIdx.x ? sh[threadIdx.x - 1] : ef_zero();
#pragma unroll
  for (int k = 0; k < SCAN_PER; k++)
    if (base + k < n) data[base + k] = ef_add(v[k], prefix);
  if (threadIdx.x == SCAN_T - 1) block_sums[blockIdx.x] = sh[SCAN_T - 1];
}

__global__ __launch_bounds__(SCAN_T) void k_scan_add(EF* __restrict__ data, size_t n,
                                                     const EF* __restrict__ block_prefix) {
  if (blockIdx.x == 0) return;
  const EF p = block_prefix[blockIdx.x - 1];
  const size_t base = (size_t)blockIdx.x * SCAN_BLOCK;
  for (int k = threadIdx.x; k < SCAN_BLOCK; k += SCAN_T)
    if (base + k < n) data[base + k] = ef_add(data[base + k], p);
}

void ef_inclusive_scan(EF* data, size_t n, hipStream_t st) {
  const size_t nb = (n + SCAN_BLOCK - 1) / SCAN_BLOCK;
  DBuf<EF> sums(nb);
  hipLaunchKernelGGL(k_scan_block, dim3((unsigned)nb), dim3(SCAN_T), 0, st, (const EF*)data, -1,
                     data, n, sums.p);
  KCHECK();
  if (nb > 1) {
    ef_inclusive_scan(sums.p, nb, st);
    hipLaunchKernelGGL(k_scan_add, dim3((unsigned)nb), dim3(SCAN_T), 0, st, data, n,
                       (const EF*)sums.p);
    KCHECK();
  }
}

// ------------------------------------------------ LogUp running sum by tiles (n >= 2^11)
// Natural row i = x 2^(L-5) + z (x < 32, z < Z = n / 32) is stored at t = rev(z) 32 + rev5(x):
// for a fixed z the 32 rows x fill one contiguous run of storage.  A block owns the tile of
// every x and PHI_Z consecutive z and reads / writes whole runs (no bit-reversed gather):
//   k_phi_sums: the tile's sum per x -> S[x nb + b] (row-major = the natural order of tile rows);
//   ef_inclusive_scan(S): the natural-order prefix of every tile row;
//   k_phi_write: the tile's scans plus that prefix, written as the last EF column.
constexpr int PHI_X = 32, PHI_Z = 64, PHI_T = 256;  // 2048 rows per tile, 8 per thread
constexpr int PHI_LOG_MIN = 11;                      // Z >= PHI_Z

struct PhiTile {
  EF m[PHI_X][PHI_Z + 1];  // natural (x, z) order, padded
  EF part[PHI_T];
};

__device__ __forceinline__ void phi_load(PhiTile& tl, const EF* __restrict__ rows, int logn,
                                         size_t z0) {
  const int lz = logn - 5;
#pragma unroll
  for (int q = 0; q < PHI_X * PHI_Z / PHI_T; q++) {
    const int e = q * PHI_T + threadIdx.x, zl = e >> 5, xr = e & 31;
    const size_t t = ((size_t)dbitrev((uint32_t)(z0 + zl), lz) << 5) | (size_t)xr;
    tl.m[dbitrev((uint32_t)xr, 5)][zl] = rows[t];
  }
}

// this thread's 8 elements of tile row x = tid / 8 (z in [8 part, 8 part + 8)): local sum
__device__ __forceinline__ EF phi_part_sum(const PhiTile& tl) {
  const int x = threadIdx.x >> 3, part = threadIdx.x & 7;
  EF s = ef_zero();
#pragma unroll
  for (int k = 0; k < 8; k++) s = ef_add(s, tl.m[x][8 * part + k]);
  return s;
}

__global__ __launch_bounds__(PHI_T) void k_phi_sums(const EF* __restrict__ rows, int logn,
                                                    EF* __restrict__ sums) {
  __shared__ PhiTile tl;
  const size_t nb = ((size_t)1 << (logn - 5)) / PHI_Z, b = blockIdx.x;
  phi_load(tl, rows, logn, b * PHI_Z);
  __syncthreads();
  tl.part[threadIdx.x] = phi_part_sum(tl);
  __syncthreads();
  if ((threadIdx.x & 7) == 0) {
    EF s = ef_zero();
#pragma unroll
    for (int k = 0; k < 8; k++) s = ef_add(s, tl.part[threadIdx.x + k]);
    sums[(size_t)(threadIdx.x >> 3) * nb + b] = s;
  }
}

__global__ __launch_bounds__(PHI_T) void k_phi_write(const EF* __restrict__ rows, int logn,
                                                     const EF* __restrict__ scanned,
                                                     uint32_t* __restrict__ perm, int col0,
                                                     EF* __restrict__ cumsum) {
  __shared__ PhiTile tl;
  const size_t n = (size_t)1 << logn, nb = (n >> 5) / PHI_Z, b = blockIdx.x;
  const int lz = logn - 5;
  phi_load(tl, rows, logn, b * PHI_Z);
  __syncthreads();
  const int x = threadIdx.x >> 3, part = threadIdx.x & 7;
  tl.part[threadIdx.x] = phi_part_sum(tl);
  __syncthreads();
  // prefix of this thread's run: every earlier tile row (scan of S), then the earlier parts
  const size_t r = (size_t)x * nb + b;
  EF run = r ? scanned[r - 1] : ef_zero();
  for (int k = 0; k < part; k++) run = ef_add(run, tl.part[threadIdx.x - part + k]);
  __syncthreads();  // every part read before the tile is overwritten
#pragma unroll
  for (int k = 0; k < 8; k++) {
    run = ef_add(run, tl.m[x][8 * part + k]);
    tl.m[x][8 * part + k] = run;
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < PHI_X * PHI_Z / PHI_T; q++) {
    const int e = q * PHI_T + threadIdx.x, zl = e >> 5, xr = e & 31;
    const size_t t = ((size_t)dbitrev((uint32_t)(b * PHI_Z + zl), lz) << 5) | (size_t)xr;
    const EF v = tl.m[dbitrev((uint32_t)xr, 5)][zl];
#pragma unroll
    for (int c = 0; c < 4; c++) perm[(size_t)(col0 + c) * n + t] = v.c[c];
    if (t == n - 1) *cumsum = v;
  }
}

static bool phi_tiles_on() {  // BFZ_PHI_TILES=0: the round-5 gather scan (A/B)
  static const bool on = [] {
    const char* e = std::getenv("BFZ_PHI_TILES");
    return !(e && e[0] == '0');
  }();
  return on;
}

template <int CHIP>
static void launch_rows(const uint32_t* mainc, const uint32_t* prepc, size_t n,
                        const PermChallenges* ch, uint32_t* perm, EF* rowsum, hipStream_t st) {
  hipLaunchKernelGGL(k_perm_rows<CHIP>, dim3(ceil_div(n, 256)), dim3(256), 0, st, mainc, prepc, n,
                     ch, perm, rowsum);
  KCHECK();
}

void perm_trace(int chip, const uint32_t* mainc, const uint32_t* prepc, size_t n,
                const PermChallenges* ch, uint32_t* perm, EF* cumsum_dev, hipStream_t st) {
  const int logn = log2i(n);
  DBuf<EF> rows(n);
  switch (chip) {
    case CHIP_CPU: launch_rows<CHIP_CPU>(mainc, prepc, n, ch, perm, rows.p, st); break;
    case CHIP_PROGRAM: launch_rows<CHIP_PROGRAM>(mainc, prepc, n, ch, perm, rows.p, st); break;
    case CHIP_ADDSUB: launch_rows<CHIP_ADDSUB>(mainc, prepc, n, ch, perm, rows.p, st); break;
    case CHIP_JUMP: launch_rows<CHIP_JUMP>(mainc, prepc, n, ch, perm, rows.p, st); break;
    case CHIP_MEMORY: launch_rows<CHIP_MEMORY>(mainc, prepc, n, ch, perm, rows.p, st); break;
    case CHIP_BYTE: launch_rows<CHIP_BYTE>(mainc, prepc, n, ch, perm, rows.p, st); break;
    case CHIP_MEMINSTRS: launch_rows<CHIP_MEMINSTRS>(mainc, prepc, n, ch, perm, rows.p, st); break;
    case CHIP_IO: launch_rows<CHIP_IO>(mainc, prepc, n, ch, perm, rows.p, st); break;
    default: throw std::runtime_error("perm_trace: bad chip");
  }
  const int col0 = 4 * (perm_width(chip) - 1);
  if (logn >= PHI_LOG_MIN && phi_tiles_on()) {  // running sum by tiles of whole storage runs
    const size_t nt = (n >> 5) / PHI_Z;          // tiles per tile row
    DBuf<EF> sums(PHI_X * nt);
    hipLaunchKernelGGL(k_phi_sums, dim3((unsigned)nt), dim3(PHI_T), 0, st, (const EF*)rows.p, logn,
                       sums.p);
    KCHECK();
    ef_inclusive_scan(sums.p, PHI_X * nt, st);
    hipLaunchKernelGGL(k_phi_write, dim3((unsigned)nt), dim3(PHI_T), 0, st, (const EF*)rows.p,
                       logn, (const EF*)sums.p, perm, col0, cumsum_dev);
    KCHECK();
    return;
  }
  // running sum in natural row order: block-local scans read the bit-reversed row sums
  // directly, the block sums are scanned, and k_write_phi adds each block's prefix while
  // scattering phi back to bit-reversed storage
  const size_t nb = (n + SCAN_BLOCK - 1) / SCAN_BLOCK;
  DBuf<EF> sums(nb), nat(n);
  hipLaunchKernelGGL(k_scan_block, dim3((unsigned)nb), dim3(SCAN_T), 0, st, (const EF*)rows.p,
                     logn, nat.p, n, sums.p);
  KCHECK();
  if (nb > 1) ef_inclusive_scan(sums.p, nb, st);
  hipLaunchKernelGGL(k_write_phi, dim3(ceil_div(n, 256)), dim3(256), 0, st, (const EF*)nat.p, n,
                     logn, nb > 1 ? (const EF*)sums.p : nullptr, perm, col0, cumsum_dev);
  KCHECK();
}

__global__ __launch_bounds__(256) void k_write_phi(const EF* __restrict__ local, size_t n, int logn,
                                                   const EF* __restrict__ block_prefix,
                                                   uint32_t* __restrict__ perm, int col0,
                                                   EF* __restrict__ cumsum) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const size_t i = dbitrev((uint32_t)t, logn);
  EF v = local[i];
  const size_t b = i / SCAN_BLOCK;
  if (block_prefix && b > 0) v = ef_add(v, block_prefix[b - 1]);
#pragma unroll
  for (int e = 0; e < 4; e++) perm[(size_t)(col0 + e) * n + t] = v.c[e];
  if (t == n - 1) *cumsum = v;
}

// The LogUp challenges on the device (challenger.h): observe the main root, sample alpha, beta.
__global__ __launch_bounds__(64) void k_challenge_perm(DevChallenger* __restrict__ c,
                                                       const uint32_t* __restrict__ root,
                                                       PermChallenges* __restrict__ out) {
  LaneSponge sp;
  sp.load(c);
  for (int i = 0; i < 8; i++) sp.observe(root[i]);
  const EF alpha = sp.sample_ef();
  const EF beta = sp.sample_ef();
  sp.store(c);
  if (threadIdx.x == 0) {
    out->alpha = alpha;
    EF p = ef_one();
    for (int j = 0; j < 8; j++) {
      out->beta_pows[j] = p;
      p = ef_mul(p, beta);
    }
  }
}

void challenge_perm(DevChallenger* ch, const uint32_t* root, PermChallenges* out, hipStream_t st) {
  hipLaunchKernelGGL(k_challenge_perm, dim3(1), dim3(64), 0, st, ch, root, out);
  KCHECK();
}

__global__ __launch_bounds__(64) void k_challenge_zeta(DevChallenger* __restrict__ c,
                                                       const uint32_t* __restrict__ root,
                                                       EF* __restrict__ zeta) {
  LaneSponge sp;
  sp.load(c);
  for (int i = 0; i < 8; i++) sp.observe(root[i]);
  const EF z = sp.sample_ef();
  sp.store(c);
  if (threadIdx.x == 0) *zeta = z;
}

void challenge_zeta(DevChallenger* ch, const uint32_t* root, EF* zeta, hipStream_t st) {
  hipLaunchKernelGGL(k_challenge_zeta, dim3(1), dim3(64), 0, st, ch, root, zeta);
  KCHECK();
}

// kernels a proof launches (gpu.h PreloadKernels)
static PreloadKernels preload_logup{
    (const void*)&k_perm_rows<0>,
    (const void*)&k_perm_rows<1>,
    (const void*)&k_perm_rows<2>,
    (const void*)&k_perm_rows<3>,
    (const void*)&k_perm_rows<4>,
    (const void*)&k_perm_rows<5>,
    (const void*)&k_perm_rows<6>,
    (const void*)&k_perm_rows<7>,
    (const void*)&k_write_phi,
    (const void*)&k_scan_block,
    (const void*)&k_scan_add,
    (const void*)&k_phi_sums,
    (const void*)&k_phi_write,
    (const void*)&k_challenge_perm,
    (const void*)&k_challenge_zeta};

}  // namespace bfz
