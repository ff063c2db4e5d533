// Quotient evaluation on the device: quotient_values (crates/stark/src/quotient.rs:18-165)
// with the ProverConstraintFolder fold (folder.rs:68-89) and Chip::eval (chip.rs:222-228).
//
// Point i of the quotient domain 3*H_2n (natural index) sits at storage position
// t = bitrev(i) of every LDE; its "next" row is i+2 (quotient.rs:41-42, next_step = 2).
// Selectors [p3-recalled selectors_on_coset]: Z_H(x) = x^n - 1 (= 3^n (-1)^i - 1),
// is_first = Z_H/(x-1), is_last = Z_H/(x - w_n^-1), is_transition = x - w_n^-1.
// The Horner fold acc = acc*alpha + c_k is computed as sum_k alpha^(K-1-k) c_k (identical
// value): base-valued AIR constraints cost 4 base multiplies each instead of an EF multiply.
// Output: Q(x_i) for storage position t lands in quotient chunk (t >> log n) at row
// (t mod n) -- the bit-reversed evaluation order of chunk i mod 2 on its domain
// 3 w_2n^k H_n (split_evals / split_domains), ready for the chunk LDE.
#include "quotient.h"

#include <mutex>

#include <array>
#include <map>

#include "air.h"

namespace bfz {

using namespace kb;

constexpr int QMAIN_W[NUM_CHIPS] = {31, 1, 7, 45, 12, 2, 41, 5};
constexpr int QPREP_W[NUM_CHIPS] = {0, 6, 0, 0, 0, 2, 0, 0};
constexpr int QPERM_W[NUM_CHIPS] = {9, 2, 4, 2, 3, 2, 2, 2};

// Lazy fold of the constraints: raw 64-bit products of Montgomery values accumulate with
// v_mad_u64_u32 (a base constraint times its EF alpha power is one multiply-add per
// component instead of a Montgomery product + modular add).  Budget: a raw product is < p^2
// (1 unit), a reduced EF term added at scale 2^32 is < 2 p^2 (2 units); the accumulator is
// folded (hi * (2^32 mod p) + lo < 2^57) before 4 units would be exceeded (4 p^2 + 2^57 <
// 2^64), and reduced once at the end -- the same field element as the eager sum.
struct PowAcc {
  static constexpr uint32_t C32 = (1u << 25) - 2;  // 2^32 mod p
  uint64_t a64[4];
  int units;
  // alpha powers, read through the constant address space: the pointer now comes from device
  // memory (QuotParams), and through a generic pointer the reads became vector flat loads (+19
  // VGPRs, k_quotient<0> 930 -> 1031 us); as constant-space loads they stay scalar.
  const __attribute__((address_space(4))) uint32_t* ap;
  int k;
  __device__ __forceinline__ EF pow_k() {
    EF a;
#pragma unroll
    for (int e = 0; e < 4; e++) a.c[e] = ap[4 * k + e];
    k++;
    return a;
  }
  __device__ __forceinline__ void fold() {
#pragma unroll
    for (int e = 0; e < 4; e++) a64[e] = (uint64_t)(uint32_t)(a64[e] >> 32) * C32 + (uint32_t)a64[e];
    units = 0;
  }
  __device__ __forceinline__ void emit(uint32_t c) {
    if (units + 1 > 4) fold();
    const EF a = pow_k();
#pragma unroll
    for (int e = 0; e < 4; e++) a64[e] += (uint64_t)a.c[e] * c;
    units += 1;
  }
  __device__ __forceinline__ void emit_ext(const EF& c) {
    if (units + 2 > 4) fold();
    const EF r = ef_mul(pow_k(), c);
#pragma unroll
    for (int e = 0; e < 4; e++) a64[e] += (uint64_t)r.c[e] << 32;
    units += 2;
  }
  __device__ __forceinline__ EF value() {
    fold();
    EF r;
#pragma unroll
    for (int e = 0; e < 4; e++) r.c[e] = mred_lt_p(a64[e]);  // folded: < 2^57
    return r;
  }
};

// x_i = 3 w_N^i, the natural point i of the quotient domain 3 H_N (twf[N/2 + j] = w_N^j).
__device__ __forceinline__ uint32_t quot_point(uint32_t i, uint32_t half, uint32_t shift,
                                               const uint32_t* __restrict__ twf) {
  const uint32_t w = i < half ? twf[half + i] : mneg(twf[i]);  // twf[half + (i - half)]
  return mmul(shift, w);
}

// 1 / ((x - 1)(x - w_n^-1)) at every point of 3 H_N, stored by LDE position t (point
// bitrev(t)): the selector denominators depend on the domain alone, so one table per log N
// serves every chip of that height in every proof (built once, cached).
__global__ __launch_bounds__(256) void k_sel_inv(int logN, uint32_t shift, uint32_t wn_inv,
                                                 const uint32_t* __restrict__ twf,
                                                 uint32_t* __restrict__ out) {
  const size_t N = (size_t)1 << logN;
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= N) return;
  const uint32_t x = quot_point(dbitrev((uint32_t)t, logN), (uint32_t)(N >> 1), shift, twf);
  out[t] = minv(mmul(msub(x, ONE), msub(x, wn_inv)));
}

// Register budget sized for 3 blocks per CU (4 spilled and was slower,
// profiles/r02/ab_quotient_occupancy.txt).
template <int CHIP>
__global__ __launch_bounds__(256, 3) void k_quotient(QuotRows in, int logN,
                                                  const QuotParams* __restrict__ qpp,
                                                  const uint32_t* __restrict__ twf,
                                                  const uint32_t* __restrict__ sel_inv,
                                                  QuotOut qo) {
  const QuotParams qp = *qpp;  // device memory (the challenges are sampled on the device)
  constexpr int MW = QMAIN_W[CHIP];
  constexpr int PWD = QPREP_W[CHIP] > 0 ? QPREP_W[CHIP] : 1;
  constexpr int PMW = QPERM_W[CHIP];
  const size_t N = (size_t)1 << logN, n = N >> 1;
  const size_t t = in.t0 + (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= in.t0 + in.count) return;
  const uint32_t i = dbitrev((uint32_t)t, logN);
  const uint32_t inext = (i + 2) & (uint32_t)(N - 1);
  const size_t tn = dbitrev(inext, logN);

  // buffer loads: one descriptor per column (its base is wave-uniform: scalar arithmetic), the
  // row is the voffset -- no 64-bit address per column in VGPRs, and no 2 GiB limit on a whole
  // column set (a 2^24-row LDE of 36 columns spans 2.4 GB)
  uint32_t L[MW], Nx[MW], PL[PWD], PN[PWD];
  const uint32_t vt = (uint32_t)(t - in.t0) * 4u, vn = (uint32_t)tn * 4u;
#pragma unroll
  for (int c = 0; c < MW; c++) {
    L[c] = ld_b(rsrc_of(in.main_l + (size_t)c * in.stride + in.t0), vt, 0);
    Nx[c] = ld_b(rsrc_of(in.main_n + (size_t)in.nmain[c] * in.stride), vn, 0);
  }
#pragma unroll
  for (int c = 0; c < PWD; c++) {
    PL[c] = QPREP_W[CHIP] > 0 ? in.prep[(size_t)c * N + t] : 0;
    PN[c] = QPREP_W[CHIP] > 0 ? in.prep[(size_t)c * N + tn] : 0;
  }
  EF pl[PMW], pn[PMW];
#pragma unroll
  for (int e = 0; e < PMW; e++)
#pragma unroll
    for (int k = 0; k < 4; k++) {
      pl[e].c[k] = ld_b(rsrc_of(in.perm_l + (size_t)(4 * e + k) * in.stride + in.t0), vt, 0);
      pn[e].c[k] = ld_b(rsrc_of(in.perm_n + (size_t)in.nperm[4 * e + k] * in.stride), vn, 0);
    }

  const uint32_t x = quot_point(i, (uint32_t)n, qp.shift, twf);
  const uint32_t zh = (i & 1) ? qp.zh_odd : qp.zh_even;
  const uint32_t zh_inv = (i & 1) ? qp.zh_odd_inv : qp.zh_even_inv;
  const uint32_t a = msub(x, ONE), b = msub(x, qp.wn_inv);
  const uint32_t inv_ab = sel_inv[t];  // 1 / (a b)
  const uint32_t zi = mmul(zh, inv_ab);
  const uint32_t is_first = mmul(zi, b), is_last = mmul(zi, a), is_trans = b;

  PowAcc acc{{0, 0, 0, 0}, 0,
             (const __attribute__((address_space(4))) uint32_t*)qp.alpha_pows, 0};
  Air<BaseOps, PowAcc> air{L, Nx, PL, PN, is_first, is_last, is_trans, acc};
  air.template eval_air<CHIP>();
  air.template eval_perm<CHIP>(pl, pn, qp.perm_alpha, qp.beta_pows, qp.cumsum, ef_base(is_first),
                               ef_base(is_last), ef_base(is_trans));
  const EF q = ef_mul_base(acc.value(), zh_inv);
  const size_t chunk = t >> (logN - 1), pos = t & (n - 1);
#pragma unroll
  for (int e = 0; e < 4; e++) qo.chunk[chunk][e * qo.stride + pos] = q.c[e];
}

template <int CHIP>
static void launch_q(const QuotRows& in, int logN, const QuotParams* qp_dev, const uint32_t* sel,
                     const QuotOut& qo, hipStream_t st) {
  hipLaunchKernelGGL(k_quotient<CHIP>, dim3(ceil_div(in.count, 256)), dim3(256), 0, st, in, logN,
                     qp_dev, (const uint32_t*)twiddles().fwd(), sel, qo);
  KCHECK();
}

// The selector-denominator table of 3 H_N (k_sel_inv), built on first use per log N.  It is
// written on the prover stream, so every later reader on that stream sees it complete.
static const uint32_t* sel_inv_table(int logN, const QuotParams& qp, hipStream_t st) {
  static std::mutex mu;  // shared by the proof lanes
  std::lock_guard<std::mutex> lk(mu);
  static auto* cache = new std::map<int, DBuf<uint32_t>>();
  auto it = cache->find(logN);
  if (it != cache->end()) return it->second.p;
  const size_t N = (size_t)1 << logN;
  ResidentScope rs;  // cached for the process, not part of the lane's working set
  DBuf<uint32_t> d(N);
  hipLaunchKernelGGL(k_sel_inv, dim3(ceil_div(N, 256)), dim3(256), 0, st, logN, qp.shift,
                     qp.wn_inv, (const uint32_t*)twiddles().fwd(), d.p);
  KCHECK();
  HIP_CHECK(hipStreamSynchronize(st));  // complete before another lane's stream reads it
  const uint32_t* p = d.p;
  cache->emplace(logN, std::move(d));
  return p;
}

void prepare_quotient_tables(int logN) {
  twiddles().ensure(logN);
  QuotParams qp{};  // the fields k_sel_inv reads (prover.hip quotient stage)
  qp.shift = to_mont(3);
  qp.wn_inv = minv(two_adic_gen(logN - 1));
  (void)sel_inv_table(logN, qp, stream());
}

void quotient(int chip, const uint32_t* mainc, const uint32_t* prepc, const uint32_t* permc,
              int logN, const QuotParams& qp, uint32_t* qout, hipStream_t st) {
  const size_t N = (size_t)1 << logN;
  QuotRows in{mainc, mainc, permc, permc, prepc, N, 0, N, {}, {}};
  for (int c = 0; c < 64; c++) in.nmain[c] = in.nperm[c] = (uint8_t)c;
  quotient_rows(chip, in, logN, qp, qout, st);
}

void quotient_rows(int chip, const QuotRows& in, int logN, const QuotParams& qp, uint32_t* qout,
                   hipStream_t st, const QuotParams* qp_dev) {
  const size_t n = (size_t)1 << (logN - 1);
  quotient_into(chip, in, logN, qp, QuotOut{{qout, qout + 4 * n}, n}, st, qp_dev);
}

void quotient_into(int chip, const QuotRows& in, int logN, const QuotParams& qp, const QuotOut& qout,
                   hipStream_t st, const QuotParams* qp_dev) {
  twiddles().ensure(logN);
  const uint32_t* sel = sel_inv_table(logN, qp, st);
  DBuf<QuotParams> up;
  if (!qp_dev) {  // the host's parameters, uploaded (stream-ordered: freed after the launch is fine)
    up.reset(1);
    upload_async(up.p, &qp, sizeof(qp), st);
    qp_dev = up.p;
  }
  switch (chip) {
    case CHIP_CPU: launch_q<CHIP_CPU>(in, logN, qp_dev, sel, qout, st); break;
    case CHIP_PROGRAM: launch_q<CHIP_PROGRAM>(in, logN, qp_dev, sel, qout, st); break;
    case CHIP_ADDSUB: launch_q<CHIP_ADDSUB>(in, logN, qp_dev, sel, qout, st); break;
    case CHIP_JUMP: launch_q<CHIP_JUMP>(in, logN, qp_dev, sel, qout, st); break;
    case CHIP_MEMORY: launch_q<CHIP_MEMORY>(in, logN, qp_dev, sel, qout, st); break;
    case CHIP_BYTE: launch_q<CHIP_BYTE>(in, logN, qp_dev, sel, qout, st); break;
    case CHIP_MEMINSTRS: launch_q<CHIP_MEMINSTRS>(in, logN, qp_dev, sel, qout, st); break;
    case CHIP_IO: launch_q<CHIP_IO>(in, logN, qp_dev, sel, qout, st); break;
    default: throw std::runtime_error("quotient: bad chip");
  }
}

// The quotient challenge on the device (challenger.h): the sponge observes the permutation
// root and every chip's cumulative sum, samples alpha (prover.rs:336-342); each chip's alpha
// powers alpha^(K-1-j) and the challenge fields of its QuotParams are written.
// Every 16-lane row runs the sponge (the same values); the powers are then spread over the whole
// block, one (chip, j) pair per thread (64 threads looping over the chips took 28 us).
constexpr int QCH_THREADS = 1024;
__global__ __launch_bounds__(QCH_THREADS) void k_challenge_quot(DevChallenger* __restrict__ c,
                                                                const uint32_t* __restrict__ root,
                                                                const EF* __restrict__ cums, int nc,
                                                                const PermChallenges* __restrict__ pc,
                                                                QuotParams* __restrict__ qps,
                                                                QuotAlphaTargets tg) {
  __shared__ EF s_alpha;
  if (threadIdx.x < 64) {  // one wave: the sponge
    LaneSponge sp;
    sp.load(c);
    for (int i = 0; i < 8; i++) sp.observe(root[i]);
    for (int k = 0; k < nc; k++)
      for (int e = 0; e < 4; e++) sp.observe(cums[k].c[e]);
    const EF alpha = sp.sample_ef();
    sp.store(c);
    if (threadIdx.x == 0) {
      s_alpha = alpha;
      if (tg.alpha_out) *tg.alpha_out = alpha;
    }
  }
  __syncthreads();
  const EF a = s_alpha;
  int total = 0;
  for (int k = 0; k < nc; k++) total += tg.K[k];
  for (int t = threadIdx.x; t < total; t += blockDim.x) {
    int k = 0, j = t;
    while (j >= tg.K[k]) j -= tg.K[k++];
    tg.apows[k][j] = ef_pow(a, (uint64_t)(tg.K[k] - 1 - j));
  }
  if (threadIdx.x < nc) {
    QuotParams& q = qps[threadIdx.x];
    q.perm_alpha = pc->alpha;
    for (int j = 0; j < 8; j++) q.beta_pows[j] = pc->beta_pows[j];
    q.cumsum = cums[threadIdx.x];
  }
}

void challenge_quot(DevChallenger* ch, const uint32_t* root, const EF* cums, int nc,
                    const PermChallenges* pc, QuotParams* qps, const QuotAlphaTargets& tg,
                    hipStream_t st) {
  if (nc > QUOT_MAX_CHIPS) throw std::runtime_error("challenge_quot: too many chips");
  hipLaunchKernelGGL(k_challenge_quot, dim3(1), dim3(QCH_THREADS), 0, st, ch, root, cums, nc, pc, qps, tg);
  KCHECK();
}

}  // namespace bfz

namespace bfz {

template <int CHIP>
static int count_chip() {
  EF z[64];
  for (auto& e : z) e = kb::ef_zero();
  CountAcc acc;
  Air<ExtOps, CountAcc> air{z, z, z, z, z[0], z[0], z[0], acc};
  air.template eval_air<CHIP>();
  EF bp[8];
  for (auto& e : bp) e = kb::ef_zero();
  air.template eval_perm<CHIP>(z, z, z[0], bp, z[0], z[0], z[0], z[0]);
  return acc.n;
}

// The count is a property of the AIR: evaluated symbolically once per chip and cached (the
// prover needs it for every chip of every proof).
static int num_constraints_eval(int chip) {
  switch (chip) {
    case CHIP_CPU: return count_chip<CHIP_CPU>();
    case CHIP_PROGRAM: return count_chip<CHIP_PROGRAM>();
    case CHIP_ADDSUB: return count_chip<CHIP_ADDSUB>();
    case CHIP_JUMP: return count_chip<CHIP_JUMP>();
    case CHIP_MEMORY: return count_chip<CHIP_MEMORY>();
    case CHIP_BYTE: return count_chip<CHIP_BYTE>();
    case CHIP_MEMINSTRS: return count_chip<CHIP_MEMINSTRS>();
    case CHIP_IO: return count_chip<CHIP_IO>();
  }
  return 0;
}

int num_constraints(int chip) {
  static const auto counts = [] {
    std::array<int, NUM_CHIPS> c{};
    for (int i = 0; i < NUM_CHIPS; i++) c[i] = num_constraints_eval(i);
    return c;
  }();
  if (chip < 0 || chip >= NUM_CHIPS) return 0;
  return counts[chip];
}

// kernels a proof launches (gpu.h PreloadKernels)
static PreloadKernels preload_quotient{
    (const void*)&k_quotient<0>,
    (const void*)&k_quotient<1>,
    (const void*)&k_quotient<2>,
    (const void*)&k_quotient<3>,
    (const void*)&k_quotient<4>,
    (const void*)&k_quotient<5>,
    (const void*)&k_quotient<6>,
    (const void*)&k_quotient<7>,
    (const void*)&k_sel_inv,
    (const void*)&k_challenge_quot};

}  // namespace bfz
