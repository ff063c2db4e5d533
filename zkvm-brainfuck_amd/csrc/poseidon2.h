// Poseidon2KoalaBear<16> exactly as configured by the reference's my_perm()
// (crates/stark/src/kb31_poseidon2.rs:35-50 == crates/primitives/src/lib.rs:1101-1117):
// 8 external rounds (4 initial from RC rows 0..4, 4 terminal from rows 17..21), 13 internal
// rounds (first element of rows 4..17), S-box x^3.  Algorithm per the published Plonky3
// Poseidon2 [p3-recalled]: MDS-light (M4 = [[2,3,1,1],[1,2,3,1],[1,1,2,3],[3,1,1,2]] per
// 4-lane block + lane-wise block sum) before round 1 and after every external round;
// internal layer s_i <- sum + d_i * s_i, d = [-2,1,2,1/2,3,4,-1/2,-3,-4,1/2^8,1/8,1/2^24,
// -1/2^8,-1/8,-1/16,-1/2^24].
//
// All constants are folded to Montgomery form at compile time; with the rounds fully
// unrolled they become instruction literals / SGPR operands on gfx950.
#pragma once
#include "kb.h"

namespace kb {

struct P2Tables {
  uint32_t ext_init[4][16];
  uint32_t ext_term[4][16];
  uint32_t ext_init_r2[4][16];  // rc^M * R mod p: added to a 64-bit R^2-form value
  uint32_t ext_term_r2[4][16];
  uint32_t internal[13];
  uint32_t diag[16];
  uint32_t dabs[16];  // |d_i| (Montgomery)
};

constexpr uint32_t RC_RAW[30 * 16] = {
#include "rc_16_30.inc"
};

constexpr uint32_t cinv(uint32_t a) { return cpow(a, P - 2); }
constexpr uint32_t cneg(uint32_t a) { return a ? P - a : 0; }

constexpr P2Tables make_p2_tables() {
  P2Tables t{};
  for (int r = 0; r < 4; r++)
    for (int i = 0; i < 16; i++) {
      t.ext_init[r][i] = to_mont_c(RC_RAW[r * 16 + i] % P);
      t.ext_term[r][i] = to_mont_c(RC_RAW[(17 + r) * 16 + i] % P);
      t.ext_init_r2[r][i] = to_mont_c(t.ext_init[r][i]);
      t.ext_term_r2[r][i] = to_mont_c(t.ext_term[r][i]);
    }
  for (int r = 0; r < 13; r++) t.internal[r] = to_mont_c(RC_RAW[(4 + r) * 16] % P);
  uint32_t d[16] = {cneg(2),        1,          2,         cinv(2),          3,
                    4,              cneg(cinv(2)), cneg(3), cneg(4),          cinv(256),
                    cinv(8),        cinv(1u << 24), cneg(cinv(256)), cneg(cinv(8)), cneg(cinv(16)),
                    cneg(cinv(1u << 24))};
  uint32_t da[16] = {2, 1, 2, cinv(2), 3, 4, cinv(2), 3, 4, cinv(256), cinv(8), cinv(1u << 24),
                     cinv(256), cinv(8), cinv(16), cinv(1u << 24)};
  for (int i = 0; i < 16; i++) {
    t.diag[i] = to_mont_c(d[i]);
    t.dabs[i] = to_mont_c(da[i]);
  }
  return t;
}

constexpr P2Tables P2 = make_p2_tables();

// x^3: the square is left unreduced as a signed value in (-p, p/2) and fed to a signed
// Montgomery product (v_mad_i64_i32 / v_mul_hi_i32), whose result lies in (-p, p):
// one correction instead of two.
KB_HD uint32_t cube(uint32_t x) {
  const uint64_t t = (uint64_t)x * x;
  const uint32_t m = (uint32_t)t * MU;
  const int32_t x2 = (int32_t)(opaque((uint32_t)(t >> 32)) - (uint32_t)(((uint64_t)m * P) >> 32));
  const int64_t u = (int64_t)x2 * (int64_t)(int32_t)x;  // |u| < p^2 (x < p < 2^31)
  const uint32_t m2 = (uint32_t)u * MU;
  const int32_t mh = (int32_t)(((int64_t)(int32_t)m2 * (int64_t)P) >> 32);
  const uint32_t r = (uint32_t)((int32_t)(u >> 32) - mh);  // (-p, p)
  return umin(r, r + P);
}

// MDS-light in 64-bit adds (one half-rate v_lshl_add_u64 each, no reductions): M4 =
// [[2,3,1,1],[1,2,3,1],[1,1,2,3],[3,1,1,2]] per 4-element block, then each element gets the
// sum of the 4 blocks at its position.  A row's coefficients sum to 35.
constexpr uint32_t C32 = (1u << 25) - 2;  // 2^32 mod p
KB_HD void mds_light64(uint64_t s[16]) {
#pragma unroll
  for (int b = 0; b < 16; b += 4) {
    const uint64_t x0 = s[b], x1 = s[b + 1], x2 = s[b + 2], x3 = s[b + 3];
    const uint64_t t01 = x0 + x1, t23 = x2 + x3, t0123 = t01 + t23;
    const uint64_t t01123 = t0123 + x1, t01233 = t0123 + x3;
    s[b + 3] = t01233 + (x0 + x0);  // 3x0 + x1 + x2 + 2x3
    s[b + 1] = t01123 + (x2 + x2);  // x0 + 2x1 + 3x2 + x3
    s[b + 0] = t01123 + t01;        // 2x0 + 3x1 + x2 + x3
    s[b + 2] = t01233 + t23;        // x0 + x1 + 2x2 + 3x3
  }
  uint64_t sums[4];
#pragma unroll
  for (int k = 0; k < 4; k++) sums[k] = (s[k] + s[4 + k]) + (s[8 + k] + s[12 + k]);
#pragma unroll
  for (int i = 0; i < 16; i++) s[i] += sums[i & 3];
}
// ---- signed lazy form ------------------------------------------------------------------
// Between reductions every state element is a SIGNED Montgomery value (int32, |.| < p), and
// nothing is corrected back to [0, p) until the permutation's output.  The reduction uses a
// signed Montgomery factor: m = (int32)(lo p^-1), r = hi - mulhi_i32(m, p).  It is exact for
// any 64-bit two's-complement input (the low words cancel) and, with |mulhi| <= p/2, lands
// within p/2 of the input's high word — so no bias or correction is needed anywhere:
//  * external round (R^2-form, 64-bit): S-box a -> a^2 (reduced, in (-p/2, p)) -> a^2 * a
//    (x^3 R^2, |.| < p^2) -> fold to |.| < 2^55.1 -> MDS-light in 64-bit adds (|.| < 2^60.2)
//    -> + rc R^2 -> one reduction (|.| < p/2 + 2^28.2) = next S-box input, constant included.
//  * internal round: c = reduce(t0^3 R^2); T = c + sum t_i (exact, |T| < 16p);
//    S = reduce(T) (|S| < p/2 + 8) = sum of the plain values; t_i <- reduce(D_i t_i + S K [+ rc])
//    with D_i = d_i R and K = R^2 as centred residues (|.| <= p/2): |input| < 3p^2/4, so
//    |t_i| < 7p/8; the result is sum + d_i x_i in Montgomery form.  The next round's constant
//    rides on t_0's reduction (the terminal external round's on every element after the last
//    internal round).
constexpr int32_t centred(uint32_t x) { return x > P / 2 ? (int32_t)(x - P) : (int32_t)x; }
struct P2Signed {
  int32_t rc_init[4][16];  // centred rc R^2 (R^2-form constants)
  int32_t rc_term[4][16];
  int32_t rc_int[13];
  int32_t d[16];           // centred d_i R
  int32_t k;               // centred R^2
};
constexpr P2Signed make_p2_signed() {
  P2Signed t{};
  for (int r = 0; r < 4; r++)
    for (int i = 0; i < 16; i++) {
      t.rc_init[r][i] = centred(P2.ext_init_r2[r][i]);
      t.rc_term[r][i] = centred(P2.ext_term_r2[r][i]);
    }
  for (int r = 0; r < 13; r++) t.rc_int[r] = centred(to_mont_c(P2.internal[r]));
  for (int i = 0; i < 16; i++) t.d[i] = centred(P2.diag[i]);
  t.k = centred(R2);
  return t;
}
constexpr P2Signed P2S = make_p2_signed();

// Round constants moved in front of the MDS-light: the MDS layer M is linear
// and invertible, so M y + rc = M (y + K) with K = M^-1 rc (mod p).  K rides on the 64-bit
// addend of the S-box's last product (x^3 = m a + K, one v_mad_i64_i32 either way; |K| < p/2)
// or of the initial s * C32, and the separate 64-bit "+ rc" before each reduction is gone.
// M^-1 = (I4 (x) M4^-1)(I - J/5): M = (I + J (x) I4)(I4 (x) M4) with J the 4 x 4 all-ones
// block matrix, (I + J)^-1 = I - J/5 since J^2 = 4J.
struct P2Pre {
  int32_t init0[16];     // M^-1 rc_init[0], added to s * C32
  int32_t init[4][16];   // round r's S-box addend: M^-1 rc_init[r+1]; r = 3: M^-1 (rc_int[0] e0)
  int32_t term[4][16];   // M^-1 rc_term[r+1]; r = 3: none
};
constexpr uint32_t cmul_mod(uint32_t a, uint32_t b) { return (uint32_t)((uint64_t)a * b % P); }
constexpr void m4_inverse(uint32_t inv[4][4]) {
  constexpr uint32_t m4[4][4] = {{2, 3, 1, 1}, {1, 2, 3, 1}, {1, 1, 2, 3}, {3, 1, 1, 2}};
  uint32_t a[4][8] = {};
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 4; j++) {
      a[i][j] = m4[i][j];
      a[i][4 + j] = i == j;
    }
  for (int c = 0; c < 4; c++) {
    int piv = c;
    while (a[piv][c] == 0) piv++;
    for (int j = 0; j < 8; j++) {
      const uint32_t t = a[c][j];
      a[c][j] = a[piv][j];
      a[piv][j] = t;
    }
    const uint32_t iv = cpow(a[c][c], P - 2);
    for (int j = 0; j < 8; j++) a[c][j] = cmul_mod(a[c][j], iv);
    for (int i = 0; i < 4; i++)
      if (i != c && a[i][c]) {
        const uint32_t f = a[i][c];
        for (int j = 0; j < 8; j++) a[i][j] = (a[i][j] + P - cmul_mod(f, a[c][j])) % P;
      }
  }
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 4; j++) inv[i][j] = a[i][4 + j];
}
// canonical residues in, centred M^-1 v out
constexpr void mds_light_inverse(const uint32_t v[16], int32_t out[16]) {
  uint32_t inv[4][4] = {};
  m4_inverse(inv);
  const uint32_t inv5 = cpow(5, P - 2);
  uint32_t w[16] = {};
  for (int k = 0; k < 4; k++) {
    uint64_t sum = 0;
    for (int b = 0; b < 4; b++) sum += v[4 * b + k];
    const uint32_t s5 = cmul_mod((uint32_t)(sum % P), inv5);
    for (int b = 0; b < 4; b++) w[4 * b + k] = (v[4 * b + k] + P - s5) % P;
  }
  for (int b = 0; b < 4; b++)
    for (int i = 0; i < 4; i++) {
      uint64_t acc = 0;
      for (int j = 0; j < 4; j++) acc += (uint64_t)inv[i][j] * w[4 * b + j] % P;
      out[4 * b + i] = centred((uint32_t)(acc % P));
    }
}
constexpr P2Pre make_p2_pre() {
  P2Pre t{};
  mds_light_inverse(P2.ext_init_r2[0], t.init0);
  for (int r = 0; r < 3; r++) {
    mds_light_inverse(P2.ext_init_r2[r + 1], t.init[r]);
    mds_light_inverse(P2.ext_term_r2[r + 1], t.term[r]);
  }
  uint32_t e0[16] = {};
  e0[0] = to_mont_c(P2.internal[0]);  // rc_int[0] in R^2 form
  mds_light_inverse(e0, t.init[3]);
  return t;
}
constexpr P2Pre P2PRE = make_p2_pre();

// The diagonal entries d_i R include powers of two, and a sum of int32 terms into 64 bits
// sign-extends each term; the compiler would turn d * t + acc into 64-bit shifts and
// add/sub pairs, and t + acc into ashr + 64-bit add (2-3 half-rate ops where one
// v_mad_i64_i32 does).  On the device the multipliers therefore come from a constant-memory
// table the compiler cannot see into (scalar loads, hoisted into SGPRs); a distinct 1 per sum
// term stops it from factoring t_1 * 1 + t_2 * 1 + ... back into one sum.
struct P2Mul {
  int32_t d[16];
  int32_t k;
  int32_t one[16];
  int32_t dd[16];  // centred d_i R^2 (a plain value times it is R^2-form)
};
constexpr P2Mul make_p2_mul() {
  P2Mul m{};
  for (int i = 0; i < 16; i++) {
    m.d[i] = P2S.d[i];
    m.one[i] = 1;
    m.dd[i] = centred(to_mont_c(P2.diag[i]));
  }
  m.k = P2S.k;
  return m;
}
#ifdef __HIP_DEVICE_COMPILE__
__constant__ P2Mul P2M_DEV = make_p2_mul();
#define P2M P2M_DEV
#else
constexpr P2Mul P2M_HOST = make_p2_mul();
#define P2M P2M_HOST
#endif
// y R^-1 mod p, within p/2 of y's (signed) high word
// Optimization barrier for a 64-bit value (no instruction).
KB_HD int64_t opaque64(int64_t x) {
#ifdef __HIP_DEVICE_COMPILE__
  asm("" : "+v"(x));
#endif
  return x;
}
// With m = -y p^-1 (mod 2^32, signed), y + m p is a multiple of 2^32 and the reduction is
// its high word: v_mul_lo_u32 + one v_mad_i64_i32 (y the 64-bit addend).  |m p| < 2^62 and
// every caller keeps |y| < 2^62, so the sum stays inside int64.
// On the device the multiply-add is written as the instruction itself: expressed in C++ the
// same code takes the AMDGPU backend minutes per Merkle kernel (12 s -> 8 min for merkle.hip).
KB_HD int32_t mred_s(int64_t y) {
  const int32_t m = (int32_t)((uint32_t)y * MU_NEG);
#ifdef __HIP_DEVICE_COMPILE__
  int64_t r;
  uint64_t carry;  // VOP3b carry-out, unused
  asm("v_mad_i64_i32 %0, %1, %2, %3, %4" : "=v"(r), "=s"(carry) : "v"(m), "s"(P), "v"(y));
  return (int32_t)(r >> 32);
#else  // host (transcript, verifier): the same residue as hi(y) - hi(m' p), m' = -m
  const uint32_t mh = (uint32_t)(((int64_t)(int32_t)(0u - (uint32_t)m) * (int64_t)P) >> 32);
  return (int32_t)((uint32_t)((uint64_t)y >> 32) - mh);
#endif
}
// (a << sh) + b in one v_lshl_add_u64 (the compiler turns a small-constant multiple of a
// 64-bit value into v_mad_u64_u32 pairs and moves otherwise)
template <int SH>
KB_HD int64_t lshl_add64(int64_t a, int64_t b) {
#ifdef __HIP_DEVICE_COMPILE__
  int64_t r;
  asm("v_lshl_add_u64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "n"(SH), "v"(b));
  return r;
#else
  return (int64_t)(((uint64_t)a << SH) + (uint64_t)b);
#endif
}
// a = x R, |a| < p  ->  x^3 R^2 (mod p), |.| < p^2
KB_HD int64_t cube_s(int32_t a) {
  const int64_t A = (int64_t)a * a;
  return (int64_t)mred_s(A) * a;
}
// same residue, |.| < 2^55 + 2^32
KB_HD int64_t fold_s(int64_t u) {
  return (int64_t)(int32_t)(u >> 32) * (int64_t)C32 + (int64_t)(uint32_t)u;
}
// External rounds with the constants already in front of the MDS layers (P2Pre): a[i] are the
// first round's S-box inputs (constant included); round r's S-box output gets K[r] (the M^-1
// image of the constant the reduction after its MDS would add).  Leaves the 4th MDS output
// (64-bit R^2-form) in y.
KB_HD void external_rounds_pre(const int32_t a[16], int64_t y[16], const int32_t (&K)[4][16]) {
  uint64_t* u = reinterpret_cast<uint64_t*>(y);
#pragma unroll
  for (int r = 0; r < 4; r++) {
#pragma unroll
    for (int i = 0; i < 16; i++) {
      const int32_t x = r ? mred_s(y[i]) : a[i];
      const int64_t c3 = (int64_t)mred_s((int64_t)x * x) * x + K[r][i];
      y[i] = fold_s(c3);
    }
    mds_light64(u);
  }
}
KB_HD void poseidon2_permute(uint32_t s[16]) {
  int64_t y[16];
  int32_t t[16];
  // initial MDS-light on x R^2 + M^-1 rc_0 (s C32 < 2^56, rows sum to 35: < 2^61.2)
#pragma unroll
  for (int i = 0; i < 16; i++) y[i] = (int64_t)((uint64_t)s[i] * C32) + P2PRE.init0[i];
  mds_light64(reinterpret_cast<uint64_t*>(y));
#pragma unroll
  for (int i = 0; i < 16; i++) t[i] = mred_s(y[i]);
  external_rounds_pre(t, y, P2PRE.init);
#pragma unroll
  for (int i = 0; i < 16; i++) t[i] = mred_s(y[i]);  // rc_int[0] already in y[0]
  // Elements 1, 2, 4, 5 (d = 1, 2, 3, 4) stay unreduced 64-bit R-form values through rounds
  // 0..11: u <- d u + T_R with T_R = reduce(q) the R-form round sum (|T_R| < p/2 + 2^28), a
  // 64-bit shift-add instead of multiply + reduction.  Growth: |u_5| < 4^12 2^30.2 + 4^12 p/6
  // < 2^54.7, so every sum stays below 2^58 (mred_s needs < 2^62).  Round 12 reduces them to
  // plain values x = reduce(u) and applies d_i R^2 x + q + rc, the other elements' form.
  int64_t u1 = t[1], u2 = t[2], u4 = t[4], u5 = t[5];
#pragma unroll
  for (int r = 0; r < 13; r++) {
    const int32_t c = mred_s(cube_s(t[0]));
    int64_t part[2];
    part[0] = (int64_t)P2M.one[0] * c;
    part[0] = (int64_t)P2M.one[3] * t[3] + part[0];
    part[0] = (int64_t)P2M.one[6] * t[6] + part[0];
    part[0] = (int64_t)P2M.one[7] * t[7] + part[0];
    part[0] = part[0] + u1;
    part[0] = part[0] + u2;
    part[1] = (int64_t)P2M.one[8] * t[8];
#pragma unroll
    for (int i = 9; i < 16; i++) part[1] = (int64_t)P2M.one[i] * t[i] + part[1];
    part[1] = part[1] + u4;
    part[1] = part[1] + u5;
    const int32_t sp = mred_s(part[0] + part[1]);
    const int64_t q = opaque64((int64_t)P2M.k * sp);
    if (r < 12) {
      const int64_t tr = (int64_t)mred_s(q);
      t[0] = mred_s((int64_t)P2M.d[0] * c + (q + P2S.rc_int[r + 1]));
#pragma unroll
      for (int i = 3; i < 16; i++)
        if (i != 4 && i != 5) t[i] = mred_s((int64_t)P2M.d[i] * t[i] + q);
      u1 = lshl_add64<0>(u1, tr);
      u2 = lshl_add64<1>(u2, tr);
      u4 = lshl_add64<0>(lshl_add64<1>(u4, u4), tr);
      u5 = lshl_add64<2>(u5, tr);
    } else {
      t[0] = mred_s((int64_t)P2M.d[0] * c + (q + P2S.rc_term[0][0]));
#pragma unroll
      for (int i = 3; i < 16; i++)
        if (i != 4 && i != 5) t[i] = mred_s((int64_t)P2M.d[i] * t[i] + (q + P2S.rc_term[0][i]));
      t[1] = mred_s((int64_t)P2M.dd[1] * mred_s(u1) + (q + P2S.rc_term[0][1]));
      t[2] = mred_s((int64_t)P2M.dd[2] * mred_s(u2) + (q + P2S.rc_term[0][2]));
      t[4] = mred_s((int64_t)P2M.dd[4] * mred_s(u4) + (q + P2S.rc_term[0][4]));
      t[5] = mred_s((int64_t)P2M.dd[5] * mred_s(u5) + (q + P2S.rc_term[0][5]));
    }
  }
  external_rounds_pre(t, y, P2PRE.term);
#pragma unroll
  for (int i = 0; i < 16; i++) {
    const uint32_t r = (uint32_t)mred_s(y[i]);
    s[i] = umin(r, r + P);
  }
}
// ---------------------------------------------------------------------------------------
// Latency-optimised permutation: one state element per lane, a state per 16-lane DPP row
// (lane = threadIdx.x & 15).  Cross-lane steps use DPP: quad_perm rotations for the M4 blocks,
// row_ror for the block sums and the internal-round total.  About 1/6 of the single-lane
// latency; used where only a few permutations are in flight (top layers of Merkle trees).
template <int CTRL>
__device__ __forceinline__ uint32_t dpp(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xf, 0xf, false);
}
constexpr int DPP_QROT1 = 0x39, DPP_QROT2 = 0x4E, DPP_QROT3 = 0x93;  // quad_perm x_{j+1,2,3}
constexpr int DPP_ROR1 = 0x121, DPP_ROR2 = 0x122, DPP_ROR4 = 0x124, DPP_ROR8 = 0x128;

// Signed lazy form in lane mode: the throughput permutation's
// arithmetic (poseidon2_permute above: R^2-form 64-bit S-box outputs folded to < 2^55.1,
// MDS-light in 64-bit adds, one signed reduction per element and round, round constants in front
// of the MDS layer) with lane l holding element l and the cross-lane terms moved by DPP (both
// halves of a 64-bit value): 619 VALU instructions per lane against 836 for the canonical form
// below (three-instruction modular adds, five-instruction products).  Lane mode is latency-bound
// (tree tops, the FRI tail, the device challenger): k_compress_top 18.0 -> 15.3 us and k_fri_tail
// 107 -> 91 us per launch (profiles/r04/ab_lane_signed.txt).
// (mov_dpp: every lane of the row is a valid source for these controls, so no "old" value is
// needed -- update_dpp(0, ...) would cost a v_mov of zero into every destination first)
template <int CTRL>
__device__ __forceinline__ int64_t dpp64(int64_t v) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)(uint64_t)v, CTRL, 0xf, 0xf, false);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)((uint64_t)v >> 32), CTRL, 0xf, 0xf, false);
  return (int64_t)(((uint64_t)hi << 32) | lo);
}
// mds_light64 with one element per lane: M4 inside each quad, then the four blocks' sums.
// (Plain 64-bit C++ adds instead of lshl_add64 compile to more instructions here: the compiler
// rebuilds each DPP'd value as lo + (hi << 32), two 64-bit adds per use.)
__device__ __forceinline__ int64_t mds_light64_lane(int64_t y) {
  const int64_t a1 = dpp64<DPP_QROT1>(y), a2 = dpp64<DPP_QROT2>(y), a3 = dpp64<DPP_QROT3>(y);
  const int64_t p1 = lshl_add64<1>(y, a1);                      // 2 y + a1
  const int64_t m = lshl_add64<0>(p1, lshl_add64<0>(lshl_add64<1>(a1, a2), a3));  // + 2 a1 + a2 + a3
  const int64_t t = lshl_add64<0>(m, dpp64<DPP_ROR8>(m));
  return lshl_add64<0>(m, lshl_add64<0>(t, dpp64<DPP_ROR4>(t)));
}
__device__ __forceinline__ int64_t sum_lanes16_64(int64_t v) {
  v = lshl_add64<0>(v, dpp64<DPP_ROR1>(v));
  v = lshl_add64<0>(v, dpp64<DPP_ROR2>(v));
  v = lshl_add64<0>(v, dpp64<DPP_ROR4>(v));
  return lshl_add64<0>(v, dpp64<DPP_ROR8>(v));
}

// The lane's round constants, loaded once per kernel by callers that permute in a loop (the
// loads are a memory round trip on a latency-bound chain).
struct LaneConsts {
  int32_t kin[4], kte[3];  // P2PRE.init[r][lane], P2PRE.term[r][lane]
  int32_t init0, d, rct;   // P2PRE.init0[lane], P2M.d[lane], P2S.rc_term[0][lane]
};
__device__ __forceinline__ LaneConsts lane_consts(int lane) {
  LaneConsts k;
#pragma unroll
  for (int r = 0; r < 4; r++) k.kin[r] = P2PRE.init[r][lane];
#pragma unroll
  for (int r = 0; r < 3; r++) k.kte[r] = P2PRE.term[r][lane];
  k.init0 = P2PRE.init0[lane];
  k.d = P2M.d[lane];
  k.rct = P2S.rc_term[0][lane];
  return k;
}

// One external round per r (as external_rounds_pre): x -> x^3 R^2 + K[r] -> fold -> MDS-light.
__device__ __forceinline__ int64_t external_rounds_lane(int32_t x, const int32_t* K, int nk) {
  int64_t y = 0;
#pragma unroll
  for (int r = 0; r < 4; r++) {
    if (r) x = mred_s(y);
    const int64_t c3 = (int64_t)mred_s((int64_t)x * x) * x + (r < nk ? K[r] : 0);
    y = mds_light64_lane(fold_s(c3));
  }
  return y;
}
__device__ __forceinline__ uint32_t poseidon2_permute_lane(uint32_t v, int lane,
                                                           const LaneConsts& kc) {
  // initial MDS-light on x R^2 + M^-1 rc_0 (x = v, Montgomery form, canonical)
  int64_t y = mds_light64_lane((int64_t)((uint64_t)v * C32) + kc.init0);
  y = external_rounds_lane(mred_s(y), kc.kin, 4);
  int32_t t = mred_s(y);  // rc_int[0] already in lane 0's value
#pragma unroll
  for (int r = 0; r < 13; r++) {
    // lane 0 carries the S-box element; every lane computes a cube, lane 0's is used
    const int32_t c = mred_s(cube_s(t));
    const int32_t u = lane == 0 ? c : t;
    const int32_t sp = mred_s(sum_lanes16_64((int64_t)u));  // the plain sum of the state
    const int64_t q = opaque64((int64_t)P2S.k * sp);
    const int32_t add = r < 12 ? (lane == 0 ? P2S.rc_int[r + 1] : 0) : kc.rct;
    t = mred_s((int64_t)kc.d * u + (q + add));
  }
  y = external_rounds_lane(t, kc.kte, 3);
  const uint32_t r = (uint32_t)mred_s(y);
  return umin(r, r + P);
}
__device__ __forceinline__ uint32_t poseidon2_permute_lane(uint32_t v, int lane) {
  return poseidon2_permute_lane(v, lane, lane_consts(lane));
}

}  // namespace kb
