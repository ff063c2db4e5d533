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

// Sum of 16 reduced values.  Pair sums are < 2p and fit 32 bits; the 8 pairs accumulate
// exactly in 64 bits with v_mad_u64_u32 (x * 1 + acc: one half-rate op, where a reduced
// modular add costs add + sub + min), then one reduction: 2^32 = 2^25 - 2 (mod p).
KB_HD uint32_t sum16(const uint32_t s[16]) {
#ifdef __HIP_DEVICE_COMPILE__
  uint32_t one;  // opaque 1 keeps the multiply-add form (an add_co/addc pair costs more)
  asm("s_mov_b32 %0, 1" : "=s"(one));
#else
  const uint32_t one = 1;
#endif
  uint64_t acc = (uint64_t)(s[0] + s[1]);
#pragma unroll
  for (int k = 1; k < 8; k++) acc = (uint64_t)(s[2 * k] + s[2 * k + 1]) * one + acc;
  constexpr uint32_t C = (1u << 25) - 2;  // < 16p < 2^35, so hi < 8
  const uint64_t t = (uint64_t)(uint32_t)(acc >> 32) * C + (uint32_t)acc;  // < 2^32 + 2^28
  const uint32_t hi2 = (uint32_t)(t >> 32);                                // 0 or 1
  const uint32_t r = (uint32_t)t + ((0u - hi2) & C);                       // any u32 < 2.02p
  return umin(r, umin(r - P, r - 2 * P));
}

KB_HD void mds_light(uint32_t s[16]) {
#pragma unroll
  for (int b = 0; b < 16; b += 4) {
    uint32_t x0 = s[b], x1 = s[b + 1], x2 = s[b + 2], x3 = s[b + 3];
    uint32_t t01 = madd(x0, x1), t23 = madd(x2, x3), t0123 = madd(t01, t23);
    uint32_t t01123 = madd(t0123, x1), t01233 = madd(t0123, x3);
    s[b + 3] = madd(t01233, mdbl(x0));  // 3x0 + x1 + x2 + 2x3
    s[b + 1] = madd(t01123, mdbl(x2));  // x0 + 2x1 + 3x2 + x3
    s[b + 0] = madd(t01123, t01);       // 2x0 + 3x1 + x2 + x3
    s[b + 2] = madd(t01233, t23);       // x0 + x1 + 2x2 + 3x3
  }
  uint32_t sums[4];
#pragma unroll
  for (int k = 0; k < 4; k++) sums[k] = madd(madd(s[k], s[4 + k]), madd(s[8 + k], s[12 + k]));
#pragma unroll
  for (int i = 0; i < 16; i++) s[i] = madd(s[i], sums[i & 3]);
}

// N independent permutations advanced round by round, so the scheduler can interleave their
// dependency chains (the internal rounds are one serial chain per state).
// ---- external rounds in 64-bit R^2-form -------------------------------------------------
// The S-box leaves its last product unreduced (x2^M * x^M = x^3 R^2 mod p, folded below 2^57),
// the MDS-light layer adds in 64 bits (a half-rate v_lshl_add_u64 each, no reductions; a
// row's coefficients sum to 35, so values stay below 2^62.2), the next round constant is
// added as rc^M R mod p (the high word grows by at most 1, so it stays below p) and one
// Montgomery reduction returns the next S-box input in Montgomery form.
constexpr uint32_t C32 = (1u << 25) - 2;  // 2^32 mod p
KB_HD uint64_t fold64(uint64_t x) { return (uint64_t)(uint32_t)(x >> 32) * C32 + (uint32_t)x; }
KB_HD uint64_t cube_r2(uint32_t x) { return fold64((uint64_t)mmul(x, x) * x); }
// Montgomery reduction of y with hi(y) < p: result in [0, p)
KB_HD uint32_t mred1(uint64_t y) {
  const uint32_t m = (uint32_t)y * MU;
  const uint32_t r = opaque((uint32_t)(y >> 32)) - (uint32_t)(((uint64_t)m * P) >> 32);
  return umin(r, r + P);
}
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
// Four external rounds from Montgomery state s (round constants rc / rc_r2 per round).
KB_HD void external_rounds(uint32_t s[16], const uint32_t (&rc)[4][16],
                           const uint32_t (&rc_r2)[4][16]) {
  uint64_t y[16];
#pragma unroll
  for (int i = 0; i < 16; i++) y[i] = cube_r2(madd(s[i], rc[0][i]));
  mds_light64(y);
#pragma unroll
  for (int r = 1; r < 4; r++) {
#pragma unroll
    for (int i = 0; i < 16; i++) y[i] = cube_r2(mred1(y[i] + rc_r2[r][i]));
    mds_light64(y);
  }
#pragma unroll
  for (int i = 0; i < 16; i++) s[i] = mred1(y[i]);
}

template <int N>
KB_HD void poseidon2_permute_n(uint32_t (&s)[N][16]) {
#pragma unroll
  for (int k = 0; k < N; k++) {
    mds_light(s[k]);
    external_rounds(s[k], P2.ext_init, P2.ext_init_r2);
  }
#pragma unroll
  for (int r = 0; r < 13; r++) {
#pragma unroll
    for (int k = 0; k < N; k++) {
      uint32_t* t = s[k];
      t[0] = cube(madd(t[0], P2.internal[r]));
      const uint32_t sum = sum16(t);
      // s_i <- sum + d_i s_i with d = [-2,1,2,1/2,3,4,-1/2,-3,-4,1/2^8,1/8,1/2^24,-1/2^8,-1/8,
      // -1/16,-1/2^24].
      // d = -2, 1, 2: doublings; the rest in one step: d^M s + (sum in R^2-form) < p^2 + p
      // has its high word below p, so one Montgomery reduction gives sum + d s.
      const uint32_t sum_r2 = mmul(sum, R2);
      t[0] = msub(sum, mdbl(t[0]));
      t[1] = madd(sum, t[1]);
      t[2] = madd(sum, mdbl(t[2]));
#pragma unroll
      for (int i = 3; i < 16; i++) t[i] = mred1((uint64_t)P2.diag[i] * t[i] + sum_r2);
    }
  }
#pragma unroll
  for (int k = 0; k < N; k++) external_rounds(s[k], P2.ext_term, P2.ext_term_r2);
}

KB_HD void poseidon2_permute(uint32_t s[16]) {
  poseidon2_permute_n<1>(*reinterpret_cast<uint32_t(*)[1][16]>(s));
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

__device__ __forceinline__ uint32_t mds_light_lane(uint32_t x) {
  const uint32_t a1 = dpp<DPP_QROT1>(x), a2 = dpp<DPP_QROT2>(x), a3 = dpp<DPP_QROT3>(x);
  const uint32_t s4 = madd(madd(x, a1), madd(a2, a3));
  const uint32_t y = madd(madd(s4, x), mdbl(a1));  // 2x_j + 3x_{j+1} + x_{j+2} + x_{j+3}
  const uint32_t t = madd(y, dpp<DPP_ROR8>(y));
  return madd(y, madd(t, dpp<DPP_ROR4>(t)));      // + sum of the 4 blocks at this position
}

__device__ __forceinline__ uint32_t sum_lanes16(uint32_t v) {
  v = madd(v, dpp<DPP_ROR1>(v));
  v = madd(v, dpp<DPP_ROR2>(v));
  v = madd(v, dpp<DPP_ROR4>(v));
  return madd(v, dpp<DPP_ROR8>(v));
}

__device__ __forceinline__ uint32_t poseidon2_permute_lane(uint32_t v, int lane) {
  uint32_t rce[8];
#pragma unroll
  for (int r = 0; r < 4; r++) {
    rce[r] = P2.ext_init[r][lane];
    rce[4 + r] = P2.ext_term[r][lane];
  }
  const uint32_t dg = P2.diag[lane];
  v = mds_light_lane(v);
#pragma unroll
  for (int r = 0; r < 4; r++) v = mds_light_lane(cube(madd(v, rce[r])));
#pragma unroll
  for (int r = 0; r < 13; r++) {
    const uint32_t c = cube(madd(v, P2.internal[r]));
    v = lane == 0 ? c : v;
    v = madd(sum_lanes16(v), mmul(v, dg));
  }
#pragma unroll
  for (int r = 0; r < 4; r++) v = mds_light_lane(cube(madd(v, rce[4 + r])));
  return v;
}

}  // namespace kb
