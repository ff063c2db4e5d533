// KoalaBear field (p = 2^31 - 2^24 + 1) and its quartic extension, for host and device.
//
// Storage is MONTGOMERY form (x * 2^32 mod p), byte-identical to Plonky3's MontyField31 —
// the representation the reference keeps `[KoalaBear]` slices in (crates/stark/src/
// kb31_poseidon2.rs:20 `Val = KoalaBear`).  EF = BinomialExtensionField<KoalaBear, 4>
// (kb31_poseidon2.rs:21) with x^4 = W = 3.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

#define KB_HD __host__ __device__ __forceinline__

namespace kb {

constexpr uint32_t P = 0x7f000001u;

constexpr uint32_t inv_mod_2_32(uint32_t p) {
  uint32_t x = p;  // p*p = 1 mod 8
  for (int i = 0; i < 5; i++) x *= 2u - p * x;
  return x;
}
constexpr uint32_t MU = inv_mod_2_32(P);  // p^-1 mod 2^32
static_assert(uint32_t(P * MU) == 1u, "MU");

// p = 1 + 127*2^24, so p^-1 = 1 - 127*2^24 = 1 + 2^24 - 2^31 (mod 2^32): the Montgomery
// factor m = lo * p^-1 is two shifts and two adds instead of a 32-bit multiply.
static_assert(MU == (uint32_t)(1u + (1u << 24) - (1u << 31)), "MU shape");
KB_HD uint32_t mont_m(uint32_t lo) { return lo + (lo << 24) - (lo << 31); }
KB_HD uint32_t umin(uint32_t a, uint32_t b) { return a < b ? a : b; }
// Optimization barrier for one VGPR value (no instruction): stops the compiler from fusing a
// 32-bit "hi - mh" back into a 64-bit borrow chain around it.
KB_HD uint32_t opaque(uint32_t x) {
#ifdef __HIP_DEVICE_COMPILE__
  asm("" : "+v"(x));
#endif
  return x;
}

KB_HD uint32_t mred_lt_p(uint64_t y);
KB_HD uint64_t fold32(uint64_t x);
// Montgomery reduction of any t < 2^64: result in [0, p) (fold to < 2^57, then mred_lt_p).
KB_HD uint32_t mreduce(uint64_t t) { return mred_lt_p(fold32(t)); }
// Any a < 2^32, b < p: with m = -t p^-1 mod 2^32, t + m p is a multiple of 2^32 below
// 2^32 p + 2^32 p < 2^64, so r = (t + m p) / 2^32 lies in [0, 2p) (one v_mad_u64_u32 forms
// t + m p: mad, mul_lo, mad, sub, min -- five instructions).
constexpr uint32_t MU_NEG = 0u - MU;
KB_HD uint32_t mmul(uint32_t a, uint32_t b) {
  const uint64_t t = (uint64_t)a * b;
  const uint32_t m = (uint32_t)t * MU_NEG;
  const uint32_t r = (uint32_t)(((uint64_t)m * P + t) >> 32);
  return umin(r, r - P);
}
// Signed a in (-p, p), b < p: t = a b and the signed factor m give |t + m p| < 2^63 and
// r = (t + m p) / 2^32 in (-p, p); one min() folds the sign.  Used for the DIF difference
// (u - v) w, which then needs no + p before the product.
KB_HD uint32_t mmul_s(int32_t a, uint32_t b) {
  const int64_t t = (int64_t)a * (int64_t)(int32_t)b;
  const int32_t m = (int32_t)((uint32_t)t * MU_NEG);
  const uint32_t r = (uint32_t)(((int64_t)m * (int64_t)P + t) >> 32);
  return umin(r, r + P);
}
KB_HD uint32_t madd(uint32_t a, uint32_t b) {
  uint32_t s = a + b;  // < 2p < 2^32
  return umin(s, s - P);
}
KB_HD uint32_t msub(uint32_t a, uint32_t b) {
  uint32_t d = a - b;
  return umin(d, d + P);
}
KB_HD uint32_t mneg(uint32_t a) { return a ? P - a : 0; }
// 2a: on gfx950 the compiler's a << 1 is a half-rate v_lshlrev; v_add_u32 a, a is full rate.
KB_HD uint32_t mdbl(uint32_t a) {
#ifdef __HIP_DEVICE_COMPILE__
  uint32_t s;
  asm("v_add_u32 %0, %1, %1" : "=v"(s) : "v"(a));
#else
  const uint32_t s = a + a;
#endif
  return umin(s, s - P);
}

constexpr uint32_t to_mont_c(uint32_t x) {
  return (uint32_t)((((uint64_t)(x % P)) << 32) % P);
}
constexpr uint32_t from_mont_c(uint32_t x) {
  // x * 2^-32 mod p
  uint64_t r = x;
  for (int i = 0; i < 32; i++) r = (r & 1) ? (r + P) >> 1 : r >> 1;
  return (uint32_t)r;
}
constexpr uint32_t R2 = (uint32_t)((((uint64_t)1 << 32) % P) * (((uint64_t)1 << 32) % P) % P);
KB_HD uint32_t to_mont(uint32_t x) { return mmul(x % P, R2); }
KB_HD uint32_t from_mont(uint32_t x) { return mmul(x, 1u); }

constexpr uint32_t ONE = to_mont_c(1);
constexpr uint32_t TWO = to_mont_c(2);

KB_HD uint32_t mpow(uint32_t a, uint64_t e) {
  uint32_t r = ONE;
  while (e) {
    if (e & 1) r = mmul(r, a);
    a = mmul(a, a);
    e >>= 1;
  }
  return r;
}
KB_HD uint32_t minv(uint32_t a) { return mpow(a, P - 2); }

// two_adic_generator(bits) = (3^127)^(2^(24-bits))  (Montgomery form)
inline uint32_t two_adic_gen(int bits) {
  uint32_t g = mpow(to_mont_c(3), 127);
  for (int i = bits; i < 24; i++) g = mmul(g, g);
  return g;
}

// ---------------------------------------------------------------- quartic extension
struct EF {
  uint32_t c[4];
};

KB_HD EF ef_zero() { return EF{{0, 0, 0, 0}}; }
KB_HD EF ef_one() { return EF{{ONE, 0, 0, 0}}; }
KB_HD EF ef_base(uint32_t a) { return EF{{a, 0, 0, 0}}; }
KB_HD EF ef_add(const EF& a, const EF& b) {
  return EF{{madd(a.c[0], b.c[0]), madd(a.c[1], b.c[1]), madd(a.c[2], b.c[2]), madd(a.c[3], b.c[3])}};
}
KB_HD EF ef_sub(const EF& a, const EF& b) {
  return EF{{msub(a.c[0], b.c[0]), msub(a.c[1], b.c[1]), msub(a.c[2], b.c[2]), msub(a.c[3], b.c[3])}};
}
KB_HD EF ef_neg(const EF& a) { return EF{{mneg(a.c[0]), mneg(a.c[1]), mneg(a.c[2]), mneg(a.c[3])}}; }
KB_HD EF ef_mul_base(const EF& a, uint32_t b) {
  return EF{{mmul(a.c[0], b), mmul(a.c[1], b), mmul(a.c[2], b), mmul(a.c[3], b)}};
}
KB_HD EF ef_add_base(EF a, uint32_t b) {
  a.c[0] = madd(a.c[0], b);
  return a;
}
KB_HD uint32_t mul3(uint32_t x) { return madd(madd(x, x), x); }
// x mod p as a smaller 64-bit value: hi * (2^32 mod p) + lo  (< 2^57 for any x)
KB_HD uint64_t fold32(uint64_t x) { return (uint64_t)(uint32_t)(x >> 32) * ((1u << 25) - 2) + (uint32_t)x; }
// Montgomery reduction of y with hi(y) < p: result in [0, p).  y + m p (m = -y p^-1 mod
// 2^32) < 2^63 + 2^63 is a multiple of 2^32 whose high word lies in [0, 2p).
KB_HD uint32_t mred_lt_p(uint64_t y) {
  const uint32_t m = (uint32_t)y * MU_NEG;
  const uint32_t r = (uint32_t)(((uint64_t)m * P + y) >> 32);
  return umin(r, r - P);
}
KB_HD EF ef_mul(const EF& a, const EF& b) {
  // Coefficient k = d_k + 3 w_k (x^4 = 3).  Each d_k, w_k is a sum of <= 4 raw products
  // (< 4 p^2 < 2^64).  3 fold(w) < 2^58.2 and fold(d) < 2^57 keep d + 3 w below p 2^32, so
  // one Montgomery reduction with a single correction gives the coefficient.
  const uint64_t w0 = (uint64_t)a.c[1] * b.c[3] + (uint64_t)a.c[2] * b.c[2] + (uint64_t)a.c[3] * b.c[1];
  const uint64_t w1 = (uint64_t)a.c[2] * b.c[3] + (uint64_t)a.c[3] * b.c[2];
  const uint64_t w2 = (uint64_t)a.c[3] * b.c[3];
  const uint64_t d0 = (uint64_t)a.c[0] * b.c[0];  // < p^2: hi < p / 2, no fold needed
  const uint64_t d1 = (uint64_t)a.c[0] * b.c[1] + (uint64_t)a.c[1] * b.c[0];
  const uint64_t d2 = (uint64_t)a.c[0] * b.c[2] + (uint64_t)a.c[1] * b.c[1] + (uint64_t)a.c[2] * b.c[0];
  const uint64_t d3 = (uint64_t)a.c[0] * b.c[3] + (uint64_t)a.c[1] * b.c[2] +
                      (uint64_t)a.c[2] * b.c[1] + (uint64_t)a.c[3] * b.c[0];  // < 4p^2: hi < 2p
  const uint64_t f0 = fold32(w0), f1 = fold32(w1), f2 = fold32(w2);
  EF r;
  r.c[0] = mred_lt_p(d0 + 3 * f0);
  r.c[1] = mred_lt_p(fold32(d1) + 3 * f1);
  r.c[2] = mred_lt_p(fold32(d2) + 3 * f2);
  r.c[3] = mreduce(d3);
  return r;
}
KB_HD bool ef_eq(const EF& a, const EF& b) {
  return a.c[0] == b.c[0] && a.c[1] == b.c[1] && a.c[2] == b.c[2] && a.c[3] == b.c[3];
}
KB_HD bool ef_is_zero(const EF& a) { return !(a.c[0] | a.c[1] | a.c[2] | a.c[3]); }

// Frobenius constants: z = W^((p-1)/4); phi^k multiplies coefficient i by z^(i*k).
// z^1, z^2, z^3 in Montgomery form (computed at compile time).
constexpr uint32_t cmul(uint32_t a, uint32_t b) { return (uint32_t)((uint64_t)a * b % P); }
constexpr uint32_t cpow(uint32_t a, uint64_t e) {
  uint32_t r = 1;
  while (e) {
    if (e & 1) r = cmul(r, a);
    a = cmul(a, a);
    e >>= 1;
  }
  return r;
}
constexpr uint32_t FZ1 = cpow(3, (P - 1) / 4);
constexpr uint32_t FZ2 = cmul(FZ1, FZ1);
constexpr uint32_t FZ3 = cmul(FZ2, FZ1);
constexpr uint32_t FZ1M = to_mont_c(FZ1), FZ2M = to_mont_c(FZ2), FZ3M = to_mont_c(FZ3);

KB_HD EF ef_frob1(const EF& a) {  // z^i
  return EF{{a.c[0], mmul(a.c[1], FZ1M), mmul(a.c[2], FZ2M), mmul(a.c[3], FZ3M)}};
}
KB_HD EF ef_frob2(const EF& a) {  // z^(2i): 1, z^2, z^4 = 1, z^6 = z^2
  return EF{{a.c[0], mmul(a.c[1], FZ2M), a.c[2], mmul(a.c[3], FZ2M)}};
}
KB_HD EF ef_frob3(const EF& a) {  // z^(3i): 1, z^3, z^6 = z^2, z^9 = z
  return EF{{a.c[0], mmul(a.c[1], FZ3M), mmul(a.c[2], FZ2M), mmul(a.c[3], FZ1M)}};
}
KB_HD EF ef_inv(const EF& a) {
  EF t = ef_mul(ef_mul(ef_frob1(a), ef_frob2(a)), ef_frob3(a));
  // norm = (a * t).c0
  uint64_t w0 = (uint64_t)a.c[1] * t.c[3] + (uint64_t)a.c[2] * t.c[2] + (uint64_t)a.c[3] * t.c[1];
  uint32_t n = madd(mreduce((uint64_t)a.c[0] * t.c[0]), mul3(mreduce(w0)));
  return ef_mul_base(t, minv(n));
}
KB_HD EF ef_pow(EF a, uint64_t e) {
  EF r = ef_one();
  while (e) {
    if (e & 1) r = ef_mul(r, a);
    a = ef_mul(a, a);
    e >>= 1;
  }
  return r;
}

// Lazy dot products: raw 64-bit products of Montgomery values (each < p^2) accumulate with
// v_mad_u64_u32; every 4 products the accumulator is folded, acc = hi * (2^32 mod p) + lo
// (< 2^57, one more v_mad_u64_u32), which leaves room for 4 more (4 p^2 + 2^57 < 2^64).  One
// Montgomery reduction at the end (fold < 2^57: its high word is far below 2p).
struct LazyEF {
  static constexpr uint32_t C32 = (1u << 25) - 2;  // 2^32 mod p
  uint64_t acc[4];
  int pending;
  KB_HD void init() {
#pragma unroll
    for (int e = 0; e < 4; e++) acc[e] = 0;
    pending = 0;
  }
  KB_HD void fold() {
#pragma unroll
    for (int e = 0; e < 4; e++) acc[e] = (uint64_t)(uint32_t)(acc[e] >> 32) * C32 + (uint32_t)acc[e];
    pending = 0;
  }
  KB_HD void add(const EF& coef, uint32_t v) {
#pragma unroll
    for (int e = 0; e < 4; e++) acc[e] += (uint64_t)coef.c[e] * v;
    if (++pending == 4) fold();
  }
  KB_HD EF get() {
    fold();
    EF r;
#pragma unroll
    for (int e = 0; e < 4; e++) r.c[e] = mred_lt_p(acc[e]);  // folded: < 2^57
    return r;
  }
};


// ---------------------------------------------------------------- global loads
// Pointers read out of a device-side descriptor lose their address space: reading through them
// compiles to flat loads, which count against lgkmcnt as well, so every scalar-load or LDS wait
// also waits for the column loads in flight.  These read through the global address space.
typedef uint32_t kb_u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint32_t ld_global(const uint32_t* p, size_t i) {
  return ((const __attribute__((address_space(1))) uint32_t*)p)[i];
}
__device__ __forceinline__ EF ld_global(const EF* p, size_t i) {
  const kb_u32x4 u = ((const __attribute__((address_space(1))) kb_u32x4*)p)[i];
  return EF{{u.x, u.y, u.z, u.w}};
}

// Buffer loads / stores through a descriptor built from a wave-uniform base: the per-thread
// part of an address is the 32-bit voffset and the uniform part (column, stage, element index)
// the scalar soffset, so an access costs no VALU address arithmetic and no VGPR pair (a flat
// global access with an offset beyond the 12-bit immediate costs two half-rate 64-bit adds per
// load).  Offsets stay below 2 GiB of the base.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_of(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), /*stride*/ 0, /*bytes*/ 0x7fffffff,
                                           0x00020000);
}
__device__ __forceinline__ uint32_t ld_b(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
  return (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(r, (int)voff, (int)soff, 0);
}
__device__ __forceinline__ void st_b(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff, uint32_t v) {
  __builtin_amdgcn_raw_buffer_store_b32(v, r, (int)voff, (int)soff, 0);
}

}  // namespace kb
