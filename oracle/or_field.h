/*
 * ORACLE — test infrastructure only.  Nothing in the product path may include, link or
 * call this code; only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg do.
 *
 * KoalaBear prime field and its degree-4 binomial extension, in CANONICAL form
 * (values in [0, p)), deliberately independent of the product's Montgomery arithmetic.
 *
 *   Val       = KoalaBear, p = 2^31 - 2^24 + 1      (crates/stark/src/kb31_poseidon2.rs:20)
 *   Challenge = BinomialExtensionField<Val, 4>       (crates/stark/src/kb31_poseidon2.rs:21)
 *               x^4 = W with W = 3  [p3-recalled: p3-koala-bear BinomialExtensionData<4>]
 *   two_adic_generator(k) = (3^127)^(2^(24-k)); 3 = multiplicative generator
 *               [p3-recalled: p3-koala-bear TWO_ADIC_GENERATORS; checked in tests]
 */
#ifndef OR_FIELD_H
#define OR_FIELD_H
#include <stdint.h>
#include <stddef.h>

#define OR_P 0x7f000001u
#define OR_W 3u
#define OR_GEN 3u
#define OR_TWO_ADICITY 24

typedef uint32_t fp;
typedef struct { fp c[4]; } ef;

static inline fp fp_add(fp a, fp b) { fp s = a + b; return s >= OR_P ? s - OR_P : s; }
static inline fp fp_sub(fp a, fp b) { return a >= b ? a - b : a + OR_P - b; }
static inline fp fp_neg(fp a) { return a ? OR_P - a : 0; }
static inline fp fp_mul(fp a, fp b) { return (fp)(((uint64_t)a * b) % OR_P); }
static inline fp fp_from_u64(uint64_t v) { return (fp)(v % OR_P); }

fp fp_pow(fp a, uint64_t e);
fp fp_inv(fp a);
fp fp_two_adic_gen(int bits);

static inline ef ef_zero(void) { ef r = {{0, 0, 0, 0}}; return r; }
static inline ef ef_one(void) { ef r = {{1, 0, 0, 0}}; return r; }
static inline ef ef_from_fp(fp a) { ef r = {{a, 0, 0, 0}}; return r; }
static inline ef ef_add(ef a, ef b) {
  ef r; for (int i = 0; i < 4; i++) r.c[i] = fp_add(a.c[i], b.c[i]); return r;
}
static inline ef ef_sub(ef a, ef b) {
  ef r; for (int i = 0; i < 4; i++) r.c[i] = fp_sub(a.c[i], b.c[i]); return r;
}
static inline ef ef_neg(ef a) {
  ef r; for (int i = 0; i < 4; i++) r.c[i] = fp_neg(a.c[i]); return r;
}
static inline ef ef_mul_fp(ef a, fp b) {
  ef r; for (int i = 0; i < 4; i++) r.c[i] = fp_mul(a.c[i], b); return r;
}
static inline ef ef_add_fp(ef a, fp b) { a.c[0] = fp_add(a.c[0], b); return a; }
static inline ef ef_mul(ef a, ef b) {
  uint64_t t[7] = {0, 0, 0, 0, 0, 0, 0};
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 4; j++) t[i + j] = (t[i + j] + (uint64_t)a.c[i] * b.c[j] % OR_P) % OR_P;
  ef r;
  for (int i = 0; i < 4; i++) {
    uint64_t v = t[i];
    if (i + 4 < 7) v = (v + t[i + 4] * OR_W) % OR_P;
    r.c[i] = (fp)v;
  }
  return r;
}
static inline int ef_eq(ef a, ef b) {
  return a.c[0] == b.c[0] && a.c[1] == b.c[1] && a.c[2] == b.c[2] && a.c[3] == b.c[3];
}
static inline int ef_is_zero(ef a) { return !(a.c[0] | a.c[1] | a.c[2] | a.c[3]); }
ef ef_inv(ef a);
ef ef_pow(ef a, uint64_t e);
ef ef_exp_power_of_2(ef a, int k);

#endif
