/* ORACLE — test infrastructure only (see or_field.h). */
#include "or_field.h"

fp fp_pow(fp a, uint64_t e) {
  fp r = 1;
  while (e) {
    if (e & 1) r = fp_mul(r, a);
    a = fp_mul(a, a);
    e >>= 1;
  }
  return r;
}

fp fp_inv(fp a) { return fp_pow(a, OR_P - 2); }

fp fp_two_adic_gen(int bits) {
  /* 3^((p-1)/2^24) = 3^127 generates the 2^24-subgroup; square down to 2^bits. */
  fp g = fp_pow(OR_GEN, 127);
  for (int i = bits; i < OR_TWO_ADICITY; i++) g = fp_mul(g, g);
  return g;
}

ef ef_pow(ef a, uint64_t e) {
  ef r = ef_one();
  while (e) {
    if (e & 1) r = ef_mul(r, a);
    a = ef_mul(a, a);
    e >>= 1;
  }
  return r;
}

ef ef_exp_power_of_2(ef a, int k) {
  for (int i = 0; i < k; i++) a = ef_mul(a, a);
  return a;
}

/* Frobenius: phi^k(sum c_i x^i) = sum c_i z^(i*k) x^i with z = W^((p-1)/4). */
static ef frob(ef a, int k) {
  static fp z = 0;
  if (!z) z = fp_pow(OR_W, (OR_P - 1) / 4);
  fp zk = fp_pow(z, (uint64_t)k);
  ef r;
  fp m = 1;
  for (int i = 0; i < 4; i++) {
    r.c[i] = fp_mul(a.c[i], m);
    m = fp_mul(m, zk);
  }
  return r;
}

ef ef_inv(ef a) {
  /* a^-1 = a^(r-1) / a^r, r = 1+p+p^2+p^3, a^(r-1) = phi(a) phi^2(a) phi^3(a), a^r in Fp. */
  ef t = ef_mul(ef_mul(frob(a, 1), frob(a, 2)), frob(a, 3));
  ef n = ef_mul(t, a);
  fp ninv = fp_inv(n.c[0]);
  return ef_mul_fp(t, ninv);
}
