/*
 * ORACLE — test infrastructure only.
 *
 * Coset low-degree extension as used by TwoAdicFriPcs::commit [p3-recalled] (called from
 * crates/stark/src/prover.rs:227,334,411 and machine.rs:196): for a matrix of evaluations
 * on a domain (shift s, size n), interpolate, and evaluate the same polynomial on
 * GENERATOR * H_{n<<log_blowup} in natural order, then bit-reverse the rows.  The output
 * is mathematically unique, so any correct NTT reproduces Radix2DitParallel bit for bit.
 * This restatement uses a textbook iterative radix-2 NTT (tests cross-check it against an
 * O(n^2) DFT at small n).
 */
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif
#include "or_field.h"
#include "or_dft.h"

size_t or_bitrev(size_t x, int bits) {
  size_t r = 0;
  for (int i = 0; i < bits; i++) { r = (r << 1) | (x & 1); x >>= 1; }
  return r;
}

int or_log2(size_t n) {
  int l = 0;
  while (((size_t)1 << l) < n) l++;
  return l;
}

/* In-place natural->natural NTT of size n=2^lg with root w (order n). */
void or_ntt(fp* a, int lg, fp w) {
  size_t n = (size_t)1 << lg;
  for (size_t i = 0; i < n; i++) {
    size_t j = or_bitrev(i, lg);
    if (i < j) { fp t = a[i]; a[i] = a[j]; a[j] = t; }
  }
  for (int s = 1; s <= lg; s++) {
    size_t m = (size_t)1 << s, h = m >> 1;
    fp wm = fp_pow(w, n / m);
    fp* tw = malloc(sizeof(fp) * h);
    tw[0] = 1;
    for (size_t j = 1; j < h; j++) tw[j] = fp_mul(tw[j - 1], wm);
    for (size_t k = 0; k < n; k += m)
      for (size_t j = 0; j < h; j++) {
        fp u = a[k + j], v = fp_mul(a[k + j + h], tw[j]);
        a[k + j] = fp_add(u, v);
        a[k + j + h] = fp_sub(u, v);
      }
    free(tw);
  }
}

/* evaluations (natural order on H_n) -> coefficients */
void or_intt(fp* a, int lg) {
  fp w = fp_inv(fp_two_adic_gen(lg));
  or_ntt(a, lg, w);
  fp ninv = fp_inv((fp)(((size_t)1 << lg) % OR_P));
  size_t n = (size_t)1 << lg;
  for (size_t i = 0; i < n; i++) a[i] = fp_mul(a[i], ninv);
}

/* Columns are transformed one at a time (textbook NTT per column), in groups of up to 16
 * adjacent columns so the row-major gather and scatter touch whole cache lines; groups are
 * small enough that every thread gets one (a 31-column trace is 16 groups, not 2). */
void or_coset_lde(const fp* in, size_t n, size_t w, fp shift, int log_blowup, fp* out) {
  int lg = or_log2(n);
  int lgN = lg + log_blowup;
  size_t N = n << log_blowup;
  fp gN = fp_two_adic_gen(lgN);
  int nthreads = 1;
#ifdef _OPENMP
  nthreads = omp_get_max_threads();
#endif
  size_t G = w / (size_t)nthreads;
  if (G < 1) G = 1;
  if (G > 16) G = 16;
  long ngroups = (long)((w + G - 1) / G);
#pragma omp parallel for schedule(dynamic, 1)
  for (long g = 0; g < ngroups; g++) {
    size_t c0 = (size_t)g * G;
    size_t gw = w - c0 < G ? w - c0 : G;
    fp* a = calloc(N * gw, sizeof(fp)); /* column k of the group at a + k N */
    for (size_t i = 0; i < n; i++)
      for (size_t k = 0; k < gw; k++) a[k * N + i] = in[i * w + c0 + k];
    for (size_t k = 0; k < gw; k++) {
      fp* col = a + k * N;
      or_intt(col, lg);
      fp p = 1;
      for (size_t j = 0; j < n; j++) { col[j] = fp_mul(col[j], p); p = fp_mul(p, shift); }
      or_ntt(col, lgN, gN);
    }
    for (size_t r = 0; r < N; r++) {
      size_t src = or_bitrev(r, lgN);
      for (size_t k = 0; k < gw; k++) out[r * w + c0 + k] = a[k * N + src];
    }
    free(a);
  }
}

/* Evaluate (at EF point z) the polynomial q with q(shift * w_n^i) = evals[i*stride + c]. */
void or_eval_columns_at(const fp* evals, size_t n, size_t w, fp shift, ef z, ef* out) {
  int lg = or_log2(n);
  ef zs = ef_mul_fp(z, fp_inv(shift));
#pragma omp parallel for schedule(dynamic, 1)
  for (long c = 0; c < (long)w; c++) {
    fp* a = malloc(sizeof(fp) * n);
    for (size_t i = 0; i < n; i++) a[i] = evals[i * w + c];
    or_intt(a, lg);
    ef acc = ef_zero();
    for (size_t k = n; k-- > 0;) acc = ef_add_fp(ef_mul(acc, zs), a[k]);
    out[c] = acc;
    free(a);
  }
}
