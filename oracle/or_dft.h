/* ORACLE — test infrastructure only.  NTT / coset LDE / polynomial evaluation. */
#ifndef OR_DFT_H
#define OR_DFT_H
#include "or_field.h"

size_t or_bitrev(size_t x, int bits);
int or_log2(size_t n);
void or_ntt(fp* a, int lg, fp w);
void or_intt(fp* a, int lg);
void or_coset_lde(const fp* in, size_t n, size_t w, fp shift, int log_blowup, fp* out);
void or_eval_columns_at(const fp* evals, size_t n, size_t w, fp shift, ef z, ef* out);

#endif
