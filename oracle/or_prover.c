/*
 * ORACLE — test infrastructure only.
 *
 * CPU restatement of the core-proof pipeline:
 *   StarkMachine::setup            crates/stark/src/machine.rs:154-224
 *   MachineProver::prove           crates/stark/src/prover.rs:560-582 (+ observe_into :595-601)
 *   CpuProver::commit / open       crates/stark/src/prover.rs:209-553
 *   generate_permutation_trace     crates/stark/src/permutation.rs:75-148
 *   quotient_values                crates/stark/src/quotient.rs:18-165
 *   TwoAdicFriPcs::{commit, open} + fri::prover  [p3-recalled, zkMIPS/Plonky3 @93967fce]
 *   Verifier::verify_shard         crates/stark/src/verifier.rs:27-329 (+ PCS / FRI verify)
 *
 * Proofs are emitted in the "BFZ1" NORMAL FORM: memory events sorted by
 * address, smallest PoW witness, chip_ordering written as the ordered chip list, all field
 * elements as canonical u32 little-endian.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "or_field.h"
#include "or_hash.h"
#include "or_dft.h"
#include "or_machine.h"
#include "or_api.h"

#define LOG_BLOWUP 1
#define POW_BITS 16

static int g_num_queries = 84;
void or_set_num_queries(int q) { g_num_queries = q; }
/* Decision D1 ([p3-recalled] TwoAdicFriPcs::open): 1 = every opened value is
 * observed before the FRI batching challenge is sampled; 0 = the challenge is sampled first. */
void or_set_pcs_variant(int observe_openings) { or_variant.observe_openings = observe_openings != 0; }

/* ------------------------------------------------------------------ byte buffer */
typedef struct { uint8_t* p; size_t n, cap; } buf;
static void bput(buf* b, const void* d, size_t n) {
  if (b->n + n > b->cap) { b->cap = (b->n + n) * 2 + 1024; b->p = realloc(b->p, b->cap); }
  memcpy(b->p + b->n, d, n); b->n += n;
}
static void bu32(buf* b, uint32_t v) { bput(b, &v, 4); }
static void bef(buf* b, ef v) { bput(b, v.c, 16); }
static void bdig(buf* b, const fp* d) { bput(b, d, 32); }

/* ------------------------------------------------------------------ committed rounds */
typedef struct {
  size_t n, w;
  int log_n;
  fp shift;   /* domain shift */
  fp* evals;  /* natural order, row-major n x w */
  fp* lde;    /* bit-reversed rows, row-major 2n x w */
} cmat;

typedef struct {
  int nmats;
  cmat* m;
  or_mat* lm;
  or_merkle tree;
} round_t;

static void round_commit(round_t* r) {
  r->lm = calloc(r->nmats, sizeof(or_mat));
  for (int i = 0; i < r->nmats; i++) {
    cmat* c = &r->m[i];
    size_t N = c->n << LOG_BLOWUP;
    c->lde = malloc(sizeof(fp) * N * c->w);
    /* TwoAdicFriPcs::commit: shift = GENERATOR / domain.shift */
    or_coset_lde(c->evals, c->n, c->w, fp_mul(OR_GEN, fp_inv(c->shift)), LOG_BLOWUP, c->lde);
    r->lm[i].values = c->lde;
    r->lm[i].height = N;
    r->lm[i].width = c->w;
  }
  or_merkle_build(&r->tree, r->lm, r->nmats);
}

static void round_free(round_t* r, int free_evals) {
  for (int i = 0; i < r->nmats; i++) {
    if (free_evals) free(r->m[i].evals);
    free(r->m[i].lde);
  }
  free(r->m);
  free(r->lm);
  or_merkle_free(&r->tree);
}

/* MerkleTreeMmcs::open_batch [p3-recalled] */
static void open_batch(buf* b, const round_t* r, size_t index) {
  size_t maxh = or_merkle_max_height(&r->tree);
  int lmax = or_log2(maxh);
  bu32(b, (uint32_t)r->nmats);
  for (int i = 0; i < r->nmats; i++) {
    int lh = or_log2(r->lm[i].height);
    size_t ri = index >> (lmax - lh);
    bu32(b, (uint32_t)r->lm[i].width);
    bput(b, &r->lm[i].values[ri * r->lm[i].width], 4 * r->lm[i].width);
  }
  bu32(b, (uint32_t)lmax);
  for (int L = 0; L < lmax; L++) bdig(b, &r->tree.layers[L][8 * ((index >> L) ^ 1)]);
}

/* ------------------------------------------------------------------ setup */
typedef struct {
  round_t prep;
  int chip_of[2];   /* prep matrix i -> chip id */
  int idx_of_chip[NUM_CHIPS]; /* chip -> prep matrix index or -1 */
} pk_t;

static int cmp_name(int a, int b) { return strcmp(OR_CHIPS[a].name, OR_CHIPS[b].name); }

static void setup(const or_program* p, pk_t* pk) {
  memset(pk, 0, sizeof *pk);
  for (int c = 0; c < NUM_CHIPS; c++) pk->idx_of_chip[c] = -1;
  int chips[2] = {CHIP_PROGRAM, CHIP_BYTE};
  size_t h[2];
  fp* t[2];
  for (int i = 0; i < 2; i++) h[i] = or_prep_trace(chips[i], p, &t[i]);
  /* sort by (Reverse(height), name) (machine.rs:182-183) */
  int o0 = 0, o1 = 1;
  if (h[1] > h[0] || (h[1] == h[0] && cmp_name(chips[1], chips[0]) < 0)) { o0 = 1; o1 = 0; }
  int ord[2] = {o0, o1};
  pk->prep.nmats = 2;
  pk->prep.m = calloc(2, sizeof(cmat));
  for (int k = 0; k < 2; k++) {
    int i = ord[k];
    cmat* c = &pk->prep.m[k];
    c->n = h[i]; c->w = OR_CHIPS[chips[i]].prep_w; c->log_n = or_log2(h[i]);
    c->shift = 1; c->evals = t[i];
    pk->chip_of[k] = chips[i];
    pk->idx_of_chip[chips[i]] = k;
  }
  round_commit(&pk->prep);
}

/* ------------------------------------------------------------------ prover */
typedef struct {
  int chip;
  size_t n;
  int log_n;
  fp* main;     /* row-major n x main_w */
  ef* perm;     /* row-major n x pw (EF) */
  int pw;
  ef cumsum;
  ef* q;        /* 2n quotient values (natural order) */
} chipdata;

static int cmp_chip_sort(const void* a, const void* b) {
  const chipdata* x = a; const chipdata* y = b;
  if (x->n != y->n) return x->n > y->n ? -1 : 1;
  return cmp_name(x->chip, y->chip);
}

static ef vcol_base(const or_vcol* v, const fp* prep, const fp* main) {
  fp r = v->c;
  for (int i = 0; i < v->n; i++)
    r = fp_add(r, fp_mul(v->w[i], v->src[i] == 1 ? prep[v->col[i]] : main[v->col[i]]));
  return ef_from_fp(r);
}

/* generate_permutation_trace (permutation.rs:75-148) */
static void perm_trace(chipdata* cd, const fp* prep, size_t prep_w, ef alpha, ef beta) {
  or_chip_lookups lu;
  or_chip_lookups_get(cd->chip, &lu);
  int nint = lu.nsends + lu.nrecvs;
  int pw = (nint + 1) / 2 + 1;
  cd->pw = pw;
  cd->perm = calloc(cd->n * pw, sizeof(ef));
  const or_lookup* all[32];
  int is_send[32];
  for (int i = 0; i < lu.nsends; i++) { all[i] = &lu.sends[i]; is_send[i] = 1; }
  for (int i = 0; i < lu.nrecvs; i++) { all[lu.nsends + i] = &lu.recvs[i]; is_send[lu.nsends + i] = 0; }
  size_t mw = OR_CHIPS[cd->chip].main_w;
#pragma omp parallel for schedule(static)
  for (long r = 0; r < (long)cd->n; r++) {
    const fp* mrow = &cd->main[r * mw];
    const fp* prow = prep ? &prep[r * prep_w] : NULL;
    ef* out = &cd->perm[r * pw];
    for (int b = 0; b < pw - 1; b++) {
      ef acc = ef_zero();
      for (int j = 2 * b; j < 2 * b + 2 && j < nint; j++) {
        const or_lookup* l = all[j];
        ef den = alpha, bp = ef_one();
        den = ef_add(den, ef_mul_fp(bp, (fp)l->kind));
        for (int k = 0; k < l->nvals; k++) {
          bp = ef_mul(bp, beta);
          den = ef_add(den, ef_mul(bp, vcol_base(&l->vals[k], prow, mrow)));
        }
        ef m = vcol_base(&l->mult, prow, mrow);
        if (!is_send[j]) m = ef_neg(m);
        acc = ef_add(acc, ef_mul(m, ef_inv(den)));
      }
      out[b] = acc;
    }
  }
  ef run = ef_zero();
  for (size_t r = 0; r < cd->n; r++) {
    ef* out = &cd->perm[r * pw];
    for (int b = 0; b < pw - 1; b++) run = ef_add(run, out[b]);
    out[pw - 1] = run;
  }
  cd->cumsum = run;
}

/* quotient_values (quotient.rs:18-165) with selectors_on_coset [p3-recalled] */
static void quotient(chipdata* cd, const cmat* prep_m, const cmat* main_m, const cmat* perm_m,
                     ef perm_alpha, ef perm_beta, ef alpha) {
  size_t n = cd->n, N = 2 * n;
  int lgN = cd->log_n + 1;
  cd->q = malloc(sizeof(ef) * N);
  fp wN = fp_two_adic_gen(lgN);
  fp wn_inv = fp_inv(fp_two_adic_gen(cd->log_n));
  size_t mw = main_m->w, pw = perm_m->w / 4, prw = prep_m ? prep_m->w : 0;
#pragma omp parallel for schedule(static)
  for (long i = 0; i < (long)N; i++) {
    size_t il = or_bitrev((size_t)i, lgN), in = or_bitrev((size_t)((i + 2) % N), lgN);
    ef ml[64], mn[64], pl[16], pn[16], prl[8], prn[8];
    for (size_t c = 0; c < mw; c++) {
      ml[c] = ef_from_fp(main_m->lde[il * mw + c]);
      mn[c] = ef_from_fp(main_m->lde[in * mw + c]);
    }
    for (size_t c = 0; c < prw; c++) {
      prl[c] = ef_from_fp(prep_m->lde[il * prw + c]);
      prn[c] = ef_from_fp(prep_m->lde[in * prw + c]);
    }
    for (size_t e = 0; e < pw; e++)
      for (int k = 0; k < 4; k++) {
        pl[e].c[k] = perm_m->lde[il * perm_m->w + 4 * e + k];
        pn[e].c[k] = perm_m->lde[in * perm_m->w + 4 * e + k];
      }
    fp x = fp_mul(OR_GEN, fp_pow(wN, (uint64_t)i));
    fp zh = fp_sub(fp_pow(x, n), 1);
    or_folder f;
    f.prep_l = prl; f.prep_n = prn; f.main_l = ml; f.main_n = mn; f.perm_l = pl; f.perm_n = pn;
    f.perm_alpha = perm_alpha; f.perm_beta = perm_beta; f.cumsum = cd->cumsum;
    f.is_first = ef_from_fp(fp_mul(zh, fp_inv(fp_sub(x, 1))));
    f.is_last = ef_from_fp(fp_mul(zh, fp_inv(fp_sub(x, wn_inv))));
    if (or_variant.selectors_normalized) { /* D8 alternative: L_0 = Z/(n(x-1)), L_last = w^-1 Z/(n(x-w^-1)) */
      fp ninv = fp_inv((fp)(n % OR_P));
      f.is_first = ef_mul_fp(f.is_first, ninv);
      f.is_last = ef_mul_fp(f.is_last, fp_mul(ninv, wn_inv));
    }
    f.is_trans = ef_from_fp(fp_sub(x, wn_inv));
    f.alpha = alpha; f.acc = ef_zero();
    or_eval_chip(cd->chip, &f);
    cd->q[i] = ef_mul_fp(f.acc, fp_inv(zh));
  }
}

/* One FRI commit-phase layer (fri::prover::commit_phase [p3-recalled]): the folded vector of
 * `len` EF values (bit-reversed order) committed as len/2 leaves, leaf i = the pair (2i, 2i+1)
 * with each EF flattened to its 4 base coefficients (D5; the D5 alternative interleaves them). */
void or_fri_commit_layer(const ef* folded, size_t len, or_merkle* tree) {
  or_mat m;
  m.values = (fp*)folded;
  m.height = len / 2;
  m.width = 8;
  fp* cm = NULL;
  if (or_variant.fri_coeff_major) { /* D5 alternative: [a0 b0 a1 b1 a2 b2 a3 b3] per leaf */
    cm = malloc(sizeof(fp) * 4 * len);
    for (size_t i = 0; i < len / 2; i++)
      for (int k = 0; k < 4; k++) {
        cm[8 * i + 2 * k] = folded[2 * i].c[k];
        cm[8 * i + 2 * k + 1] = folded[2 * i + 1].c[k];
      }
    m.values = cm;
  }
  or_merkle_build(tree, &m, 1);
  tree->mats = NULL; /* m is local: a caller that opens the layer keeps its own matrix */
  free(cm);
}

/* The fold of a committed layer with challenge beta (TwoAdicFriFolding::fold_row
 * [p3-recalled]): out[i] = (1/2 + beta/2 x_i^-1) lo + (1/2 - beta/2 x_i^-1) hi, where (lo, hi) =
 * (in[2i], in[2i+1]) are the evaluations at +-x_i and x_i = g_{2h}^bitrev(i). */
void or_fri_fold(const ef* in, size_t len, ef beta, ef* out) {
  size_t h = len / 2;
  int lgh = or_log2(h);
  fp g_inv = fp_inv(fp_two_adic_gen(lgh + 1));
  fp half = fp_inv(2);
  ef half_beta = ef_mul_fp(beta, half);
  for (size_t i = 0; i < h; i++) {
    ef pw = ef_mul_fp(half_beta, fp_pow(g_inv, or_bitrev(i, lgh)));
    ef lo = in[2 * i], hi = in[2 * i + 1];
    out[i] = ef_add(ef_mul(ef_add_fp(pw, half), lo), ef_mul(ef_sub(ef_from_fp(half), pw), hi));
  }
}

/* reduced openings + FRI (TwoAdicFriPcs::open, fri::prover::prove) [p3-recalled] */
typedef struct { int nmats; const cmat* m; int npts[16]; ef pts[16][2]; ef* vals[16][2]; } oround;

static void fri_prove(buf* b, or_challenger* ch, round_t* rounds, oround* orr, int nrounds) {
  ef alpha = or_ch_sample_ef(ch);
  ef* ro[32] = {0};
  size_t num_red[32] = {0};
  int lg_max = 0;
  for (int r = 0; r < nrounds; r++)
    for (int i = 0; i < orr[r].nmats; i++) {
      const cmat* c = &orr[r].m[i];
      int lh = c->log_n + LOG_BLOWUP;
      size_t H = (size_t)1 << lh;
      if (lh > lg_max) lg_max = lh;
      if (!ro[lh]) ro[lh] = calloc(H, sizeof(ef));
      fp wH = fp_two_adic_gen(lh);
      for (int p = 0; p < orr[r].npts[i]; p++) {
        ef z = orr[r].pts[i][p];
        ef off = ef_pow(alpha, num_red[lh]);
        num_red[lh] += c->w;
        ef* ys = orr[r].vals[i][p];
        ef ysum = ef_zero(), ap = ef_one();
        ef* apow = malloc(sizeof(ef) * c->w);
        for (size_t k = 0; k < c->w; k++) { apow[k] = ap; ysum = ef_add(ysum, ef_mul(ap, ys[k])); ap = ef_mul(ap, alpha); }
#pragma omp parallel for schedule(static)
        for (long row = 0; row < (long)H; row++) {
          fp x = fp_mul(OR_GEN, fp_pow(wH, or_bitrev((size_t)row, lh)));
          ef s = ef_zero();
          for (size_t k = 0; k < c->w; k++) s = ef_add(s, ef_mul_fp(apow[k], c->lde[row * c->w + k]));
          ef num = ef_sub(s, ysum);
          ef inv = ef_inv(ef_sub(ef_from_fp(x), z));
          ro[lh][row] = ef_add(ro[lh][row], ef_mul(off, ef_mul(num, inv)));
        }
        free(apow);
      }
    }
  /* commit phase */
  size_t len = (size_t)1 << lg_max;
  ef* folded = ro[lg_max];
  ro[lg_max] = NULL;
  int ncommit = 0;
  round_t* fr = calloc(32, sizeof(round_t));
  ef* layers[32];
  ef betas[32];
  while (len > (1u << LOG_BLOWUP)) {
    round_t* R = &fr[ncommit];
    R->nmats = 1;
    R->lm = calloc(1, sizeof(or_mat));
    R->lm[0].values = (fp*)folded; /* EF pairs flattened: width 8 base */
    R->lm[0].height = len / 2;
    R->lm[0].width = 8;
    or_fri_commit_layer(folded, len, &R->tree);
    R->tree.mats = R->lm;
    or_ch_observe_digest(ch, R->tree.root);
    ef beta = or_ch_sample_ef(ch);
    betas[ncommit] = beta;
    layers[ncommit] = folded;
    size_t h = len / 2;
    ef* nf = malloc(sizeof(ef) * h);
    or_fri_fold(folded, len, beta, nf);
    folded = nf;
    len = h;
    ncommit++;
    int lgl = or_log2(len);
    if (ro[lgl]) {
      for (size_t i = 0; i < len; i++) folded[i] = ef_add(folded[i], ro[lgl][i]);
      free(ro[lgl]); ro[lgl] = NULL;
    }
  }
  ef final_poly = folded[0];
  or_ch_observe_ef(ch, final_poly);
  fp pow_w = or_ch_grind(ch, POW_BITS);
  /* serialize commit-phase roots */
  bu32(b, (uint32_t)ncommit);
  for (int i = 0; i < ncommit; i++) bdig(b, fr[i].tree.root);
  bu32(b, (uint32_t)g_num_queries);
  for (int q = 0; q < g_num_queries; q++) {
    size_t index = or_ch_sample_bits(ch, lg_max + or_variant.query_extra_bits) >>
                   or_variant.query_extra_bits; /* D6 */
    bu32(b, (uint32_t)nrounds);
    for (int r = 0; r < nrounds; r++) {
      int lmr = or_log2(or_merkle_max_height(&rounds[r].tree));
      open_batch(b, &rounds[r], index >> (lg_max - lmr));
    }
    bu32(b, (uint32_t)ncommit);
    for (int i = 0; i < ncommit; i++) {
      size_t ii = index >> i;
      bef(b, layers[i][ii ^ 1]);
      size_t pair = ii >> 1;
      int lmax = fr[i].tree.nlayers - 1;
      bu32(b, (uint32_t)lmax);
      for (int L = 0; L < lmax; L++) bdig(b, &fr[i].tree.layers[L][8 * ((pair >> L) ^ 1)]);
    }
  }
  bef(b, final_poly);
  bu32(b, pow_w);
  for (int i = 0; i < ncommit; i++) {
    or_merkle_free(&fr[i].tree);
    free(fr[i].lm);
    free(layers[i]);
  }
  free(fr);
  free(folded);
  for (int i = 0; i < 32; i++) free(ro[i]);
  (void)betas;
}

static void write_opened(buf* b, const ef* v, size_t n) {
  bu32(b, (uint32_t)n);
  for (size_t i = 0; i < n; i++) bef(b, v[i]);
}

int or_prove_record(const or_program* prog, or_record* rec, uint8_t** out, size_t* outlen,
                    or_timing* tm) {
  pk_t pk;
  setup(prog, &pk);
  or_generate_dependencies(rec);
  or_challenger ch0;
  or_ch_init(&ch0);
  /* observe_into: commit + 7 zeros (prover.rs:595-601) */
  or_ch_observe_digest(&ch0, pk.prep.tree.root);
  for (int i = 0; i < 7; i++) or_ch_observe(&ch0, 0);
  or_challenger ch = ch0; /* open() works on challenger.clone() (prover.rs:578) */

  /* generate_traces + commit (prover.rs:58-81,209-236) */
  chipdata cds[NUM_CHIPS];
  int nc = 0;
  for (int c = 0; c < NUM_CHIPS; c++) {
    if (!or_chip_included(c, rec)) continue;
    memset(&cds[nc], 0, sizeof(chipdata));
    cds[nc].chip = c;
    cds[nc].n = or_main_trace(c, rec, &cds[nc].main);
    cds[nc].log_n = or_log2(cds[nc].n);
    nc++;
  }
  qsort(cds, nc, sizeof(chipdata), cmp_chip_sort);
  round_t main_r;
  main_r.nmats = nc;
  main_r.m = calloc(nc, sizeof(cmat));
  for (int i = 0; i < nc; i++) {
    cmat* c = &main_r.m[i];
    c->n = cds[i].n; c->w = OR_CHIPS[cds[i].chip].main_w; c->log_n = cds[i].log_n;
    c->shift = 1; c->evals = cds[i].main;
  }
  round_commit(&main_r);

  /* open (prover.rs:242-553) */
  or_ch_observe_digest(&ch, main_r.tree.root);
  ef perm_alpha = or_ch_sample_ef(&ch);
  ef perm_beta = or_ch_sample_ef(&ch);
  round_t perm_r;
  perm_r.nmats = nc;
  perm_r.m = calloc(nc, sizeof(cmat));
  for (int i = 0; i < nc; i++) {
    int pi = pk.idx_of_chip[cds[i].chip];
    const fp* prep = pi >= 0 ? pk.prep.m[pi].evals : NULL;
    size_t prep_w = pi >= 0 ? pk.prep.m[pi].w : 0;
    perm_trace(&cds[i], prep, prep_w, perm_alpha, perm_beta);
    cmat* c = &perm_r.m[i];
    c->n = cds[i].n; c->w = 4 * cds[i].pw; c->log_n = cds[i].log_n; c->shift = 1;
    c->evals = malloc(sizeof(fp) * c->n * c->w);
    memcpy(c->evals, cds[i].perm, sizeof(fp) * c->n * c->w); /* flatten_to_base */
  }
  round_commit(&perm_r);
  or_ch_observe_digest(&ch, perm_r.tree.root);
  for (int i = 0; i < nc; i++) or_ch_observe_ef(&ch, cds[i].cumsum);
  ef alpha = or_ch_sample_ef(&ch);

  round_t quot_r;
  quot_r.nmats = 2 * nc;
  quot_r.m = calloc(2 * nc, sizeof(cmat));
  for (int i = 0; i < nc; i++) {
    int pi = pk.idx_of_chip[cds[i].chip];
    quotient(&cds[i], pi >= 0 ? &pk.prep.m[pi] : NULL, &main_r.m[i], &perm_r.m[i], perm_alpha,
             perm_beta, alpha);
    fp wN = fp_two_adic_gen(cds[i].log_n + 1);
    for (int k = 0; k < 2; k++) {
      cmat* c = &quot_r.m[2 * i + k];
      c->n = cds[i].n; c->w = 4; c->log_n = cds[i].log_n;
      c->shift = fp_mul(OR_GEN, k ? wN : 1); /* split_domains: shift * gen^k */
      c->evals = malloc(sizeof(fp) * c->n * 4);
      for (size_t m = 0; m < c->n; m++) memcpy(&c->evals[4 * m], cds[i].q[2 * m + k].c, 16);
    }
  }
  round_commit(&quot_r);
  or_ch_observe_digest(&ch, quot_r.tree.root);
  ef zeta = or_ch_sample_ef(&ch);

  /* opening points (prover.rs:417-458) */
  oround orr[4];
  memset(orr, 0, sizeof orr);
  round_t* rounds[4] = {&pk.prep, &main_r, &perm_r, &quot_r};
  for (int r = 0; r < 4; r++) {
    orr[r].nmats = rounds[r]->nmats;
    orr[r].m = rounds[r]->m;
    for (int i = 0; i < rounds[r]->nmats; i++) {
      const cmat* c = &rounds[r]->m[i];
      int lo;
      if (r == 0) lo = OR_CHIPS[pk.chip_of[i]].local_only;
      else if (r == 1) lo = OR_CHIPS[cds[i].chip].local_only;
      else lo = (r == 3);
      orr[r].npts[i] = lo ? 1 : 2;
      orr[r].pts[i][0] = zeta;
      orr[r].pts[i][1] = ef_mul_fp(zeta, fp_two_adic_gen(c->log_n));
      for (int p = 0; p < orr[r].npts[i]; p++) {
        orr[r].vals[i][p] = malloc(sizeof(ef) * c->w);
        or_eval_columns_at(c->evals, c->n, c->w, c->shift, orr[r].pts[i][p], orr[r].vals[i][p]);
        if (or_variant.observe_openings)
          for (size_t k = 0; k < c->w; k++) or_ch_observe_ef(&ch, orr[r].vals[i][p][k]);
      }
    }
  }

  /* ---- serialize the proof (normal form) */
  buf b = {0};
  bu32(&b, 0x315a4642u);
  bu32(&b, (uint32_t)nc);
  for (int i = 0; i < nc; i++) {
    const char* nm = OR_CHIPS[cds[i].chip].name;
    bu32(&b, (uint32_t)cds[i].chip);
    bu32(&b, (uint32_t)strlen(nm));
    bput(&b, nm, strlen(nm));
  }
  bdig(&b, main_r.tree.root);
  bdig(&b, perm_r.tree.root);
  bdig(&b, quot_r.tree.root);
  for (int i = 0; i < nc; i++) {
    bu32(&b, (uint32_t)cds[i].log_n);
    int pi = pk.idx_of_chip[cds[i].chip];
    if (pi >= 0) {
      size_t w = pk.prep.m[pi].w;
      write_opened(&b, orr[0].vals[pi][0], w);
      write_opened(&b, orr[0].vals[pi][1], w);
    } else {
      bu32(&b, 0); bu32(&b, 0);
    }
    size_t mw = main_r.m[i].w;
    write_opened(&b, orr[1].vals[i][0], mw);
    if (orr[1].npts[i] == 2) write_opened(&b, orr[1].vals[i][1], mw);
    else { ef* z = calloc(mw, sizeof(ef)); write_opened(&b, z, mw); free(z); }
    write_opened(&b, orr[2].vals[i][0], perm_r.m[i].w);
    write_opened(&b, orr[2].vals[i][1], perm_r.m[i].w);
    bu32(&b, 2);
    write_opened(&b, orr[3].vals[2 * i][0], 4);
    write_opened(&b, orr[3].vals[2 * i + 1][0], 4);
    bef(&b, cds[i].cumsum);
  }
  round_t rr[4] = {pk.prep, main_r, perm_r, quot_r};
  fri_prove(&b, &ch, rr, orr, 4);

  for (int r = 0; r < 4; r++)
    for (int i = 0; i < orr[r].nmats; i++)
      for (int p = 0; p < orr[r].npts[i]; p++) free(orr[r].vals[i][p]);
  for (int i = 0; i < nc; i++) { free(cds[i].perm); free(cds[i].q); }
  round_free(&main_r, 1);
  round_free(&perm_r, 1);
  round_free(&quot_r, 1);
  round_free(&pk.prep, 1);
  (void)tm;
  *out = b.p;
  *outlen = b.n;
  return 0;
}

/* generate_permutation_trace of one chip on given traces (canonical, row-major): the EF
 * permutation trace flattened to base (n x 4 pw, flatten_to_base, prover.rs:318-334) and the
 * cumulative sum.  Returns pw (EF columns). */
int or_api_perm_trace(int chip, const uint32_t* main, const uint32_t* prep, size_t n,
                      const uint32_t alpha[4], const uint32_t beta[4], uint32_t* out,
                      uint32_t cumsum[4]) {
  chipdata cd;
  memset(&cd, 0, sizeof cd);
  cd.chip = chip;
  cd.n = n;
  cd.log_n = or_log2(n);
  cd.main = (fp*)main;
  ef a, b;
  memcpy(a.c, alpha, 16);
  memcpy(b.c, beta, 16);
  perm_trace(&cd, prep, prep ? (size_t)OR_CHIPS[chip].prep_w : 0, a, b);
  memcpy(out, cd.perm, sizeof(ef) * n * cd.pw);
  memcpy(cumsum, cd.cumsum.c, 16);
  free(cd.perm);
  return cd.pw;
}

/* Preprocessed commitment (vk.commit) for a program, canonical form. */
void or_setup_root(const or_program* p, uint32_t root[8]) {
  pk_t pk;
  setup(p, &pk);
  memcpy(root, pk.prep.tree.root, 32);
  round_free(&pk.prep, 1);
}

/* ====================================================================== verifier */
typedef struct { const uint8_t* p; size_t n, off; int err; } rd;
static uint32_t ru32(rd* r) {
  if (r->off + 4 > r->n) { r->err = 1; return 0; }
  uint32_t v; memcpy(&v, r->p + r->off, 4); r->off += 4; return v;
}
static ef ref_(rd* r) { ef v; for (int i = 0; i < 4; i++) v.c[i] = ru32(r) % OR_P; return v; }
static void rdig(rd* r, fp* d) { for (int i = 0; i < 8; i++) d[i] = ru32(r); }
static ef* rvec(rd* r, uint32_t* n) {
  *n = ru32(r);
  if (*n > 4096) { r->err = 1; *n = 0; return NULL; }
  ef* v = malloc(sizeof(ef) * (*n + 1));
  for (uint32_t i = 0; i < *n; i++) v[i] = ref_(r);
  return v;
}

typedef struct { size_t height; size_t width; } dims;

/* MerkleTreeMmcs::verify_batch [p3-recalled] (heights are powers of two) */
static int verify_batch(const fp root[8], const dims* d, int nm, size_t index, fp** rows,
                        const fp* path, int pathlen) {
  int order[64];
  for (int i = 0; i < nm; i++) order[i] = i;
  for (int i = 1; i < nm; i++) /* stable sort by descending height */
    for (int j = i; j > 0 && d[order[j]].height > d[order[j - 1]].height; j--) {
      int t = order[j]; order[j] = order[j - 1]; order[j - 1] = t;
    }
  size_t cur = d[order[0]].height;
  int k = 0;
  or_sponge sp; or_sponge_begin(&sp);
  while (k < nm && d[order[k]].height == cur) {
    for (size_t c = 0; c < d[order[k]].width; c++) or_sponge_absorb(&sp, rows[order[k]][c]);
    k++;
  }
  fp h[8]; or_sponge_finish(&sp, h);
  for (int L = 0; L < pathlen; L++) {
    const fp* sib = &path[8 * L];
    if (index & 1) or_compress(sib, h, h); else or_compress(h, sib, h);
    index >>= 1;
    cur >>= 1;
    if (k < nm && d[order[k]].height == cur) {
      or_sponge_begin(&sp);
      while (k < nm && d[order[k]].height == cur) {
        for (size_t c = 0; c < d[order[k]].width; c++) or_sponge_absorb(&sp, rows[order[k]][c]);
        k++;
      }
      fp rh[8]; or_sponge_finish(&sp, rh);
      if (or_variant.inject_first) or_compress(rh, h, h); /* D4 alternative */
      else or_compress(h, rh, h);
    }
  }
  return memcmp(h, root, 32) == 0 && k == nm;
}

static ef zp_at(int log_n, fp shift, ef x) { /* Z(x) = (x/s)^n - 1 */
  ef u = ef_mul_fp(x, fp_inv(shift));
  u = ef_exp_power_of_2(u, log_n);
  return ef_sub(u, ef_one());
}

int or_verify_proof(const or_program* prog, const uint8_t* proof, size_t len) {
  pk_t pk;
  setup(prog, &pk);
  rd r = {proof, len, 0, 0};
  int ok = 0;
  if (ru32(&r) != 0x315a4642u) return -1;
  uint32_t nc = ru32(&r);
  if (nc == 0 || nc > NUM_CHIPS) { round_free(&pk.prep, 1); return -2; }
  int chip[NUM_CHIPS];
  for (uint32_t i = 0; i < nc; i++) {
    chip[i] = (int)ru32(&r);
    uint32_t l = ru32(&r);
    r.off += l;
    if (chip[i] < 0 || chip[i] >= NUM_CHIPS) { r.err = 1; break; }
  }
  fp main_root[8], perm_root[8], quot_root[8];
  rdig(&r, main_root); rdig(&r, perm_root); rdig(&r, quot_root);
  uint32_t log_deg[NUM_CHIPS];
  ef *prl[NUM_CHIPS], *prn[NUM_CHIPS], *ml[NUM_CHIPS], *mn[NUM_CHIPS], *pl[NUM_CHIPS],
      *pn[NUM_CHIPS], *q0[NUM_CHIPS], *q1[NUM_CHIPS];
  uint32_t nprl[NUM_CHIPS], nml[NUM_CHIPS], npl[NUM_CHIPS], dummy;
  ef cum[NUM_CHIPS];
  for (uint32_t i = 0; i < nc; i++) {
    log_deg[i] = ru32(&r);
    prl[i] = rvec(&r, &nprl[i]); prn[i] = rvec(&r, &dummy);
    ml[i] = rvec(&r, &nml[i]); mn[i] = rvec(&r, &dummy);
    pl[i] = rvec(&r, &npl[i]); pn[i] = rvec(&r, &dummy);
    ru32(&r);
    q0[i] = rvec(&r, &dummy); q1[i] = rvec(&r, &dummy);
    cum[i] = ref_(&r);
  }
  if (r.err) goto fail;
  /* shape checks */
  for (uint32_t i = 0; i < nc; i++) {
    if (nml[i] != (uint32_t)OR_CHIPS[chip[i]].main_w) goto fail;
    if (npl[i] != (uint32_t)(4 * or_perm_width(chip[i]))) goto fail;
    if (nprl[i] != (uint32_t)OR_CHIPS[chip[i]].prep_w) goto fail;
    if (log_deg[i] > 22 + 1) goto fail;
  }
  /* transcript (verifier.rs:76-101) */
  or_challenger ch;
  or_ch_init(&ch);
  or_ch_observe_digest(&ch, pk.prep.tree.root);
  for (int i = 0; i < 7; i++) or_ch_observe(&ch, 0);
  or_ch_observe_digest(&ch, main_root);
  ef perm_alpha = or_ch_sample_ef(&ch), perm_beta = or_ch_sample_ef(&ch);
  or_ch_observe_digest(&ch, perm_root);
  for (uint32_t i = 0; i < nc; i++) or_ch_observe_ef(&ch, cum[i]);
  ef alpha = or_ch_sample_ef(&ch);
  or_ch_observe_digest(&ch, quot_root);
  ef zeta = or_ch_sample_ef(&ch);

  /* rounds: (commit, [(domain log_n, shift, width, points, values)]) */
  typedef struct { int log_n; fp shift; size_t w; int np; ef pt[2]; ef* v[2]; } vmat;
  vmat vm[4][2 * NUM_CHIPS];
  int vn[4] = {0, 0, 0, 0};
  for (int k = 0; k < 2; k++) { /* vk.chip_information order */
    int c = pk.chip_of[k];
    int i = -1;
    for (uint32_t j = 0; j < nc; j++) if (chip[j] == c) i = (int)j;
    if (i < 0) goto fail;
    vmat* m = &vm[0][vn[0]++];
    m->log_n = pk.prep.m[k].log_n; m->shift = 1; m->w = pk.prep.m[k].w;
    m->np = OR_CHIPS[c].local_only ? 1 : 2;
    m->pt[0] = zeta; m->pt[1] = ef_mul_fp(zeta, fp_two_adic_gen(m->log_n));
    m->v[0] = prl[i]; m->v[1] = prn[i];
  }
  for (uint32_t i = 0; i < nc; i++) {
    vmat* m = &vm[1][vn[1]++];
    m->log_n = (int)log_deg[i]; m->shift = 1; m->w = nml[i];
    m->np = OR_CHIPS[chip[i]].local_only ? 1 : 2;
    m->pt[0] = zeta; m->pt[1] = ef_mul_fp(zeta, fp_two_adic_gen(m->log_n));
    m->v[0] = ml[i]; m->v[1] = mn[i];
    m = &vm[2][vn[2]++];
    m->log_n = (int)log_deg[i]; m->shift = 1; m->w = npl[i]; m->np = 2;
    m->pt[0] = zeta; m->pt[1] = ef_mul_fp(zeta, fp_two_adic_gen(m->log_n));
    m->v[0] = pl[i]; m->v[1] = pn[i];
    fp wN = fp_two_adic_gen((int)log_deg[i] + 1);
    for (int k = 0; k < 2; k++) {
      m = &vm[3][vn[3]++];
      m->log_n = (int)log_deg[i]; m->shift = fp_mul(OR_GEN, k ? wN : 1); m->w = 4; m->np = 1;
      m->pt[0] = zeta; m->v[0] = k ? q1[i] : q0[i];
    }
  }
  /* PCS verify: observe openings (decision D1), sample alpha */
  if (or_variant.observe_openings) for (int rr_ = 0; rr_ < 4; rr_++)
    for (int i = 0; i < vn[rr_]; i++)
      for (int p = 0; p < vm[rr_][i].np; p++)
        for (size_t k = 0; k < vm[rr_][i].w; k++) or_ch_observe_ef(&ch, vm[rr_][i].v[p][k]);
  ef fri_alpha = or_ch_sample_ef(&ch);
  uint32_t ncommit = ru32(&r);
  if (ncommit > 30) goto fail;
  fp croots[32][8];
  ef betas[32];
  for (uint32_t i = 0; i < ncommit; i++) {
    rdig(&r, croots[i]);
    or_ch_observe_digest(&ch, croots[i]);
    betas[i] = or_ch_sample_ef(&ch);
  }
  /* queries are after the final poly in our layout: read them into memory first */
  uint32_t nq = ru32(&r);
  if (nq != (uint32_t)g_num_queries || r.err) goto fail;
  size_t qstart = r.off;
  /* skip queries to reach final poly + pow witness */
  for (uint32_t q = 0; q < nq && !r.err; q++) {
    uint32_t nr = ru32(&r);
    for (uint32_t x = 0; x < nr && !r.err; x++) {
      uint32_t nm = ru32(&r);
      for (uint32_t i = 0; i < nm && !r.err; i++) { uint32_t w = ru32(&r); r.off += 4 * (size_t)w; }
      uint32_t pl_ = ru32(&r); r.off += 32 * (size_t)pl_;
    }
    uint32_t ns = ru32(&r);
    for (uint32_t s = 0; s < ns && !r.err; s++) { r.off += 16; uint32_t pl_ = ru32(&r); r.off += 32 * (size_t)pl_; }
  }
  if (r.err) goto fail;
  ef final_poly = ref_(&r);
  fp pow_w = ru32(&r);
  if (r.err) goto fail;
  or_ch_observe_ef(&ch, final_poly);
  if (!or_ch_check_witness(&ch, POW_BITS, pow_w)) goto fail;
  int log_max_h = (int)ncommit + LOG_BLOWUP;
  r.off = qstart;
  for (uint32_t q = 0; q < nq; q++) {
    size_t index = or_ch_sample_bits(&ch, log_max_h + or_variant.query_extra_bits) >>
                   or_variant.query_extra_bits; /* D6 */
    uint32_t nr = ru32(&r);
    if (nr != 4) goto fail;
    ef ro[32];
    int have[32] = {0};
    ef apow[32];
    const fp* roots[4] = {pk.prep.tree.root, main_root, perm_root, quot_root};
    for (int rr_ = 0; rr_ < 4; rr_++) {
      uint32_t nm = ru32(&r);
      if ((int)nm != vn[rr_]) goto fail;
      fp* rows[2 * NUM_CHIPS];
      dims d[2 * NUM_CHIPS];
      int lbmax = 0;
      for (uint32_t i = 0; i < nm; i++) {
        uint32_t w = ru32(&r);
        if (w != vm[rr_][i].w || r.err) goto fail;
        rows[i] = (fp*)(r.p + r.off);
        r.off += 4 * (size_t)w;
        d[i].height = (size_t)1 << (vm[rr_][i].log_n + LOG_BLOWUP);
        d[i].width = w;
        if (vm[rr_][i].log_n + LOG_BLOWUP > lbmax) lbmax = vm[rr_][i].log_n + LOG_BLOWUP;
      }
      uint32_t pathlen = ru32(&r);
      const fp* path = (const fp*)(r.p + r.off);
      r.off += 32 * (size_t)pathlen;
      if (r.err || r.off > r.n || (int)pathlen != lbmax) goto fail;
      size_t ridx = index >> (log_max_h - lbmax);
      if (!verify_batch(roots[rr_], d, (int)nm, ridx, rows, path, (int)pathlen)) goto fail;
      for (uint32_t i = 0; i < nm; i++) {
        int lh = vm[rr_][i].log_n + LOG_BLOWUP;
        size_t rev = or_bitrev(index >> (log_max_h - lh), lh);
        fp x = fp_mul(OR_GEN, fp_pow(fp_two_adic_gen(lh), rev));
        if (!have[lh]) { have[lh] = 1; ro[lh] = ef_zero(); apow[lh] = ef_one(); }
        for (int p = 0; p < vm[rr_][i].np; p++) {
          ef inv = ef_inv(ef_sub(ef_from_fp(x), vm[rr_][i].pt[p]));
          for (size_t k = 0; k < vm[rr_][i].w; k++) {
            ef quo = ef_mul(ef_sub(ef_from_fp(rows[i][k] % OR_P), vm[rr_][i].v[p][k]), inv);
            ro[lh] = ef_add(ro[lh], ef_mul(apow[lh], quo));
            apow[lh] = ef_mul(apow[lh], fri_alpha);
          }
        }
      }
    }
    /* verify_query */
    uint32_t ns = ru32(&r);
    if (ns != ncommit) goto fail;
    ef folded = ef_zero();
    size_t idx = index;
    for (uint32_t s = 0; s < ns; s++) {
      int lfh = log_max_h - 1 - (int)s;
      if (have[lfh + 1]) { folded = ef_add(folded, ro[lfh + 1]); have[lfh + 1] = 0; }
      ef sib = ref_(&r);
      uint32_t pl_ = ru32(&r);
      const fp* path = (const fp*)(r.p + r.off);
      r.off += 32 * (size_t)pl_;
      if (r.err || r.off > r.n || (int)pl_ != lfh) goto fail;
      ef ev[2];
      ev[idx & 1] = folded;
      ev[(idx & 1) ^ 1] = sib;
      fp row[8];
      memcpy(row, ev[0].c, 16); memcpy(row + 4, ev[1].c, 16);
      if (or_variant.fri_coeff_major) /* D5 alternative */
        for (int k = 0; k < 4; k++) { row[2 * k] = ev[0].c[k]; row[2 * k + 1] = ev[1].c[k]; }
      fp* rowp = row;
      dims d1 = {(size_t)1 << lfh, 8};
      if (!verify_batch(croots[s], &d1, 1, idx >> 1, &rowp, path, (int)pl_)) goto fail;
      idx >>= 1;
      /* fold_row: e0 + (beta - xs0)(e1 - e0)/(xs1 - xs0), xs = bitrev([g, -g]) */
      fp sub_start = fp_pow(fp_two_adic_gen(lfh + 1), or_bitrev(idx, lfh));
      fp xs0 = sub_start, xs1 = fp_neg(sub_start); /* reverse_slice_index_bits on 2 elems: no-op */
      ef t = ef_mul(ef_sub(betas[s], ef_from_fp(xs0)), ef_sub(ev[1], ev[0]));
      folded = ef_add(ev[0], ef_mul_fp(t, fp_inv(fp_sub(xs1, xs0))));
    }
    /* a height-2 input (a 1-row trace) joins after the last fold, as in the commit phase above
     * (decision D11) */
    {
      int lfin = log_max_h - (int)ns;
      if (lfin >= 0 && lfin < 32 && have[lfin]) { folded = ef_add(folded, ro[lfin]); have[lfin] = 0; }
    }
    for (int lh = 0; lh < 32; lh++) if (have[lh]) goto fail;
    if (!ef_eq(folded, final_poly)) goto fail;
  }
  /* constraint checks (verifier.rs:194-213) */
  {
    ef total = ef_zero();
    for (uint32_t i = 0; i < nc; i++) {
      int c = chip[i];
      int log_n = (int)log_deg[i];
      fp wN = fp_two_adic_gen(log_n + 1);
      fp sh[2] = {OR_GEN, fp_mul(OR_GEN, wN)};
      /* recompute_quotient */
      ef zps[2];
      for (int a = 0; a < 2; a++) {
        int o = 1 - a;
        ef num = zp_at(log_n, sh[o], zeta);
        ef den = zp_at(log_n, sh[o], ef_from_fp(sh[a]));
        zps[a] = ef_mul(num, ef_inv(den));
      }
      ef quot = ef_zero();
      ef* qs[2] = {q0[i], q1[i]};
      for (int a = 0; a < 2; a++)
        for (int e = 0; e < 4; e++) {
          ef mono = ef_zero(); mono.c[e] = 1;
          quot = ef_add(quot, ef_mul(ef_mul(zps[a], mono), qs[a][e]));
        }
      /* selectors_at_point */
      fp gn_inv = fp_inv(fp_two_adic_gen(log_n));
      ef zh = ef_sub(ef_exp_power_of_2(zeta, log_n), ef_one());
      or_folder f;
      ef plv[16], pnv[16];
      int pw = or_perm_width(c);
      for (int e = 0; e < pw; e++) {
        plv[e] = ef_zero(); pnv[e] = ef_zero();
        for (int k = 0; k < 4; k++) {
          ef mono = ef_zero(); mono.c[k] = 1;
          plv[e] = ef_add(plv[e], ef_mul(mono, pl[i][4 * e + k]));
          pnv[e] = ef_add(pnv[e], ef_mul(mono, pn[i][4 * e + k]));
        }
      }
      f.prep_l = prl[i]; f.prep_n = prn[i]; f.main_l = ml[i]; f.main_n = mn[i];
      f.perm_l = plv; f.perm_n = pnv;
      f.perm_alpha = perm_alpha; f.perm_beta = perm_beta; f.cumsum = cum[i];
      f.is_first = ef_mul(zh, ef_inv(ef_sub(zeta, ef_one())));
      f.is_last = ef_mul(zh, ef_inv(ef_sub(zeta, ef_from_fp(gn_inv))));
      if (or_variant.selectors_normalized) { /* D8 alternative */
        fp ninv = fp_inv((fp)(((uint64_t)1 << log_n) % OR_P));
        f.is_first = ef_mul_fp(f.is_first, ninv);
        f.is_last = ef_mul_fp(f.is_last, fp_mul(ninv, gn_inv));
      }
      f.is_trans = ef_sub(zeta, ef_from_fp(gn_inv));
      f.alpha = alpha; f.acc = ef_zero();
      or_eval_chip(c, &f);
      if (!ef_eq(ef_mul(f.acc, ef_inv(zh)), quot)) goto fail;
      total = ef_add(total, cum[i]);
    }
    if (!ef_is_zero(total)) goto fail;
  }
  ok = 1;
fail:
  for (uint32_t i = 0; i < nc && i < NUM_CHIPS; i++) {
    if (r.err && i > 0) break;
  }
  round_free(&pk.prep, 1);
  return ok ? 0 : -10;
}
