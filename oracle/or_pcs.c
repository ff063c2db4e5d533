/* ORACLE — test infrastructure only (tests/test_pcs_sharded.py): the checker of
 * bfz_commit_fri_sharded (zkvm-brainfuck_amd/csrc/pcs_sharded.hip), BASELINE configs 4/5 and
 * SURVEY.md §8(e) -- one n x w trace committed the way TwoAdicFriPcs::commit commits a matrix
 * (crates/stark/src/prover.rs:209-236: coset LDE with shift GENERATOR, bit-reversed rows,
 * MerkleTreeMmcs) followed by FRI's commit phase (prover.rs:460-470 -> p3 fri::prover::commit_phase
 * [p3-recalled]) on the batched column f = sum_c alpha^c col_c, where alpha is sampled from a fresh
 * DuplexChallenger after it observes the root (the batching step of the reduced opening with
 * every column opened at one point; no quotient by (x - z), so f has degree < n and its fold
 * ends in a constant).  The commit-phase rounds are fri_prove's (or_prover.c): the same layer
 * commitment (or_fri_commit_layer) and fold (or_fri_fold), with no reduced openings injected. */
#include <stdlib.h>
#include <string.h>
#include "or_api.h"
#include "or_dft.h"
#include "or_field.h"
#include "or_hash.h"

int or_api_pcs_commit_fri(const uint32_t* m, size_t n, size_t w, uint32_t root[8],
                          uint32_t* fri_roots, size_t cap_rounds, size_t* nrounds, uint32_t fin[4],
                          uint32_t* challenges) {
  const size_t H = 2 * n;
  fp* lde = malloc(sizeof(fp) * H * w);
  if (!lde) return -2;
  or_coset_lde((const fp*)m, n, w, OR_GEN, 1, lde);
  or_mat mat = {lde, H, w, 0};
  or_merkle t;
  or_merkle_build(&t, &mat, 1);
  memcpy(root, t.root, 32);
  or_merkle_free(&t);

  or_challenger ch;
  or_ch_init(&ch);
  or_ch_observe_digest(&ch, root);
  const ef alpha = or_ch_sample_ef(&ch);
  if (challenges) memcpy(challenges, alpha.c, 16);
  ef* apow = malloc(sizeof(ef) * w);
  ef a = ef_one();
  for (size_t c = 0; c < w; c++) { apow[c] = a; a = ef_mul(a, alpha); }
  ef* cur = malloc(sizeof(ef) * H);
#pragma omp parallel for schedule(static)
  for (long r = 0; r < (long)H; r++) {
    ef s = ef_zero();
    for (size_t c = 0; c < w; c++) s = ef_add(s, ef_mul_fp(apow[c], lde[(size_t)r * w + c]));
    cur[r] = s;
  }
  free(apow);
  free(lde);

  size_t len = H, k = 0;
  while (len > 2) {
    or_merkle ft;
    or_fri_commit_layer(cur, len, &ft);
    if (k < cap_rounds) memcpy(&fri_roots[8 * k], ft.root, 32);
    or_ch_observe_digest(&ch, ft.root);
    or_merkle_free(&ft);
    const ef beta = or_ch_sample_ef(&ch);
    if (challenges && k < cap_rounds) memcpy(&challenges[4 + 4 * k], beta.c, 16);
    ef* next = malloc(sizeof(ef) * (len / 2));
    or_fri_fold(cur, len, beta, next);
    free(cur);
    cur = next;
    len /= 2;
    k++;
  }
  *nrounds = k;
  memcpy(fin, cur[0].c, 16);
  const int constant = memcmp(cur[0].c, cur[1].c, 16) == 0;
  free(cur);
  return constant ? 0 : -1;
}
