/* ORACLE — test infrastructure only.  Exported entry points (ctypes) for tests / bench. */
#ifndef OR_API_H
#define OR_API_H
#include <stdint.h>
#include <stddef.h>
#include "or_machine.h"

typedef struct { double t[8]; } or_timing;

int or_prove_record(const or_program* prog, or_record* rec, uint8_t** out, size_t* outlen,
                    or_timing* tm);
int or_verify_proof(const or_program* prog, const uint8_t* proof, size_t len);
void or_set_num_queries(int q);
void or_set_pcs_variant(int observe_openings);
/* D1-D9 switches (or_hash.h or_variant_t) */
void or_variant_reset(void);
int or_variant_set(const char* name, uint32_t value);
void or_setup_root(const or_program* p, uint32_t root[8]);
int or_api_setup_root(const char* program, uint32_t root[8]);

/* ctypes-facing API (canonical u32 field values everywhere) */
int or_api_execute(const char* program, const uint8_t* in, size_t nin, uint8_t* out,
                   size_t outcap, size_t* outlen, uint64_t* cycles, uint32_t* final_pc,
                   uint32_t* final_mp);
int or_api_prove(const char* program, const uint8_t* in, size_t nin, uint8_t** proof,
                 size_t* len);
int or_api_verify(const char* program, const uint8_t* proof, size_t len);
void or_api_free(void* p);
int or_api_trace(const char* program, const uint8_t* in, size_t nin, int chip, int prep,
                 uint32_t** out, size_t* h, size_t* w);
void or_api_poseidon2(uint32_t* states, size_t n);
void or_api_hash(const uint32_t* in, size_t n, uint32_t out[8]);
void or_api_coset_lde(const uint32_t* in, size_t n, size_t w, uint32_t shift, uint32_t* out);
void or_api_merkle_root(const uint32_t* const* mats, const size_t* heights, const size_t* widths,
                        int nmats, uint32_t root[8]);
uint32_t or_api_two_adic_gen(int bits);
void or_api_ef_mul(const uint32_t a[4], const uint32_t b[4], uint32_t out[4]);
void or_api_ef_inv(const uint32_t a[4], uint32_t out[4]);
int or_api_perm_trace(int chip, const uint32_t* main, const uint32_t* prep, size_t n,
                      const uint32_t alpha[4], const uint32_t beta[4], uint32_t* out,
                      uint32_t cumsum[4]);
/* FRI commit-phase helpers shared by the prover and the column-sharded PCS restatement */
#include "or_hash.h"
void or_fri_commit_layer(const ef* folded, size_t len, or_merkle* tree);
void or_fri_fold(const ef* in, size_t len, ef beta, ef* out);
/* Column-sharded PCS commit + FRI commit phase of one n x w trace (or_pcs.c; the product is
 * bfz_commit_fri_sharded): root[8], fri_roots[8 * rounds] (at most cap_rounds), *nrounds, fin[4],
 * and (if challenges is not NULL) alpha then each round's beta, 4 words each.  m: canonical
 * words, natural row order, row-major.  Returns -1 if the fold is not constant. */
int or_api_pcs_commit_fri(const uint32_t* m, size_t n, size_t w, uint32_t root[8],
                          uint32_t* fri_roots, size_t cap_rounds, size_t* nrounds, uint32_t fin[4],
                          uint32_t* challenges);
/* sample a challenger transcript: observe `n` values then squeeze `m` samples */
void or_api_challenger(const uint32_t* obs, size_t n, uint32_t* samples, size_t m);

#endif
