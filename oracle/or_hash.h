/* ORACLE — test infrastructure only.  Poseidon2 / sponge / Merkle / challenger. */
#ifndef OR_HASH_H
#define OR_HASH_H
#include "or_field.h"

void or_poseidon2_permute(fp s[16]);

typedef struct { fp st[16]; int pos; } or_sponge;
void or_sponge_begin(or_sponge* sp);
void or_sponge_absorb(or_sponge* sp, fp x);
void or_sponge_finish(or_sponge* sp, fp out[8]);
void or_hash(const fp* in, size_t n, fp out[8]);
void or_compress(const fp l[8], const fp r[8], fp out[8]);

/* Row-major matrix (canonical values). */
typedef struct {
  fp* values;
  size_t height, width;
  int order; /* position in the commit call (used for stable sorting) */
} or_mat;

typedef struct {
  or_mat* mats; /* not owned */
  int nmats;
  int nlayers;  /* layers[0] = leaves (max height digests), layers[nlayers-1] = root */
  fp** layers;  /* layers[L] has (max_height >> L) digests of 8 elements */
  fp root[8];
} or_merkle;

void or_merkle_build(or_merkle* t, or_mat* mats, int nmats);
void or_merkle_free(or_merkle* t);
size_t or_merkle_max_height(const or_merkle* t);

typedef struct {
  fp st[16];
  fp in[8];
  int nin;
  fp out[8];
  int nout;
} or_challenger;

void or_ch_init(or_challenger* c);
void or_ch_observe(or_challenger* c, fp v);
void or_ch_observe_digest(or_challenger* c, const fp d[8]);
void or_ch_observe_ef(or_challenger* c, ef v);
fp or_ch_sample(or_challenger* c);
ef or_ch_sample_ef(or_challenger* c);
uint32_t or_ch_sample_bits(or_challenger* c, int bits);
int or_ch_check_witness(or_challenger* c, int bits, fp w);
fp or_ch_grind(or_challenger* c, int bits);

#endif
