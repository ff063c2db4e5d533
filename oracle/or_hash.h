/* ORACLE — test infrastructure only.  Poseidon2 / sponge / Merkle / challenger. */
#ifndef OR_HASH_H
#define OR_HASH_H
#include "or_field.h"

/* The [p3-recalled] decisions of DESIGN.md §2 (D1-D9) as switches, oracle only: the default
 * (all zero except observe_openings) is the product's choice; scripts/localize_parity.py flips
 * them to find which combination reproduces a reference proof byte for byte.  Every switch is
 * honoured by the oracle prover AND its verifier, so a proof made under a variant verifies
 * under the same variant. */
typedef struct {
  int observe_openings;     /* D1: opened values observed before the FRI alpha (1, default) */
  int diag_alt;             /* D2: 1 = the alternative internal diagonal (OR_DIAG_ALT) */
  int m4_horizen;           /* D3a: 1 = HorizenLabs M4 [[5,7,1,3],[4,6,1,1],[1,3,5,7],[1,1,4,6]] */
  int no_initial_mds;       /* D3b: 1 = no external linear layer before round 1 */
  int inject_first;         /* D4: 1 = node = compress(injected digest, node) */
  int fri_coeff_major;      /* D5: 1 = FRI leaf pair flattened coefficient-major */
  int query_extra_bits;     /* D6: k > 0 = sample log_max_height + k bits, open index >> k */
  int sample_front;         /* D7: 1 = samples pop from the front of the duplex outputs */
  int selectors_normalized; /* D8: 1 = Lagrange-normalized first/last-row selectors */
  int force_witness;        /* D9: 1 = use `witness` as the PoW witness (not the smallest);
                               2 = the second-smallest valid witness */
  uint32_t witness;
} or_variant_t;
extern or_variant_t or_variant;
void or_variant_reset(void);
/* by name ("observe_openings", "diag_alt", ...); 0 on success, -1 for an unknown name */
int or_variant_set(const char* name, uint32_t value);

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
