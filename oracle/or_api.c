/* ORACLE — test infrastructure only.  ctypes-facing wrappers. */
#include <stdlib.h>
#include <string.h>
#include "or_api.h"
#include "or_dft.h"
#include "or_hash.h"

int or_api_execute(const char* program, const uint8_t* in, size_t nin, uint8_t* out,
                   size_t outcap, size_t* outlen, uint64_t* cycles, uint32_t* final_pc,
                   uint32_t* final_mp) {
  or_program p;
  if (or_parse_program(program, &p)) return -1;
  or_record r;
  int err = or_execute(&p, in, nin, &r);
  if (!err) {
    size_t n = r.noutput < outcap ? r.noutput : outcap;
    if (n) memcpy(out, r.output, n);
    *outlen = r.noutput;
    *cycles = r.global_clk;
    *final_pc = r.final_pc;
    *final_mp = r.final_mp;
  }
  or_record_free(&r);
  free(p.ins);
  return err;
}

int or_api_prove(const char* program, const uint8_t* in, size_t nin, uint8_t** proof,
                 size_t* len) {
  or_program p;
  if (or_parse_program(program, &p)) return -1;
  or_record r;
  int err = or_execute(&p, in, nin, &r);
  if (!err) err = or_prove_record(&p, &r, proof, len, NULL);
  or_record_free(&r);
  free(p.ins);
  return err;
}

int or_api_verify(const char* program, const uint8_t* proof, size_t len) {
  or_program p;
  if (or_parse_program(program, &p)) return -1;
  int err = or_verify_proof(&p, proof, len);
  free(p.ins);
  return err;
}

void or_api_free(void* p) { free(p); }

int or_api_setup_root(const char* program, uint32_t root[8]) {
  or_program p;
  if (or_parse_program(program, &p)) return -1;
  or_setup_root(&p, root);
  free(p.ins);
  return 0;
}

int or_api_trace(const char* program, const uint8_t* in, size_t nin, int chip, int prep,
                 uint32_t** out, size_t* h, size_t* w) {
  or_program p;
  if (or_parse_program(program, &p)) return -1;
  int err = 0;
  if (prep) {
    *h = or_prep_trace(chip, &p, out);
    *w = (size_t)OR_CHIPS[chip].prep_w;
    if (!*h) err = -2;
  } else {
    or_record r;
    err = or_execute(&p, in, nin, &r);
    if (!err) {
      or_generate_dependencies(&r);
      if (!or_chip_included(chip, &r)) err = -2;
      else { *h = or_main_trace(chip, &r, out); *w = (size_t)OR_CHIPS[chip].main_w; }
    }
    or_record_free(&r);
  }
  free(p.ins);
  return err;
}

void or_api_poseidon2(uint32_t* states, size_t n) {
  for (size_t i = 0; i < n; i++) or_poseidon2_permute(&states[16 * i]);
}

void or_api_hash(const uint32_t* in, size_t n, uint32_t out[8]) { or_hash(in, n, out); }

void or_api_coset_lde(const uint32_t* in, size_t n, size_t w, uint32_t shift, uint32_t* out) {
  or_coset_lde(in, n, w, shift, 1, out);
}

void or_api_merkle_root(const uint32_t* const* mats, const size_t* heights, const size_t* widths,
                        int nmats, uint32_t root[8]) {
  or_mat* m = calloc(nmats, sizeof(or_mat));
  for (int i = 0; i < nmats; i++) {
    m[i].values = (fp*)mats[i]; m[i].height = heights[i]; m[i].width = widths[i];
  }
  or_merkle t;
  or_merkle_build(&t, m, nmats);
  memcpy(root, t.root, 32);
  or_merkle_free(&t);
  free(m);
}

uint32_t or_api_two_adic_gen(int bits) { return fp_two_adic_gen(bits); }

void or_api_ef_mul(const uint32_t a[4], const uint32_t b[4], uint32_t out[4]) {
  ef x, y;
  memcpy(x.c, a, 16); memcpy(y.c, b, 16);
  ef z = ef_mul(x, y);
  memcpy(out, z.c, 16);
}

void or_api_ef_inv(const uint32_t a[4], uint32_t out[4]) {
  ef x;
  memcpy(x.c, a, 16);
  ef z = ef_inv(x);
  memcpy(out, z.c, 16);
}

void or_api_challenger(const uint32_t* obs, size_t n, uint32_t* samples, size_t m) {
  or_challenger c;
  or_ch_init(&c);
  for (size_t i = 0; i < n; i++) or_ch_observe(&c, obs[i]);
  for (size_t i = 0; i < m; i++) samples[i] = or_ch_sample(&c);
}
