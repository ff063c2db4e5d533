// Device NTT / coset LDE (see ntt.hip).
#pragma once
#include <algorithm>
#include <utility>
#include <vector>

#include "gpu.h"

namespace bfz {

// All device work of a proof is ordered on one stream (bfz::stream()); pooled buffers released
// on the host may be reused immediately by later work on that stream.

// In-place/out-of-place radix-2 passes over `ncols` columns of size 2^L.
// dif=false: inverse DIT (bit-reversed in -> natural out, twiddles w^-1, no 1/n scaling)
// dif=true : forward DIF (natural in -> bit-reversed out)
void ntt_passes(const uint32_t* src, uint32_t* dst, size_t src_stride, size_t dst_stride, int ncols,
                int L, bool dif, hipStream_t st);

// evals: column-major, bit-reversed rows (n x w).  lde: column-major 2n x w, bit-reversed
// rows = evaluations of the interpolant on shift * H_2n (shift = GENERATOR / domain shift).
// Builds (once per process) the twiddle and coset-power tables a proof's LDEs of height 2^L use,
// so no proof builds a table between its launches (bfz_record_* call it for the record's heights).
void prepare_lde_tables(int L);
void coset_lde(const uint32_t* evals, size_t n, int w, uint32_t shift, uint32_t* lde,
               hipStream_t st);
// The same with the input columns at stride src_stride, and only_half = 0 / 1: write only
// LDE rows [0, n) / [n, 2n) of each column (the other half is left untouched -- a quotient
// chunk's own domain is that half, so the caller has its values already; -1: both halves).
void coset_lde_ex(const uint32_t* evals, size_t src_stride, size_t n, int w, uint32_t shift,
                  uint32_t* lde, int only_half, hipStream_t st);

// Sharded LDE.  lde_coefficients: coef = n * (coefficients of the interpolant
// over H_n), natural order (the iDFT alone).  coset_residue: the rank shard of the coset LDE
// on shift * H_2n for G = 2^logG ranks and residue r = bitrev_G(rank): bit-reversed positions
// [rank m, (rank+1) m), m = 2n / G, column-major (m x w) -- word-for-word the same rows as
// coset_lde's.
void lde_coefficients(const uint32_t* evals, size_t n, int w, uint32_t* coef, hipStream_t st);
void coset_residue(const uint32_t* coef, size_t n, int w, uint32_t shift, int logG, int r,
                   uint32_t* out, hipStream_t st);
// The same for the listed columns only (out column y = coefficient column cols[y]).
void coset_residue_cols(const uint32_t* coef, size_t n, const std::vector<int>& cols,
                        uint32_t shift, int logG, int r, uint32_t* out, hipStream_t st);

// The same in one pass over the coefficients (k_coef_fold): the iDFT's second pass keeps each
// column's coefficients in registers, writes coef only for [j0, j0 + len) (column stride n) and
// folds them into out (residue r, m x w, m = 2n / G) and, with next_cols, into nxt (residue r2,
// the listed columns) -- natural order; residue_dft then finishes each (the forward DFT).
// Returns false (nothing launched) where it does not apply (log n <= 14 or > 23, G > 32);
// else *dft_low is what residue_dft has left to do for out and nxt alike: -1 = the whole DFT,
// s >= 0 = only its stages [0, s) (2, 4 and 8 ranks: at 2 ranks without a next residue out is
// k_lde_mid's half r, at 4 and 8 the fold kernel continues with the strided DIF stages).
bool coef_fold_residues(const uint32_t* evals, size_t n, int w, uint32_t* coef, size_t j0,
                        size_t len, uint32_t shift, int logG, int r, uint32_t* out,
                        const std::vector<int>* next_cols, int r2, uint32_t* nxt, int* dft_low,
                        hipStream_t st);
void residue_dft(uint32_t* out, size_t m, int w, int dft_low, hipStream_t st);

// Row-major natural-order host layout -> column-major bit-reversed device layout.
void transpose_bitrev(const uint32_t* rowmajor, size_t n, int w, uint32_t* colmajor,
                      hipStream_t st);

// Number of waves that saw a word >= p in d[0..n) (0 iff every word is canonical); syncs st.
size_t count_noncanonical(const uint32_t* d, size_t n, hipStream_t st);

// Column-major (H x w) -> row-major, row order unchanged.
void transpose_to_rowmajor(const uint32_t* colmajor, size_t H, int w, uint32_t* rowmajor,
                           hipStream_t st);

}  // namespace bfz
