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
void coset_lde(const uint32_t* evals, size_t n, int w, uint32_t shift, uint32_t* lde,
               hipStream_t st);

// Row-major natural-order host layout -> column-major bit-reversed device layout.
void transpose_bitrev(const uint32_t* rowmajor, size_t n, int w, uint32_t* colmajor,
                      hipStream_t st);

// Number of waves that saw a word >= p in d[0..n) (0 iff every word is canonical); syncs st.
size_t count_noncanonical(const uint32_t* d, size_t n, hipStream_t st);

// Column-major (H x w) -> row-major, row order unchanged.
void transpose_to_rowmajor(const uint32_t* colmajor, size_t H, int w, uint32_t* rowmajor,
                           hipStream_t st);

}  // namespace bfz
