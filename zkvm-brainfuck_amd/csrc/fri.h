// Device PCS-open / FRI kernels (see fri.hip).
#pragma once
#include <vector>

#include "challenger.h"
#include "gpu.h"
#include "merkle.h"

namespace bfz {

struct RedCol {            // one committed column at a given LDE height
  const uint32_t* col;     // device column (bit-reversed rows)
  kb::EF ca;               // alpha-power coefficient at the first opening point
};
struct RedMat {            // the columns [first, first + count) of one matrix
  int first, count;
  int has_b;               // opened at the second point too: coefficient there = kb * ca
  int pad;
  kb::EF kb;               // alpha^width
};

// out[t] = 1 / (x_t - z), x_t = 3 * w_H^bitrev(t), t < 2^logH
void inv_denoms(const kb::EF& z, int logH, kb::EF* out, hipStream_t st);
// out[t - t0] = 1 / (x_t - z) for the positions t in [t0, t0 + count) of an LDE of height 2^logH
void inv_denoms_range(const kb::EF& z, int logH, size_t t0, size_t count, kb::EF* out,
                      hipStream_t st);
// out[t] = z^(j0 + t), t < count
void pow_table(const kb::EF& z, size_t j0, size_t count, kb::EF* out, hipStream_t st);
// Several of either in one launch (a sharded proof's openings: one table per point and height,
// one denominator range per height and point)
struct PowJob {
  kb::EF z;
  size_t j0, count;
  kb::EF* out;
};
void pow_tables(const std::vector<PowJob>& jobs, hipStream_t st);
struct InvJob {
  kb::EF z;
  int logH;
  size_t t0, count;
  kb::EF* out;
};
void inv_denoms_ranges(const std::vector<InvJob>& jobs, hipStream_t st);
// Coefficient-form opening (sharded proofs): out[c] = scale * sum_(t < count) coef[c * col_stride
// + t] tab[t] for each point (tab = powers of the point from the range's first exponent).
void open_coefficients(const uint32_t* coef, size_t col_stride, int w, size_t count,
                       const kb::EF* tab_a, const kb::EF& scale_a, kb::EF* out_a,
                       const kb::EF* tab_b, const kb::EF& scale_b, kb::EF* out_b, hipStream_t st);
// One matrix of a batched barycentric opening (open_batch): columns of an LDE of height
// `height` (column stride) opened over its low coset at one or two points; out_a[c] / out_b[c]
// = scale_a / scale_b times the weighted column sums.  chunk0 .. part_off are filled in by
// open_batch.
struct OpenDesc {
  const uint32_t* mat;
  uint64_t height;
  int w, logH;
  // two matrices of one height opened at the same points share a descriptor (open_batch merges
  // them: one weight computation per row for both): columns [0, w1) from mat, [w1, w) from mat2,
  // opened values to out_a / out_b and out_a2 / out_b2
  const uint32_t* mat2;
  int w1;
  kb::EF* out_a2;
  kb::EF* out_b2;
  // wtab != nullptr: the weights x_t / (x_t - z) are read from this table (inv_denoms_dev's wout)
  // for both points (the second at t', see open_tile_body) and zb must be 1
  const kb::EF* wtab;
  const kb::EF* invd_a;
  const kb::EF* invd_b;  // nullptr: derived from invd_a (w_n^-1 folded into scale_b, see k_reduce)
  kb::EF scale_a, scale_b;
  kb::EF* out_a;
  kb::EF* out_b;
  uint32_t chunk0, col0, nchunks, nslab;  // first block, first column, row chunks, column slabs
  int slab_w;                              // columns per slab (a multiple of 4)
  uint64_t part_off;
  // zeta != nullptr: the point lives on the device (sampled there) and k_open_final_batch
  // computes the scales itself: scale_a = (zeta^n - 3^n) * zc with n = 2^zlog, zc = 1/(3^n n);
  // scale_b = scale_a * zb ((zeta w_n)^n = zeta^n; zb = w_n^-1 when invd_b is derived, else 1)
  const kb::EF* zeta;
  int zlog;
  uint32_t z3n, zc, zb;
  // tab != 0: the coefficient form of a sharded matrix (open_coefficients): mat = the first of
  // `rows` coefficients of each column (column stride height), invd_a / invd_b = the points'
  // power tables (the weights), scales unnegated.  rows = 0: the low coset (height / 2).
  uint64_t rows;
  int tab;
};
// Every descriptor of ds is opened at np (1 or 2) points: one partial-sum launch over all of
// their row chunks, one final launch over all of their columns.
void open_batch(std::vector<OpenDesc>& ds, int np, hipStream_t st);
// 1 / (x_t - z) over the whole 2^logH coset with z read from device memory (sampled there)
// wout != nullptr: also the low coset's barycentric weights x_t / (x_t - z), t < 2^(logH-1)
// (every smaller height's low coset is a prefix, as for out)
void inv_denoms_dev(const kb::EF* z, int logH, kb::EF* out, hipStream_t st, kb::EF* wout = nullptr);
// ro[t] = (sum_c ca_c v_c[t] - ya) invd_a[t] + (sum_m kb_m sum_(c in m) ca_c v_c[t] - yb) invd_b[t]
// for the positions [t0, t0 + count) of a height-`height` LDE (all of it, or a shard's range);
// cols / mats: device descriptor arrays of one height (RedMat::first indexes cols); every
// pointer is indexed by the global position.  invd_b == nullptr with has_b: the second point is zeta w_n and its
// denominators are read from invd_a at the position of natural index i - 2 -- the caller has
// folded w_n^-1 into every RedMat::kb and into yb.
// yab: DEVICE pointer to {ya, yb} (reduce_prep writes them)
void reduce_range(const RedCol* cols, const RedMat* mats, int nmats, size_t height, size_t t0,
                  size_t count, const kb::EF* invd_a, const kb::EF* invd_b, const kb::EF* yab,
                  bool has_b, kb::EF* ro, hipStream_t st, int ncols = 0);
// The alpha-dependent fields of the reduced-opening descriptors, computed on the device once the
// FRI batching challenge alpha is known (the host builds the rest while the openings run):
//   column c: ca = alpha^e0 (its position in the height's reduction order), and the job's
//   ya = sum ca y_a, yb = yb_fold * sum ca alpha^w(m) y_b  (y from the opened-value buffer);
//   matrix m: kb = alpha^w * fold.
struct RedColPrep {
  uint32_t e0, ia, ib;  // ib = UINT32_MAX: the matrix is opened at one point
  uint32_t w;           // the column's matrix width (alpha^w for the second point)
};
struct RedMatPrep {
  uint32_t w, fold;     // kb = alpha^w * fold (fold: Montgomery base-field factor)
};
struct RedJobPrep {
  uint32_t col0, ncols, mat0, nmats;
  uint32_t yb_fold, pad[3];
};
void reduce_prep(RedCol* cols, const RedColPrep* cp, RedMat* mats, const RedMatPrep* mp,
                 const RedJobPrep* jp, int njobs, const kb::EF* opened, const kb::EF* alpha,
                 kb::EF* yab, hipStream_t st);
// The transcript after the commit phase, on the device (prover.rs:470 open -> TwoAdicFriPcs
// [p3-recalled]: observe the final constant, grind, sample the query indices) with no host round
// trip.  c: the challenger, in device memory -- taken as is when fri_state is null (no FRI round),
// otherwise rebuilt from the commit phase's sponge state (the last round's duplex, 4 outputs
// left).  It ends as the host challenger would after the last query index.  res[0] = the smallest
// witness w with sample_bits(bits) == 0 after observe(w), res[1] = 1 when the replayed check
// holds; qidx[q] = sample_bits(log_max), q < nq.
void fri_transcript_tail(DevChallenger* c, const uint32_t* fri_state, const kb::EF* fin, int bits,
                         int nq, int log_max, uint32_t* qidx, uint32_t* res, hipStream_t st);
// One FRI commit-phase transcript step on the device (DuplexChallenger with an empty input
// buffer): observe the 8-word root, duplex, sample an EF (pops out[7], out[6], out[5], out[4]).
// state: 16 words (Montgomery), updated in place; beta: EF written for the fold.
void fri_challenge(uint32_t* state, const uint32_t* root, kb::EF* beta, hipStream_t st);
// Fold with beta read from device memory.
void fri_fold_dev(const kb::EF* in, kb::EF* out, size_t h, const kb::EF* beta, const kb::EF* add,
                  hipStream_t st);
// Outputs [i0, i0 + count) of the same fold; in, out and add hold only that range.
void fri_fold_range(const kb::EF* in, kb::EF* out, size_t h, size_t i0, size_t count,
                    const kb::EF* beta, const kb::EF* add, hipStream_t st);
// The fold of layer `in` (4 h values) fused with the next round's leaf hashes: out[k] =
// fold(in[2k], in[2k+1]) (+ add[k]) for k < 2 h, and leaf i = P(out[2i] || out[2i+1])[0..8] into
// digests[8 i ..] (k_fri_fold_dev + k_hash_rows8 in one pass).  Thread mode only: the
// prover uses it where the leaves are hashed one permutation per thread (h > FRI_FUSE_MIN / 2).
// (A lane-mode form, 16 lanes per leaf with every fold computed by four lanes, took 14.7 us per
// round against 4.7 + 4.8 us for the separate fold and lane-mode hash.)
constexpr size_t FRI_FUSE_MIN = (size_t)1 << 15;  // merkle.hip: lane-mode leaves up to 2^14
void fri_fold_leaves(const kb::EF* in, kb::EF* out, size_t h, const kb::EF* beta,
                     const kb::EF* add, uint32_t* digests, hipStream_t st);
// The last commit-phase rounds (at most FRI_TAIL_MAXH leaves) in one single-workgroup launch:
// per round the leaf hashes, every tree layer, the transcript step (observe the root, duplex,
// beta) and the fold, with the layer and the digests kept in LDS between the steps.  Every
// digest and fold output is also written to its buffer (the query openings read them).
// (same-box A/B, profiles/r03/ab_open_and_tops.txt: FRI stage 2.675 -> 2.624 ms with the fused
// folds and a 128-leaf tail; 64 and 256 leaves were no better)
constexpr int FRI_TAIL_MAXH = 128;
constexpr int FRI_TAIL_MAXR = 10;
struct FriTailRounds {
  int nr = 0;                             // rounds: h = 2^logh0, 2^(logh0-1), ...
  int logh0 = 0;
  const kb::EF* in = nullptr;             // the first round's layer (2 h values)
  kb::EF* layer[FRI_TAIL_MAXR] = {};      // round r's fold output (h_r values)
  uint32_t* tree[FRI_TAIL_MAXR] = {};     // round r's tree: layers of 8 h_r, 4 h_r, ..., 8 words
  const kb::EF* add[FRI_TAIL_MAXR] = {};  // reduced openings added to round r's fold, or null
  uint32_t* state = nullptr;              // device challenger state (16 words), in/out
  kb::EF* beta = nullptr;                 // the rounds' betas
};
void fri_tail_rounds(const FriTailRounds& a, hipStream_t st);
// Query openings: word k of segment s for query index I is
//   base[((I >> shift) ^ xr) * unit + k * stride],  k < count
// (matrix rows: unit 1, stride = height; Merkle siblings: unit 8; FRI siblings: unit 4).
// When the tree is sharded, word k of a segment is owned by rank (element >> own_shift)
// (own_shift < 0: replicated data, owned by rank 0); other ranks write 0 and the ranks' words
// are summed.
struct GatherSeg {
  const uint32_t* base;
  uint64_t stride;
  uint32_t shift, xr, unit, count;
  int32_t own_shift;
  int32_t pad;
};
// Words per query of a segment list.
size_t query_words(const std::vector<GatherSeg>& segs);
// out[q * query_words(segs) + ...] = the segments' words for qidx[q] (device), q < nq, segments
// in order, canonical form; a segment with base == nullptr is `count` literal words of value xr.
// In a sharded proof (shard != nullptr, world > 1) every rank writes the words it owns and one
// sum all-reduce over the device buffer completes them.
void gather_queries(const std::vector<GatherSeg>& segs, const uint32_t* qidx, int nq, uint32_t* out,
                    const ShardCtx* shard, hipStream_t st);

}  // namespace bfz
