// Device quotient evaluation (see quotient.hip).
#pragma once
#include "gpu.h"
#include "machine.h"
#include "logup.h"

namespace bfz {

struct QuotParams {
  kb::EF perm_alpha;
  kb::EF beta_pows[8];
  kb::EF cumsum;
  const kb::EF* alpha_pows;  // device array: alpha^(K-1-k), k = 0..K-1
  uint32_t zh_even, zh_odd, zh_even_inv, zh_odd_inv;  // Z_H at even / odd natural index
  uint32_t wn_inv;  // w_n^-1
  uint32_t shift;   // GENERATOR = 3
};

// Number of constraints (AIR + LogUp) emitted by a chip's eval.
int num_constraints(int chip);

// Writes Q at all 2n points into qout: 8 base columns of n rows (chunk k, coefficient e at
// column 4k+e), rows in bit-reversed order of the chunk domain.
// Builds (once per process) the selector-denominator table of the quotient domain 3 H_N, N = 2^logN.
void prepare_quotient_tables(int logN);
void quotient(int chip, const uint32_t* mainc, const uint32_t* prepc, const uint32_t* permc,
              int logN, const QuotParams& qp, uint32_t* qout, hipStream_t st);

// Row-range form (sharded proofs): LDE positions [t0, t0 + count) only.  Every
// pointer is indexed by the GLOBAL position: column c of main/perm at ptr[c * stride + t]
// (a shard buffer passes its base minus its first position), prep at prep[c * N + t] (full).
// main_l/perm_l serve the points' own rows, main_n/perm_n their next rows (i + 2); in the
// unsharded form both are the full LDE (identity column maps); a sharded proof's next-row
// shards hold only the columns the chip reads at the next row.  qout is the full 8 x n chunk buffer; only the
// range's entries are written.
struct QuotRows {
  const uint32_t *main_l, *main_n, *perm_l, *perm_n, *prep;
  size_t stride, t0, count;
  uint8_t nmain[64], nperm[64];  // column c's next row: main_n / perm_n column nmain[c] / nperm[c]
};
// qp_dev: the same parameters in device memory (nullptr: qp is uploaded for the launch).
void quotient_rows(int chip, const QuotRows& in, int logN, const QuotParams& qp, uint32_t* qout,
                   hipStream_t st, const QuotParams* qp_dev = nullptr);
// Output placement: chunk k's coefficient column e at chunk[k] + e * stride (row = position
// within the chunk).  qout above is {qout, qout + 4n}, stride n; the single-GPU prover writes
// each chunk straight into its own half of the chunk's LDE buffer ({lde0, lde1 + n}, stride 2n).
struct QuotOut {
  uint32_t* chunk[2];
  size_t stride;
};
void quotient_into(int chip, const QuotRows& in, int logN, const QuotParams& qp, const QuotOut& out,
                   hipStream_t st, const QuotParams* qp_dev = nullptr);
// The quotient challenge on the device after the LogUp commit (see k_challenge_quot): ch is the
// device sponge (updated), root the permutation root, cums the chips' cumulative sums, pc the
// LogUp challenges; qps[k]'s perm_alpha / beta_pows / cumsum and apows[k] (K[k] powers) are
// written.  The host replays the step when it fetches the roots.
constexpr int QUOT_MAX_CHIPS = 8;
struct QuotAlphaTargets {
  kb::EF* apows[QUOT_MAX_CHIPS];
  int K[QUOT_MAX_CHIPS];
  kb::EF* alpha_out;  // optional: the sampled alpha itself (checked against the host replay)
};
void challenge_quot(DevChallenger* ch, const uint32_t* root, const kb::EF* cums, int nc,
                    const PermChallenges* pc, QuotParams* qps, const QuotAlphaTargets& tg,
                    hipStream_t st);

}  // namespace bfz
