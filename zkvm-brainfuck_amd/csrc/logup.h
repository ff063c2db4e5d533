// Device LogUp permutation trace (see logup.hip).
#pragma once
#include "challenger.h"
#include "air.h"
#include "gpu.h"
#include "machine.h"

namespace bfz {

struct PermChallenges {
  kb::EF alpha;          // LogUp alpha (prover.rs:269-272, first sample)
  kb::EF beta_pows[8];   // beta^0 .. beta^7
};

// mainc/prepc: column-major bit-reversed trace evaluations (n rows).  perm: 4*perm_width(chip)
// base columns (n rows, bit-reversed).  cumsum_dev: device EF receiving the cumulative sum.
// ch: DEVICE memory (the prover samples the challenges on the device, challenge_perm).
void perm_trace(int chip, const uint32_t* mainc, const uint32_t* prepc, size_t n,
                const PermChallenges* ch, uint32_t* perm, kb::EF* cumsum_dev, hipStream_t st);
// Device transcript step after the main commit: the DuplexChallenger state `ch` (device
// memory, updated in place) observes the 8-word root and samples the LogUp alpha and beta
// (prover.rs:269-272); out receives alpha and beta^0..7.  The host replays the same step when
// it fetches the root later, so its transcript stays in step.
void challenge_perm(DevChallenger* ch, const uint32_t* root, PermChallenges* out, hipStream_t st);
// The out-of-domain point after the quotient commit (prover.rs:415 challenger.sample_ext_element
// after observing the quotient root), on the device: observe root, *zeta = sample_ef.  The host
// replays it when the roots come back and fails on a mismatch.
void challenge_zeta(DevChallenger* ch, const uint32_t* root, kb::EF* zeta, hipStream_t st);

void ef_inclusive_scan(kb::EF* data, size_t n, hipStream_t st);

}  // namespace bfz
