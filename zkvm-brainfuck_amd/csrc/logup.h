// Device LogUp permutation trace (see logup.hip).
#pragma once
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
void perm_trace(int chip, const uint32_t* mainc, const uint32_t* prepc, size_t n,
                const PermChallenges& ch, uint32_t* perm, kb::EF* cumsum_dev, hipStream_t st);

void ef_inclusive_scan(kb::EF* data, size_t n, hipStream_t st);

}  // namespace bfz
