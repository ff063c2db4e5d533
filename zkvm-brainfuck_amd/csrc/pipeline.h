// Proof pipeline (pipeline.hip): execute + upload of proof k+1 under prove(k).
#pragma once
#include <vector>

#include "machine.h"
#include "prover.h"

namespace bfz {

struct Job {
  const uint8_t* stdin_data;
  size_t nin;
};
struct BatchStats {
  double wall_ms = 0;    // whole batch, first execute to last proof
  double exec_ms = 0;    // sum over jobs (several executor threads run at once)
  double upload_ms = 0;  // sum over jobs of the event DMA (copy stream)
  double prove_ms = 0;   // sum over jobs of tracegen + proof on the prover stream
  int exec_threads = 0;
};

// Proofs of `jobs` (stdins of pk.program), in order; byte-identical to prove() per job.
// inflight: proofs on the GPU at once (1..MAX_LANES lanes, gpu.h Lane).
std::vector<std::vector<uint8_t>> prove_batch(const ProvingKey& pk, const std::vector<Job>& jobs,
                                              const ProveOptions& opt, int exec_threads,
                                              int inflight, BatchStats* stats);

// Process-wide pinned HostEvents for single proofs (bfz_prove, bfz_record_new); callers hold the
// C ABI lock.
HostEvents& scratch_events();

}  // namespace bfz
