// Column-sharded PCS commit + FRI commit phase over the GPUs of a node (SURVEY.md §8(e);
// BASELINE configs 4 and 5: a synthetic 2^24 x 64 trace over 4 GPUs, 2^26 rows over 8).
#pragma once
#include <array>
#include <functional>
#include <vector>

#include "kb.h"
#include "prover.h"

namespace bfz {

struct PcsShardedResult {
  uint32_t root[8];                             // commitment to the trace LDE (Montgomery)
  std::vector<std::array<uint32_t, 8>> fri_roots;  // commit-phase roots, one per fold round
  kb::EF final_value;                           // the constant the FRI input folds down to
};

// cols: this rank's w_local columns of an n = 2^log_n row trace, column-major with
// bit-reversed rows (the device trace layout), columns [rank w_local, (rank+1) w_local).
// send/recv: caller-owned device buffers of 2n * w_local words each (unused when world == 1);
// alltoall() exchanges equal blocks of send into recv (block j goes to rank j).  The shard
// context (shard_ctx()) supplies rank, world and the all-gather; without one, world = 1.
PcsShardedResult commit_fri_sharded(const uint32_t* cols, int log_n, int w_local, uint32_t* send,
                                    uint32_t* recv, const std::function<void()>& alltoall,
                                    hipStream_t st);

}  // namespace bfz
