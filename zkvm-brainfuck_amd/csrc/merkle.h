// Poseidon2 Merkle commitment on the device: MerkleTreeMmcs<.., PaddingFreeSponge<Perm,16,8,8>,
// TruncatedPermutation<Perm,2,8,16>, 8> (crates/stark/src/kb31_poseidon2.rs:24-28).
#pragma once
#include <deque>
#include <functional>
#include <vector>

#include "gpu.h"

namespace bfz {

struct MatRef {           // column-major, bit-reversed rows
  const uint32_t* base;   // column c at base + c * (stride ? stride : height)
  size_t height;
  int width;
  size_t stride = 0;
};

struct MerkleTree {
  std::vector<DBuf<uint32_t>> layers;  // layers[L]: (max_height >> L) digests x 8 (Montgomery)
  std::vector<MatRef> mats;            // committed matrices in commit order
  uint32_t root[8];                    // Montgomery form
  int sharded_below = 0;               // layers [0, sharded_below) hold only this rank's range
  int shard_log = 0;                   // log2(world) when sharded
  size_t max_height() const { return mats.empty() ? 0 : ((size_t)1 << (layers.size() - 1)); }
};

// Multi-GPU sharding of the Merkle trees of one proof.  While a context
// is installed (shard_ctx() != nullptr, world > 1), trees with at least world *
// SHARD_MIN_LEAVES leaves are built as one subtree per rank plus redundant top layers.
struct ShardCtx {
  int rank = 0, world = 1;
  // Every buffer below is DEVICE memory on this rank's GPU (RCCL moves it over xGMI with no host
  // copy).  The send data is complete when a call is made (the prover stream is drained first,
  // except before the two pipelined quotient all-gathers, where later work stays queued); the
  // received data is in place on return.
  // all-gather `bytes` from every rank into recv (world * bytes, rank order)
  std::function<void(const void* send, size_t bytes, void* recv)> allgather;
  // element-wise sum over ranks, in place
  std::function<void(uint32_t* data, size_t n)> allreduce_sum_u32;
  // timing-only run of one rank's share (bfz_record_prove_shard_solo): the exchanges are
  // no-ops, so the data after them is not the proof's and its consistency checks are skipped
  bool solo = false;
  // timing runs of a solo share: GPU milliseconds of the work that runs beside the next
  // collective (set just before it, filled when the proof's events resolve; slots live in
  // overlap_store) -- bench.py's collective model subtracts them (bfz_shard_solo_overlaps)
  mutable double* pending_overlap = nullptr;
  mutable std::deque<double> overlap_store;
};
constexpr size_t SHARD_MIN_LEAVES = 1024;
ShardCtx*& shard_ctx();

// Builds the tree (heights must be powers of two) and copies the root to the host (with
// fetch_root = false the root stays on the device, tree.layers.back(), tree.root not filled).
void merkle_build(const std::vector<MatRef>& mats, MerkleTree& tree, hipStream_t st,
                  bool fetch_root = true);

// Batched Poseidon2 permutations of n 16-element states in place (device pointer).
void poseidon2_batch(uint32_t* states, size_t n, hipStream_t st);

// Same, latency-optimised (16 lanes per state; for few states).
void poseidon2_batch_small(uint32_t* states, size_t n, hipStream_t st);

// FRI transcript step fused into the launch that finishes a root: with state != nullptr the
// device DuplexChallenger state observes the root, duplexes, and beta receives the 4 outputs a
// sample_ef pops (see k_fri_challenge).
struct RootChallenge {
  uint32_t* state = nullptr;
  kb::EF* beta = nullptr;
};

// Tree over h >= 2 rows of 8 elements (FRI commit-phase leaves: pairs of EF values, one
// permutation each).  With fetch_root = false the root stays on the device
// (tree.layers.back()) and tree.root is not filled.
// leaves(r0, count, digests) replaces the leaf hashing when given (fri.hip fuses the previous
// round's fold into it).
void merkle_from_rows8(MerkleTree& tree, const uint32_t* rows, size_t h, hipStream_t st,
                       bool fetch_root = true, RootChallenge rc = {}, bool allow_shard = true,
                       const std::function<void(size_t, size_t, uint32_t*)>& leaves = {});

}  // namespace bfz
