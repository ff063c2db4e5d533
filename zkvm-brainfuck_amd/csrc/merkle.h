// Poseidon2 Merkle commitment on the device: MerkleTreeMmcs<.., PaddingFreeSponge<Perm,16,8,8>,
// TruncatedPermutation<Perm,2,8,16>, 8> (crates/stark/src/kb31_poseidon2.rs:24-28).
#pragma once
#include <vector>

#include "gpu.h"

namespace bfz {

struct MatRef {           // column-major, bit-reversed rows
  const uint32_t* base;   // column c at base + c * height
  size_t height;
  int width;
};

struct MerkleTree {
  std::vector<DBuf<uint32_t>> layers;  // layers[L]: (max_height >> L) digests x 8 (Montgomery)
  std::vector<MatRef> mats;            // committed matrices in commit order
  uint32_t root[8];                    // Montgomery form
  size_t max_height() const { return mats.empty() ? 0 : ((size_t)1 << (layers.size() - 1)); }
};

// Builds the tree (heights must be powers of two) and copies the root to the host.
void merkle_build(const std::vector<MatRef>& mats, MerkleTree& tree, hipStream_t st);

// Batched Poseidon2 permutations of n 16-element states in place (device pointer).
void poseidon2_batch(uint32_t* states, size_t n, hipStream_t st);

// Same, latency-optimised (16 lanes per state; for few states).
void poseidon2_batch_small(uint32_t* states, size_t n, hipStream_t st);

// Hash of 8-element rows (FRI commit-phase leaves: pairs of EF values), one permutation each.
void hash_rows8(const uint32_t* rows, size_t n, uint32_t* digests, hipStream_t st);

// Digest layers above an existing leaf layer (no injection).  With fetch_root = false the
// root stays on the device (tree.layers.back()) and tree.root is not filled.
void merkle_layers_from_leaves(MerkleTree& tree, hipStream_t st, bool fetch_root = true);

}  // namespace bfz
