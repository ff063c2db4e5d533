// Host verifier: Verifier::verify_shard (crates/stark/src/verifier.rs:27-329)
// + TwoAdicFriPcs::verify / fri::verifier [p3-recalled] + BfProver::verify's CPU-degree cap
// (crates/prover/src/verify.rs:10-36), over a decoded ShardProof (proof.h) -- so the same checks
// run on the BFZ1 normal form and on the reference's bincode bytes.
#pragma once
#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

#include "proof.h"

namespace bfz {

struct VerifyOptions {
  int num_queries = 84;
  bool observe_openings = true;  // PCS transcript variant (decision D1)
};

// Main and permutation (base) columns a chip's constraints read at the next row.
struct NextCols {
  std::vector<int> main, perm;
};
NextCols next_row_columns(int chip);

bool verify_shard(const std::string& program_src, const uint32_t vk_commit[8], const ShardProof& pf,
                  const VerifyOptions& opt, std::string* why);

// BFZ1 bytes (decode_bfz1 + verify_shard)
bool verify_proof(const std::string& program_src, const uint32_t vk_commit[8], const uint8_t* proof,
                  size_t len, const VerifyOptions& opt, std::string* why);

}  // namespace bfz
