// Host verifier for BFZ1 proofs: Verifier::verify_shard (crates/stark/src/verifier.rs:27-329)
// + TwoAdicFriPcs::verify / fri::verifier [p3-recalled] + BfProver::verify's CPU-degree cap
// (crates/prover/src/verify.rs:10-36).
#pragma once
#include <cstddef>
#include <cstdint>
#include <string>

namespace bfz {

bool verify_proof(const std::string& program_src, const uint32_t vk_commit[8], const uint8_t* proof,
                  size_t len, int num_queries, std::string* why);

}  // namespace bfz
