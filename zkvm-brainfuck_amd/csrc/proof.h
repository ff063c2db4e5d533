// The core proof as a value: ShardProof<KoalaBearPoseidon2> (crates/stark/src/types.rs:66-73)
// and its two byte forms.
//
//   BFZ1     the prover's normal form: what prove_device writes and the oracle
//            writes, canonical u32 words, chip_ordering as an ordered list.
//   bincode  what the reference writes: `bincode::serialize(&MachineProof)` (utils/prove.rs:46),
//            bincode 1.x default options (little-endian, u64 lengths, no varints) over the serde
//            derives of ShardProof -> ShardCommitment, ShardOpenedValues, ChipOpenedValues,
//            AirOpenedValues (types.rs:30-73) and the p3 FriProof / QueryProof /
//            CommitPhaseProofStep / BatchOpening types [p3-recalled, zkMIPS/Plonky3 @93967fce].
//            A MachineProof { shard_proof } serializes to exactly its ShardProof's bytes.
#pragma once
#include <array>
#include <cstdint>
#include <vector>

#include "kb.h"

namespace bfz {

using kb::EF;
using Digest = std::array<uint32_t, 8>;  // Montgomery words

struct ChipOpened {                  // ChipOpenedValues<Challenge> (types.rs:44-52)
  int chip = 0;                      // index in BfAir::chips() order (machine.h Chip)
  uint32_t log_degree = 0;
  std::vector<EF> prep_local, prep_next, main_local, main_next, perm_local, perm_next;
  std::vector<EF> quotient[2];       // quotient chunks opened at zeta (4 EF each)
  EF cumsum{};
};

struct BatchOpening {                // p3 BatchOpening<Val, ValMmcs>: one per input round
  std::vector<std::vector<uint32_t>> rows;  // opened row of every matrix (Montgomery)
  std::vector<Digest> path;          // MerkleTreeMmcs proof: siblings leaf -> root
};

struct CommitPhaseStep {             // p3 CommitPhaseProofStep<Challenge, ChallengeMmcs>
  EF sibling{};
  std::vector<Digest> path;
};

struct QueryProof {                  // p3 QueryProof: input_proof + commit_phase_openings
  std::vector<BatchOpening> inputs;  // 4 rounds: preprocessed, main, permutation, quotient
  std::vector<CommitPhaseStep> steps;
};

struct ShardProof {
  std::vector<int> chips;            // proof order (chip_ordering: name -> position)
  Digest main_root{}, perm_root{}, quot_root{};
  std::vector<ChipOpened> opened;
  std::vector<Digest> commit_roots;  // FRI commit-phase commitments
  std::vector<QueryProof> queries;
  EF final_poly{};
  uint32_t pow_witness = 0;          // Montgomery
};

// Field-element representation inside bincode: p3's MontyField31 serde writes the raw
// Montgomery word [p3-recalled: "faster to serialize in monty form"]; CANONICAL is the
// alternative (as_canonical_u32) kept selectable until a reference proof pins it.
enum class FieldRepr : int { MONTGOMERY = 0, CANONICAL = 1 };

ShardProof decode_bfz1(const uint8_t* p, size_t n);   // throws on malformed input
std::vector<uint8_t> encode_bfz1(const ShardProof& pf);
ShardProof decode_bincode(const uint8_t* p, size_t n, FieldRepr repr);
std::vector<uint8_t> encode_bincode(const ShardProof& pf, FieldRepr repr);

}  // namespace bfz
