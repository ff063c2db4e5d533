// HIP core prover: the MachineProver<KoalaBearPoseidon2, BfAir> drop-in
// (crates/stark/src/prover.rs:27-150), device-resident from trace upload to proof.
#pragma once
#include <array>
#include <memory>
#include <string>
#include <vector>

#include "gpu.h"
#include "machine.h"
#include "merkle.h"

namespace bfz {

using kb::EF;

// DuplexChallenger<KoalaBear, Perm, 16, 8> (crates/stark/src/kb31_poseidon2.rs:31,126-128)
// [p3-recalled]: observe -> input buffer (duplex when 8 pending, clears outputs);
// sample -> duplex if inputs pending or outputs empty, then pop from the END of the outputs.
struct Challenger {
  uint32_t st[16] = {0};
  uint32_t in[8] = {0};
  int nin = 0;
  uint32_t out[8] = {0};
  int nout = 0;
  void duplex();
  void observe(uint32_t v);  // Montgomery form
  void observe_digest(const uint32_t d[8]);
  void observe_ef(const EF& e);
  uint32_t sample();
  EF sample_ef();
  uint32_t sample_bits(int bits);
  bool check_witness(int bits, uint32_t w);
};

struct CMat {               // a committed matrix: LDE on 3*H_2n (bit-reversed, column-major)
  DevMatrix lde;            // lde.height = 2n always; a sharded matrix's buffer holds blk rows
  size_t n = 0;             // trace-domain size
  int log_n = 0;
  uint32_t shift = 0;       // trace-domain shift (Montgomery)
  // Sharded proofs: this rank's positions [row0, row0 + blk) of the LDE (its
  // residue class of natural rows), the interpolant's coefficients (n c_j, natural order, for
  // the coefficient-form opening) and, for G >= 4, the shard of the residue class the quotient's
  // next rows (i + 2) fall in, at positions [nxt_row0, nxt_row0 + blk).
  bool sharded = false;
  size_t blk = 0, row0 = 0, nxt_row0 = 0;
  DBuf<uint32_t> coef, nxt;
  std::array<uint8_t, 64> nmap{};  // column c's next row: column nmap[c] of next_rows()
  // column c, global position t  ->  rows()[c * stride() + t]
  const uint32_t* rows() const { return sharded ? lde.buf.p - row0 : lde.buf.p; }
  size_t stride() const { return sharded ? blk : lde.height; }
  // Next rows of a sharded matrix come from positions [nxt_row0, nxt_row0 + blk): the next-row
  // shard when one was computed (G >= 4), the rank's own shard otherwise (G = 2: the same class;
  // G >= 4 without next-row columns: never read, but every address stays inside the buffer).
  const uint32_t* next_rows() const {
    return sharded ? (nxt.p ? nxt.p : lde.buf.p) - nxt_row0 : rows();
  }
  MatRef ref() const { return MatRef{rows(), lde.height, lde.width, stride()}; }
};

struct Round {
  std::vector<CMat> mats;
  MerkleTree tree;
  void commit(hipStream_t st, bool fetch_root = true);
};

struct ProvingKey {
  Program program;
  Round prep;                                // Program / Byte, sorted (Reverse(height), name)
  std::vector<DBuf<uint32_t>> prep_evals;    // trace evaluations (bit-reversed, column-major)
  std::array<int, 2> chip_of{};
  std::array<int, NUM_CHIPS> idx_of_chip{};
};

struct StageTimes {          // milliseconds, measured with HIP events on the prover stream
  double trace = 0, main_commit = 0, perm = 0, quotient = 0, open = 0, fri = 0, total = 0;
  double lde_ms = 0;         // sum over coset_lde calls
  double lde_bytes = 0;      // algorithmic bytes: 12 * n * w per call
  int lde_calls = 0;
  double ntt_kernel_ms = 0;     // k_ntt_r16 launches, one event pair per launch
  double ntt_kernel_bytes = 0;  // 8 B per element per pass
  int ntt_kernel_launches = 0;
  double p2_kernel_ms = 0;   // throughput Poseidon2 kernels (leaves, compress, FRI rows)
  double p2_perms = 0;       // permutations they computed
  int p2_launches = 0;
  double lde_elem_stages = 0;  // iDFT n + DFT n on each coset half: 3 * n * log2(n) * w per call
  double open_kernel_ms = 0, open_kernel_bytes = 0;  // k_open_partial_batch (algorithmic bytes)
  int open_kernel_launches = 0;
  double reduce_kernel_ms = 0, reduce_kernel_bytes = 0;  // k_reduce
  int reduce_kernel_launches = 0;
  // the LogUp stage in parts (bfz.h bfz_timings)
  double perm_rows = 0, perm_idft = 0, perm_dft = 0, perm_hash = 0;
  // the main commit in parts: iDFT of the main columns, fold + forward DFT, Merkle hashing
  double main_idft = 0, main_dft = 0, main_hash = 0;
  // base-field cells (sum of n x w) of the main and permutation traces
  double main_cells = 0, perm_cells = 0;
  // timed runs of a solo share: the spins that isolate the collective-overlap windows (taken
  // back out of quotient and total when the events resolve)
  double spin = 0;
};

std::unique_ptr<ProvingKey> setup(const std::string& program_src);

// Coset LDE of trace evaluations (bit-reversed, column-major) into a committed matrix.
void commit_lde(CMat& cm, const uint32_t* evals, size_t n, int w, uint32_t domain_shift,
                hipStream_t st);

struct ProveOptions {
  int num_queries = 84;
  bool timing = false;
  // Decision D1 ([p3-recalled]): TwoAdicFriPcs::open observes every opened
  // value before sampling the FRI batching challenge alpha (true), or samples alpha first (false)
  bool observe_openings = true;
  // Test-only fault injection (bfz_set_fault_injection): perturb the device challenger's
  // uploaded sponge so the host replay must report the divergence.
  bool fault_device_challenger = false;
};

// Full core proof of (program, stdin) in the BFZ1 normal form.
std::vector<uint8_t> prove(const ProvingKey& pk, const uint8_t* stdin_data, size_t nin,
                           const ProveOptions& opt, StageTimes* times,
                           std::vector<uint8_t>* output_stream = nullptr,
                           uint64_t* cycles = nullptr);

// Prove from pre-generated main traces already resident on the device (bench path).
struct DeviceTraces {
  std::vector<int> chips;                     // included chips (any order)
  std::vector<DBuf<uint32_t>> evals;          // column-major bit-reversed evaluations
  std::vector<size_t> heights;
};
// Host main traces as MachineProver::generate_traces returns them (row-major Montgomery,
// one per included chip); validates chip ids, widths and power-of-two heights.
void upload_host_traces(const int* chips, const uint32_t* const* mats, const size_t* heights,
                        const size_t* widths, size_t n, DeviceTraces& dt, hipStream_t st);
std::vector<uint8_t> prove_device(const ProvingKey& pk, DeviceTraces& dt, const ProveOptions& opt,
                                  StageTimes* times);

// The split MachineProver surface (crates/stark/src/prover.rs:209-236 commit, :242-553 open).
// MainData is ShardMainData (types.rs:13-18) kept in HBM: the traces' evaluations, the
// committed LDEs and their Merkle tree, alive from commit until the owner frees it.
// BFZ_HOST_TRACE=1: prints the host time (us since the proof started) with a label
void host_mark(const char* what);
// A buffer for the next proof's bytes (a returned one when available) / hand one back.
std::vector<uint8_t> acquire_proof_buffer();
void release_proof_buffer(std::vector<uint8_t>&& v);

struct MainData {
  DeviceTraces dt;
  std::vector<int> order;   // dt index of the k-th committed matrix
  std::vector<int> chip;    // chip of the k-th committed matrix, sorted (Reverse(height), name)
  std::vector<size_t> hn;   // its height
  Round mainr;              // the main commit (LDEs + tree)
  bool root_on_host = true; // mainr.tree.root filled (false: on the device only, prove_device)
};
void commit_main(MainData& md);  // md.dt holds the traces
// Challenger state after pk.observe_into (prover.rs:595-601) on a fresh DuplexChallenger.
Challenger challenger_after_pk(const ProvingKey& pk);
// ch = the prover's challenger after pk.observe_into.  *after (optional) receives the state at
// the end of the opening (the trait's open advances its &mut challenger; prove opens on a
// clone, prover.rs:578).  md may be opened more than once.
std::vector<uint8_t> open_main(const ProvingKey& pk, MainData& md, const Challenger& ch,
                               const ProveOptions& opt, Challenger* after = nullptr);

int num_queries_from_env();
bool observe_openings_from_env();  // BFZ_OBSERVE_OPENINGS = 1 (default) | 0

}  // namespace bfz
