/*
 * bfz — C ABI of the MI355X core-proof prover for the felicityin/zkvm-brainfuck zkVM.
 *
 * This is the drop-in boundary.  Each entry point replaces one reference interface
 * (paths relative to the reference repository):
 *
 *   bfz_execute      ProverClient::execute().run()        crates/sdk/src/lib.rs:57-59,
 *                    -> BfProver::execute                 crates/prover/src/lib.rs:60-65
 *   bfz_setup        ProverClient::setup / MachineProver::setup
 *                                                         crates/sdk/src/lib.rs:133-135,
 *                                                         crates/stark/src/prover.rs:49,197,
 *                                                         crates/stark/src/machine.rs:154-224
 *   bfz_prove        ProverClient::prove().run() / MachineProver::prove
 *                                                         crates/sdk/src/action.rs:58-61,
 *                                                         crates/stark/src/prover.rs:112,560-582
 *   bfz_verify       ProverClient::verify / StarkMachine::verify
 *                                                         crates/sdk/src/lib.rs:110-116,
 *                                                         crates/stark/src/machine.rs:258-284
 *   bfz_commit       MachineProver::commit -> Pcs::commit (coset LDE + MerkleTreeMmcs)
 *                                                         crates/stark/src/prover.rs:209-236
 *   bfz_coset_lde    Radix2DitParallel::coset_lde_batch + bit_reverse_rows (inside
 *                    TwoAdicFriPcs::commit, called at prover.rs:227,334,411)
 *   bfz_poseidon2_permute  Poseidon2KoalaBear<16> (kb31_poseidon2.rs:35-50)
 *
 * Conventions: field elements are uint32_t in MONTGOMERY form (x * 2^32 mod p), i.e.
 * byte-identical to a Rust `[KoalaBear]` slice; matrices are row-major.  Every function
 * returns 0 on success and a negative status on failure (bfz_last_error() describes it);
 * the Rust wrapper panics on a non-zero status, matching the reference (which unwraps).
 * Calls are serialized internally (one mutex); one process drives ONE GPU: bfz_init binds
 * the device on first use and fails if a later call names another one.  The stream,
 * allocator pool, twiddle/selector caches and pinned staging are process-wide, so ranks are
 * separate processes (one per GPU), never threads of one process -- the sharded entry points
 * hold the mutex while they run the caller's collective callbacks.
 * Proofs are byte strings in the BFZ1 normal form described in DESIGN.md.
 */
#ifndef BFZ_H
#define BFZ_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct bfz_pk bfz_pk;         /* device-resident proving key (DeviceProvingKey) */
typedef struct bfz_record bfz_record; /* executed record with traces resident in HBM  */
/* ShardMainData<SC, DeviceMatrix, DeviceProverData> (crates/stark/src/types.rs:13-18): the main
 * traces' evaluations, their coset LDEs and Merkle tree, resident in HBM from bfz_main_commit
 * until bfz_main_data_free. */
typedef struct bfz_main_data bfz_main_data;
/* p3 DuplexChallenger<KoalaBear, Poseidon2KoalaBear<16>, 16, 8> (kb31_poseidon2.rs:31) as plain
 * data, words in Montgomery form (the in-memory MontyField31 value): sponge_state, then
 * input_buffer[0..n_input) and output_buffer[0..n_output) exactly as the Rust Vecs hold them
 * (samples pop from the end of output_buffer). */
typedef struct {
  uint32_t sponge_state[16];
  uint32_t input_buffer[8];
  uint32_t n_input;
  uint32_t output_buffer[8];
  uint32_t n_output;
} bfz_challenger;

typedef struct {
  double trace_ms, main_commit_ms, perm_ms, quotient_ms, open_ms, fri_ms, total_ms;
  double lde_ms, lde_bytes; /* whole coset LDEs: 12*n*w algorithmic bytes per call */
  int lde_calls;
  double ntt_kernel_ms, ntt_kernel_bytes; /* NTT pass kernel, per-launch events, 8 B/element */
  int ntt_kernel_launches;
  double p2_kernel_ms, p2_perms; /* Poseidon2 leaf/compress kernels: time and permutations */
  int p2_launches;
  double lde_elem_stages; /* radix-2 element-stages of the coset LDEs: 3*n*log2(n)*w per call */
  /* Openings (k_open_partial_batch: 4*n*w + 16*n*points B per matrix, the low coset) and reduced
   * openings (k_reduce: 4*H*w + 16*H*(2 or 3) B per LDE height): per-launch events, algorithmic
   * bytes. */
  double open_kernel_ms, open_kernel_bytes;
  int open_kernel_launches;
  double reduce_kernel_ms, reduce_kernel_bytes;
  int reduce_kernel_launches;
  /* The LogUp stage (perm_ms, prover.rs:280-334) in parts: permutation rows + cumulative-sum scan
   * (replicated on every rank of a sharded proof), iDFT of the permutation columns (replicated;
   * 0 unsharded), fold + forward DFT (this rank's residue and its next-residue shards when
   * sharded; the whole coset LDE unsharded), Merkle hashing (split). */
  double perm_rows_ms, perm_idft_ms, perm_dft_ms, perm_hash_ms;
  /* The main commit (main_commit_ms, prover.rs:209-236) in the same parts: iDFT of the main
   * columns (replicated when sharded; 0 unsharded), fold + forward DFT, Merkle hashing. */
  double main_idft_ms, main_dft_ms, main_hash_ms;
  /* Base-field cells (sum of height x width) of the main and permutation traces. */
  double main_cells, perm_cells;
} bfz_timings;

/* Binds the process to `device` and looks up every kernel a proof launches (code objects and
 * launch objects, ~5 ms), so none of that runs between the first proof's launches. */
int bfz_init(int device);
const char* bfz_last_error(void);
/* Hash of the sources the library was built from (bfz/srchash.py); bfz/_lib.py refuses a
 * library whose hash differs from the sources beside it. */
const char* bfz_build_id(void);
int bfz_device_name(char* buf, size_t cap);
void bfz_free(void* p);
int bfz_synchronize(void); /* hipDeviceSynchronize on the bound device */
/* Host-only self-tests of the boundary's own bookkeeping (no device needed): "emit_rollback" =
 * a batch hand-over that fails part-way releases the proofs already handed out. 0 = passed. */
int bfz_selftest(const char* name);

int bfz_execute(const char* elf, const uint8_t* stdin_data, size_t nin, uint8_t* out,
                size_t out_cap, size_t* out_len, uint64_t* cycles);

/* MachineProver::generate_traces (crates/stark/src/prover.rs:58-81) after
 * generate_dependencies (machine.rs:228-248): row-major Montgomery trace of one chip
 * (chip index in BfAir::chips() order, brainfuck/mod.rs:53-81; prep != 0 selects the
 * preprocessed trace).  *out is malloc'd (bfz_free).  Returns 1 if the chip is not
 * included in the record. */
int bfz_trace(const char* elf, const uint8_t* stdin_data, size_t nin, int chip, int prep,
              uint32_t** out, size_t* height, size_t* width);

/* Diagnostic: the executor's event stream (Executor::run + emit_events, crates/core/executor/src/
 * executor.rs:71-326) serialized field by field: executor 0 = the record executor (bfz_trace,
 * oracle-checked traces), 1 = the prover pipeline's executor (bfz_record_new, bfz_prove,
 * bfz_prove_batch).  Host only; *out is malloc'd (bfz_free). */
int bfz_execute_events(const char* elf, const uint8_t* stdin_data, size_t nin, int executor,
                       uint8_t** out, size_t* out_len);

/* generate_permutation_trace (crates/stark/src/permutation.rs:75-148, called at
 * prover.rs:280-296) of one chip on the device: main (and, for Program/Byte, prep) are
 * row-major Montgomery traces of `height` rows, alpha/beta the LogUp challenges (EF,
 * Montgomery).  *out (malloc'd, bfz_free) = the permutation trace flattened to base
 * (flatten_to_base, prover.rs:318-334), row-major height x *width; cumsum = its last row's
 * running sum.  Diagnostic entry (the prover keeps the trace in HBM). */
int bfz_perm_trace(int chip, const uint32_t* main, const uint32_t* prep, size_t height,
                   const uint32_t alpha[4], const uint32_t beta[4], uint32_t** out, size_t* width,
                   uint32_t cumsum[4]);

/* Same trace generated on the device from the uploaded events (the prover's own path),
 * returned row-major in natural row order for comparison. */
int bfz_trace_device(const char* elf, const uint8_t* stdin_data, size_t nin, int chip,
                     uint32_t** out, size_t* height, size_t* width);

/* The preprocessed commit is made once per program text and cached (16 most recent programs):
 * a repeated setup of the same ELF returns a handle to the same device-resident key. */
int bfz_setup(const char* elf, bfz_pk** pk, uint32_t vk_commit[8]);
void bfz_pk_free(bfz_pk* pk);

/* MachineProver::pk_to_device (crates/stark/src/prover.rs:52,201-203): the device key of a
 * StarkProvingKey kept on the host.  BfProver::setup keeps only pk_to_host(pk)
 * (crates/prover/src/lib.rs:51) and BfProver::prove rebuilds the device key from it on every
 * proof (:76).  Arguments are the key's preprocessed traces (StarkProvingKey::traces,
 * machine.rs:49-60, in the key's order): chips[i] the chip id (BfAir::chips() order) of
 * traces[i], a row-major Montgomery heights[i] x widths[i] matrix, and the key's commit.
 * The program is recovered from the Program chip's preprocessed trace (pc, opcode, op_a bytes;
 * program/mod.rs:66-94); both traces must be exactly that program's (machine.rs:154-224), and
 * the device commitment of them must equal commit, or the call fails.  The device key is the
 * per-program setup cache's (a cache hit costs the trace comparison only). */
int bfz_pk_from_host(const int* chips, const uint32_t* const* traces, const size_t* heights,
                     const size_t* widths, size_t n, const uint32_t commit[8], bfz_pk** pk);
/* The preprocessed commitment of a device key (StarkProvingKey::commit / vk.commit). */
int bfz_pk_commit(const bfz_pk* pk, uint32_t commit[8]);

/* The split MachineProver surface, for a Rust HipProver:
 *   bfz_main_commit         MachineProver::commit (crates/stark/src/prover.rs:209-236): host
 *                           row-major main traces (as bfz_prove_traces) -> LDE + MerkleTreeMmcs
 *                           commit in HBM; root = main_commit (8 Montgomery words, as vk_commit).
 *                           pk may be NULL (the trait's commit takes no key); if given, bfz_open
 *                           refuses the data for any other key.
 *   bfz_record_main_commit  the same from a device-resident record (traces generated on device).
 *   bfz_challenger_observe_pk  MachineProvingKey::observe_into (prover.rs:595-601).
 *   bfz_open                MachineProver::open (prover.rs:242-553) on the challenger state
 *                           after observe_into.  Like the trait method (which takes the
 *                           challenger &mut), ch is advanced: on success it holds the state
 *                           after the whole opening (PCS open, FRI commit phase, grind, query
 *                           sampling).  MachineProver::prove opens on a clone (prover.rs:578):
 *                           pass a copy to keep the caller's state.  Output = the same BFZ1
 *                           proof bfz_prove* returns.  The main data stays valid (it may be
 *                           opened again).
 *   bfz_main_data_free      drops ShardMainData (frees its HBM). */
int bfz_main_commit(const bfz_pk* pk, const int* chips, const uint32_t* const* traces,
                    const size_t* heights, const size_t* widths, size_t nchips, bfz_main_data** out,
                    uint32_t root[8]);
int bfz_record_main_commit(const bfz_pk* pk, const bfz_record* rec, bfz_main_data** out,
                           uint32_t root[8]);
int bfz_challenger_observe_pk(const bfz_pk* pk, bfz_challenger* ch);
int bfz_open(const bfz_pk* pk, bfz_main_data* data, bfz_challenger* ch, uint8_t** proof,
             size_t* proof_len);
void bfz_main_data_free(bfz_main_data* data);

int bfz_prove(const bfz_pk* pk, const uint8_t* stdin_data, size_t nin, uint8_t** proof,
              size_t* proof_len);
/* MachineProver::prove from host traces (crates/stark/src/prover.rs:560-582 after
 * generate_dependencies + generate_traces, prover.rs:58-81): chips[i] is the chip index in
 * BfAir::chips() order, traces[i] its row-major Montgomery main trace (heights[i] x
 * widths[i], height a power of two).  Preprocessed traces come from the proving key. */
int bfz_prove_traces(const bfz_pk* pk, const int* chips, const uint32_t* const* traces,
                     const size_t* heights, const size_t* widths, size_t nchips, uint8_t** proof,
                     size_t* proof_len);
int bfz_verify(const char* elf, const uint32_t vk_commit[8], const uint8_t* proof,
               size_t proof_len);

/* Pipelined proofs of one program over many inputs (the reference's execute-then-prove loop,
 * crates/core/machine/src/utils/prove.rs:23-66, with execution off the critical path):
 * exec_threads host threads run the executor into pinned memory, a copy stream uploads job
 * k+1's events while the GPU proves job k.  proofs[i] (malloc'd, bfz_free) is byte-identical to
 * bfz_prove(pk, stdins[i]).  exec_threads <= 0: environment BFZ_EXEC_THREADS or 3.
 * stats (optional): wall time of the batch and per-stage sums over jobs. */
typedef struct {
  double wall_ms, exec_ms, upload_ms, prove_ms;
  int exec_threads;
} bfz_batch_stats;
int bfz_prove_batch(const bfz_pk* pk, const uint8_t* const* stdins, const size_t* nins,
                    size_t njobs, int exec_threads, uint8_t** proofs, size_t* proof_lens,
                    bfz_batch_stats* stats);

/* Split prove: bfz_record_new executes the program and copies its events to HBM (the
 * proof's inputs); bfz_record_prove generates every chip trace on the device
 * (generate_dependencies + generate_traces, prover.rs:58-81) and proves. */
int bfz_record_new(const bfz_pk* pk, const uint8_t* stdin_data, size_t nin, bfz_record** rec,
                   uint64_t* cycles);
int bfz_record_prove(const bfz_pk* pk, const bfz_record* rec, uint8_t** proof, size_t* proof_len,
                     bfz_timings* timings);
void bfz_record_free(bfz_record* rec);

/* The reference's ExecutionRecord (crates/core/executor/src/record.rs:15-34) as plain arrays,
 * one C struct per event type of crates/core/executor/src/events (explicit padding, no
 * compiler-inserted gaps; opcodes are the Opcode discriminants of opcode.rs:13-30).
 * bfz_memory_access is Option<MemoryRecordEnum> (events/memory.rs:31-79): kind 0 = None,
 * 1 = Read (prev_value unused), 2 = Write. */
typedef struct {
  uint8_t kind, value, prev_value, _pad;
  uint32_t timestamp, prev_timestamp;
} bfz_memory_access;
typedef struct { /* CpuEvent, events/cpu.rs */
  uint32_t clk, pc, next_pc, mp, next_mp;
  uint8_t mv, next_mv, _pad[2];
  bfz_memory_access mv_access, next_mv_access;
} bfz_cpu_event;
typedef struct { /* AluEvent, events/instr.rs */
  uint32_t pc;
  uint8_t opcode, next_mv, mv, _pad;
} bfz_alu_event;
typedef struct { /* JumpEvent */
  uint32_t pc, next_pc;
  uint8_t opcode, _pad[3];
  uint32_t dst;
  uint8_t mv, _pad2[3];
} bfz_jump_event;
typedef struct { /* MemInstrEvent */
  uint32_t clk, pc;
  uint8_t opcode, _pad[3];
  uint32_t mp, next_mp;
} bfz_mem_instr_event;
typedef struct { /* IoEvent */
  uint32_t pc;
  uint8_t opcode, _pad[3];
  uint32_t mp;
  uint8_t mv, _pad2[3];
} bfz_io_event;
typedef struct { /* MemoryEvent: addr, initial_mem_access, final_mem_access (events/memory.rs:6-13) */
  uint32_t addr, initial_timestamp, final_timestamp;
  uint8_t initial_value, final_value, _pad[2];
} bfz_memory_event;
typedef struct {
  const bfz_cpu_event* cpu;                 size_t n_cpu;          /* cpu_events */
  const bfz_alu_event* add;                 size_t n_add;          /* add_events */
  const bfz_alu_event* sub;                 size_t n_sub;          /* sub_events */
  const bfz_jump_event* jump;               size_t n_jump;         /* jump_events */
  const bfz_io_event* io;                   size_t n_io;           /* io_events */
  const bfz_mem_instr_event* memory_instr;  size_t n_memory_instr; /* memory_instr_events */
  const bfz_memory_event* memory;           size_t n_memory;       /* cpu_memory_access */
} bfz_events;
/* A device record from the reference's own events (the record utils::prove hands to
 * MachineProver::prove, crates/core/machine/src/utils/prove.rs:38-44): the arrays go to HBM
 * (add_events then sub_events as one AddSub stream, alu/mod.rs:72), the memory events are put
 * in the normal form (sorted by address; the reference drains a HashMap, executor.rs:74), and
 * bfz_record_prove / bfz_record_main_commit then generate every chip trace and the byte-lookup
 * multiplicities on the device (generate_dependencies + generate_traces, prover.rs:58-81,
 * machine.rs:228-248).  The program is pk's.  Events are validated (pc inside the program,
 * opcodes, access kinds, unique memory addresses, at least one cycle) before any kernel reads
 * them.  Host pointers (pageable is fine). */
int bfz_record_from_events(const bfz_pk* pk, const bfz_events* events, bfz_record** rec);

/* The same record from a compact hand-over: one 16-byte bfz_cycle per CpuEvent (in
 * record.cpu_events order) plus cpu_memory_access.  Everything else in the record is a function
 * of these and the program: clk = 2 i (executor.rs:131), next_pc / next_mp = the next cycle's pc
 * / mp (the last cycle's next_pc is the program length, its next_mp follows its opcode),
 * next_mv and both access records follow the opcode (executor.rs:140-205: the read at clk + 1,
 * the ALU write at clk + 2), and every add/jump/memory_instr/io event is the cycle's own fields
 * (emit_events, executor.rs:196-239) -- so the device rebuilds them (tracegen.hip
 * expand_cycles) instead of receiving ~64 B per cycle.  Cycles that no reference record holds
 * (pc outside the program, an access on a memory step, prev_timestamp >= clk + 1, prev_value
 * outside an Input, nonzero padding, a successor pc / mp the executor would not step to, a last
 * cycle that does not leave the program) are refused before any trace kernel runs. */
typedef struct {
  uint32_t pc;         /* CpuEvent::pc */
  uint32_t mp;         /* CpuEvent::mp */
  uint32_t prev_ts;    /* mv_access's prev_timestamp; 0 when mv_access is None (memory steps) */
  uint8_t mv;          /* CpuEvent::mv */
  uint8_t prev_value;  /* Input (mv_access is a Write): its prev_value; 0 otherwise */
  uint8_t _pad[2];
} bfz_cycle;
int bfz_record_from_cycles(const bfz_pk* pk, const bfz_cycle* cycles, size_t n_cycles,
                           const bfz_memory_event* memory, size_t n_memory, bfz_record** rec);

/* The same hand-over in chunks, so the host conversion of record.cpu_events overlaps the DMA:
 * bfz_cycles_begin announces n_cycles; each bfz_cycles_push queues one converted chunk
 * (cycles[first, first + n)) on a copy stream and returns at once -- from page-locked
 * (bfz_host_alloc) memory the copy is a DMA that runs while the caller converts the next chunk,
 * and the chunk must then stay unchanged until bfz_cycles_finish returns; chunks may come from
 * several threads, in any order.  bfz_cycles_finish checks that every cycle was pushed exactly
 * once, then validates and expands them exactly as bfz_record_from_cycles (same record, same
 * proof) and consumes the handle, also on error; bfz_cycles_abort drops an unfinished one.
 * Replaces the single-array call of HipProver::prove (crates/bf-hip-prover) with a pipelined
 * CycleArrays::new; the reference hands the record over in memory (utils/prove.rs:44-46). */
typedef struct bfz_cycle_upload bfz_cycle_upload;
int bfz_cycles_begin(const bfz_pk* pk, size_t n_cycles, bfz_cycle_upload** up);
int bfz_cycles_push(bfz_cycle_upload* up, size_t first, const bfz_cycle* cycles, size_t n);
int bfz_cycles_finish(bfz_cycle_upload* up, const bfz_memory_event* memory, size_t n_memory,
                      bfz_record** rec);
void bfz_cycles_abort(bfz_cycle_upload* up);

/* Page-locked host memory for the hand-over arrays (the Rust CycleArrays builds its bfz_cycle
 * vector in it): bfz_record_from_cycles / bfz_record_from_events then DMA straight from the
 * caller's array instead of staging it through the library's pinned chunks (PCIe-bound: ~60 GB/s
 * against ~35-40 GB/s staged).  Any host memory is still accepted; this only makes the upload
 * faster.  Pairs with bfz_host_free (not bfz_free); freed blocks are kept page-locked for reuse
 * (up to 8 GiB), so a per-proof allocation of the same size does not pin memory again.  Host-side replacement of the reference's
 * Vec allocation in ExecutionRecord hand-off (crates/core/machine/src/utils/prove.rs:44-46). */
int bfz_host_alloc(size_t bytes, void** out);
void bfz_host_free(void* p);

/* One proof sharded over `world` GPUs (one process per GPU, every rank calls this with the
 * same record): each rank computes its residue-class row shard of every large LDE, hashes its
 * subtree of every large Merkle tree, evaluates the quotient at its points and computes its
 * slice of the openings, reduced openings and large FRI rounds (the commits, quotient and
 * open of crates/stark/src/prover.rs:209-236,344-470); the ranks exchange subtree roots,
 * quotient values, opened-value slices, one FRI layer and the query openings through the
 * callbacks (torch.distributed / RCCL on the host side).  Every rank returns the same proof,
 * byte-identical to bfz_record_prove's.  The
 * callbacks return 0 on success.  Their buffers (send / recv / data) are DEVICE pointers on the
 * rank's GPU: ncclAllGather / ncclAllReduce run on them directly.  When a callback is entered the
 * send data is complete; the library's stream is drained first except at the two quotient
 * all-gathers, where later GPU work is already queued to run beside the collective (a callback
 * that synchronizes the whole device waits for that work too, which is correct).  The received
 * data must be in place when the callback returns. */
typedef int (*bfz_allgather_fn)(void* ctx, const void* send, size_t bytes, void* recv);
typedef int (*bfz_allreduce_u32_fn)(void* ctx, uint32_t* data, size_t n);
/* `count` proofs of one record back to back with `inflight` (1..4) of them in flight, each on
 * its own stream, pool and pinned mailboxes ("lane", one host thread each): one proof's
 * latency-bound launches (Merkle tree tops, the FRI tail, the transcript steps) then run beside
 * the other's bulk hashing.  Every proof must be byte-identical to the first (an error
 * otherwise); *proof receives the first; wall_ms (optional) the whole run.  The steady-state
 * throughput of the bfz_record_prove loop; the reference proves one shard at a time
 * (utils/prove.rs:38-66). */
int bfz_record_prove_repeat(const bfz_pk* pk, const bfz_record* rec, int count, int inflight,
                            uint8_t** proof, size_t* len, double* wall_ms);

int bfz_record_prove_sharded(const bfz_pk* pk, const bfz_record* rec, int rank, int world,
                             bfz_allgather_fn allgather, bfz_allreduce_u32_fn allreduce_sum,
                             void* ctx, uint8_t** proof, size_t* proof_len, bfz_timings* timings);

/* Timing of ONE rank's share of a world-rank sharded proof, run alone on this GPU: the same
 * kernels and sizes bfz_record_prove_sharded runs on rank `rank`, with every exchange a no-op
 * (receive buffers keep whatever they hold, so the result is not a proof and is discarded;
 * the FRI final-constant check is skipped).  Stage times and kernel counters go to *timings;
 * timings == NULL runs the share without stage events or per-launch kernel probes (the caller
 * times it on the wall clock, as the single-GPU headline is timed).  Predicts the per-rank
 * critical path of an N-GPU proof without N GPUs. */
int bfz_record_prove_shard_solo(const bfz_pk* pk, const bfz_record* rec, int rank, int world,
                                bfz_timings* timings);

/* The collectives of the last bfz_record_prove_shard_solo run, in call order: kinds[i] = 0 for an
 * all-gather (bytes[i] = this rank's contribution; it receives world - 1 times that), 1 for a sum
 * all-reduce of u32 words (bytes[i] = the vector's size).  *n = the number of collectives; at most
 * cap entries are written.  Feeds bench.py's collective-time model of the N-GPU curve; the
 * reference has no multi-GPU prover. */
int bfz_shard_solo_exchanges(int* kinds, uint64_t* bytes, size_t cap, size_t* n);

/* For the same collectives: ms[i] = GPU milliseconds of the work this rank has queued to run
 * while collective i is in flight (the sharded prover issues the quotient exchange in two
 * all-gathers, each after the work it overlaps is queued), 0 where nothing overlaps.  Measured
 * only by a bfz_record_prove_shard_solo run WITH timings (0 otherwise).  bench.py's collective
 * model charges max(0, collective time - ms[i]). */
int bfz_shard_solo_overlaps(double* ms, size_t cap, size_t* n);

/* Device memory held by proof lane `lane`'s buffer pool (0..3, the lanes of
 * bfz_record_prove_repeat / bfz_prove_batch; 0 = the default
 * lane): every buffer a proof on that lane allocated, in use or cached for the next proof -- the
 * resident set of one proof in flight (bench.py reports it beside the lanes' throughput).  The
 * process-wide device data -- twiddle, power and selector tables, proving keys, the records'
 * device events -- lives in a separate resident pool and is not included.  0 for a lane never
 * used. */
int bfz_device_pool_bytes(int lane, uint64_t* bytes);

/* Column-sharded PCS commit + FRI commit phase of a synthetic trace (BASELINE.json configs 4
 * and 5).  Replaces, for one n x (world * w_local) trace, TwoAdicFriPcs::commit
 * (crates/stark/src/prover.rs:209-236: coset LDE with shift GENERATOR, bit-reversed rows,
 * MerkleTreeMmcs) followed by the FRI commit phase of fri::prover (prover.rs:460-470) on the
 * batched column sum_c alpha^c col_c.  Rank r passes its columns [r w_local, (r+1) w_local) as a
 * DEVICE buffer d_cols (column-major, bit-reversed rows, Montgomery form, n = 2^log_n) and two
 * device exchange buffers of 2n * w_local words; alltoall(ctx) must exchange equal blocks of
 * d_send into d_recv (block j to rank j, e.g. ncclAllToAll / torch all_to_all_single), and
 * allgather is as above.  out receives [root (8) | FRI roots (8 per round) | final value (4)]
 * (*nwords words, identical on every rank and to world = 1).  cap = capacity of out in words.
 * As above, the allgather buffers are device pointers. */
typedef int (*bfz_alltoall_fn)(void* ctx);
int bfz_commit_fri_sharded(const uint32_t* d_cols, int log_n, size_t w_local, int rank, int world,
                           uint32_t* d_send, uint32_t* d_recv, bfz_alltoall_fn alltoall,
                           bfz_allgather_fn allgather, void* ctx, uint32_t* out, size_t cap,
                           size_t* nwords);

/* FRI_QUERIES (kb31_poseidon2.rs:59-62): 1..4096, or 0 = environment FRI_QUERIES / 84. */
int bfz_set_num_queries(int num_queries);

/* PCS transcript variant, decision D1 of DESIGN.md §2 ([p3-recalled] TwoAdicFriPcs::open at
 * zkMIPS/Plonky3 93967fce): 1 = every opened value is observed before the FRI batching
 * challenge alpha is sampled (default), 0 = alpha is sampled first; -1 = environment
 * BFZ_OBSERVE_OPENINGS.  Applies to bfz_prove*, bfz_verify*, identically in the oracle. */
int bfz_set_pcs_variant(int observe_openings);

/* Test-only fault injection, no reference counterpart: bit 0 perturbs the device challenger's
 * uploaded sponge state, so the host's replay of the device-sampled challenges must fail the
 * proof with "device transcript diverged" (tests/test_gpu.py).  0 (default) = off. */
int bfz_set_fault_injection(int mask);

/* Proof wire format.  bfz_prove* return the BFZ1 normal form; bfz_proof_to_bincode turns it
 * into the reference's bytes: bincode::serialize(&MachineProof<KoalaBearPoseidon2>)
 * (crates/core/machine/src/utils/prove.rs:46), i.e. ShardProof (crates/stark/src/types.rs:66-73)
 * with bincode 1.x default options, chip_ordering entries in proof order.  field_repr selects
 * how a KoalaBear word is serialized: 0 = Montgomery word (p3 MontyField31 serde, default,
 * [p3-recalled]), 1 = canonical value.  bfz_proof_from_bincode is the inverse;
 * bfz_verify_bincode verifies the bincode bytes directly.  *out is malloc'd (bfz_free). */
int bfz_proof_to_bincode(const uint8_t* proof, size_t len, int field_repr, uint8_t** out,
                         size_t* out_len);
int bfz_proof_from_bincode(const uint8_t* bytes, size_t len, int field_repr, uint8_t** out,
                           size_t* out_len);
int bfz_verify_bincode(const char* elf, const uint32_t vk_commit[8], const uint8_t* bytes,
                       size_t len, int field_repr);

int bfz_coset_lde(const uint32_t* evals, size_t n, size_t w, uint32_t shift, uint32_t* lde_out);
int bfz_commit(const uint32_t* const* mats, const size_t* heights, const size_t* widths,
               size_t nmats, uint32_t root[8]);
int bfz_poseidon2_permute(uint32_t* states, size_t n);
/* The latency-optimised form used for small Merkle layers (16 lanes per state, DPP). */
int bfz_poseidon2_permute_small(uint32_t* states, size_t n);

#ifdef __cplusplus
}
#endif
#endif
