// Device trace generation: the executor's events are uploaded once
// (compact, ~50 B per cycle) and every chip's main trace is filled on the device directly in
// the prover's layout (column-major, bit-reversed rows), together with the byte-lookup and
// program multiplicities of StarkMachine::generate_dependencies (machine.rs:228-248).
#pragma once
#include "gpu.h"
#include "machine.h"
#include "prover.h"

namespace bfz {

struct DeviceEvents {
  DBuf<CpuEvent> cpu;
  DBuf<AluEvent> alu;
  DBuf<JumpEvent> jump;
  DBuf<MemInstrEvent> meminstr;
  DBuf<IoEvent> io;
  DBuf<MemoryEvent> memory;
  DBuf<Instruction> prog;
  size_t n[NUM_CHIPS] = {};   // events per chip (Program: instructions, Byte: 0)
  size_t height[NUM_CHIPS] = {};
  bool included[NUM_CHIPS] = {};
  uint64_t global_clk = 0;
};

// Host -> HBM copy of the record's events (the proof's inputs).
void upload_events(const ExecutionRecord& rec, DeviceEvents& ev, hipStream_t st);

// The same from the pipeline executor's events (machine.h HostEvents; pinned host memory gives
// one DMA per event array).  Returns when the copies are done.
void upload_events(const HostEvents& h, const Program& prog, DeviceEvents& ev, hipStream_t st);
// Chip inclusion, heights and counts of ev from the event counts (the device buffers are set
// by the caller); builds the process-wide tables a proof of these heights reads (prepare_*).
void set_event_meta(DeviceEvents& ev, const EventCounts& n, uint64_t global_clk);
// Events that came from outside (bfz_record_from_events): the number of events a kernel must
// not read -- a cpu pc outside the program (k_trace_cpu / k_deps index by it), an opcode or
// memory-access kind out of range.  Counted on the device after the upload.
size_t count_invalid_events(const DeviceEvents& ev, hipStream_t st);
// The record's event vectors from the compact per-cycle form (bfz_record_from_cycles): d holds
// n cycles in HBM, ev.prog the program (uploaded by the caller).  Fills ev.cpu, ev.alu, ev.jump,
// ev.meminstr, ev.io on the device (chip events in cycle order, as the executor pushes them) and
// returns their counts in n_out (cpu, alu, jump, meminstr, io); *invalid = cycles that are not
// a reference record's (pc outside the program, a memory step with an access, a previous
// timestamp at or after the cycle's own, a prev_value outside an Input, nonzero padding).  The
// kernels never index the program with an out-of-range pc.
void expand_cycles(const Cycle* d, size_t n, DeviceEvents& ev, EventCounts& n_out, size_t* invalid,
                   hipStream_t st);
// Pinned host memory for HostEvents (hipHostMalloc / hipHostFree).
void* pinned_alloc(size_t bytes);
void pinned_free(void* p);

// generate_dependencies + generate_traces on the device, into dt (replaces its contents).
void generate_traces_device(const DeviceEvents& ev, DeviceTraces& dt, hipStream_t st);

// Device trace generation + prove_device; with timing, StageTimes::trace covers the former.
std::vector<uint8_t> prove_events(const ProvingKey& pk, const DeviceEvents& ev,
                                  const ProveOptions& opt, StageTimes* times);

}  // namespace bfz
