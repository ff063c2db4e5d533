// Brainfuck machine: program, executor, execution record, chip traces.
// Host-side C++ mirror of crates/core/executor (parser, interpreter, events) and of the
// per-chip generate_trace / generate_dependencies of crates/core/machine.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace bfz {

enum Opcode : uint8_t {
  OP_LOOP_START = 0, OP_LOOP_END = 1, OP_ADD = 2, OP_SUB = 3,
  OP_MEM_FWD = 4, OP_MEM_BWD = 5, OP_INPUT = 6, OP_OUTPUT = 7,
};

struct Instruction {
  uint8_t opcode;
  uint32_t op_a;
};

struct Program {
  std::vector<Instruction> instructions;
  // Program::from (crates/core/executor/src/program.rs:22-45). Throws on bad input.
  static Program parse(const std::string& code);
};

struct MemAccess {  // MemoryRecordEnum (events/memory.rs:31-79); kind 0 = none
  uint8_t kind = 0;  // 1 = Read, 2 = Write
  uint8_t value = 0, prev_value = 0;
  uint32_t ts = 0, prev_ts = 0;
};
struct CpuEvent {
  uint32_t clk, pc, next_pc, mp, next_mp;
  uint8_t mv, next_mv;
  MemAccess mv_access, next_mv_access;
};
struct AluEvent { uint32_t pc; uint8_t opcode, next_mv, mv; };
struct JumpEvent { uint32_t pc, next_pc; uint8_t opcode; uint32_t dst; uint8_t mv; };
struct MemInstrEvent { uint32_t clk, pc; uint8_t opcode; uint32_t mp, next_mp; };
struct IoEvent { uint32_t pc; uint8_t opcode; uint32_t mp; uint8_t mv; };
struct MemoryEvent { uint32_t addr, init_ts, final_ts; uint8_t init_v, final_v; };
// One executed cycle in the compact hand-over form (include/bfz.h bfz_cycle): every other field
// of the CpuEvent and every chip event of the cycle follow from these, the next cycle and the
// program (executor.rs:108-129,196-239); tracegen.hip expand_cycles rebuilds them on the device.
struct Cycle {
  uint32_t pc, mp, prev_ts;  // pc, mp, mv_access.prev_timestamp (0 without an access)
  uint8_t mv, prev_value;    // mv; Input: the cell's value before the write
  uint8_t pad[2];
};

struct ExecutionRecord {
  const Program* program = nullptr;
  std::vector<CpuEvent> cpu;
  std::vector<AluEvent> alu;
  std::vector<JumpEvent> jump;
  std::vector<MemInstrEvent> meminstr;
  std::vector<IoEvent> io;
  std::vector<MemoryEvent> memory;  // NORMAL FORM: sorted by address
  std::vector<uint64_t> u8_mult, u16_mult;  // byte-lookup multiplicities
  std::vector<uint8_t> output;
  uint64_t global_clk = 0;
  uint32_t pc = 0, mp = 0;
};

// Executor::run (crates/core/executor/src/executor.rs:71-326). Throws on missing input.
void execute(const Program& prog, const uint8_t* in, size_t nin, ExecutionRecord& rec);
// StarkMachine::generate_dependencies (crates/stark/src/machine.rs:228-248)
void generate_dependencies(ExecutionRecord& rec);

// The prover pipeline's executor: the same events as execute(), written into growable arrays
// whose memory the caller chooses (pinned host memory, so the upload to HBM is one DMA per array
// with no staging), memory cells in a dense offset-indexed array reused across runs, and the
// memory events emitted in address order from the final cells (the normal form) with no sort.
// Reused across runs, a HostEvents stops allocating once it has seen the largest run.
struct HostEvents {
  using AllocFn = void* (*)(size_t);
  using FreeFn = void (*)(void*);
  template <class T>
  struct Arr {
    T* p = nullptr;
    size_t n = 0, cap = 0;
  };
  AllocFn alloc = nullptr;  // malloc / free when null
  FreeFn dealloc = nullptr;
  Arr<CpuEvent> cpu;
  Arr<AluEvent> alu;
  Arr<JumpEvent> jump;
  Arr<MemInstrEvent> meminstr;
  Arr<IoEvent> io;
  Arr<MemoryEvent> memory;
  std::vector<uint8_t> output;
  uint64_t global_clk = 0;
  uint32_t pc = 0, mp = 0;
  struct Cell {
    uint32_t ts;
    uint8_t value, touched;
  };
  std::vector<Cell> cells;  // cells[off - cell_lo] for memory offset off (address = (u32)off)
  int64_t cell_lo = 0;
  HostEvents() = default;
  HostEvents(const HostEvents&) = delete;
  HostEvents& operator=(const HostEvents&) = delete;
  ~HostEvents();
  template <class T>
  void grow(Arr<T>& a, size_t need);
};
void execute_into(const Program& prog, const uint8_t* in, size_t nin, HostEvents& ev);

// Chips in machine order (crates/core/machine/src/brainfuck/mod.rs:53-81).
enum Chip : int {
  CHIP_CPU = 0, CHIP_PROGRAM, CHIP_ADDSUB, CHIP_JUMP, CHIP_MEMORY, CHIP_BYTE,
  CHIP_MEMINSTRS, CHIP_IO, NUM_CHIPS
};
struct ChipInfo {
  const char* name;
  int main_w, prep_w;
  bool local_only;
  int n_interactions;
};
extern const ChipInfo CHIP_INFO[NUM_CHIPS];
inline int perm_width(int chip) {  // permutation_trace_width (permutation.rs:15-21), in EF
  int n = CHIP_INFO[chip].n_interactions;
  return n ? (n + 1) / 2 + 1 : 0;
}

// What chip inclusion and main-trace heights depend on: the event count of each kind.
struct EventCounts {
  size_t cpu = 0, alu = 0, jump = 0, meminstr = 0, io = 0, memory = 0, program = 0;
};
EventCounts counts_of(const ExecutionRecord& rec);
EventCounts counts_of(const HostEvents& ev, const Program& prog);
bool chip_included(int chip, const EventCounts& n);
size_t main_trace_height(int chip, const EventCounts& n);

bool chip_included(int chip, const ExecutionRecord& rec);
// Row-major main trace in Montgomery form; returns height.
size_t main_trace(int chip, const ExecutionRecord& rec, std::vector<uint32_t>& out);
size_t main_trace_height(int chip, const ExecutionRecord& rec);
// Preprocessed trace (Program, Byte); returns 0 for chips without one.
size_t prep_trace(int chip, const Program& prog, std::vector<uint32_t>& out);

}  // namespace bfz
