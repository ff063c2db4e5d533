// Brainfuck executor and chip trace generation (host C++).  See machine.h.
#include "machine.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <unordered_map>

#include "kb.h"

namespace bfz {

using kb::to_mont;

const ChipInfo CHIP_INFO[NUM_CHIPS] = {
    {"Cpu", 31, 0, false, 16},     {"Program", 1, 6, false, 1}, {"AddSub", 7, 0, true, 5},
    {"Jump", 45, 0, true, 1},      {"Memory", 12, 0, false, 4}, {"Byte", 2, 2, false, 2},
    {"MemoryInstrs", 41, 0, false, 1}, {"IO", 5, 0, true, 1},
};

Program Program::parse(const std::string& code) {
  Program p;
  std::vector<size_t> stack;
  for (char c : code) {
    switch (c) {
      case '>': p.instructions.push_back({OP_MEM_FWD, 0}); break;
      case '<': p.instructions.push_back({OP_MEM_BWD, 0}); break;
      case '+': p.instructions.push_back({OP_ADD, 0}); break;
      case '-': p.instructions.push_back({OP_SUB, 0}); break;
      case '.': p.instructions.push_back({OP_OUTPUT, 0}); break;
      case ',': p.instructions.push_back({OP_INPUT, 0}); break;
      case '[':
        p.instructions.push_back({OP_LOOP_START, 0});
        stack.push_back(p.instructions.size() - 1);
        break;
      case ']': {
        if (stack.empty()) throw std::runtime_error("unmatched ']'");
        size_t start = stack.back();
        stack.pop_back();
        p.instructions[start].op_a = (uint32_t)p.instructions.size();
        p.instructions.push_back({OP_LOOP_END, (uint32_t)(start + 1)});
        break;
      }
      case ' ': case '\n': case '\r': break;
      default: throw std::runtime_error(std::string("invalid program character '") + c + "'");
    }
  }
  return p;
}

namespace {
struct Cell { uint8_t value = 0; uint32_t ts = 0; int64_t ev = -1; };
struct Memory {
  std::vector<Cell> dense;  // addresses < 2^20
  std::unordered_map<uint32_t, Cell> sparse;
  Memory() : dense(1u << 20) {}
  Cell& at(uint32_t a) { return a < dense.size() ? dense[a] : sparse[a]; }
};
}  // namespace

void execute(const Program& prog, const uint8_t* in, size_t nin, ExecutionRecord& rec) {
  rec = ExecutionRecord();
  rec.program = &prog;
  if (prog.instructions.empty()) throw std::runtime_error("empty program");
  Memory mem;
  uint32_t pc = 0, mp = 0, clk = 0;
  size_t inptr = 0;
  uint64_t gclk = 0;
  // rr_traced / rw_traced (executor.rs:262-326)
  auto access = [&](uint32_t addr, uint32_t ts, bool write, uint8_t val) {
    Cell& c = mem.at(addr);
    MemAccess a;
    a.prev_value = c.value;
    a.prev_ts = c.ts;
    if (write) c.value = val;
    c.ts = ts;
    if (c.ev < 0) {
      c.ev = (int64_t)rec.memory.size();
      rec.memory.push_back({addr, a.prev_ts, 0, a.prev_value, 0});
    }
    rec.memory[c.ev].final_ts = c.ts;
    rec.memory[c.ev].final_v = c.value;
    a.kind = write ? 2 : 1;
    a.value = c.value;
    a.ts = c.ts;
    return a;
  };
  const size_t n = prog.instructions.size();
  for (;;) {
    const Instruction ins = prog.instructions[pc];
    uint32_t next_pc = pc + 1, jmp_dst = 0;
    uint8_t mv = 0, next_mv = 0;
    const uint32_t mp0 = mp;
    MemAccess a_mv, a_next;
    switch (ins.opcode) {
      case OP_MEM_FWD: mp = mp + 1; break;
      case OP_MEM_BWD: mp = mp - 1; break;
      case OP_ADD: case OP_SUB:
        a_mv = access(mp, clk + 1, false, 0);
        mv = a_mv.value;
        next_mv = ins.opcode == OP_ADD ? (uint8_t)(mv + 1) : (uint8_t)(mv - 1);
        a_next = access(mp, clk + 2, true, next_mv);
        break;
      case OP_LOOP_START: case OP_LOOP_END:
        a_mv = access(mp, clk + 1, false, 0);
        mv = a_mv.value;
        if (ins.opcode == OP_LOOP_START) next_pc = mv == 0 ? ins.op_a : pc + 1;
        else next_pc = mv != 0 ? ins.op_a : pc + 1;
        jmp_dst = next_pc;
        break;
      case OP_INPUT: {
        if (inptr >= nin) throw std::runtime_error("input stream exhausted");
        uint8_t v = in[inptr];  // the reference never advances input_stream_ptr
        a_mv = access(mp, clk + 1, true, v);
        mv = v;
        break;
      }
      case OP_OUTPUT:
        a_mv = access(mp, clk + 1, false, 0);
        mv = a_mv.value;
        rec.output.push_back(mv);
        break;
    }
    // emit_events (executor.rs:178-239)
    rec.cpu.push_back({clk, pc, next_pc, mp0, mp, mv, next_mv, a_mv, a_next});
    switch (ins.opcode) {
      case OP_ADD: case OP_SUB: rec.alu.push_back({pc, ins.opcode, next_mv, mv}); break;
      case OP_LOOP_START: case OP_LOOP_END:
        rec.jump.push_back({pc, next_pc, ins.opcode, jmp_dst, mv});
        break;
      case OP_MEM_FWD: case OP_MEM_BWD: rec.meminstr.push_back({clk, pc, ins.opcode, mp0, mp}); break;
      default: rec.io.push_back({pc, ins.opcode, mp0, mv}); break;
    }
    pc = next_pc;
    clk += 2;
    gclk++;
    if (pc == n) break;
  }
  std::sort(rec.memory.begin(), rec.memory.end(),
            [](const MemoryEvent& a, const MemoryEvent& b) { return a.addr < b.addr; });
  rec.global_clk = gclk;
  rec.pc = pc;
  rec.mp = mp;
}

// ---------------------------------------------------------------- pipeline executor
HostEvents::~HostEvents() {
  FreeFn f = dealloc ? dealloc : std::free;
  f(cpu.p);
  f(alu.p);
  f(jump.p);
  f(meminstr.p);
  f(io.p);
  f(memory.p);
}

template <class T>
void HostEvents::grow(Arr<T>& a, size_t need) {
  if (need <= a.cap) return;
  size_t cap = std::max<size_t>(a.cap ? a.cap : 1024, 1024);
  while (cap < need) cap *= 2;
  T* p = static_cast<T*>((alloc ? alloc : std::malloc)(cap * sizeof(T)));
  if (!p) throw std::runtime_error("executor: out of host memory");
  if (a.n) std::memcpy(p, a.p, a.n * sizeof(T));
  (dealloc ? dealloc : std::free)(a.p);
  a.p = p;
  a.cap = cap;
}

// Executor::run (crates/core/executor/src/executor.rs:71-326) with emit_events (:178-239) and
// rr_traced / rw_traced (:262-326) -- the same event stream as execute() above.
void execute_into(const Program& prog, const uint8_t* in, size_t nin, HostEvents& ev) {
  if (prog.instructions.empty()) throw std::runtime_error("empty program");
  ev.cpu.n = ev.alu.n = ev.jump.n = ev.meminstr.n = ev.io.n = ev.memory.n = 0;
  ev.output.clear();
  // memory cells: offsets [lo, hi) relative to address 0 (mp moves by one, so the cells a run
  // touches form one interval); the array is cleared here, sized by the previous run
  std::fill(ev.cells.begin(), ev.cells.end(), HostEvents::Cell{0, 0, 0});
  if (ev.cells.empty()) {
    ev.cells.assign(1 << 16, HostEvents::Cell{0, 0, 0});
    ev.cell_lo = -(1 << 12);
  }
  int64_t lo = ev.cell_lo, hi = lo + (int64_t)ev.cells.size();
  HostEvents::Cell* cells = ev.cells.data();
  const Instruction* code = prog.instructions.data();
  const uint32_t n = (uint32_t)prog.instructions.size();
  uint32_t pc = 0, clk = 0;
  int64_t off = 0;  // memory pointer as an unwrapped offset; mp = (u32)off
  uint64_t gclk = 0;
  auto ensure_cell = [&](int64_t o) {
    if (o >= lo && o < hi) return;
    const int64_t span = hi - lo;
    const int64_t nlo = o < lo ? std::min(o, lo - span) : lo;
    const int64_t nhi = o >= hi ? std::max(o + 1, hi + span) : hi;
    std::vector<HostEvents::Cell> nc((size_t)(nhi - nlo), HostEvents::Cell{0, 0, 0});
    std::memcpy(&nc[(size_t)(lo - nlo)], cells, (size_t)span * sizeof(HostEvents::Cell));
    ev.cells.swap(nc);
    lo = nlo;
    hi = nhi;
    cells = ev.cells.data();
  };
  ensure_cell(0);
  for (;;) {
    if (ev.cpu.n == ev.cpu.cap) {  // every cycle emits one Cpu event and at most one other
      const size_t want = ev.cpu.cap ? 2 * ev.cpu.cap : (size_t)1 << 16;
      ev.grow(ev.cpu, want);
      ev.grow(ev.alu, std::min(want, std::max(ev.alu.cap, ev.alu.n + want / 2)));
      ev.grow(ev.jump, std::min(want, std::max(ev.jump.cap, ev.jump.n + want / 2)));
      ev.grow(ev.meminstr, std::min(want, std::max(ev.meminstr.cap, ev.meminstr.n + want / 2)));
      ev.grow(ev.io, std::min(want, std::max(ev.io.cap, ev.io.n + 1024)));
    }
    const Instruction ins = code[pc];
    CpuEvent& ce = ev.cpu.p[ev.cpu.n++];
    const uint32_t mp0 = (uint32_t)off;
    uint32_t next_pc = pc + 1;
    ce.clk = clk;
    ce.pc = pc;
    ce.mp = mp0;
    ce.mv = ce.next_mv = 0;
    ce.mv_access = MemAccess();
    ce.next_mv_access = MemAccess();
    const uint8_t op = ins.opcode;
    if (op == OP_MEM_FWD || op == OP_MEM_BWD) {
      off += op == OP_MEM_FWD ? 1 : -1;
      if (ev.meminstr.n == ev.meminstr.cap) ev.grow(ev.meminstr, ev.meminstr.n + 1);
      ev.meminstr.p[ev.meminstr.n++] = {clk, pc, op, mp0, (uint32_t)off};
    } else {
      ensure_cell(off);
      HostEvents::Cell& c = cells[off - lo];
      c.touched = 1;
      MemAccess& a = ce.mv_access;  // the first access of the cycle: read, or the input write
      a.prev_value = c.value;
      a.prev_ts = c.ts;
      const bool input = op == OP_INPUT;
      if (input) {
        if (nin == 0) throw std::runtime_error("input stream exhausted");
        c.value = in[0];  // the reference never advances input_stream_ptr
      }
      c.ts = clk + 1;
      a.kind = input ? 2 : 1;
      a.value = c.value;
      a.ts = c.ts;
      const uint8_t mv = c.value;
      ce.mv = mv;
      switch (op) {
        case OP_ADD:
        case OP_SUB: {
          const uint8_t nv = op == OP_ADD ? (uint8_t)(mv + 1) : (uint8_t)(mv - 1);
          MemAccess& b = ce.next_mv_access;
          b.prev_value = c.value;
          b.prev_ts = c.ts;
          c.value = nv;
          c.ts = clk + 2;
          b.kind = 2;
          b.value = nv;
          b.ts = c.ts;
          ce.next_mv = nv;
          if (ev.alu.n == ev.alu.cap) ev.grow(ev.alu, ev.alu.n + 1);
          ev.alu.p[ev.alu.n++] = {pc, op, nv, mv};
          break;
        }
        case OP_LOOP_START:
        case OP_LOOP_END:
          if (op == OP_LOOP_START) next_pc = mv == 0 ? ins.op_a : pc + 1;
          else next_pc = mv != 0 ? ins.op_a : pc + 1;
          if (ev.jump.n == ev.jump.cap) ev.grow(ev.jump, ev.jump.n + 1);
          ev.jump.p[ev.jump.n++] = {pc, next_pc, op, next_pc, mv};
          break;
        default:  // OP_INPUT / OP_OUTPUT
          if (op == OP_OUTPUT) ev.output.push_back(mv);
          if (ev.io.n == ev.io.cap) ev.grow(ev.io, ev.io.n + 1);
          ev.io.p[ev.io.n++] = {pc, op, mp0, mv};
          break;
      }
    }
    ce.next_pc = next_pc;
    ce.next_mp = (uint32_t)off;
    pc = next_pc;
    clk += 2;
    gclk++;
    if (pc == n) break;
  }
  // memory events in address order: offsets [0, hi) are addresses 0.., offsets [lo, 0) wrap to
  // 2^32 + off, above every non-negative one; first access saw (value 0, ts 0)
  size_t touched = 0;
  for (int64_t o = lo; o < hi; o++) touched += cells[o - lo].touched;
  ev.grow(ev.memory, touched);
  ev.memory.n = 0;
  auto emit = [&](int64_t a, int64_t b) {
    for (int64_t o = a; o < b; o++) {
      const HostEvents::Cell& c = cells[o - lo];
      if (c.touched) ev.memory.p[ev.memory.n++] = {(uint32_t)o, 0, c.ts, 0, c.value};
    }
  };
  emit(std::max<int64_t>(0, lo), hi);
  emit(lo, std::min<int64_t>(0, hi));
  ev.cell_lo = lo;
  ev.global_clk = gclk;
  ev.pc = pc;
  ev.mp = (uint32_t)off;
}

void generate_dependencies(ExecutionRecord& rec) {
  // CpuChip (cpu/trace.rs:58-79,86-150), MemoryAccessCols::populate_access
  // (memory/consistency/trace.rs:52-77), AddSubChip (alu/mod.rs:95-116; operations/add.rs:20-40).
  rec.u8_mult.assign(256, 0);
  rec.u16_mult.assign(65536, 0);
  for (const CpuEvent& e : rec.cpu) {
    rec.u16_mult[e.clk & 0xffff]++;
    rec.u8_mult[(e.clk >> 16) & 0xff]++;
    if (e.mv_access.kind) {
      uint32_t d = e.mv_access.ts - e.mv_access.prev_ts - 1;
      rec.u16_mult[d & 0xffff]++;
      rec.u8_mult[(d >> 16) & 0xff]++;
    }
    if (e.next_mv_access.kind == 2) {
      uint32_t d = e.next_mv_access.ts - e.next_mv_access.prev_ts - 1;
      rec.u16_mult[d & 0xffff]++;
      rec.u8_mult[(d >> 16) & 0xff]++;
    }
    rec.u8_mult[e.mv]++;
  }
  for (const AluEvent& e : rec.alu) {
    uint8_t a = e.opcode == OP_ADD ? e.mv : e.next_mv;
    rec.u8_mult[a]++;
    rec.u8_mult[1]++;
    rec.u8_mult[(uint8_t)(a + 1)]++;
  }
}

EventCounts counts_of(const ExecutionRecord& r) {
  EventCounts n;
  n.cpu = r.cpu.size();
  n.alu = r.alu.size();
  n.jump = r.jump.size();
  n.meminstr = r.meminstr.size();
  n.io = r.io.size();
  n.memory = r.memory.size();
  n.program = r.program ? r.program->instructions.size() : 0;
  return n;
}

EventCounts counts_of(const HostEvents& e, const Program& prog) {
  EventCounts n;
  n.cpu = e.cpu.n;
  n.alu = e.alu.n;
  n.jump = e.jump.n;
  n.meminstr = e.meminstr.n;
  n.io = e.io.n;
  n.memory = e.memory.n;
  n.program = prog.instructions.size();
  return n;
}

bool chip_included(int chip, const EventCounts& n) {
  switch (chip) {
    case CHIP_CPU: return n.cpu != 0;
    case CHIP_PROGRAM: return true;
    case CHIP_ADDSUB: return n.alu != 0;
    case CHIP_JUMP: return n.jump != 0;
    case CHIP_MEMORY: return n.memory != 0;
    case CHIP_BYTE: return true;
    case CHIP_MEMINSTRS: return n.meminstr != 0;
    case CHIP_IO: return n.io != 0;
  }
  return false;
}
bool chip_included(int chip, const ExecutionRecord& r) { return chip_included(chip, counts_of(r)); }

static size_t npot(size_t n) {
  size_t p = 1;
  while (p < n) p <<= 1;
  return p;
}
static size_t npot16(size_t n) { return std::max<size_t>(16, npot(n)); }

size_t main_trace_height(int chip, const EventCounts& n) {
  switch (chip) {
    case CHIP_CPU: return npot(n.cpu);  // no minimum (cpu/trace.rs:33)
    case CHIP_PROGRAM: return npot16(n.program);
    case CHIP_ADDSUB: return npot16(n.alu);
    case CHIP_JUMP: return npot16(n.jump);
    case CHIP_MEMORY: return npot16((n.memory + 1) / 2);
    case CHIP_BYTE: return 1u << 16;
    case CHIP_MEMINSTRS: return npot16(n.meminstr);
    case CHIP_IO: return npot16(n.io);
  }
  return 0;
}
size_t main_trace_height(int chip, const ExecutionRecord& r) {
  return main_trace_height(chip, counts_of(r));
}

namespace {
const uint32_t M1 = kb::ONE;
inline uint32_t mb(bool b) { return b ? M1 : 0; }
inline void put_word(uint32_t* c, uint32_t v) {
  for (int i = 0; i < 4; i++) c[i] = to_mont((v >> (8 * i)) & 0xff);
}
// KoalaBearWordRangeChecker::populate (operations/koala_bear_word.rs:29-45)
inline void put_word_rc(uint32_t* c, uint32_t v) {
  uint32_t b[8];
  for (int i = 0; i < 8; i++) b[i] = (v >> (i + 24)) & 1;
  for (int i = 0; i < 8; i++) c[i] = mb(b[i]);
  uint32_t a = b[0] & b[1];
  c[8] = mb(a);
  for (int k = 2; k <= 6; k++) { a &= b[k]; c[7 + k] = mb(a); }
}
// Memory{ReadWrite,Write}Cols::populate + MemoryAccessCols::populate_access
inline void put_access(uint32_t* prev_value, uint32_t* acc, const MemAccess& a) {
  *prev_value = to_mont(a.kind == 2 ? a.prev_value : a.value);
  acc[0] = to_mont(a.value);
  acc[1] = to_mont(a.prev_ts);
  uint32_t d = a.ts - a.prev_ts - 1;
  acc[2] = to_mont(d & 0xffff);
  acc[3] = to_mont((d >> 16) & 0xff);
}
}  // namespace

size_t main_trace(int chip, const ExecutionRecord& r, std::vector<uint32_t>& out) {
  const size_t h = main_trace_height(chip, r);
  const size_t w = (size_t)CHIP_INFO[chip].main_w;
  out.assign(h * w, 0);
  const Program& prog = *r.program;
  switch (chip) {
    case CHIP_CPU:  // cpu/trace.rs:28-55,86-150; layout cpu/cols.rs:29-71
      for (size_t i = 0; i < r.cpu.size(); i++) {
        const CpuEvent& e = r.cpu[i];
        uint32_t* c = &out[i * w];
        const Instruction& ins = prog.instructions[e.pc];
        const int op = ins.opcode;
        c[0] = to_mont(e.clk & 0xffff);
        c[1] = to_mont((e.clk >> 16) & 0xff);
        c[2] = to_mont(e.pc);
        c[3] = to_mont(e.next_pc);
        c[4] = to_mont(e.mp);
        c[5] = to_mont(e.next_mp);
        c[6] = to_mont(e.mv);
        c[7] = to_mont(e.next_mv);
        c[8] = to_mont((uint32_t)op);
        put_word(&c[9], ins.op_a);
        c[14] = to_mont(e.mv);
        c[19] = to_mont(e.next_mv);
        if (e.mv_access.kind) { put_access(&c[13], &c[14], e.mv_access); c[23] = M1; }
        if (e.next_mv_access.kind == 2) { put_access(&c[18], &c[19], e.next_mv_access); c[24] = M1; }
        const bool alu = op == OP_ADD || op == OP_SUB;
        const bool jump = op == OP_LOOP_START || op == OP_LOOP_END;
        const bool mi = op == OP_MEM_FWD || op == OP_MEM_BWD;
        const bool io = op == OP_INPUT || op == OP_OUTPUT;
        c[25] = mb(alu || jump || op == OP_OUTPUT);
        c[26] = mb(alu);
        c[27] = mb(jump);
        c[28] = mb(io);
        c[29] = mb(mi);
        c[30] = to_mont((uint32_t)alu + jump + mi + io);
      }
      break;
    case CHIP_PROGRAM: {  // program/mod.rs:100-135
      std::vector<uint32_t> cnt(prog.instructions.size(), 0);
      for (const CpuEvent& e : r.cpu) cnt[e.pc]++;
      for (size_t i = 0; i < cnt.size(); i++) out[i] = to_mont(cnt[i]);
      break;
    }
    case CHIP_ADDSUB:  // alu/mod.rs:63-146
      for (size_t i = 0; i < r.alu.size(); i++) {
        const AluEvent& e = r.alu[i];
        uint32_t* c = &out[i * w];
        uint8_t a = e.opcode == OP_ADD ? e.mv : e.next_mv;
        c[0] = to_mont(e.pc);
        c[1] = to_mont((uint8_t)(a + 1));
        c[2] = mb((unsigned)a + 1u > 255u);
        c[3] = to_mont(a);
        c[4] = M1;
        c[5] = mb(e.opcode == OP_ADD);
        c[6] = mb(e.opcode == OP_SUB);
      }
      break;
    case CHIP_JUMP:  // jump/trace.rs:32-97; layout jump/cols.rs:12-31
      for (size_t i = 0; i < r.jump.size(); i++) {
        const JumpEvent& e = r.jump[i];
        uint32_t* c = &out[i * w];
        put_word(&c[0], e.pc);
        put_word_rc(&c[4], e.pc);
        put_word(&c[18], e.next_pc);
        put_word_rc(&c[22], e.next_pc);
        put_word(&c[36], e.dst);
        c[40] = to_mont(e.mv);
        c[41] = e.mv ? kb::minv(to_mont(e.mv)) : 0;  // IsZeroOperation::populate
        c[42] = mb(e.mv == 0);
        c[43] = mb(e.opcode == OP_LOOP_START);
        c[44] = mb(e.opcode == OP_LOOP_END);
      }
      break;
    case CHIP_MEMORY:  // memory/memory.rs:84-129 (2 entries per row)
      for (size_t i = 0; i < r.memory.size(); i++) {
        const MemoryEvent& e = r.memory[i];
        uint32_t* c = &out[(i / 2) * w + 6 * (i % 2)];
        c[0] = to_mont(e.addr);
        c[1] = to_mont(e.init_ts);
        c[2] = to_mont(e.final_ts);
        c[3] = to_mont(e.init_v);
        c[4] = to_mont(e.final_v);
        c[5] = M1;
      }
      break;
    case CHIP_BYTE:  // bytes/trace.rs:39-60
      for (size_t v = 0; v < 256; v++) out[v * 2 + 0] = to_mont((uint32_t)(r.u8_mult[v] % kb::P));
      for (size_t v = 0; v < 65536; v++) out[v * 2 + 1] = to_mont((uint32_t)(r.u16_mult[v] % kb::P));
      break;
    case CHIP_MEMINSTRS:  // memory/instructions/trace.rs:30-97; cols.rs:13-35
      for (size_t i = 0; i < r.meminstr.size(); i++) {
        const MemInstrEvent& e = r.meminstr[i];
        uint32_t* c = &out[i * w];
        c[0] = to_mont(e.pc);
        c[1] = to_mont(e.clk);
        put_word(&c[2], e.mp);
        put_word_rc(&c[6], e.mp);
        put_word(&c[20], e.next_mp);
        put_word_rc(&c[24], e.next_mp);
        c[38] = mb(e.opcode == OP_MEM_FWD);
        c[39] = mb(e.opcode == OP_MEM_BWD);
        c[40] = M1;
      }
      break;
    case CHIP_IO:  // io/mod.rs:72-121
      for (size_t i = 0; i < r.io.size(); i++) {
        const IoEvent& e = r.io[i];
        uint32_t* c = &out[i * w];
        c[0] = to_mont(e.pc);
        c[1] = to_mont(e.mp);
        c[2] = to_mont(e.mv);
        c[3] = mb(e.opcode == OP_INPUT);
        c[4] = mb(e.opcode == OP_OUTPUT);
      }
      break;
  }
  return h;
}

size_t prep_trace(int chip, const Program& prog, std::vector<uint32_t>& out) {
  if (chip == CHIP_PROGRAM) {  // program/mod.rs:66-98
    size_t h = npot16(prog.instructions.size());
    out.assign(h * 6, 0);
    for (size_t i = 0; i < prog.instructions.size(); i++) {
      out[i * 6 + 0] = to_mont((uint32_t)i);
      out[i * 6 + 1] = to_mont(prog.instructions[i].opcode);
      put_word(&out[i * 6 + 2], prog.instructions[i].op_a);
    }
    return h;
  }
  if (chip == CHIP_BYTE) {  // bytes/mod.rs:31-62
    size_t h = 1u << 16;
    out.assign(h * 2, 0);
    for (size_t i = 0; i < h; i++) {
      out[2 * i] = to_mont(i & 0xff);
      out[2 * i + 1] = to_mont((uint32_t)i);
    }
    return h;
  }
  out.clear();
  return 0;
}

}  // namespace bfz
