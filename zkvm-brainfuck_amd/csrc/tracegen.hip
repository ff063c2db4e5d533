// Device trace generation (see tracegen.h).  One thread per output position t of a chip's
// column-major, bit-reversed evaluation matrix: it reads event bitrev(t) (or writes a zero
// padding row) and stores every column at [c][t], so each column store of a wave is one
// contiguous segment.  Column layouts and values follow the host mirror in machine.cpp,
// which cites the reference's generate_trace for every chip.
#include "tracegen.h"
#include "ntt.h"
#include "quotient.h"

namespace bfz {

using namespace kb;

namespace {

__device__ __forceinline__ uint32_t mb(bool b) { return b ? ONE : 0u; }

__device__ __forceinline__ void put_word(uint32_t* c, uint32_t v) {
#pragma unroll
  for (int i = 0; i < 4; i++) c[i] = to_mont((v >> (8 * i)) & 0xff);
}

// KoalaBearWordRangeChecker::populate (operations/koala_bear_word.rs:29-45)
__device__ __forceinline__ void put_word_rc(uint32_t* c, uint32_t v) {
  uint32_t b[8];
#pragma unroll
  for (int i = 0; i < 8; i++) b[i] = (v >> (i + 24)) & 1;
#pragma unroll
  for (int i = 0; i < 8; i++) c[i] = mb(b[i]);
  uint32_t a = b[0] & b[1];
  c[8] = mb(a);
#pragma unroll
  for (int k = 2; k <= 6; k++) {
    a &= b[k];
    c[7 + k] = mb(a);
  }
}

// Memory{ReadWrite,Write}Cols::populate + MemoryAccessCols::populate_access
__device__ __forceinline__ void put_access(uint32_t* prev_value, uint32_t* acc, const MemAccess& a) {
  *prev_value = to_mont(a.kind == 2 ? a.prev_value : a.value);
  acc[0] = to_mont(a.value);
  acc[1] = to_mont(a.prev_ts);
  const uint32_t d = a.ts - a.prev_ts - 1;
  acc[2] = to_mont(d & 0xffff);
  acc[3] = to_mont((d >> 16) & 0xff);
}

template <int W>
__device__ __forceinline__ void store_row(uint32_t* out, size_t h, size_t t, const uint32_t (&c)[W]) {
#pragma unroll
  for (int k = 0; k < W; k++) out[(size_t)k * h + t] = c[k];
}

// ---------------------------------------------------------------- generate_dependencies
constexpr int LOW16 = 8192;    // u16 bins kept in LDS per block (small timestamp gaps dominate)
constexpr int PROG_LDS = 4096; // program counts in LDS when the program is this short

// Histogram increment with wave aggregation: in execution order neighbouring lanes mostly
// share a key (clock high byte, timestamp gap, loop pcs), so the lanes matching the first
// active lane's key add their count with one atomic; the rest add individually.
__device__ __forceinline__ void agg_add(uint32_t* h, uint32_t key) {
  const uint32_t k0 = __builtin_amdgcn_readfirstlane(key);
  const uint64_t active = __ballot(1);
  const uint64_t same = __ballot(key == k0);
  if (key == k0) {
    if (__lane_id() == (unsigned)(__ffsll((unsigned long long)active) - 1))
      atomicAdd(&h[k0], (uint32_t)__popcll(same));
  } else {
    atomicAdd(&h[key], 1u);
  }
}

__device__ __forceinline__ void bump16(uint32_t* lds16, uint32_t* g16, uint32_t v) {
  if (v < LOW16) agg_add(lds16, v);
  else atomicAdd(&g16[v], 1u);
}

// CpuChip (cpu/trace.rs:58-79,86-150) + AddSubChip (alu/mod.rs:95-116) byte lookups and
// the Program chip's per-pc execution counts (program/mod.rs:100-135).
__global__ __launch_bounds__(256) void k_deps(const CpuEvent* __restrict__ cpu, size_t ncpu,
                                              const AluEvent* __restrict__ alu, size_t nalu,
                                              uint32_t* __restrict__ g8, uint32_t* __restrict__ g16,
                                              uint32_t* __restrict__ gprog, int nprog) {
  __shared__ uint32_t h8[256];
  __shared__ uint32_t h16[LOW16];
  __shared__ uint32_t hp[PROG_LDS];
  const bool prog_lds = nprog <= PROG_LDS;
  for (int i = threadIdx.x; i < LOW16; i += blockDim.x) h16[i] = 0;
  for (int i = threadIdx.x; i < PROG_LDS; i += blockDim.x) hp[i] = 0;
  if (threadIdx.x < 256) h8[threadIdx.x] = 0;
  __syncthreads();
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < ncpu; i += stride) {
    const CpuEvent e = cpu[i];
    bump16(h16, g16, e.clk & 0xffff);
    agg_add(h8, (e.clk >> 16) & 0xff);
    if (e.mv_access.kind) {
      const uint32_t d = e.mv_access.ts - e.mv_access.prev_ts - 1;
      bump16(h16, g16, d & 0xffff);
      agg_add(h8, (d >> 16) & 0xff);
    }
    if (e.next_mv_access.kind == 2) {
      const uint32_t d = e.next_mv_access.ts - e.next_mv_access.prev_ts - 1;
      bump16(h16, g16, d & 0xffff);
      agg_add(h8, (d >> 16) & 0xff);
    }
    agg_add(h8, e.mv);
    if (prog_lds) agg_add(hp, e.pc);
    else if (e.pc < (uint32_t)nprog) atomicAdd(&gprog[e.pc], 1u);
  }
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < nalu; i += stride) {
    const AluEvent e = alu[i];
    const uint8_t a = e.opcode == OP_ADD ? e.mv : e.next_mv;
    agg_add(h8, a);
    agg_add(h8, 1);
    agg_add(h8, (uint8_t)(a + 1));
  }
  __syncthreads();
  for (int i = threadIdx.x; i < LOW16; i += blockDim.x)
    if (h16[i]) atomicAdd(&g16[i], h16[i]);
  if (prog_lds)
    for (int i = threadIdx.x; i < nprog; i += blockDim.x)
      if (hp[i]) atomicAdd(&gprog[i], hp[i]);
  if (threadIdx.x < 256 && h8[threadIdx.x]) atomicAdd(&g8[threadIdx.x], h8[threadIdx.x]);
}

// ---------------------------------------------------------------- per-chip traces
// CpuChip: cpu/trace.rs:28-55,86-150; layout cpu/cols.rs:29-71
__global__ __launch_bounds__(256) void k_trace_cpu(const CpuEvent* __restrict__ ev, size_t n,
                                                   const Instruction* __restrict__ prog,
                                                   uint32_t* __restrict__ out, size_t h, int logh) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= h) return;
  const size_t i = dbitrev((uint32_t)t, logh);
  uint32_t c[31] = {};
  if (i < n) {
    const CpuEvent e = ev[i];
    const Instruction ins = prog[e.pc];
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
    if (e.mv_access.kind) {
      put_access(&c[13], &c[14], e.mv_access);
      c[23] = ONE;
    }
    if (e.next_mv_access.kind == 2) {
      put_access(&c[18], &c[19], e.next_mv_access);
      c[24] = ONE;
    }
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
  store_row(out, h, t, c);
}

// AddSubChip: alu/mod.rs:63-146
__global__ __launch_bounds__(256) void k_trace_addsub(const AluEvent* __restrict__ ev, size_t n,
                                                      uint32_t* __restrict__ out, size_t h,
                                                      int logh) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= h) return;
  const size_t i = dbitrev((uint32_t)t, logh);
  uint32_t c[7] = {};
  if (i < n) {
    const AluEvent e = ev[i];
    const uint8_t a = e.opcode == OP_ADD ? e.mv : e.next_mv;
    c[0] = to_mont(e.pc);
    c[1] = to_mont((uint8_t)(a + 1));
    c[2] = mb((unsigned)a + 1u > 255u);
    c[3] = to_mont(a);
    c[4] = ONE;
    c[5] = mb(e.opcode == OP_ADD);
    c[6] = mb(e.opcode == OP_SUB);
  }
  store_row(out, h, t, c);
}

// JumpChip: jump/trace.rs:32-97; layout jump/cols.rs:12-31 (IsZero inverse from a table)
__global__ __launch_bounds__(256) void k_trace_jump(const JumpEvent* __restrict__ ev, size_t n,
                                                    uint32_t* __restrict__ out, size_t h, int logh) {
  __shared__ uint32_t inv[256];
  if (threadIdx.x < 256) inv[threadIdx.x] = threadIdx.x ? minv(to_mont(threadIdx.x)) : 0u;
  __syncthreads();
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= h) return;
  const size_t i = dbitrev((uint32_t)t, logh);
  uint32_t c[45] = {};
  if (i < n) {
    const JumpEvent e = ev[i];
    put_word(&c[0], e.pc);
    put_word_rc(&c[4], e.pc);
    put_word(&c[18], e.next_pc);
    put_word_rc(&c[22], e.next_pc);
    put_word(&c[36], e.dst);
    c[40] = to_mont(e.mv);
    c[41] = inv[e.mv];  // IsZeroOperation::populate (operations/is_zero.rs:29-40)
    c[42] = mb(e.mv == 0);
    c[43] = mb(e.opcode == OP_LOOP_START);
    c[44] = mb(e.opcode == OP_LOOP_END);
  }
  store_row(out, h, t, c);
}

// MemoryChip: memory/memory.rs:84-129 (two address entries per row)
__global__ __launch_bounds__(256) void k_trace_memory(const MemoryEvent* __restrict__ ev, size_t n,
                                                      uint32_t* __restrict__ out, size_t h,
                                                      int logh) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= h) return;
  const size_t i = dbitrev((uint32_t)t, logh);
  uint32_t c[12] = {};
#pragma unroll
  for (int k = 0; k < 2; k++) {
    const size_t j = 2 * i + k;
    if (j < n) {
      const MemoryEvent e = ev[j];
      c[6 * k + 0] = to_mont(e.addr);
      c[6 * k + 1] = to_mont(e.init_ts);
      c[6 * k + 2] = to_mont(e.final_ts);
      c[6 * k + 3] = to_mont(e.init_v);
      c[6 * k + 4] = to_mont(e.final_v);
      c[6 * k + 5] = ONE;
    }
  }
  store_row(out, h, t, c);
}

// MemoryInstructionsChip: memory/instructions/trace.rs:30-97; cols.rs:13-35
__global__ __launch_bounds__(256) void k_trace_meminstr(const MemInstrEvent* __restrict__ ev,
                                                        size_t n, uint32_t* __restrict__ out,
                                                        size_t h, int logh) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= h) return;
  const size_t i = dbitrev((uint32_t)t, logh);
  uint32_t c[41] = {};
  if (i < n) {
    const MemInstrEvent e = ev[i];
    c[0] = to_mont(e.pc);
    c[1] = to_mont(e.clk);
    put_word(&c[2], e.mp);
    put_word_rc(&c[6], e.mp);
    put_word(&c[20], e.next_mp);
    put_word_rc(&c[24], e.next_mp);
    c[38] = mb(e.opcode == OP_MEM_FWD);
    c[39] = mb(e.opcode == OP_MEM_BWD);
    c[40] = ONE;
  }
  store_row(out, h, t, c);
}

// IoChip: io/mod.rs:72-121
__global__ __launch_bounds__(256) void k_trace_io(const IoEvent* __restrict__ ev, size_t n,
                                                  uint32_t* __restrict__ out, size_t h, int logh) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= h) return;
  const size_t i = dbitrev((uint32_t)t, logh);
  uint32_t c[5] = {};
  if (i < n) {
    const IoEvent e = ev[i];
    c[0] = to_mont(e.pc);
    c[1] = to_mont(e.mp);
    c[2] = to_mont(e.mv);
    c[3] = mb(e.opcode == OP_INPUT);
    c[4] = mb(e.opcode == OP_OUTPUT);
  }
  store_row(out, h, t, c);
}

// ProgramChip main trace (program/mod.rs:100-135): execution count per instruction.
__global__ __launch_bounds__(256) void k_trace_program(const uint32_t* __restrict__ cnt, size_t n,
                                                       uint32_t* __restrict__ out, size_t h,
                                                       int logh) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= h) return;
  const size_t i = dbitrev((uint32_t)t, logh);
  out[t] = i < n ? to_mont(cnt[i]) : 0u;
}

// ByteChip main trace (bytes/trace.rs:39-60): row v = (u8 multiplicity of v if v < 256,
// u16 multiplicity of v).
__global__ __launch_bounds__(256) void k_trace_byte(const uint32_t* __restrict__ m8,
                                                    const uint32_t* __restrict__ m16,
                                                    uint32_t* __restrict__ out) {
  const size_t h = (size_t)1 << 16;
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= h) return;
  const uint32_t v = dbitrev((uint32_t)t, 16);
  out[t] = v < 256 ? to_mont(m8[v]) : 0u;
  out[h + t] = to_mont(m16[v]);
}

template <class T>
void put(DBuf<T>& d, const std::vector<T>& v, hipStream_t st) {
  d.reset(std::max<size_t>(v.size(), 1));
  if (!v.empty())
    HIP_CHECK(hipMemcpyAsync(d.p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, st));
}

}  // namespace

void set_event_meta(DeviceEvents& ev, const EventCounts& n, uint64_t global_clk) {
  ev.n[CHIP_CPU] = n.cpu;
  ev.n[CHIP_PROGRAM] = n.program;
  ev.n[CHIP_ADDSUB] = n.alu;
  ev.n[CHIP_JUMP] = n.jump;
  ev.n[CHIP_MEMORY] = n.memory;
  ev.n[CHIP_BYTE] = 0;
  ev.n[CHIP_MEMINSTRS] = n.meminstr;
  ev.n[CHIP_IO] = n.io;
  for (int c = 0; c < NUM_CHIPS; c++) {
    ev.included[c] = chip_included(c, n);
    ev.height[c] = main_trace_height(c, n);
  }
  ev.global_clk = global_clk;
  // every twiddle / coset-power / selector table a proof of these heights reads, built now
  // (once per process and height) instead of between the first proof's launches
  for (int c = 0; c < NUM_CHIPS; c++)
    if (ev.included[c] && ev.height[c]) {
      const int L = log2i(ev.height[c]);
      prepare_lde_tables(L);
      prepare_quotient_tables(L + 1);
    }
}

void upload_events(const ExecutionRecord& rec, DeviceEvents& ev, hipStream_t st) {
  put(ev.cpu, rec.cpu, st);
  put(ev.alu, rec.alu, st);
  put(ev.jump, rec.jump, st);
  put(ev.meminstr, rec.meminstr, st);
  put(ev.io, rec.io, st);
  put(ev.memory, rec.memory, st);
  put(ev.prog, rec.program->instructions, st);
  set_event_meta(ev, counts_of(rec), rec.global_clk);
  HIP_CHECK(hipStreamSynchronize(st));  // the host vectors may be freed after this returns
}

namespace {
template <class T>
void put_arr(DBuf<T>& d, const HostEvents::Arr<T>& a, hipStream_t st) {
  d.reset(std::max<size_t>(a.n, 1));
  if (a.n) HIP_CHECK(hipMemcpyAsync(d.p, a.p, a.n * sizeof(T), hipMemcpyHostToDevice, st));
}
}  // namespace

void upload_events(const HostEvents& h, const Program& prog, DeviceEvents& ev, hipStream_t st) {
  put_arr(ev.cpu, h.cpu, st);
  put_arr(ev.alu, h.alu, st);
  put_arr(ev.jump, h.jump, st);
  put_arr(ev.meminstr, h.meminstr, st);
  put_arr(ev.io, h.io, st);
  put_arr(ev.memory, h.memory, st);
  put(ev.prog, prog.instructions, st);
  set_event_meta(ev, counts_of(h, prog), h.global_clk);
  HIP_CHECK(hipStreamSynchronize(st));
}

namespace {
__global__ __launch_bounds__(256) void k_check_events(const CpuEvent* __restrict__ cpu, size_t ncpu,
                                                      const AluEvent* __restrict__ alu, size_t nalu,
                                                      const JumpEvent* __restrict__ jump, size_t njump,
                                                      const MemInstrEvent* __restrict__ mi, size_t nmi,
                                                      const IoEvent* __restrict__ io, size_t nio,
                                                      uint32_t nprog, unsigned* __restrict__ bad) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  const size_t i0 = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  unsigned b = 0;
  for (size_t i = i0; i < ncpu; i += stride) {
    const CpuEvent e = cpu[i];
    b += e.pc >= nprog || e.mv_access.kind > 2 || e.next_mv_access.kind > 2;
  }
  for (size_t i = i0; i < nalu; i += stride) b += alu[i].opcode != OP_ADD && alu[i].opcode != OP_SUB;
  for (size_t i = i0; i < njump; i += stride)
    b += jump[i].opcode != OP_LOOP_START && jump[i].opcode != OP_LOOP_END;
  for (size_t i = i0; i < nmi; i += stride) b += mi[i].opcode != OP_MEM_FWD && mi[i].opcode != OP_MEM_BWD;
  for (size_t i = i0; i < nio; i += stride) b += io[i].opcode != OP_INPUT && io[i].opcode != OP_OUTPUT;
  if (b) atomicAdd(bad, b);
}
}  // namespace

size_t count_invalid_events(const DeviceEvents& ev, hipStream_t st) {
  DBuf<unsigned> bad(1);
  HIP_CHECK(hipMemsetAsync(bad.p, 0, sizeof(unsigned), st));
  size_t most = 0;
  for (int c : {CHIP_CPU, CHIP_ADDSUB, CHIP_JUMP, CHIP_MEMINSTRS, CHIP_IO}) most = std::max(most, ev.n[c]);
  const unsigned grid = std::max(1u, std::min<unsigned>(ceil_div(most, 256 * 4), 2048));
  hipLaunchKernelGGL(k_check_events, dim3(grid), dim3(256), 0, st, (const CpuEvent*)ev.cpu.p,
                     ev.n[CHIP_CPU], (const AluEvent*)ev.alu.p, ev.n[CHIP_ADDSUB],
                     (const JumpEvent*)ev.jump.p, ev.n[CHIP_JUMP], (const MemInstrEvent*)ev.meminstr.p,
                     ev.n[CHIP_MEMINSTRS], (const IoEvent*)ev.io.p, ev.n[CHIP_IO],
                     (uint32_t)ev.n[CHIP_PROGRAM], bad.p);
  KCHECK();
  unsigned h = 0;
  fetch(&h, bad.p, sizeof h, st);
  return h;
}

// ------------------------------------------------------------ compact cycles -> events
namespace {
constexpr int XB = 256;  // cycles per block of the expansion passes
enum { CAT_ALU = 0, CAT_JUMP, CAT_MEM, CAT_IO, NCAT };
__device__ __forceinline__ int cat_of(int op) {
  return (op == OP_ADD || op == OP_SUB)              ? CAT_ALU
         : (op == OP_LOOP_START || op == OP_LOOP_END) ? CAT_JUMP
         : (op == OP_MEM_FWD || op == OP_MEM_BWD)     ? CAT_MEM
                                                      : CAT_IO;
}
// A cycle the reference executor could have emitted (executor.rs:108-239): memory steps have
// no access (mv = 0), only Input writes (prev_value), and an access's previous timestamp lies
// before the cycle's first access at clk + 1.  k_cycles_count adds the step rules between a
// cycle and its successor.
__device__ __forceinline__ bool cycle_ok(const Cycle& c, uint32_t clk, int cat, int op) {
  if (c.pad[0] | c.pad[1]) return false;
  if (cat == CAT_MEM) return c.mv == 0 && c.prev_ts == 0 && c.prev_value == 0;
  if (op != OP_INPUT && c.prev_value != 0) return false;
  return c.prev_ts <= clk;
}
__device__ __forceinline__ uint64_t lanes_below() {
  return (1ull << __lane_id()) - 1ull;  // lane_id < 64
}

// Pass 1: each block's count per category; invalid cycles counted into cnt[NCAT].
__global__ __launch_bounds__(XB) void k_cycles_count(const Cycle* __restrict__ cyc, size_t n,
                                                     const Instruction* __restrict__ prog,
                                                     uint32_t nprog, uint32_t* __restrict__ bc,
                                                     uint32_t* __restrict__ cnt) {
  __shared__ uint32_t wc[XB / 64][NCAT];
  const size_t i = (size_t)blockIdx.x * XB + threadIdx.x;
  int cat = -1;
  bool bad = false;
  if (i < n) {
    const Cycle c = cyc[i];
    if (c.pc >= nprog) {
      bad = true;
    } else {
      const Instruction ins = prog[c.pc];
      const int op = ins.opcode;
      cat = cat_of(op);
      bad = !cycle_ok(c, (uint32_t)(2 * i), cat, op);
      // the successor the executor steps to (executor.rs:107-141,157-176): pc + 1, or a loop's
      // op_a chosen by mv; mp moves only on a memory step; the last cycle leaves the program
      uint32_t npc = c.pc + 1;
      if (op == OP_LOOP_START && c.mv == 0) npc = ins.op_a;
      if (op == OP_LOOP_END && c.mv != 0) npc = ins.op_a;
      const uint32_t nmp = op == OP_MEM_FWD ? c.mp + 1 : op == OP_MEM_BWD ? c.mp - 1 : c.mp;
      if (i + 1 < n) {
        const Cycle nx = cyc[i + 1];
        bad = bad || nx.pc != npc || nx.mp != nmp;
      } else {
        bad = bad || npc != nprog;
      }
    }
  }
  const int wv = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < NCAT; k++) {
    const uint32_t m = (uint32_t)__popcll(__ballot(cat == k));
    if (__lane_id() == 0) wc[wv][k] = m;
  }
  const uint32_t nb = (uint32_t)__popcll(__ballot(bad));
  if (__lane_id() == 0 && nb) atomicAdd(&cnt[NCAT], nb);
  __syncthreads();
  if (threadIdx.x < NCAT) {
    uint32_t t = 0;
    for (int w = 0; w < XB / 64; w++) t += wc[w][threadIdx.x];
    bc[(size_t)blockIdx.x * NCAT + threadIdx.x] = t;
  }
}

// Pass 2 (one block): exclusive scan of the block counts per category, totals into cnt[0..NCAT).
__global__ __launch_bounds__(1024) void k_cycles_scan(uint32_t* __restrict__ bc, size_t nb,
                                                      uint32_t* __restrict__ cnt) {
  __shared__ uint32_t part[1024][NCAT];
  const size_t per = (nb + 1023) / 1024;
  const size_t b0 = threadIdx.x * per, b1 = b0 + per < nb ? b0 + per : nb;
  uint32_t s[NCAT] = {};
  for (size_t b = b0; b < b1; b++)
#pragma unroll
    for (int k = 0; k < NCAT; k++) s[k] += bc[b * NCAT + k];
#pragma unroll
  for (int k = 0; k < NCAT; k++) part[threadIdx.x][k] = s[k];
  __syncthreads();
  if (threadIdx.x < NCAT) {  // 1024 chunk sums per category, serially (tiny)
    uint32_t run = 0;
    for (int t = 0; t < 1024; t++) {
      const uint32_t v = part[t][threadIdx.x];
      part[t][threadIdx.x] = run;
      run += v;
    }
    cnt[threadIdx.x] = run;
  }
  __syncthreads();
  uint32_t run[NCAT];
#pragma unroll
  for (int k = 0; k < NCAT; k++) run[k] = part[threadIdx.x][k];
  for (size_t b = b0; b < b1; b++)
#pragma unroll
    for (int k = 0; k < NCAT; k++) {
      const uint32_t v = bc[b * NCAT + k];
      bc[b * NCAT + k] = run[k];
      run[k] += v;
    }
}

// Pass 3: the CpuEvent of every cycle and its chip event at its category's running position.
__global__ __launch_bounds__(XB) void k_cycles_expand(const Cycle* __restrict__ cyc, size_t n,
                                                      const Instruction* __restrict__ prog,
                                                      uint32_t nprog, const uint32_t* __restrict__ bc,
                                                      CpuEvent* __restrict__ cpu, AluEvent* __restrict__ alu,
                                                      JumpEvent* __restrict__ jump,
                                                      MemInstrEvent* __restrict__ mi,
                                                      IoEvent* __restrict__ io) {
  __shared__ uint32_t wc[XB / 64][NCAT];
  const size_t i = (size_t)blockIdx.x * XB + threadIdx.x;
  Cycle c{};
  int op = 0, cat = -1;
  if (i < n) {
    c = cyc[i];
    if (c.pc < nprog) {  // an out-of-range pc fails the whole call (pass 1): write nothing
      op = prog[c.pc].opcode;
      cat = cat_of(op);
    }
  }
  const int wv = threadIdx.x >> 6;
  uint32_t rank = 0;
#pragma unroll
  for (int k = 0; k < NCAT; k++) {
    const uint64_t m = __ballot(cat == k);
    if (cat == k) rank = (uint32_t)__popcll(m & lanes_below());
    if (__lane_id() == 0) wc[wv][k] = (uint32_t)__popcll(m);
  }
  __syncthreads();
  if (cat < 0) return;
  uint32_t pos = bc[(size_t)blockIdx.x * NCAT + cat] + rank;
  for (int w = 0; w < wv; w++) pos += wc[w][cat];
  const uint32_t clk = (uint32_t)(2 * i);
  const bool last = i + 1 == n;
  const Cycle nx = last ? c : cyc[i + 1];
  CpuEvent e{};
  e.clk = clk;
  e.pc = c.pc;
  e.mp = c.mp;
  e.mv = c.mv;
  e.next_pc = last ? nprog : nx.pc;  // the run ends when pc reaches the program's end
  e.next_mp = !last ? nx.mp : op == OP_MEM_FWD ? c.mp + 1 : op == OP_MEM_BWD ? c.mp - 1 : c.mp;
  e.next_mv = op == OP_ADD ? (uint8_t)(c.mv + 1) : op == OP_SUB ? (uint8_t)(c.mv - 1) : (uint8_t)0;
  if (cat != CAT_MEM) {  // rr_cpu / rw_cpu at clk + 1 (executor.rs:145-205)
    e.mv_access.kind = op == OP_INPUT ? 2 : 1;
    e.mv_access.value = c.mv;
    e.mv_access.prev_value = op == OP_INPUT ? c.prev_value : c.mv;
    e.mv_access.ts = clk + 1;
    e.mv_access.prev_ts = c.prev_ts;
  }
  if (cat == CAT_ALU) {  // the write of next_mv at clk + 2 (executor.rs:148-158)
    e.next_mv_access.kind = 2;
    e.next_mv_access.value = e.next_mv;
    e.next_mv_access.prev_value = c.mv;
    e.next_mv_access.ts = clk + 2;
    e.next_mv_access.prev_ts = clk + 1;
  }
  cpu[i] = e;
  switch (cat) {  // emit_events (executor.rs:196-239)
    case CAT_ALU: alu[pos] = AluEvent{c.pc, (uint8_t)op, e.next_mv, c.mv}; break;
    case CAT_JUMP: jump[pos] = JumpEvent{c.pc, e.next_pc, (uint8_t)op, e.next_pc, c.mv}; break;
    case CAT_MEM: mi[pos] = MemInstrEvent{clk, c.pc, (uint8_t)op, c.mp, e.next_mp}; break;
    default: io[pos] = IoEvent{c.pc, (uint8_t)op, c.mp, c.mv}; break;
  }
}
}  // namespace

void expand_cycles(const Cycle* d, size_t n, DeviceEvents& ev, EventCounts& n_out, size_t* invalid,
                   hipStream_t st) {
  if (n == 0 || n > ((size_t)1 << 30)) throw std::runtime_error("expand_cycles: cycle count out of range");
  const uint32_t nprog = (uint32_t)ev.n[CHIP_PROGRAM];
  const size_t nb = ceil_div(n, XB);
  DBuf<uint32_t> bc(nb * NCAT), cnt(NCAT + 1);
  HIP_CHECK(hipMemsetAsync(cnt.p, 0, (NCAT + 1) * 4, st));
  hipLaunchKernelGGL(k_cycles_count, dim3((unsigned)nb), dim3(XB), 0, st, d, n,
                     (const Instruction*)ev.prog.p, nprog, bc.p, cnt.p);
  KCHECK();
  hipLaunchKernelGGL(k_cycles_scan, dim3(1), dim3(1024), 0, st, bc.p, nb, cnt.p);
  KCHECK();
  uint32_t h[NCAT + 1];
  fetch(h, cnt.p, sizeof h, st);
  *invalid = h[NCAT];
  n_out.cpu = n;
  n_out.alu = h[CAT_ALU];
  n_out.jump = h[CAT_JUMP];
  n_out.meminstr = h[CAT_MEM];
  n_out.io = h[CAT_IO];
  ev.cpu.reset(n);
  ev.alu.reset(std::max<size_t>(n_out.alu, 1));
  ev.jump.reset(std::max<size_t>(n_out.jump, 1));
  ev.meminstr.reset(std::max<size_t>(n_out.meminstr, 1));
  ev.io.reset(std::max<size_t>(n_out.io, 1));
  if (*invalid) return;
  hipLaunchKernelGGL(k_cycles_expand, dim3((unsigned)nb), dim3(XB), 0, st, d, n,
                     (const Instruction*)ev.prog.p, nprog, (const uint32_t*)bc.p, ev.cpu.p, ev.alu.p,
                     ev.jump.p, ev.meminstr.p, ev.io.p);
  KCHECK();
}

void* pinned_alloc(size_t bytes) {
  void* p = nullptr;
  if (hipHostMalloc(&p, bytes, hipHostMallocDefault) != hipSuccess) return nullptr;
  return p;
}
void pinned_free(void* p) {
  if (p) (void)hipHostFree(p);
}

void generate_traces_device(const DeviceEvents& ev, DeviceTraces& dt, hipStream_t st) {
  dt.chips.clear();
  dt.evals.clear();
  dt.heights.clear();
  if (ev.n[CHIP_CPU] > 0xffffffffull / 4) throw std::runtime_error("tracegen: too many cycles");
  const int nprog = (int)ev.n[CHIP_PROGRAM];
  DBuf<uint32_t> m8(256), m16(65536), mprog(std::max(nprog, 1));
  HIP_CHECK(hipMemsetAsync(m8.p, 0, 256 * 4, st));
  HIP_CHECK(hipMemsetAsync(m16.p, 0, 65536 * 4, st));
  HIP_CHECK(hipMemsetAsync(mprog.p, 0, std::max(nprog, 1) * 4, st));
  {
    const size_t work = std::max(ev.n[CHIP_CPU], ev.n[CHIP_ADDSUB]);
    const unsigned grid = std::max(1u, std::min<unsigned>(ceil_div(work, 256 * 16), 1024));
    hipLaunchKernelGGL(k_deps, dim3(grid), dim3(256), 0, st, (const CpuEvent*)ev.cpu.p,
                       ev.n[CHIP_CPU], (const AluEvent*)ev.alu.p, ev.n[CHIP_ADDSUB], m8.p, m16.p,
                       mprog.p, nprog);
    KCHECK();
  }
  for (int c = 0; c < NUM_CHIPS; c++) {
    if (!ev.included[c]) continue;
    const size_t h = ev.height[c];
    const int w = CHIP_INFO[c].main_w;
    const int logh = log2i(h);
    DBuf<uint32_t> out(h * (size_t)w);
    const dim3 grid(ceil_div(h, 256)), blk(256);
    switch (c) {
      case CHIP_CPU:
        hipLaunchKernelGGL(k_trace_cpu, grid, blk, 0, st, (const CpuEvent*)ev.cpu.p, ev.n[c],
                           (const Instruction*)ev.prog.p, out.p, h, logh);
        break;
      case CHIP_PROGRAM:
        hipLaunchKernelGGL(k_trace_program, grid, blk, 0, st, (const uint32_t*)mprog.p, ev.n[c],
                           out.p, h, logh);
        break;
      case CHIP_ADDSUB:
        hipLaunchKernelGGL(k_trace_addsub, grid, blk, 0, st, (const AluEvent*)ev.alu.p, ev.n[c],
                           out.p, h, logh);
        break;
      case CHIP_JUMP:
        hipLaunchKernelGGL(k_trace_jump, grid, blk, 0, st, (const JumpEvent*)ev.jump.p, ev.n[c],
                           out.p, h, logh);
        break;
      case CHIP_MEMORY:
        hipLaunchKernelGGL(k_trace_memory, grid, blk, 0, st, (const MemoryEvent*)ev.memory.p,
                           ev.n[c], out.p, h, logh);
        break;
      case CHIP_BYTE:
        hipLaunchKernelGGL(k_trace_byte, grid, blk, 0, st, (const uint32_t*)m8.p,
                           (const uint32_t*)m16.p, out.p);
        break;
      case CHIP_MEMINSTRS:
        hipLaunchKernelGGL(k_trace_meminstr, grid, blk, 0, st, (const MemInstrEvent*)ev.meminstr.p,
                           ev.n[c], out.p, h, logh);
        break;
      case CHIP_IO:
        hipLaunchKernelGGL(k_trace_io, grid, blk, 0, st, (const IoEvent*)ev.io.p, ev.n[c], out.p, h,
                           logh);
        break;
    }
    KCHECK();
    dt.chips.push_back(c);
    dt.evals.push_back(std::move(out));
    dt.heights.push_back(h);
  }
}

// kernels a proof launches (gpu.h PreloadKernels)
static PreloadKernels preload_tracegen{
    (const void*)&k_deps,
    (const void*)&k_trace_cpu,
    (const void*)&k_trace_addsub,
    (const void*)&k_trace_jump,
    (const void*)&k_trace_memory,
    (const void*)&k_trace_meminstr,
    (const void*)&k_trace_io,
    (const void*)&k_trace_program,
    (const void*)&k_trace_byte};

}  // namespace bfz
