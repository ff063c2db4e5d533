// extern "C" boundary (include/bfz.h).  Exceptions never cross it: every entry point
// catches, records the message for bfz_last_error(), and returns a negative status.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstddef>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/bfz.h"
#include "fri.h"
#include "logup.h"
#include "merkle.h"
#include "ntt.h"
#include "pcs_sharded.h"
#include "pipeline.h"
#include "proof.h"
#include "prover.h"
#include "tracegen.h"
#include "verifier.h"

struct bfz_pk {
  std::shared_ptr<const bfz::ProvingKey> pk;  // shared with the per-program setup cache
};
struct bfz_main_data {
  std::shared_ptr<const bfz::ProvingKey> pk;  // the key the commit was made for
  bfz::MainData md;
};
struct bfz_record {
  bfz::DeviceEvents ev;  // executor events resident in HBM
  uint64_t cycles = 0;
};
struct bfz_cycle_upload {  // a chunked hand-over in progress (bfz_cycles_begin .. finish)
  const bfz_pk* pk = nullptr;
  size_t n = 0;
  bfz::DBuf<bfz::Cycle> d;
  std::vector<std::pair<size_t, size_t>> ranges;  // pushed (first, count)
  hipEvent_t copied = nullptr;
  ~bfz_cycle_upload() {
    if (copied) (void)hipEventDestroy(copied);
  }
};

namespace {
std::mutex g_mu;
thread_local std::string g_err;
// proofs handed out by emit, by data pointer (bfz_free releases them)
std::mutex& emitted_mu() {
  static std::mutex m;
  return m;
}
std::unordered_map<void*, std::vector<uint8_t>*>& emitted() {
  static auto* m = new std::unordered_map<void*, std::vector<uint8_t>*>();
  return *m;
}
int g_num_queries = -1;
int g_observe_openings = -1;  // -1: BFZ_OBSERVE_OPENINGS / default
int g_fault = 0;              // bfz_set_fault_injection (tests only)

int fail(const std::exception& e, int code = -1) {
  g_err = e.what();
  return code;
}
bfz::ProveOptions opts() {
  bfz::ProveOptions o;
  o.num_queries = g_num_queries > 0 ? g_num_queries : bfz::num_queries_from_env();
  o.observe_openings = g_observe_openings >= 0 ? g_observe_openings != 0 : bfz::observe_openings_from_env();
  o.fault_device_challenger = (g_fault & 1) != 0;
  return o;
}
template <class F>
int guarded(F&& f) {
  std::lock_guard<std::mutex> lk(g_mu);
  bfz::ApiLockScope held;  // open_impl's process-global pinned buffers rely on it
  try {
    return f();
  } catch (const bfz::HipError& e) {
    bfz::quiesce();  // nothing queued may still write a pinned mailbox after the error returns
    return fail(e, -2);
  } catch (const std::exception& e) {
    bfz::quiesce();
    return fail(e, -1);
  }
}
}  // namespace

extern "C" {

// One process drives one device: the stream, the allocator pool, the twiddle and selector
// caches and the pinned staging arena are process-wide and belong to the first device bound.
int bfz_init(int device) {
  return guarded([&] {
    static int bound = -1;
    int n = 0;
    HIP_CHECK(hipGetDeviceCount(&n));
    if (n <= 0) throw std::runtime_error("no HIP device");
    if (device < 0 || device >= n) throw std::runtime_error("bfz_init: device index out of range");
    if (bound >= 0 && bound != device)
      throw std::runtime_error("bfz_init: this process is already bound to device " +
                               std::to_string(bound) + " (one process per GPU)");
    HIP_CHECK(hipSetDevice(device));
    (void)bfz::stream();
    // every kernel a proof launches, looked up now rather than between the first proof's launches
    const double pre_ms = bfz::preload_kernels();
    if (pre_ms > 0 && std::getenv("BFZ_HOST_TRACE"))
      std::fprintf(stderr, "preload: kernels looked up in %.2f ms\n", pre_ms);
    bound = device;
    return 0;
  });
}

const char* bfz_last_error(void) { return g_err.c_str(); }

#ifndef BFZ_SRC_HASH
#error "BFZ_SRC_HASH must be defined by the Makefile (bfz/srchash.py)"
#endif
const char* bfz_build_id(void) { return BFZ_SRC_HASH; }

int bfz_device_name(char* buf, size_t cap) {
  return guarded([&] {
    hipDeviceProp_t p;
    int dev = 0;
    HIP_CHECK(hipGetDevice(&dev));
    HIP_CHECK(hipGetDeviceProperties(&p, dev));
    std::snprintf(buf, cap, "%s (%s)", p.name, p.gcnArchName);
    return 0;
  });
}

void bfz_free(void* p) {
  if (!p) return;
  {
    std::lock_guard<std::mutex> lk(emitted_mu());
    auto it = emitted().find(p);
    if (it != emitted().end()) {
      bfz::release_proof_buffer(std::move(*it->second));
      delete it->second;
      emitted().erase(it);
      return;
    }
  }
  std::free(p);
}

int bfz_execute(const char* elf, const uint8_t* in, size_t nin, uint8_t* out, size_t cap,
                size_t* out_len, uint64_t* cycles) {
  return guarded([&] {
    bfz::Program p = bfz::Program::parse(elf);
    bfz::ExecutionRecord rec;
    bfz::execute(p, in, nin, rec);
    const size_t n = std::min(cap, rec.output.size());
    if (n) std::memcpy(out, rec.output.data(), n);
    *out_len = rec.output.size();
    if (cycles) *cycles = rec.global_clk;
    return 0;
  });
}

int bfz_trace(const char* elf, const uint8_t* in, size_t nin, int chip, int prep, uint32_t** out,
              size_t* height, size_t* width) {
  return guarded([&] {
    if (chip < 0 || chip >= bfz::NUM_CHIPS) throw std::runtime_error("bad chip index");
    bfz::Program p = bfz::Program::parse(elf);
    std::vector<uint32_t> t;
    size_t h = 0;
    if (prep) {
      h = bfz::prep_trace(chip, p, t);
      if (!h) return 1;
      *width = bfz::CHIP_INFO[chip].prep_w;
    } else {
      bfz::ExecutionRecord rec;
      bfz::execute(p, in, nin, rec);
      bfz::generate_dependencies(rec);
      if (!bfz::chip_included(chip, rec)) return 1;
      h = bfz::main_trace(chip, rec, t);
      *width = bfz::CHIP_INFO[chip].main_w;
    }
    uint32_t* o = (uint32_t*)std::malloc(t.size() * 4 + 4);
    if (!o) throw std::runtime_error("out of host memory");
    std::memcpy(o, t.data(), t.size() * 4);
    *out = o;
    *height = h;
    return 0;
  });
}

// A proof (about 1 MB) is handed to the caller without a copy: the vector moves to the heap
// and bfz_free finds it by its data pointer.
static int emit(std::vector<uint8_t>&& v, uint8_t** proof, size_t* len) {
  if (v.empty()) {
    uint8_t* p = (uint8_t*)std::malloc(1);
    if (!p) throw std::runtime_error("out of host memory");
    *proof = p;
    *len = 0;
    return 0;
  }
  auto* h = new std::vector<uint8_t>(std::move(v));
  {
    std::lock_guard<std::mutex> lk(emitted_mu());
    emitted()[h->data()] = h;
  }
  *proof = h->data();
  *len = h->size();
  return 0;
}

// Hands every proof of a batch to the caller.  If one hand-over fails, the proofs already
// handed out are released the way the caller would (bfz_free: they are emitted() vectors, not
// malloc'd), every slot is cleared, and the error propagates.  fail_at injects that failure at
// job fail_at (bfz_selftest only).
static void emit_all(std::vector<std::vector<uint8_t>>& v, uint8_t** proofs, size_t* lens,
                     size_t fail_at) {
  for (size_t i = 0; i < v.size(); i++) {
    try {
      if (i == fail_at) throw std::runtime_error("emit: injected failure");
      emit(std::move(v[i]), &proofs[i], &lens[i]);
    } catch (...) {
      for (size_t k = 0; k < i; k++) {
        bfz_free(proofs[k]);
        proofs[k] = nullptr;
        lens[k] = 0;
      }
      throw;
    }
  }
}

int bfz_selftest(const char* name) {
  return guarded([&] {
    const std::string what = name ? name : "";
    if (what == "emit_rollback") {
      size_t before;
      {
        std::lock_guard<std::mutex> lk(emitted_mu());
        before = emitted().size();
      }
      std::vector<std::vector<uint8_t>> v(4, std::vector<uint8_t>(1000, 7));
      uint8_t* proofs[4] = {};
      size_t lens[4] = {};
      bool threw = false;
      try {
        emit_all(v, proofs, lens, 2);
      } catch (const std::exception&) {
        threw = true;
      }
      size_t after;
      {
        std::lock_guard<std::mutex> lk(emitted_mu());
        after = emitted().size();
      }
      if (!threw) throw std::runtime_error("selftest emit_rollback: no failure raised");
      for (int k = 0; k < 4; k++)
        if (proofs[k] || lens[k]) throw std::runtime_error("selftest emit_rollback: slot not cleared");
      if (after != before) throw std::runtime_error("selftest emit_rollback: emitted proofs leaked");
      return 0;
    }
    if (what == "twiddles") {  // the device-built table == the host's running products
      bfz::Twiddles& T = bfz::twiddles();
      T.ensure(bfz::TWIDDLE_LOG_MAX);
      const int L = T.logmax;
      for (int inverse = 0; inverse < 2; inverse++) {
        // the table's levels below 2^20 (host reference in seconds) and the top level's head
        const std::vector<uint32_t> want = bfz::host_twiddles(20, inverse);
        std::vector<uint32_t> got((size_t)1 << L);
        HIP_CHECK(hipMemcpy(got.data(), inverse ? T.inv() : T.fwd(), got.size() * 4,
                            hipMemcpyDeviceToHost));
        if (std::memcmp(got.data(), want.data(), want.size() * 4) != 0)
          throw std::runtime_error("selftest twiddles: levels < 20 differ from the host table");
        for (int k = 20; k < L; k++) {  // every level: first 4096 words and a strided sample
          uint32_t w = kb::two_adic_gen(k + 1);
          if (inverse) w = kb::minv(w);
          const size_t h = (size_t)1 << k;
          uint32_t a = kb::ONE;
          for (size_t j = 0; j < 4096; j++, a = kb::mmul(a, w))
            if (got[h + j] != a) throw std::runtime_error("selftest twiddles: high level head differs");
          for (size_t j = 4097; j < h; j += 65521)
            if (got[h + j] != kb::mpow(w, j)) throw std::runtime_error("selftest twiddles: high level differs");
        }
      }
      return 0;
    }
    throw std::runtime_error("bfz_selftest: unknown test '" + what + "'");
  });
}

// Field-wise serialization of an event stream (no struct padding), for comparing executors.
}  // extern "C"
namespace {
struct EvBlob {
  std::vector<uint8_t> b;
  void u8(uint8_t v) { b.push_back(v); }
  void u32(uint32_t v) { for (int i = 0; i < 4; i++) b.push_back((uint8_t)(v >> (8 * i))); }
  void u64(uint64_t v) { u32((uint32_t)v); u32((uint32_t)(v >> 32)); }
  void acc(const bfz::MemAccess& a) {
    u8(a.kind); u8(a.value); u8(a.prev_value); u32(a.ts); u32(a.prev_ts);
  }
  void ev(const bfz::CpuEvent& e) {
    u32(e.clk); u32(e.pc); u32(e.next_pc); u32(e.mp); u32(e.next_mp); u8(e.mv); u8(e.next_mv);
    acc(e.mv_access); acc(e.next_mv_access);
  }
  void ev(const bfz::AluEvent& e) { u32(e.pc); u8(e.opcode); u8(e.next_mv); u8(e.mv); }
  void ev(const bfz::JumpEvent& e) { u32(e.pc); u32(e.next_pc); u8(e.opcode); u32(e.dst); u8(e.mv); }
  void ev(const bfz::MemInstrEvent& e) { u32(e.clk); u32(e.pc); u8(e.opcode); u32(e.mp); u32(e.next_mp); }
  void ev(const bfz::IoEvent& e) { u32(e.pc); u8(e.opcode); u32(e.mp); u8(e.mv); }
  void ev(const bfz::MemoryEvent& e) { u32(e.addr); u32(e.init_ts); u32(e.final_ts); u8(e.init_v); u8(e.final_v); }
  template <class T>
  void arr(const T* p, size_t n) {
    u64(n);
    for (size_t i = 0; i < n; i++) ev(p[i]);
  }
};
}  // namespace
extern "C" {

int bfz_execute_events(const char* elf, const uint8_t* in, size_t nin, int executor, uint8_t** out,
                       size_t* len) {
  return guarded([&] {
    bfz::Program p = bfz::Program::parse(elf);
    EvBlob b;
    if (executor == 0) {
      bfz::ExecutionRecord r;
      bfz::execute(p, in, nin, r);
      b.arr(r.cpu.data(), r.cpu.size());
      b.arr(r.alu.data(), r.alu.size());
      b.arr(r.jump.data(), r.jump.size());
      b.arr(r.meminstr.data(), r.meminstr.size());
      b.arr(r.io.data(), r.io.size());
      b.arr(r.memory.data(), r.memory.size());
      b.u64(r.global_clk);
      b.u32(r.pc);
      b.u32(r.mp);
      b.u64(r.output.size());
      b.b.insert(b.b.end(), r.output.begin(), r.output.end());
    } else if (executor == 1) {
      static bfz::HostEvents* h = new bfz::HostEvents();  // reused: exercises the reset path
      bfz::execute_into(p, in, nin, *h);
      b.arr(h->cpu.p, h->cpu.n);
      b.arr(h->alu.p, h->alu.n);
      b.arr(h->jump.p, h->jump.n);
      b.arr(h->meminstr.p, h->meminstr.n);
      b.arr(h->io.p, h->io.n);
      b.arr(h->memory.p, h->memory.n);
      b.u64(h->global_clk);
      b.u32(h->pc);
      b.u32(h->mp);
      b.u64(h->output.size());
      b.b.insert(b.b.end(), h->output.begin(), h->output.end());
    } else {
      throw std::runtime_error("executor must be 0 (record) or 1 (pipeline)");
    }
    return emit(std::move(b.b), out, len);
  });
}

int bfz_trace_device(const char* elf, const uint8_t* in, size_t nin, int chip, uint32_t** out,
                     size_t* height, size_t* width) {
  return guarded([&] {
    if (chip < 0 || chip >= bfz::NUM_CHIPS) throw std::runtime_error("bad chip index");
    bfz::Program p = bfz::Program::parse(elf);
    bfz::ExecutionRecord rec;
    bfz::execute(p, in, nin, rec);
    if (!bfz::chip_included(chip, rec)) return 1;
    bfz::DeviceEvents ev;
    bfz::upload_events(rec, ev, bfz::stream());
    bfz::DeviceTraces dt;
    bfz::generate_traces_device(ev, dt, bfz::stream());
    size_t k = 0;
    while (dt.chips[k] != chip) k++;
    const size_t h = dt.heights[k];
    const int w = bfz::CHIP_INFO[chip].main_w;
    std::vector<uint32_t> cm(h * w);
    HIP_CHECK(hipMemcpyAsync(cm.data(), dt.evals[k].p, cm.size() * 4, hipMemcpyDeviceToHost,
                             bfz::stream()));
    HIP_CHECK(hipStreamSynchronize(bfz::stream()));
    uint32_t* o = (uint32_t*)std::malloc(cm.size() * 4 + 4);
    if (!o) throw std::runtime_error("out of host memory");
    const int logh = bfz::log2i(h);
    for (size_t r = 0; r < h; r++)  // column-major bit-reversed -> row-major natural
      for (int c = 0; c < w; c++) o[r * w + c] = cm[(size_t)c * h + bfz::bitrev32((uint32_t)r, logh)];
    *out = o;
    *height = h;
    *width = w;
    return 0;
  });
}

int bfz_perm_trace(int chip, const uint32_t* main, const uint32_t* prep, size_t n,
                   const uint32_t alpha[4], const uint32_t beta[4], uint32_t** out, size_t* width,
                   uint32_t cumsum[4]) {
  return guarded([&] {
    if (chip < 0 || chip >= bfz::NUM_CHIPS) throw std::runtime_error("bad chip index");
    if (!main || !alpha || !beta || !out || !width || !cumsum) throw std::runtime_error("null argument");
    if (n == 0 || (n & (n - 1)) || n > ((size_t)1 << 23)) throw std::runtime_error("height must be a power of two");
    const int mw = bfz::CHIP_INFO[chip].main_w, pwid = bfz::CHIP_INFO[chip].prep_w;
    if (pwid && !prep) throw std::runtime_error("this chip has a preprocessed trace");
    hipStream_t st = bfz::stream();
    auto colmajor = [&](const uint32_t* rm, int w) {
      bfz::DBuf<uint32_t> r(n * w), c(n * w);
      bfz::upload_bulk(r.p, rm, n * w * 4, st);
      if (bfz::count_noncanonical(r.p, n * w, st)) throw std::runtime_error("non-canonical field word");
      bfz::transpose_bitrev(r.p, n, w, c.p, st);
      return c;
    };
    bfz::DBuf<uint32_t> mc = colmajor(main, mw);
    bfz::DBuf<uint32_t> pc;
    if (pwid) pc = colmajor(prep, pwid);
    bfz::PermChallenges ch;
    std::memcpy(ch.alpha.c, alpha, 16);
    kb::EF beta_e;
    std::memcpy(beta_e.c, beta, 16);
    for (int k = 0; k < 4; k++)
      if (ch.alpha.c[k] >= kb::P || beta_e.c[k] >= kb::P) throw std::runtime_error("non-canonical challenge");
    ch.beta_pows[0] = kb::ef_one();
    for (int j = 1; j < 8; j++) ch.beta_pows[j] = kb::ef_mul(ch.beta_pows[j - 1], beta_e);
    const int w = 4 * bfz::perm_width(chip);
    bfz::DBuf<uint32_t> pe(n * w);
    bfz::DBuf<kb::EF> cs(1);
    bfz::DBuf<bfz::PermChallenges> chd(1);
    bfz::upload_async(chd.p, &ch, sizeof(ch), st);
    bfz::perm_trace(chip, mc.p, pwid ? pc.p : nullptr, n, chd.p, pe.p, cs.p, st);
    std::vector<uint32_t> cm(n * w);
    HIP_CHECK(hipMemcpyAsync(cm.data(), pe.p, cm.size() * 4, hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipMemcpyAsync(cumsum, cs.p, 16, hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    uint32_t* o = (uint32_t*)std::malloc(cm.size() * 4 + 4);
    if (!o) throw std::runtime_error("out of host memory");
    const int logh = bfz::log2i(n);
    for (size_t r = 0; r < n; r++)  // column-major bit-reversed -> row-major natural
      for (int c = 0; c < w; c++) o[r * w + c] = cm[(size_t)c * n + bfz::bitrev32((uint32_t)r, logh)];
    *out = o;
    *width = w;
    return 0;
  });
}

// StarkMachine::setup (machine.rs:154-224) runs once per program: the preprocessed commit
// (Program + Byte LDEs and tree, resident in HBM) is cached by program text, so a repeated
// ProverClient::setup of the same ELF costs a map lookup.  The cache keeps the 16 most recently
// used keys; a key stays alive while any bfz_pk handle refers to it.
}  // extern "C"
namespace {
std::shared_ptr<const bfz::ProvingKey> cached_setup(const std::string& elf) {
  struct Entry {
    std::string elf;
    std::shared_ptr<const bfz::ProvingKey> pk;
  };
  static std::vector<Entry>* cache = new std::vector<Entry>();  // most recent last
  constexpr size_t CAP = 16;
  for (size_t i = 0; i < cache->size(); i++)
    if ((*cache)[i].elf == elf) {
      Entry e = std::move((*cache)[i]);
      cache->erase(cache->begin() + i);
      cache->push_back(std::move(e));
      return cache->back().pk;
    }
  std::shared_ptr<const bfz::ProvingKey> pk(bfz::setup(elf).release());
  if (cache->size() == CAP) cache->erase(cache->begin());
  cache->push_back({elf, pk});
  return pk;
}
}  // namespace
extern "C" {

int bfz_setup(const char* elf, bfz_pk** pk, uint32_t vk_commit[8]) {
  return guarded([&] {
    auto k = std::make_unique<bfz_pk>();
    k->pk = cached_setup(elf);
    if (vk_commit) std::memcpy(vk_commit, k->pk->prep.tree.root, 32);
    *pk = k.release();
    return 0;
  });
}

void bfz_pk_free(bfz_pk* pk) {
  std::lock_guard<std::mutex> lk(g_mu);
  delete pk;
}

}  // extern "C"
namespace {
// Program text of a Program chip preprocessed trace (program/mod.rs:66-94: row i = pc i, opcode,
// op_a bytes; rows past the program are zero).  Row 0 is always an instruction (the reference
// asserts a non-empty program); the first row i > 0 whose pc column is not i starts the padding.
std::string program_from_prep_trace(const uint32_t* t, size_t h, size_t w) {
  static const char OPS[8] = {'[', ']', '+', '-', '>', '<', ',', '.'};
  if (w != 6 || h == 0) throw std::runtime_error("pk_from_host: bad Program preprocessed shape");
  std::string src;
  for (size_t i = 0; i < h; i++) {
    const uint32_t pc = kb::from_mont(t[i * 6]);
    if (i > 0 && pc != i) break;
    const uint32_t op = kb::from_mont(t[i * 6 + 1]);
    if (op > 7) throw std::runtime_error("pk_from_host: bad opcode in the Program trace");
    src.push_back(OPS[op]);
  }
  return src;
}
}  // namespace
extern "C" {

int bfz_pk_from_host(const int* chips, const uint32_t* const* traces, const size_t* heights,
                     const size_t* widths, size_t n, const uint32_t commit[8], bfz_pk** pk) {
  return guarded([&] {
    if (!chips || !traces || !heights || !widths || !commit || !pk)
      throw std::runtime_error("null argument");
    if (n != 2) throw std::runtime_error("pk_from_host: expected the Program and Byte preprocessed traces");
    int ip = -1, ib = -1;
    for (size_t i = 0; i < n; i++) {
      if (chips[i] == bfz::CHIP_PROGRAM && ip < 0) ip = (int)i;
      else if (chips[i] == bfz::CHIP_BYTE && ib < 0) ib = (int)i;
      else throw std::runtime_error("pk_from_host: preprocessed chips must be Program and Byte");
    }
    for (size_t i = 0; i < n; i++) {
      const size_t need = (size_t)bfz::CHIP_INFO[chips[i]].prep_w;
      if (widths[i] != need || !traces[i] || heights[i] == 0 || heights[i] > ((size_t)1 << 23))
        throw std::runtime_error(std::string("pk_from_host: bad shape for ") +
                                 bfz::CHIP_INFO[chips[i]].name);
    }
    const std::string src = program_from_prep_trace(traces[ip], heights[ip], widths[ip]);
    const bfz::Program prog = bfz::Program::parse(src);  // unmatched brackets throw
    for (size_t i = 0; i < n; i++) {  // both traces are exactly setup(program)'s
      std::vector<uint32_t> want;
      const size_t h = bfz::prep_trace(chips[i], prog, want);
      if (h != heights[i] || std::memcmp(want.data(), traces[i], want.size() * 4) != 0)
        throw std::runtime_error(std::string("pk_from_host: preprocessed trace of ") +
                                 bfz::CHIP_INFO[chips[i]].name + " is not the program's");
    }
    auto k = std::make_unique<bfz_pk>();
    k->pk = cached_setup(src);
    if (std::memcmp(k->pk->prep.tree.root, commit, 32) != 0)
      throw std::runtime_error("pk_from_host: preprocessed commitment mismatch");
    *pk = k.release();
    return 0;
  });
}

int bfz_pk_commit(const bfz_pk* pk, uint32_t commit[8]) {
  return guarded([&] {
    if (!pk || !commit) throw std::runtime_error("null argument");
    std::memcpy(commit, pk->pk->prep.tree.root, 32);
    return 0;
  });
}

int bfz_prove(const bfz_pk* pk, const uint8_t* in, size_t nin, uint8_t** proof, size_t* len) {
  return guarded([&] { return emit(bfz::prove(*pk->pk, in, nin, opts(), nullptr), proof, len); });
}

int bfz_synchronize(void) {
  return guarded([&] {
    HIP_CHECK(hipDeviceSynchronize());
    return 0;
  });
}

int bfz_prove_traces(const bfz_pk* pk, const int* chips, const uint32_t* const* traces,
                     const size_t* heights, const size_t* widths, size_t nchips, uint8_t** proof,
                     size_t* len) {
  return guarded([&] {
    bfz::DeviceTraces dt;
    bfz::upload_host_traces(chips, traces, heights, widths, nchips, dt, bfz::stream());
    return emit(bfz::prove_device(*pk->pk, dt, opts(), nullptr), proof, len);
  });
}

// ------------------------------------------------ split MachineProver surface (commit / open)
}  // extern "C"
namespace {
bfz::Challenger from_c(const bfz_challenger* c) {
  bfz::Challenger ch;
  if (c->n_input > 8 || c->n_output > 8) throw std::runtime_error("challenger: buffer length > 8");
  for (int i = 0; i < 16; i++) ch.st[i] = c->sponge_state[i];
  for (uint32_t i = 0; i < c->n_input; i++) ch.in[i] = c->input_buffer[i];
  for (uint32_t i = 0; i < c->n_output; i++) ch.out[i] = c->output_buffer[i];
  ch.nin = (int)c->n_input;
  ch.nout = (int)c->n_output;
  // every word the challenger may permute or return must be a canonical Montgomery residue
  for (int i = 0; i < 16; i++)
    if (ch.st[i] >= kb::P) throw std::runtime_error("challenger: non-canonical word");
  for (int i = 0; i < ch.nin; i++)
    if (ch.in[i] >= kb::P) throw std::runtime_error("challenger: non-canonical input word");
  for (int i = 0; i < ch.nout; i++)
    if (ch.out[i] >= kb::P) throw std::runtime_error("challenger: non-canonical output word");
  return ch;
}
void to_c(const bfz::Challenger& ch, bfz_challenger* c) {
  std::memset(c, 0, sizeof *c);
  for (int i = 0; i < 16; i++) c->sponge_state[i] = ch.st[i];
  for (int i = 0; i < ch.nin; i++) c->input_buffer[i] = ch.in[i];
  for (int i = 0; i < ch.nout; i++) c->output_buffer[i] = ch.out[i];
  c->n_input = (uint32_t)ch.nin;
  c->n_output = (uint32_t)ch.nout;
}
}  // namespace
extern "C" {

int bfz_challenger_observe_pk(const bfz_pk* pk, bfz_challenger* ch) {
  return guarded([&] {
    if (!pk || !ch) throw std::runtime_error("null argument");
    bfz::Challenger c = from_c(ch);
    c.observe_digest(pk->pk->prep.tree.root);  // observe_into (prover.rs:595-601)
    for (int i = 0; i < 7; i++) c.observe(0);
    to_c(c, ch);
    return 0;
  });
}

int bfz_main_commit(const bfz_pk* pk, const int* chips, const uint32_t* const* traces,
                    const size_t* heights, const size_t* widths, size_t nchips, bfz_main_data** out,
                    uint32_t root[8]) {
  return guarded([&] {
    if (!out) throw std::runtime_error("null argument");
    auto d = std::make_unique<bfz_main_data>();
    if (pk) d->pk = pk->pk;  // the commit itself does not depend on the key
    bfz::upload_host_traces(chips, traces, heights, widths, nchips, d->md.dt, bfz::stream());
    bfz::commit_main(d->md);
    if (root) std::memcpy(root, d->md.mainr.tree.root, 32);
    *out = d.release();
    return 0;
  });
}

int bfz_record_main_commit(const bfz_pk* pk, const bfz_record* rec, bfz_main_data** out,
                           uint32_t root[8]) {
  return guarded([&] {
    if (!pk || !rec || !out) throw std::runtime_error("null argument");
    auto d = std::make_unique<bfz_main_data>();
    d->pk = pk->pk;
    bfz::generate_traces_device(rec->ev, d->md.dt, bfz::stream());
    bfz::commit_main(d->md);
    if (root) std::memcpy(root, d->md.mainr.tree.root, 32);
    *out = d.release();
    return 0;
  });
}

int bfz_open(const bfz_pk* pk, bfz_main_data* data, bfz_challenger* ch, uint8_t** proof,
             size_t* len) {
  return guarded([&] {
    if (!pk || !data || !ch) throw std::runtime_error("null argument");
    if (data->pk && data->pk != pk->pk)
      throw std::runtime_error("open: main data was committed for another key");
    bfz::Challenger after;
    emit(bfz::open_main(*pk->pk, data->md, from_c(ch), opts(), &after), proof, len);
    to_c(after, ch);  // MachineProver::open advances its &mut challenger
    return 0;
  });
}

void bfz_main_data_free(bfz_main_data* data) {
  std::lock_guard<std::mutex> lk(g_mu);
  delete data;
}

int bfz_prove_batch(const bfz_pk* pk, const uint8_t* const* stdins, const size_t* nins,
                    size_t njobs, int exec_threads, uint8_t** proofs, size_t* proof_lens,
                    bfz_batch_stats* stats) {
  return guarded([&] {
    if (!pk || (njobs && (!stdins || !nins || !proofs || !proof_lens)))
      throw std::runtime_error("null argument");
    for (size_t i = 0; i < njobs; i++) proofs[i] = nullptr;
    std::vector<bfz::Job> jobs(njobs);
    for (size_t i = 0; i < njobs; i++) jobs[i] = {stdins[i], nins[i]};
    int E = exec_threads;
    if (E <= 0) {
      const char* e = std::getenv("BFZ_EXEC_THREADS");
      E = e ? std::atoi(e) : 3;
    }
    if (E < 1 || E > 64) throw std::runtime_error("exec_threads must be in 1..64");
    bfz::BatchStats bs;
    static const int inflight = [] {  // proofs in flight (lanes); BFZ_INFLIGHT = 1..MAX_LANES
      const char* e = std::getenv("BFZ_INFLIGHT");
      if (!e || !*e) return bfz::DEFAULT_INFLIGHT;
      char* end = nullptr;
      const long v = std::strtol(e, &end, 10);
      if (*end || v < 1 || v > bfz::MAX_LANES)
        throw std::runtime_error(std::string("BFZ_INFLIGHT must be an integer in 1..") +
                                 std::to_string(bfz::MAX_LANES) + ", got '" + e + "'");
      return (int)v;
    }();
    auto v = bfz::prove_batch(*pk->pk, jobs, opts(), E, inflight, &bs);
    emit_all(v, proofs, proof_lens, (size_t)-1);
    if (stats) {
      stats->wall_ms = bs.wall_ms;
      stats->exec_ms = bs.exec_ms;
      stats->upload_ms = bs.upload_ms;
      stats->prove_ms = bs.prove_ms;
      stats->exec_threads = bs.exec_threads;
    }
    return 0;
  });
}

int bfz_verify(const char* elf, const uint32_t vk_commit[8], const uint8_t* proof, size_t len) {
  return guarded([&] {
    std::string why;
    const bfz::ProveOptions o = opts();
    bfz::VerifyOptions vo;
    vo.num_queries = o.num_queries;
    vo.observe_openings = o.observe_openings;
    if (!bfz::verify_proof(elf, vk_commit, proof, len, vo, &why)) {
      g_err = "verification failed: " + why;
      return -3;
    }
    return 0;
  });
}

int bfz_record_new(const bfz_pk* pk, const uint8_t* in, size_t nin, bfz_record** rec,
                   uint64_t* cycles) {
  return guarded([&] {
    bfz::ResidentScope rs;  // the record's device events live outside the lane pools
    auto r = std::make_unique<bfz_record>();
    bfz::HostEvents& h = bfz::scratch_events();
    bfz::execute_into(pk->pk->program, in, nin, h);
    bfz::upload_events(h, pk->pk->program, r->ev, bfz::stream());
    r->cycles = h.global_clk;
    if (cycles) *cycles = h.global_clk;
    *rec = r.release();
    return 0;
  });
}

// The C event structs are the device record's layout (machine.h), so the caller's arrays go to
// HBM as they are.
}  // extern "C"
namespace {
template <class C, class D>
constexpr bool same_size() { return sizeof(C) == sizeof(D) && alignof(C) == alignof(D); }
static_assert(same_size<bfz_cpu_event, bfz::CpuEvent>() && same_size<bfz_alu_event, bfz::AluEvent>() &&
              same_size<bfz_jump_event, bfz::JumpEvent>() &&
              same_size<bfz_mem_instr_event, bfz::MemInstrEvent>() &&
              same_size<bfz_io_event, bfz::IoEvent>() && same_size<bfz_memory_event, bfz::MemoryEvent>(),
              "bfz.h event structs must match machine.h");
static_assert(offsetof(bfz_cpu_event, mv) == offsetof(bfz::CpuEvent, mv) &&
              offsetof(bfz_cpu_event, mv_access) == offsetof(bfz::CpuEvent, mv_access) &&
              offsetof(bfz_cpu_event, next_mv_access) == offsetof(bfz::CpuEvent, next_mv_access) &&
              offsetof(bfz_memory_access, timestamp) == offsetof(bfz::MemAccess, ts) &&
              offsetof(bfz_memory_access, prev_timestamp) == offsetof(bfz::MemAccess, prev_ts) &&
              offsetof(bfz_memory_access, prev_value) == offsetof(bfz::MemAccess, prev_value) &&
              offsetof(bfz_alu_event, mv) == offsetof(bfz::AluEvent, mv) &&
              offsetof(bfz_jump_event, dst) == offsetof(bfz::JumpEvent, dst) &&
              offsetof(bfz_jump_event, mv) == offsetof(bfz::JumpEvent, mv) &&
              offsetof(bfz_mem_instr_event, next_mp) == offsetof(bfz::MemInstrEvent, next_mp) &&
              offsetof(bfz_io_event, mv) == offsetof(bfz::IoEvent, mv) &&
              offsetof(bfz_memory_event, final_value) == offsetof(bfz::MemoryEvent, final_v),
              "bfz.h event field offsets must match machine.h");

template <class D, class C>
void put_events(bfz::DBuf<D>& d, const C* src, size_t n, hipStream_t st) {
  if (n && !src) throw std::runtime_error("record_from_events: null event array");
  d.reset(std::max<size_t>(n, 1));
  bfz::upload_bulk(d.p, src, n * sizeof(D), st);
}
// cpu_memory_access in the normal form: sorted by address (the reference's order is that of a
// HashMap drain, executor.rs:74); one event per address.  Returns the count.
size_t put_memory_events(bfz::DeviceEvents& ev, const bfz_memory_event* src, size_t n, hipStream_t st) {
  if (n && !src) throw std::runtime_error("record_from_events: null event array");
  std::vector<bfz::MemoryEvent> mem(n);
  if (n) std::memcpy(mem.data(), src, n * sizeof(bfz::MemoryEvent));
  std::sort(mem.begin(), mem.end(), [](const bfz::MemoryEvent& a, const bfz::MemoryEvent& b) {
    return a.addr < b.addr;
  });
  for (size_t i = 1; i < mem.size(); i++)
    if (mem[i].addr == mem[i - 1].addr)
      throw std::runtime_error("record_from_events: two memory events for one address");
  put_events(ev.memory, mem.data(), mem.size(), st);
  return mem.size();
}
const bfz::Program& put_program(bfz::DeviceEvents& ev, const bfz::Program& prog, hipStream_t st) {
  ev.prog.reset(std::max<size_t>(prog.instructions.size(), 1));
  HIP_CHECK(hipMemcpyAsync(ev.prog.p, prog.instructions.data(),
                           prog.instructions.size() * sizeof(bfz::Instruction), hipMemcpyHostToDevice, st));
  return prog;
}
static_assert(sizeof(bfz_cycle) == sizeof(bfz::Cycle) && offsetof(bfz_cycle, prev_ts) == offsetof(bfz::Cycle, prev_ts) &&
                  offsetof(bfz_cycle, mv) == offsetof(bfz::Cycle, mv) &&
                  offsetof(bfz_cycle, prev_value) == offsetof(bfz::Cycle, prev_value),
              "bfz.h bfz_cycle must match machine.h Cycle");

void check_cycle_counts(size_t n_cycles, size_t n_memory) {
  if (n_cycles == 0) throw std::runtime_error("record_from_cycles: no cycles");
  const size_t lim = (size_t)1 << 26;  // beyond any committable trace (2^23 rows)
  if (n_cycles > lim || n_memory > 2 * lim)
    throw std::runtime_error("record_from_cycles: event count out of range");
}

// bfz_host_alloc / bfz_host_free: page-locked blocks are kept for reuse (rounded up to 2 MiB,
// up to 8 GiB held), because a caller such as HipProver allocates its hand-over array per proof
// and pinning tens of MB costs milliseconds each time.
class PinnedCache {
 public:
  void* take(size_t bytes) {
    bytes = (bytes + GRAIN - 1) / GRAIN * GRAIN;
    auto it = free_.find(bytes);
    if (it != free_.end() && !it->second.empty()) {
      void* p = it->second.back();
      it->second.pop_back();
      held_ -= bytes;
      return p;
    }
    void* p = bfz::pinned_alloc(bytes);
    if (p) size_of_[p] = bytes;
    return p;
  }
  void give(void* p) {
    if (!p) return;
    auto it = size_of_.find(p);
    if (it == size_of_.end()) return;  // not ours
    if (held_ + it->second > CAP) {
      bfz::pinned_free(p);
      size_of_.erase(it);
      return;
    }
    free_[it->second].push_back(p);
    held_ += it->second;
  }

 private:
  static constexpr size_t GRAIN = (size_t)2 << 20, CAP = (size_t)8 << 30;
  std::unordered_map<size_t, std::vector<void*>> free_;
  std::unordered_map<void*, size_t> size_of_;
  size_t held_ = 0;
};
PinnedCache& pinned_cache() {
  static auto* c = new PinnedCache();  // blocks stay pinned until the process exits
  return *c;
}

// The collectives of the last bfz_record_prove_shard_solo run: (0 all-gather | 1 sum all-reduce,
// this rank's bytes).
std::vector<std::pair<int, uint64_t>>& solo_exchange_log() {
  static auto* v = new std::vector<std::pair<int, uint64_t>>();
  return *v;
}
// ... and the overlapped GPU milliseconds of each (bfz_shard_solo_overlaps)
std::vector<double>& solo_overlap_log() {
  static auto* v = new std::vector<double>();
  return *v;
}

// Copies of the chunked hand-over (bfz_cycles_push) run here, beside the prover stream.
hipStream_t handover_stream() {
  static hipStream_t s = [] {
    hipStream_t st;
    HIP_CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    return st;
  }();
  return s;
}

// The record from cycles already in HBM (ordered on the prover stream): program and memory
// events uploaded, every cycle validated and expanded into the chip events (tracegen.hip).
std::unique_ptr<bfz_record> record_from_device_cycles(const bfz_pk* pk, const bfz::DBuf<bfz::Cycle>& d,
                                                      size_t n_cycles, const bfz_memory_event* memory,
                                                      size_t n_memory) {
  hipStream_t st = bfz::stream();
  auto r = std::make_unique<bfz_record>();
  bfz::DeviceEvents& ev = r->ev;
  const bfz::Program& prog = put_program(ev, pk->pk->program, st);
  ev.n[bfz::CHIP_PROGRAM] = prog.instructions.size();
  const size_t nmem = put_memory_events(ev, memory, n_memory, st);
  bfz::EventCounts n;
  size_t bad = 0;
  bfz::expand_cycles(d.p, n_cycles, ev, n, &bad, st);
  if (bad)
    throw std::runtime_error("record_from_cycles: " + std::to_string(bad) +
                             " cycles out of range (pc outside the program, fields a reference "
                             "record cannot hold, or a successor the executor would not step to)");
  n.memory = nmem;
  n.program = prog.instructions.size();
  bfz::set_event_meta(ev, n, n_cycles);
  r->cycles = n_cycles;
  return r;
}
}  // namespace
extern "C" {

int bfz_record_from_events(const bfz_pk* pk, const bfz_events* e, bfz_record** rec) {
  return guarded([&] {
    bfz::ResidentScope rs;  // the record's device events live outside the lane pools
    if (!pk || !e || !rec) throw std::runtime_error("null argument");
    if (e->n_cpu == 0) throw std::runtime_error("record_from_events: no cpu events");
    const size_t lim = (size_t)1 << 26;  // beyond any committable trace (2^23 rows)
    if (e->n_cpu > lim || e->n_add + e->n_sub > lim || e->n_jump > lim || e->n_io > lim ||
        e->n_memory_instr > lim || e->n_memory > 2 * lim)
      throw std::runtime_error("record_from_events: event count out of range");
    hipStream_t st = bfz::stream();
    auto r = std::make_unique<bfz_record>();
    bfz::DeviceEvents& ev = r->ev;
    put_events(ev.cpu, e->cpu, e->n_cpu, st);
    // AddSubChip rows: add_events then sub_events (alu/mod.rs:72)
    const size_t nalu = e->n_add + e->n_sub;
    if ((e->n_add && !e->add) || (e->n_sub && !e->sub))
      throw std::runtime_error("record_from_events: null event array");
    ev.alu.reset(std::max<size_t>(nalu, 1));
    bfz::upload_bulk(ev.alu.p, e->add, e->n_add * sizeof(bfz::AluEvent), st);
    bfz::upload_bulk(ev.alu.p + e->n_add, e->sub, e->n_sub * sizeof(bfz::AluEvent), st);
    put_events(ev.jump, e->jump, e->n_jump, st);
    put_events(ev.meminstr, e->memory_instr, e->n_memory_instr, st);
    put_events(ev.io, e->io, e->n_io, st);
    const size_t nmem = put_memory_events(ev, e->memory, e->n_memory, st);
    const bfz::Program& prog = put_program(ev, pk->pk->program, st);
    bfz::EventCounts n;
    n.cpu = e->n_cpu;
    n.alu = nalu;
    n.jump = e->n_jump;
    n.meminstr = e->n_memory_instr;
    n.io = e->n_io;
    n.memory = nmem;
    n.program = prog.instructions.size();
    bfz::set_event_meta(ev, n, e->n_cpu);
    if (const size_t bad = bfz::count_invalid_events(ev, st))
      throw std::runtime_error("record_from_events: " + std::to_string(bad) +
                               " events out of range (pc outside the program, opcode or access kind)");
    r->cycles = e->n_cpu;
    *rec = r.release();
    return 0;
  });
}

int bfz_host_alloc(size_t bytes, void** out) {
  return guarded([&] {
    if (!out) throw std::runtime_error("host_alloc: null argument");
    *out = nullptr;
    if (bytes == 0 || bytes > ((size_t)1 << 38)) throw std::runtime_error("host_alloc: size out of range");
    void* p = pinned_cache().take(bytes);
    if (!p) throw std::runtime_error("host_alloc: hipHostMalloc failed");
    *out = p;
    return 0;
  });
}

void bfz_host_free(void* p) {
  std::lock_guard<std::mutex> lk(g_mu);
  pinned_cache().give(p);
}

int bfz_record_from_cycles(const bfz_pk* pk, const bfz_cycle* cycles, size_t n_cycles,
                           const bfz_memory_event* memory, size_t n_memory, bfz_record** rec) {
  return guarded([&] {
    bfz::ResidentScope rs;  // the record's device events live outside the lane pools
    if (!pk || !rec) throw std::runtime_error("null argument");
    check_cycle_counts(n_cycles, n_memory);
    if (!cycles) throw std::runtime_error("record_from_cycles: null cycle array");
    hipStream_t st = bfz::stream();
    bfz::DBuf<bfz::Cycle> d(n_cycles);
    bfz::upload_bulk(d.p, cycles, n_cycles * sizeof(bfz::Cycle), st);
    *rec = record_from_device_cycles(pk, d, n_cycles, memory, n_memory).release();
    return 0;
  });
}

int bfz_cycles_begin(const bfz_pk* pk, size_t n_cycles, bfz_cycle_upload** up) {
  return guarded([&] {
    bfz::ResidentScope rs;  // the record's device events live outside the lane pools
    if (!pk || !up) throw std::runtime_error("null argument");
    check_cycle_counts(n_cycles, 0);
    auto u = std::make_unique<bfz_cycle_upload>();
    u->pk = pk;
    u->n = n_cycles;
    u->d.reset(n_cycles);
    // the pooled buffer may still be read by work queued on the prover stream (the pool is
    // ordered on that stream only): the copy stream starts after everything queued there
    HIP_CHECK(hipEventCreateWithFlags(&u->copied, hipEventDisableTiming));
    HIP_CHECK(hipEventRecord(u->copied, bfz::stream()));
    HIP_CHECK(hipStreamWaitEvent(handover_stream(), u->copied, 0));
    *up = u.release();
    return 0;
  });
}

int bfz_cycles_push(bfz_cycle_upload* up, size_t first, const bfz_cycle* cycles, size_t n) {
  return guarded([&] {
    if (!up || !cycles) throw std::runtime_error("null argument");
    if (n == 0 || first > up->n || n > up->n - first)
      throw std::runtime_error("cycles_push: chunk [" + std::to_string(first) + ", +" +
                               std::to_string(n) + ") outside the " + std::to_string(up->n) +
                               " announced cycles");
    up->ranges.push_back({first, n});
    HIP_CHECK(hipMemcpyAsync(up->d.p + first, cycles, n * sizeof(bfz::Cycle), hipMemcpyHostToDevice,
                             handover_stream()));
    return 0;
  });
}

int bfz_cycles_finish(bfz_cycle_upload* up, const bfz_memory_event* memory, size_t n_memory,
                      bfz_record** rec) {
  std::unique_ptr<bfz_cycle_upload> u(up);  // consumed whatever happens
  return guarded([&] {
    bfz::ResidentScope rs;  // the record's device events live outside the lane pools
    if (!u || !rec) throw std::runtime_error("null argument");
    // the prover stream waits for the last copy on the device (no host synchronisation); done
    // first, so the buffer goes back to the stream-ordered pool after the copies on any path
    HIP_CHECK(hipEventRecord(u->copied, handover_stream()));
    HIP_CHECK(hipStreamWaitEvent(bfz::stream(), u->copied, 0));
    check_cycle_counts(u->n, n_memory);
    std::sort(u->ranges.begin(), u->ranges.end());
    size_t next = 0;
    for (const auto& r : u->ranges) {
      if (r.first != next)
        throw std::runtime_error(r.first < next ? "cycles_finish: a cycle was pushed twice"
                                                : "cycles_finish: cycles missing at " + std::to_string(next));
      next = r.first + r.second;
    }
    if (next != u->n) throw std::runtime_error("cycles_finish: cycles missing at " + std::to_string(next));
    *rec = record_from_device_cycles(u->pk, u->d, u->n, memory, n_memory).release();
    return 0;
  });
}

void bfz_cycles_abort(bfz_cycle_upload* up) {
  if (!up) return;
  std::lock_guard<std::mutex> lk(g_mu);
  (void)hipStreamSynchronize(handover_stream());  // no copy may still write the buffer
  delete up;
}

namespace {
void fill_timings(const bfz::StageTimes& st, bfz_timings* t) {
  if (!t) return;
  t->trace_ms = st.trace;
  t->main_commit_ms = st.main_commit;
  t->perm_ms = st.perm;
  t->quotient_ms = st.quotient;
  t->open_ms = st.open;
  t->fri_ms = st.fri;
  t->total_ms = st.total;
  t->lde_ms = st.lde_ms;
  t->lde_bytes = st.lde_bytes;
  t->lde_calls = st.lde_calls;
  t->ntt_kernel_ms = st.ntt_kernel_ms;
  t->ntt_kernel_bytes = st.ntt_kernel_bytes;
  t->ntt_kernel_launches = st.ntt_kernel_launches;
  t->p2_kernel_ms = st.p2_kernel_ms;
  t->p2_perms = st.p2_perms;
  t->p2_launches = st.p2_launches;
  t->lde_elem_stages = st.lde_elem_stages;
  t->open_kernel_ms = st.open_kernel_ms;
  t->open_kernel_bytes = st.open_kernel_bytes;
  t->open_kernel_launches = st.open_kernel_launches;
  t->reduce_kernel_ms = st.reduce_kernel_ms;
  t->reduce_kernel_bytes = st.reduce_kernel_bytes;
  t->reduce_kernel_launches = st.reduce_kernel_launches;
  t->perm_rows_ms = st.perm_rows;
  t->perm_idft_ms = st.perm_idft;
  t->perm_dft_ms = st.perm_dft;
  t->perm_hash_ms = st.perm_hash;
  t->main_idft_ms = st.main_idft;
  t->main_dft_ms = st.main_dft;
  t->main_hash_ms = st.main_hash;
  t->main_cells = st.main_cells;
  t->perm_cells = st.perm_cells;
}
struct ShardScope {  // installs the shard context for one proof
  explicit ShardScope(bfz::ShardCtx* c) { bfz::shard_ctx() = c; }
  ~ShardScope() { bfz::shard_ctx() = nullptr; }
};
}  // namespace

int bfz_record_prove(const bfz_pk* pk, const bfz_record* rec, uint8_t** proof, size_t* len,
                     bfz_timings* t) {
  return guarded([&] {
    bfz::ProveOptions o = opts();
    o.timing = t != nullptr;
    bfz::StageTimes st;
    auto v = bfz::prove_events(*pk->pk, rec->ev, o, &st);
    fill_timings(st, t);
    const int r = emit(std::move(v), proof, len);
    bfz::host_mark("emitted");
    return r;
  });
}

int bfz_record_prove_repeat(const bfz_pk* pk, const bfz_record* rec, int count, int inflight,
                            uint8_t** proof, size_t* len, double* wall_ms) {
  return guarded([&] {
    if (!pk || !rec || !proof || !len) throw std::runtime_error("null argument");
    if (count < 1 || inflight < 1 || inflight > bfz::MAX_LANES)
      throw std::runtime_error("prove_repeat: count >= 1, inflight 1.." + std::to_string(bfz::MAX_LANES));
    HIP_CHECK(hipStreamSynchronize(bfz::stream()));  // the record is complete for every lane
    const bfz::ProveOptions o = opts();
    const auto t0 = std::chrono::steady_clock::now();
    std::vector<uint8_t> first;
    std::mutex mu;
    std::atomic<int> next{0};
    std::atomic<bool> differ{false}, failed{false};
    bfz::run_lanes(inflight, [&](int) {
      // a lane that throws stops the others at their next proof (the error returns at once,
      // not after the remaining `count` proofs)
      for (int k; !failed.load(std::memory_order_relaxed) && (k = next.fetch_add(1)) < count;) {
        std::vector<uint8_t> v;
        try {
          v = bfz::prove_events(*pk->pk, rec->ev, o, nullptr);
        } catch (...) {
          failed.store(true, std::memory_order_relaxed);
          throw;
        }
        std::lock_guard<std::mutex> lk(mu);
        if (first.empty()) {
          first = std::move(v);
        } else {
          if (v != first) differ = true;
          bfz::release_proof_buffer(std::move(v));
        }
      }
    });
    if (wall_ms)
      *wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (differ) throw std::runtime_error("prove_repeat: proofs of one record differ");
    return emit(std::move(first), proof, len);
  });
}

int bfz_record_prove_sharded(const bfz_pk* pk, const bfz_record* rec, int rank, int world,
                             bfz_allgather_fn allgather, bfz_allreduce_u32_fn allreduce_sum,
                             void* ctx, uint8_t** proof, size_t* len, bfz_timings* t) {
  return guarded([&] {
    if (world < 1 || rank < 0 || rank >= world || (world & (world - 1)))
      throw std::runtime_error("sharded prove: world must be a power of two, 0 <= rank < world");
    if (world > 1 && (!allgather || !allreduce_sum))
      throw std::runtime_error("sharded prove: collectives required");
    bfz::ShardCtx c;
    c.rank = rank;
    c.world = world;
    c.allgather = [&](const void* send, size_t bytes, void* recv) {
      if (allgather(ctx, send, bytes, recv)) throw std::runtime_error("allgather callback failed");
    };
    c.allreduce_sum_u32 = [&](uint32_t* data, size_t n) {
      if (allreduce_sum(ctx, data, n)) throw std::runtime_error("allreduce callback failed");
    };
    ShardScope scope(&c);
    bfz::ProveOptions o = opts();
    o.timing = t != nullptr;
    bfz::StageTimes st;
    auto v = bfz::prove_events(*pk->pk, rec->ev, o, &st);
    fill_timings(st, t);
    return emit(std::move(v), proof, len);
  });
}

int bfz_device_pool_bytes(int lane, uint64_t* bytes) {
  return guarded([&] {
    if (!bytes) throw std::runtime_error("null argument");
    if (lane < 0 || lane >= bfz::MAX_LANES) throw std::runtime_error("lane must be in 0..3");
    *bytes = bfz::lane_pool_bytes(lane);
    return 0;
  });
}

int bfz_shard_solo_exchanges(int* kinds, uint64_t* bytes, size_t cap, size_t* n) {
  return guarded([&] {
    if (!n) throw std::runtime_error("null argument");
    const auto& log = solo_exchange_log();
    *n = log.size();
    for (size_t i = 0; i < log.size() && i < cap; i++) {
      if (kinds) kinds[i] = log[i].first;
      if (bytes) bytes[i] = log[i].second;
    }
    return 0;
  });
}

int bfz_shard_solo_overlaps(double* ms, size_t cap, size_t* n) {
  return guarded([&] {
    if (!n) throw std::runtime_error("null argument");
    const auto& log = solo_overlap_log();
    *n = log.size();
    for (size_t i = 0; i < log.size() && i < cap; i++)
      if (ms) ms[i] = log[i];
    return 0;
  });
}

int bfz_record_prove_shard_solo(const bfz_pk* pk, const bfz_record* rec, int rank, int world,
                                bfz_timings* t) {
  return guarded([&] {
    if (!pk || !rec) throw std::runtime_error("null argument");
    if (world < 2 || rank < 0 || rank >= world || (world & (world - 1)))
      throw std::runtime_error("shard solo: world must be a power of two >= 2, 0 <= rank < world");
    bfz::ShardCtx c;
    c.rank = rank;
    c.world = world;
    c.solo = true;
    // the exchanges are no-ops (receive buffers keep what they hold), logged for the bench's
    // collective-time model (bfz_shard_solo_exchanges)
    auto& log = solo_exchange_log();
    log.clear();
    std::vector<const double*> ov;  // the overlap slot of each collective (filled by the events)
    c.allgather = [&log, &ov, &c](const void*, size_t bytes, void*) {
      log.push_back({0, bytes});
      ov.push_back(c.pending_overlap);
    };
    c.allreduce_sum_u32 = [&log, &ov](uint32_t*, size_t n) {
      log.push_back({1, n * 4});
      ov.push_back(nullptr);
    };
    ShardScope scope(&c);
    bfz::ProveOptions o = opts();
    o.timing = t != nullptr;  // t == nullptr: no stage events or kernel probes (wall-clock runs)
    bfz::StageTimes st;
    (void)bfz::prove_events(*pk->pk, rec->ev, o, t ? &st : nullptr);  // not a proof: discarded
    if (t) fill_timings(st, t);
    auto& olog = solo_overlap_log();  // the proof's events have resolved into the slots
    olog.assign(ov.size(), 0.0);
    for (size_t i = 0; i < ov.size(); i++)
      if (ov[i]) olog[i] = *ov[i];
    return 0;
  });
}

int bfz_commit_fri_sharded(const uint32_t* d_cols, int log_n, size_t w_local, int rank, int world,
                           uint32_t* d_send, uint32_t* d_recv, bfz_alltoall_fn alltoall,
                           bfz_allgather_fn allgather, void* ctx, uint32_t* out, size_t cap,
                           size_t* nwords) {
  return guarded([&] {
    if (world < 1 || rank < 0 || rank >= world || (world & (world - 1)))
      throw std::runtime_error("pcs: world must be a power of two, 0 <= rank < world");
    if (log_n < 1 || log_n > 27) throw std::runtime_error("pcs: log_n out of range");
    if (world > 1 && (!alltoall || !allgather)) throw std::runtime_error("pcs: collectives required");
    if (!d_cols || !out || !nwords) throw std::runtime_error("pcs: null argument");
    bfz::ShardCtx c;
    c.rank = rank;
    c.world = world;
    c.allgather = [&](const void* send, size_t bytes, void* recv) {
      if (allgather(ctx, send, bytes, recv)) throw std::runtime_error("allgather callback failed");
    };
    ShardScope scope(world > 1 ? &c : nullptr);
    const bfz::PcsShardedResult r = bfz::commit_fri_sharded(
        d_cols, log_n, (int)w_local, d_send, d_recv,
        [&] {
          if (alltoall(ctx)) throw std::runtime_error("alltoall callback failed");
        },
        bfz::stream());
    const size_t need = 8 + 8 * r.fri_roots.size() + 4;
    *nwords = need;
    if (cap < need) throw std::runtime_error("pcs: output buffer too small");
    std::memcpy(out, r.root, 32);
    for (size_t i = 0; i < r.fri_roots.size(); i++) std::memcpy(out + 8 + 8 * i, r.fri_roots[i].data(), 32);
    std::memcpy(out + 8 + 8 * r.fri_roots.size(), r.final_value.c, 16);
    return 0;
  });
}

void bfz_record_free(bfz_record* rec) { delete rec; }

int bfz_set_pcs_variant(int observe_openings) {
  return guarded([&] {
    if (observe_openings < -1 || observe_openings > 1)
      throw std::runtime_error("observe_openings must be -1 (environment), 0 or 1");
    g_observe_openings = observe_openings;
    return 0;
  });
}

int bfz_set_fault_injection(int mask) {
  return guarded([&] {
    if (mask & ~1) throw std::runtime_error("fault mask: bit 0 (device challenger) only");
    g_fault = mask;
    return 0;
  });
}

int bfz_proof_to_bincode(const uint8_t* proof, size_t len, int field_repr, uint8_t** out,
                         size_t* out_len) {
  return guarded([&] {
    if (field_repr != 0 && field_repr != 1) throw std::runtime_error("field_repr must be 0 or 1");
    const bfz::ShardProof pf = bfz::decode_bfz1(proof, len);
    return emit(bfz::encode_bincode(pf, (bfz::FieldRepr)field_repr), out, out_len);
  });
}

int bfz_proof_from_bincode(const uint8_t* bytes, size_t len, int field_repr, uint8_t** out,
                           size_t* out_len) {
  return guarded([&] {
    if (field_repr != 0 && field_repr != 1) throw std::runtime_error("field_repr must be 0 or 1");
    const bfz::ShardProof pf = bfz::decode_bincode(bytes, len, (bfz::FieldRepr)field_repr);
    return emit(bfz::encode_bfz1(pf), out, out_len);
  });
}

int bfz_verify_bincode(const char* elf, const uint32_t vk_commit[8], const uint8_t* bytes,
                       size_t len, int field_repr) {
  return guarded([&] {
    if (field_repr != 0 && field_repr != 1) throw std::runtime_error("field_repr must be 0 or 1");
    std::string why;
    const bfz::ProveOptions o = opts();
    bfz::VerifyOptions vo;
    vo.num_queries = o.num_queries;
    vo.observe_openings = o.observe_openings;
    bfz::ShardProof pf;
    try {
      pf = bfz::decode_bincode(bytes, len, (bfz::FieldRepr)field_repr);
    } catch (const std::exception& e) {
      g_err = std::string("verification failed: ") + e.what();
      return -3;
    }
    if (!bfz::verify_shard(elf, vk_commit, pf, vo, &why)) {
      g_err = "verification failed: " + why;
      return -3;
    }
    return 0;
  });
}

int bfz_set_num_queries(int q) {
  return guarded([&] {
    if (q < 0 || q > 4096) throw std::runtime_error("num_queries must be in [1, 4096] (0 = FRI_QUERIES/84)");
    g_num_queries = q;
    return 0;
  });
}

int bfz_coset_lde(const uint32_t* evals, size_t n, size_t w, uint32_t shift, uint32_t* out) {
  return guarded([&] {
    if (n == 0 || (n & (n - 1))) throw std::runtime_error("height must be a power of two");
    hipStream_t st = bfz::stream();
    bfz::DBuf<uint32_t> rm(n * w), ev(n * w), lde(2 * n * w), back(2 * n * w);
    HIP_CHECK(hipMemcpyAsync(rm.p, evals, n * w * 4, hipMemcpyHostToDevice, st));
    bfz::transpose_bitrev(rm.p, n, (int)w, ev.p, st);
    bfz::coset_lde(ev.p, n, (int)w, shift, lde.p, st);
    bfz::transpose_to_rowmajor(lde.p, 2 * n, (int)w, back.p, st);
    HIP_CHECK(hipMemcpyAsync(out, back.p, 2 * n * w * 4, hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    return 0;
  });
}

int bfz_commit(const uint32_t* const* mats, const size_t* heights, const size_t* widths,
               size_t nmats, uint32_t root[8]) {
  return guarded([&] {
    hipStream_t st = bfz::stream();
    bfz::Round r;
    r.mats.resize(nmats);
    std::vector<bfz::DBuf<uint32_t>> evs(nmats);
    for (size_t i = 0; i < nmats; i++) {
      const size_t n = heights[i], w = widths[i];
      if (n == 0 || (n & (n - 1))) throw std::runtime_error("height must be a power of two");
      bfz::DBuf<uint32_t> rm(n * w);
      evs[i].reset(n * w);
      HIP_CHECK(hipMemcpyAsync(rm.p, mats[i], n * w * 4, hipMemcpyHostToDevice, st));
      bfz::transpose_bitrev(rm.p, n, (int)w, evs[i].p, st);
      HIP_CHECK(hipStreamSynchronize(st));
      bfz::commit_lde(r.mats[i], evs[i].p, n, (int)w, kb::ONE, st);
    }
    r.commit(st);
    std::memcpy(root, r.tree.root, 32);
    return 0;
  });
}

int bfz_poseidon2_permute(uint32_t* states, size_t n) {
  return guarded([&] {
    hipStream_t st = bfz::stream();
    bfz::DBuf<uint32_t> d(16 * n);
    HIP_CHECK(hipMemcpyAsync(d.p, states, 16 * n * 4, hipMemcpyHostToDevice, st));
    bfz::poseidon2_batch(d.p, n, st);
    HIP_CHECK(hipMemcpyAsync(states, d.p, 16 * n * 4, hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    return 0;
  });
}

int bfz_poseidon2_permute_small(uint32_t* states, size_t n) {
  return guarded([&] {
    hipStream_t st = bfz::stream();
    bfz::DBuf<uint32_t> d(16 * n);
    HIP_CHECK(hipMemcpyAsync(d.p, states, 16 * n * 4, hipMemcpyHostToDevice, st));
    bfz::poseidon2_batch_small(d.p, n, st);
    HIP_CHECK(hipMemcpyAsync(states, d.p, 16 * n * 4, hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    return 0;
  });
}

}  // extern "C"
