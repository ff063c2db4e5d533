// Compiled stand-in of the Rust drop-in's host conversion (crates/bf-hip-prover/src/lib.rs
// CycleArrays::new), so that the part of HipProver::prove that runs before the C ABI can be timed
// here, where no Rust toolchain exists.  The reference's timer brackets
// prover.prove (crates/core/machine/src/utils/prove.rs:44-46), which for HipProver includes this
// pass over record.cpu_events (crates/core/executor/src/events/cpu.rs:10-28).
//
// The input is laid out as rustc lays out Vec<CpuEvent> (repr(Rust): fields reordered by
// alignment, the two Option<MemoryRecordEnum> as 12-byte tagged unions with the None niche in
// the tag, 48 bytes per event) -- the exact order does not matter for the cost, which is one
// 48-byte read and one 16-byte write per cycle.  Like rayon's par_iter, a persistent pool of
// threads splits the events; the output goes straight into page-locked bfz_host_alloc memory.
//
//   ca_convert   CycleArrays::new as the crate ships it: every cycle converted, then one
//                bfz_record_from_cycles (the caller times the two separately or together)
//   ca_handover  the pipelined form: the events are converted in chunks and each chunk is handed
//                to bfz_cycles_push as soon as it is written, so the DMA of chunk k runs while
//                chunk k+1 is converted; bfz_cycles_finish returns the record
#include <immintrin.h>
#include <pthread.h>
#include <sched.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstddef>
#include <cstdint>
#include <fstream>
#include <functional>
#include <sstream>
#include <string>
#include <mutex>
#include <thread>
#include <vector>

#include "../../../include/bfz.h"

namespace {

struct RsMemoryRecordOpt {  // Option<MemoryRecordEnum>: tag 0 = Read, 1 = Write, 2 = None
  uint8_t tag, value, prev_value, pad;  // prev_value: Write only
  uint32_t timestamp, prev_timestamp;
};
struct RsCpuEvent {
  uint32_t clk, pc, next_pc, mp, next_mp;
  RsMemoryRecordOpt mv_access, next_mv_access;
  uint8_t mv, next_mv, pad[2];
};
static_assert(sizeof(RsCpuEvent) == 48, "CpuEvent as rustc lays it out");
static_assert(sizeof(bfz_cycle) == 16, "bfz_cycle");

inline bfz_cycle cycle_of(const RsCpuEvent& e) {  // lib.rs CycleArrays::new's closure
  bfz_cycle c;
  c.pc = e.pc;
  c.mp = e.mp;
  c.mv = e.mv;
  c.prev_ts = e.mv_access.tag == 2 ? 0 : e.mv_access.prev_timestamp;
  c.prev_value = e.mv_access.tag == 1 ? e.mv_access.prev_value : 0;
  c._pad[0] = c._pad[1] = 0;
  return c;
}

// The CPUs of the caller's NUMA node that this process may run on (empty if unknown): the
// events were written by the executor's thread, so they sit in that node's memory, and on a
// two-socket host a worker on the other socket reads them at a fraction of the local rate.
std::vector<int> node_cpus() {
  cpu_set_t aff;
  if (sched_getaffinity(0, sizeof aff, &aff)) return {};
  const int me = sched_getcpu();
  for (int node = 0; node < 64; node++) {
    std::ifstream f("/sys/devices/system/node/node" + std::to_string(node) + "/cpulist");
    if (!f) continue;
    std::string list;
    std::getline(f, list);
    std::vector<int> cpus;
    std::stringstream ss(list);
    std::string part;
    bool mine = false;
    while (std::getline(ss, part, ',')) {
      const size_t dash = part.find('-');
      const int a = std::stoi(part.substr(0, dash));
      const int b = dash == std::string::npos ? a : std::stoi(part.substr(dash + 1));
      for (int c = a; c <= b; c++) {
        if (c == me) mine = true;
        if (c < CPU_SETSIZE && CPU_ISSET(c, &aff)) cpus.push_back(c);
      }
    }
    if (mine) return cpus;
  }
  return {};
}

// A fixed pool of workers (the caller's thread is worker 0), like rayon's global pool; the
// workers are pinned to CPUs of the caller's NUMA node when the host tells us which those are
// (rayon: ThreadPoolBuilder::spawn_handler can do the same).
class Pool {
 public:
  explicit Pool(int n) : n_(n) {
    const std::vector<int> cpus = node_cpus();
    for (int i = 1; i < n; i++) {
      th_.emplace_back([this, i] { loop(i); });
      if ((int)cpus.size() >= n) {
        cpu_set_t one;
        CPU_ZERO(&one);
        CPU_SET(cpus[(size_t)i % cpus.size()], &one);
        (void)pthread_setaffinity_np(th_.back().native_handle(), sizeof one, &one);
      }
    }
  }
  int size() const { return n_; }
  void run(const std::function<void(int)>& f) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      job_ = &f;
      pending_ = n_ - 1;
      gen_++;
    }
    cv_.notify_all();
    f(0);
    std::unique_lock<std::mutex> lk(mu_);
    done_.wait(lk, [this] { return pending_ == 0; });
    job_ = nullptr;
  }

 private:
  void loop(int id) {
    uint64_t seen = 0;
    for (;;) {
      const std::function<void(int)>* f;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return gen_ != seen; });
        seen = gen_;
        f = job_;
      }
      (*f)(id);
      std::lock_guard<std::mutex> lk(mu_);
      if (--pending_ == 0) done_.notify_one();
    }
  }
  int n_;
  std::vector<std::thread> th_;
  std::mutex mu_;
  std::condition_variable cv_, done_;
  const std::function<void(int)>* job_ = nullptr;
  uint64_t gen_ = 0;
  int pending_ = 0;
};

Pool& pool(int threads) {
  static Pool* p = nullptr;
  if (!p || p->size() != threads) p = new Pool(threads);  // one size per process in practice
  return *p;
}

// Streaming (non-temporal) 16-byte stores: the output is written once and read only by the DMA
// engine, so it need not be read into the cache first; the fence orders the stores before the
// copy that follows.
void convert_range(const RsCpuEvent* ev, bfz_cycle* out, size_t a, size_t b) {
  for (size_t i = a; i < b; i++) {
    const bfz_cycle c = cycle_of(ev[i]);
    __m128i v;
    __builtin_memcpy(&v, &c, 16);
    _mm_stream_si128(reinterpret_cast<__m128i*>(out + i), v);
  }
  _mm_sfence();
}

}  // namespace

extern "C" {

// CycleArrays::new: out[i] = the bfz_cycle of ev[i], split over `threads` workers.
int ca_convert(const void* events, size_t n, bfz_cycle* out, int threads) {
  if (!events || !out || threads < 1) return -1;
  const auto* ev = static_cast<const RsCpuEvent*>(events);
  const size_t per = (n + threads - 1) / threads;
  pool(threads).run([&](int t) {
    const size_t a = std::min(n, (size_t)t * per), b = std::min(n, a + per);
    convert_range(ev, out, a, b);
  });
  return 0;
}

// The pipelined hand-over: chunks of `chunk` cycles are claimed by the workers in order,
// converted into out (page-locked) and pushed at once; returns the bfz_cycles_* status.
// conv_ms (optional): the wall time until the last chunk was pushed.
int ca_handover(const bfz_pk* pk, const void* events, size_t n, const bfz_memory_event* memory,
                size_t n_memory, bfz_cycle* out, int threads, size_t chunk, bfz_record** rec,
                double* conv_ms) {
  if (!pk || !events || !out || !rec || threads < 1 || chunk == 0) return -1;
  const auto t0 = std::chrono::steady_clock::now();
  const auto* ev = static_cast<const RsCpuEvent*>(events);
  bfz_cycle_upload* up = nullptr;
  int rc = bfz_cycles_begin(pk, n, &up);
  if (rc) return rc;
  const size_t nchunks = (n + chunk - 1) / chunk;
  std::atomic<size_t> next{0};
  std::atomic<int> err{0};
  pool(threads).run([&](int) {
    for (size_t k; (k = next.fetch_add(1)) < nchunks;) {
      const size_t a = k * chunk, b = std::min(n, a + chunk);
      convert_range(ev, out, a, b);
      const int r = bfz_cycles_push(up, a, out + a, b - a);
      if (r) err.store(r);
    }
  });
  if (conv_ms)
    *conv_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  if (err.load()) {
    bfz_cycles_abort(up);
    return err.load();
  }
  return bfz_cycles_finish(up, memory, n_memory, rec);
}

}  // extern "C"
