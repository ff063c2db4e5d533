// Proof pipeline: execution and event upload of proof k+1 run under prove(k).
//
// The reference proves a batch strictly in sequence -- execute, then generate traces and prove
// (crates/core/machine/src/utils/prove.rs:23-66) -- so the executor sits on the critical path.
// Here three kinds of threads overlap:
//   executor threads   Executor::run into pinned HostEvents (machine.h execute_into), several
//                      jobs at once;
//   uploader thread    in job order, one DMA per event array from pinned memory into one of
//                      NSLOT device event slots, on its own HIP stream;
//   prover lanes       up to MAX_LANES (default 2) proofs in flight, each on its own lane (stream,
//                      pool, mailboxes; the calling thread is lane 0): device trace generation +
//                      the proof, jobs taken in order.
// A device slot is refilled only after the proof that read it has finished generating its
// traces (an event recorded on the prover stream right after tracegen).
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <condition_variable>
#include <cstring>
#include <exception>
#include <mutex>
#include <thread>

#include "pipeline.h"
#include "tracegen.h"

namespace bfz {

namespace {

// BFZ_HOST_TRACE=live: every step of every job on stderr as it happens (where a stalled batch
// stands: executor, uploader or a proof lane).
void btrace(const char* what, size_t j) {
  static const bool on = [] {
    const char* e = std::getenv("BFZ_HOST_TRACE");
    return e && std::strcmp(e, "live") == 0;
  }();
  if (!on) return;
  std::fprintf(stderr, "batch job %zu: %s (lane %d)\n", j, what, lane().id);
  std::fflush(stderr);
}

double ms_since(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

hipStream_t copy_stream() {
  static hipStream_t s = [] {
    hipStream_t st;
    HIP_CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    return st;
  }();
  return s;
}

// Device event arrays of one pipeline slot: plain hipMalloc memory (not the stream-ordered
// pools, which are ordered on the lanes' streams only), grown on demand and kept for the process.
// Job j uses slot j % NSLOT: every lane can hold a slot while one more takes the next upload.
constexpr int NSLOT = MAX_LANES + 1;
struct EventSlot {
  static constexpr int N = 6;  // cpu, alu, jump, meminstr, io, memory
  void* p[N] = {};
  size_t cap[N] = {};
  hipEvent_t uploaded = nullptr, consumed = nullptr;
  void ensure(int i, size_t bytes) {
    bytes = std::max<size_t>(bytes, 256);
    if (bytes <= cap[i]) return;
    if (p[i]) HIP_CHECK(hipFree(p[i]));
    HIP_CHECK(hipMalloc(&p[i], bytes));
    cap[i] = bytes;
  }
};
EventSlot* slots() {
  static EventSlot* s = [] {
    auto* x = new EventSlot[NSLOT];
    for (int i = 0; i < NSLOT; i++) {
      HIP_CHECK(hipEventCreateWithFlags(&x[i].uploaded, hipEventDisableTiming));
      HIP_CHECK(hipEventCreateWithFlags(&x[i].consumed, hipEventDisableTiming));
      HIP_CHECK(hipEventRecord(x[i].consumed, stream()));  // "never read yet"
    }
    return x;
  }();
  return s;
}

// Pinned host event buffers, reused across batches (they keep their capacity).
std::vector<HostEvents*>& host_pool() {
  static auto* v = new std::vector<HostEvents*>();
  return *v;
}

template <class T>
void copy_arr(EventSlot& s, int i, const HostEvents::Arr<T>& a, hipStream_t st) {
  s.ensure(i, a.n * sizeof(T));
  if (a.n) HIP_CHECK(hipMemcpyAsync(s.p[i], a.p, a.n * sizeof(T), hipMemcpyHostToDevice, st));
}
template <class T>
DBuf<T> view(const EventSlot& s, int i, size_t n) {
  return DBuf<T>::borrow(static_cast<T*>(s.p[i]), std::max<size_t>(n, 1));
}

}  // namespace

HostEvents& scratch_events() {
  static HostEvents* h = [] {
    auto* x = new HostEvents();
    x->alloc = pinned_alloc;
    x->dealloc = pinned_free;
    return x;
  }();
  return *h;
}

std::vector<std::vector<uint8_t>> prove_batch(const ProvingKey& pk, const std::vector<Job>& jobs,
                                              const ProveOptions& opt, int exec_threads,
                                              int inflight, BatchStats* stats) {
  const size_t n = jobs.size();
  std::vector<std::vector<uint8_t>> proofs(n);
  if (n == 0) return proofs;
  const auto t_start = std::chrono::steady_clock::now();
  const int E = std::max(1, std::min<int>(exec_threads, (int)n));
  const int F = std::max(1, std::min(inflight, MAX_LANES));  // proofs in flight (lanes)
  const size_t H = (size_t)E + F + 1;  // pinned host buffers: E executing + the rest waiting
  auto& hp = host_pool();
  while (hp.size() < H) {
    auto* h = new HostEvents();
    h->alloc = pinned_alloc;
    h->dealloc = pinned_free;
    hp.push_back(h);
  }
  EventSlot* sl = slots();
  hipStream_t cs = copy_stream();
  DBuf<Instruction> prog_d(std::max<size_t>(pk.program.instructions.size(), 1));
  HIP_CHECK(hipMemcpyAsync(prog_d.p, pk.program.instructions.data(),
                           pk.program.instructions.size() * sizeof(Instruction),
                           hipMemcpyHostToDevice, stream()));
  HIP_CHECK(hipStreamSynchronize(stream()));  // read by every lane

  std::mutex mu;
  std::condition_variable cv;
  std::vector<HostEvents*> free_h(hp.begin(), hp.begin() + H);
  std::vector<HostEvents*> executed(n, nullptr);
  std::vector<char> uploaded(n, 0), consumed(n, 0);  // consumed: the slot's event is recorded
  size_t next_job = 0, next_prove = 0;
  bool abort = false;
  std::exception_ptr err;
  std::vector<double> exec_ms(n, 0.0), up_ms(n, 0.0);
  auto fail = [&](std::exception_ptr e) {
    std::lock_guard<std::mutex> lk(mu);
    if (!err) err = e;
    abort = true;
    cv.notify_all();
  };

  auto executor = [&] {
    try {
      for (;;) {
        size_t j;
        HostEvents* h = nullptr;
        {
          // a job and its buffer are taken together, in job order: the job the prover needs
          // next always holds a buffer, so executors that run ahead cannot starve it
          std::unique_lock<std::mutex> lk(mu);
          cv.wait(lk, [&] { return abort || next_job >= n || !free_h.empty(); });
          if (abort || next_job >= n) return;
          j = next_job++;
          h = free_h.back();
          free_h.pop_back();
        }
        btrace("execute", j);
        const auto t0 = std::chrono::steady_clock::now();
        execute_into(pk.program, jobs[j].stdin_data, jobs[j].nin, *h);
        btrace("executed", j);
        exec_ms[j] = ms_since(t0);
        std::lock_guard<std::mutex> lk(mu);
        executed[j] = h;
        cv.notify_all();
      }
    } catch (...) {
      fail(std::current_exception());
    }
  };

  auto uploader = [&] {
    try {
      for (size_t j = 0; j < n; j++) {
        HostEvents* h = nullptr;
        {
          std::unique_lock<std::mutex> lk(mu);
          cv.wait(lk, [&] {
            return abort || (executed[j] && (j < NSLOT || consumed[j - NSLOT]));
          });
          if (abort) return;
          h = executed[j];
        }
        EventSlot& s = sl[j % NSLOT];
        btrace("upload: slot free?", j);
        HIP_CHECK(hipEventSynchronize(s.consumed));  // job j - NSLOT has read this slot
        btrace("upload", j);
        const auto t0 = std::chrono::steady_clock::now();
        copy_arr(s, 0, h->cpu, cs);
        copy_arr(s, 1, h->alu, cs);
        copy_arr(s, 2, h->jump, cs);
        copy_arr(s, 3, h->meminstr, cs);
        copy_arr(s, 4, h->io, cs);
        copy_arr(s, 5, h->memory, cs);
        HIP_CHECK(hipEventRecord(s.uploaded, cs));
        HIP_CHECK(hipEventSynchronize(s.uploaded));
        up_ms[j] = ms_since(t0);
        btrace("uploaded", j);
        std::lock_guard<std::mutex> lk(mu);
        uploaded[j] = 1;
        cv.notify_all();
      }
    } catch (...) {
      fail(std::current_exception());
    }
  };

  std::vector<std::thread> threads;
  for (int e = 0; e < E; e++) threads.emplace_back(executor);
  threads.emplace_back(uploader);
  double prove_ms = 0;
  // F lanes prove jobs in order of arrival (job j on whichever lane takes it), each on its own
  // stream and pool: one proof's latency-bound launches run beside another's bulk kernels
  auto prover = [&](int) {
    for (;;) {
      size_t j;
      HostEvents* h = nullptr;
      {
        std::unique_lock<std::mutex> lk(mu);
        if (abort || next_prove >= n) return;
        j = next_prove++;
        cv.wait(lk, [&] { return abort || uploaded[j]; });
        if (abort) return;
        h = executed[j];
      }
      btrace("prove", j);
      const auto t0 = std::chrono::steady_clock::now();
      EventSlot& s = sl[j % NSLOT];
      DeviceEvents ev;
      ev.cpu = view<CpuEvent>(s, 0, h->cpu.n);
      ev.alu = view<AluEvent>(s, 1, h->alu.n);
      ev.jump = view<JumpEvent>(s, 2, h->jump.n);
      ev.meminstr = view<MemInstrEvent>(s, 3, h->meminstr.n);
      ev.io = view<IoEvent>(s, 4, h->io.n);
      ev.memory = view<MemoryEvent>(s, 5, h->memory.n);
      ev.prog = DBuf<Instruction>::borrow(prog_d.p, prog_d.n);
      set_event_meta(ev, counts_of(*h, pk.program), h->global_clk);
      {  // the host buffer is no longer needed: its DMA is done
        std::lock_guard<std::mutex> lk(mu);
        free_h.push_back(h);
        executed[j] = nullptr;
        cv.notify_all();
      }
      DeviceTraces dt;
      generate_traces_device(ev, dt, stream());
      HIP_CHECK(hipEventRecord(s.consumed, stream()));
      btrace("traces queued", j);
      {
        std::lock_guard<std::mutex> lk(mu);
        consumed[j] = 1;
        cv.notify_all();
      }
      auto pf = prove_device(pk, dt, opt, nullptr);
      const double ms = ms_since(t0);
      btrace("proved", j);
      std::lock_guard<std::mutex> lk(mu);
      proofs[j] = std::move(pf);
      prove_ms += ms;
    }
  };
  try {
    run_lanes(F, [&](int i) {
      try {
        prover(i);
      } catch (...) {
        fail(std::current_exception());
      }
    });
  } catch (...) {
    fail(std::current_exception());
  }
  {
    std::lock_guard<std::mutex> lk(mu);
    if (err) abort = true;
    cv.notify_all();
  }
  for (auto& t : threads) t.join();
  HIP_CHECK(hipStreamSynchronize(stream()));
  if (err) std::rethrow_exception(err);
  if (stats) {
    stats->wall_ms = ms_since(t_start);
    stats->exec_ms = stats->upload_ms = 0;
    for (size_t j = 0; j < n; j++) {
      stats->exec_ms += exec_ms[j];
      stats->upload_ms += up_ms[j];
    }
    stats->prove_ms = prove_ms;
    stats->exec_threads = E;
  }
  return proofs;
}

}  // namespace bfz
