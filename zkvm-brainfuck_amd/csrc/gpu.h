// Device utilities: error checking, a caching device allocator, launch helpers, and the
// device-side data layout used by the prover.
//
// LAYOUT: every evaluation matrix (trace, LDE, permutation trace, quotient chunk) lives in
// HBM COLUMN-MAJOR with rows in BIT-REVERSED order (position t <-> natural row bitrev(t)).
// That is the Merkle-leaf order of TwoAdicFriPcs::commit, so leaf hashing, quotient
// evaluation, FRI reduction and openings all stream columns with unit stride.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <initializer_list>
#include <atomic>
#include <chrono>
#include <map>
#include <mutex>
#include <unordered_map>
#include <unordered_set>
#include <stdexcept>
#include <string>
#include <vector>

#include "kb.h"

namespace bfz {

struct HipError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

#define HIP_CHECK(expr)                                                                  \
  do {                                                                                   \
    hipError_t _e = (expr);                                                              \
    if (_e != hipSuccess)                                                                \
      throw ::bfz::HipError(std::string("HIP error ") + hipGetErrorString(_e) + " at " + \
                            __FILE__ + ":" + std::to_string(__LINE__) + ": " #expr);     \
  } while (0)

#define KCHECK() HIP_CHECK(hipGetLastError())

inline unsigned ceil_div(size_t a, size_t b) { return (unsigned)((a + b - 1) / b); }
inline int log2i(size_t n) {
  int l = 0;
  while (((size_t)1 << l) < n) l++;
  return l;
}
inline uint32_t bitrev32(uint32_t x, int bits) {
  return bits ? (__builtin_bitreverse32(x) >> (32 - bits)) : 0;
}
__device__ __forceinline__ uint32_t dbitrev(uint32_t x, int bits) {
  return bits ? (__brev(x) >> (32 - bits)) : 0;
}

// Size-bucketed caching allocator: proofs reuse the same buffer shapes, so after the first
// proof no hipMalloc/hipFree happens inside the timed region.  A request takes a free buffer of
// its exact size, else the smallest free one of at most twice its size, so a proof of a nearby
// shape reuses cached buffers.  Buffers are never released (trim() is not called by the prover):
// a process that proves shapes whose buffers differ by more than 2x holds a set per size class
// (tests/test_gpu.py test_pool_reuse_across_shapes measures it).
// New buffers below SLAB_BIG are carved from 256 MiB slabs (4 KiB granules), so the first proof
// of a process makes a few dozen hipMalloc calls instead of ~400 between its launches
// (BFZ_POOL_SLABS=0: one hipMalloc per buffer, as before).
class DevicePool {
 public:
  static constexpr size_t SLAB = (size_t)256 << 20, SLAB_BIG = (size_t)32 << 20, GRAIN = 4096;
  // (locked: a buffer may be released from another lane's thread than the one that allocated it)
  void* alloc(size_t bytes) {
    std::lock_guard<std::mutex> lk(mu_);
    bytes = (bytes + 255) & ~(size_t)255;
    if (bytes == 0) bytes = 256;
    const bool carve = bytes < SLAB_BIG && slabs_on();
    if (carve) bytes = (bytes + GRAIN - 1) & ~(GRAIN - 1);
    auto it = free_.lower_bound(bytes);
    if (it != free_.end() && it->first <= 2 * bytes) {
      void* p = it->second.back();
      it->second.pop_back();
      if (it->second.empty()) free_.erase(it);
      return p;
    }
    if (carve) {
      if (slab_left_ < bytes) {
        // the old slab's tail becomes a free buffer of its own size (taken by a later request
        // of half that size or more)
        if (slab_left_ >= GRAIN) {
          size_of_[slab_next_] = slab_left_;
          free_[slab_left_].push_back(slab_next_);
        }
        slab_next_ = (uint8_t*)device_malloc(SLAB);
        slab_left_ = SLAB;
      }
      void* p = slab_next_;
      slab_next_ += bytes;
      slab_left_ -= bytes;
      size_of_[p] = bytes;
      return p;
    }
    void* p = device_malloc(bytes);
    size_of_[p] = bytes;
    own_.insert(p);
    return p;
  }
  // hipMalloc calls made by this pool so far and their host time (diagnostics: host trace)
  uint64_t mallocs() const { return mallocs_; }
  double malloc_ms() const { return malloc_ns_ * 1e-6; }
  size_t bytes() {  // device memory this pool holds (in use + cached)
    std::lock_guard<std::mutex> lk(mu_);
    return held_;
  }
  void release(void* p) {
    if (!p) return;
    std::lock_guard<std::mutex> lk(mu_);
    auto it = size_of_.find(p);
    if (it == size_of_.end()) return;
    free_[it->second].push_back(p);
  }
  void trim() {  // frees the cached buffers that have an allocation of their own (not slab pieces)
    std::lock_guard<std::mutex> lk(mu_);
    for (auto kv = free_.begin(); kv != free_.end();) {
      auto& v = kv->second;
      for (size_t i = 0; i < v.size();) {
        if (!own_.count(v[i])) {
          i++;
          continue;
        }
        (void)hipFree(v[i]);
        held_ -= kv->first;
        size_of_.erase(v[i]);
        own_.erase(v[i]);
        v[i] = v.back();
        v.pop_back();
      }
      kv = v.empty() ? free_.erase(kv) : std::next(kv);
    }
  }
  ~DevicePool() {}

 private:
  static bool slabs_on() {
    static const bool on = [] {
      const char* e = std::getenv("BFZ_POOL_SLABS");
      return !(e && e[0] == '0' && !e[1]);
    }();
    return on;
  }
  void* device_malloc(size_t bytes) {  // (mu_ held)
    void* p = nullptr;
    const auto t0 = std::chrono::steady_clock::now();
    HIP_CHECK(hipMalloc(&p, bytes));
    malloc_ns_ += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
                      std::chrono::steady_clock::now() - t0).count();
    mallocs_++;
    held_ += bytes;
    return p;
  }
  // a proof allocates and releases a few hundred buffers of some tens of sizes: an ordered map of
  // the free sizes (empty lists erased) for the best-fit lookup, a hash map for the releases
  std::map<size_t, std::vector<void*>> free_;
  std::unordered_map<void*, size_t> size_of_;
  std::unordered_set<void*> own_;  // buffers with a hipMalloc of their own (trim() may free them)
  uint8_t* slab_next_ = nullptr;   // the current slab's unused tail
  size_t slab_left_ = 0;
  size_t held_ = 0;
  std::atomic<uint64_t> mallocs_{0}, malloc_ns_{0};
  std::mutex mu_;
};

// Kernel preloading.  The first launch of a kernel loads its file's code object onto the device
// and builds the kernel's launch object: host work that otherwise lands between a fresh
// process's first proof's launches.  Each .hip file registers the kernels a proof launches
// (a static PreloadKernels list); bfz_init runs hipFuncGetAttributes on every one of them, the
// same lookup a first launch makes (BFZ_PRELOAD=0: lazily, at the first launch).
void preload_register(const void* kernel);
struct PreloadKernels {
  PreloadKernels(std::initializer_list<const void*> ks) {
    for (const void* k : ks) preload_register(k);
  }
};
double preload_kernels();  // host ms spent (0 when disabled or already done)

// A proof lane: the device context one proof runs in -- its stream, the stream-ordered buffer
// pool of that stream, the pinned staging arena of its in-proof uploads and its transcript
// mailboxes.  The process has a default lane; bfz_prove_batch and bfz_record_prove_repeat keep
// up to MAX_LANES proofs in flight on as many lanes (one host thread each), so the latency-bound
// launches of one proof (tree tops, the FRI tail, transcript steps) run beside another's bulk
// kernels.
constexpr int MAX_LANES = 4;
constexpr int DEFAULT_INFLIGHT = 2;  // proofs in flight in bfz_prove_batch (profiles/r05)
struct Lane {
  int id = 0;
  hipStream_t stream = nullptr;
  DevicePool pool;
  uint8_t* stage = nullptr;  // pinned arena of upload_async, rewound by staging_reset
  size_t stage_cap = 0, stage_off = 0;
  uint8_t* box = nullptr;  // pinned mailbox of fetch
  size_t box_cap = 0;
  hipEvent_t spin = nullptr;  // spin_sync's event
  // open_impl's pinned buffers (prover.hip): the opened-value groups and the proof's tail
  static constexpr int NGEV = 4;
  hipEvent_t gev[NGEV] = {};
  void* gbox = nullptr;
  size_t gcap = 0;
  uint32_t* tbox = nullptr;
  size_t tcap = 0;
};
Lane& lane();           // this thread's lane (the default lane unless a LaneScope is active)
Lane* lane_at(int i);   // lane i (0 = the default lane), created on first use; lives for the process
size_t lane_pool_bytes(int i);  // device bytes lane i's pool holds (0 if the lane was never used)
struct LaneScope {      // runs this thread's device work on another lane while in scope
  Lane* prev;
  explicit LaneScope(Lane* l);
  ~LaneScope();
};

// body(i) on lane i for i < n, concurrently: lane 0 on the calling thread, the others on
// threads of their own; each thread counts as holding the API lock (the caller holds it for
// the whole call).  Waits for every lane's stream; rethrows the first exception.
void run_lanes(int n, const std::function<void(int)>& body);

DevicePool& pool();  // this thread's allocation pool: its lane's, or the resident pool in a ResidentScope
// Process-lifetime device data (twiddle and power tables, selector tables, proving keys) comes
// from one resident pool, not from the lane that happened to build it, so a lane's pool holds
// exactly its proofs' working set (bfz_device_pool_bytes).
DevicePool& resident_pool();
struct ResidentScope {  // DBuf allocations of this thread go to resident_pool() while in scope
  DevicePool* prev;
  ResidentScope();
  ~ResidentScope();
};

template <class T>
struct DBuf {  // RAII device buffer from the pool (or a borrowed view of memory owned elsewhere)
  T* p = nullptr;
  size_t n = 0;
  bool owned = true;
  DevicePool* from = nullptr;  // the pool it returns to (the lane it was allocated in)
  DBuf() = default;
  explicit DBuf(size_t count) { reset(count); }
  DBuf(const DBuf&) = delete;
  DBuf& operator=(const DBuf&) = delete;
  DBuf(DBuf&& o) noexcept : p(o.p), n(o.n), owned(o.owned), from(o.from) { o.p = nullptr; o.n = 0; }
  DBuf& operator=(DBuf&& o) noexcept {
    if (this != &o) { free(); p = o.p; n = o.n; owned = o.owned; from = o.from; o.p = nullptr; o.n = 0; }
    return *this;
  }
  static DBuf borrow(T* ptr, size_t count) {  // not released on destruction
    DBuf b;
    b.p = ptr;
    b.n = count;
    b.owned = false;
    return b;
  }
  void reset(size_t count) {
    free();
    n = count;
    owned = true;
    from = &pool();
    p = (T*)from->alloc(count * sizeof(T));
  }
  void free() {
    if (p && owned) from->release(p);
    p = nullptr;
    n = 0;
    owned = true;
  }
  ~DBuf() { free(); }
};

// A column-major bit-reversed-row matrix on the device.
struct DevMatrix {
  DBuf<uint32_t> buf;
  size_t height = 0;  // rows (LDE height for committed matrices)
  int width = 0;
  uint32_t* col(int c) const { return buf.p + (size_t)c * height; }
};

// Twiddle tables: T[h + j] = w_{2h}^j for h = 2^k (k < LOGMAX), j < h   (forward)
//                 and w_{2h}^-j                                          (inverse)
// The tables grow (ensure) while other lanes may read them: a grown table is filled before its
// pointer is published (release store, acquire load), and every table ever built stays allocated
// (kernels queued before a growth still read the old one; it is a prefix of the new).
struct Twiddles {
  std::atomic<int> logmax{0};
  const uint32_t* fwd() const { return fwd_.load(std::memory_order_acquire); }
  const uint32_t* inv() const { return inv_.load(std::memory_order_acquire); }
  void ensure(int log_n);

 private:
  std::atomic<const uint32_t*> fwd_{nullptr}, inv_{nullptr};
  std::vector<DBuf<uint32_t>> tables_;
};
Twiddles& twiddles();
constexpr int TWIDDLE_LOG_MAX = 24;  // the first ensure() builds this size (two-adicity of KoalaBear)
std::vector<uint32_t> host_twiddles(int log_n, bool inverse);  // host running products (selftest)

hipStream_t stream();
// Waits for everything queued on stream() if the stream exists (errors ignored): the C ABI's
// error path runs it so no copy into a process-global pinned buffer is still in flight when
// a call returns with an error (the next call may reallocate those buffers).
void quiesce() noexcept;
// roctx range push / pop, bound lazily with dlopen: without the rocprofiler-sdk runtime they
// are no-ops, so the prover does not depend on the profiler library.
void roctx_push(const char* name) noexcept;
void roctx_pop() noexcept;
// Every C entry point runs under one process-wide API lock (capi.cpp guarded()); proof code
// that keeps process-global state (open_impl's pinned mailboxes) checks that it is held.
// Profiler ranges named after the reference's tracing spans (crates/stark/src/prover.rs:63,281,
// 333,355,410,460,575): roctx push / pop, recorded by `rocprofv3 --marker-trace` beside the kernel
// trace.  They are host-side spans (launches plus the transcript's waits), as the reference's are
// host spans around its CPU work; the kernels they enqueue run on the stream under them.
struct Span {
  bool open = false;
  explicit Span(const char* name) { begin(name); }
  ~Span() { end(); }
  Span(const Span&) = delete;
  Span& operator=(const Span&) = delete;
  void begin(const char* name) {
    end();
    roctx_push(name);
    open = true;
  }
  void end() {
    if (open) roctx_pop();
    open = false;
  }
};

int& api_lock_depth();  // per thread
struct ApiLockScope {
  ApiLockScope() { api_lock_depth()++; }
  ~ApiLockScope() { api_lock_depth()--; }
};
// Small host -> device copies inside a proof through a pinned arena (runtime.hip): no host
// stall.  staging_reset() once no earlier copy can be pending (after a stream synchronize).
void upload_async(void* dst, const void* src, size_t bytes, hipStream_t st);
void staging_reset();
// Device -> host copy of a few bytes for the transcript, waited for by spinning (runtime.hip);
// spin_sync waits for everything queued on st so far.
void fetch(void* dst, const void* src, size_t bytes, hipStream_t st);
void spin_sync(hipStream_t st);
// Before a sharded proof's host-call collective: the stream drained by spinning (a blocking wait
// wakes tens of microseconds late, and the GPU idles until the collective returns);
// BFZ_COLL_SPIN=0: hipStreamSynchronize (A/B).
void coll_sync(hipStream_t st);
// The calling thread's lane's pinned staging arena, fetch mailbox and spin event, allocated now
// rather than inside its first proof (setup calls it; runtime.hip).
void lane_host_reserve();
// Timed runs only: the stream busy for `us` microseconds (a one-lane spin on the wall clock),
// so the work queued behind it runs back to back (runtime.hip).
void gpu_delay(double us, hipStream_t st);
// Large pageable host -> device copy through double-buffered pinned chunks (runtime.hip);
// returns when the data has arrived.
void upload_bulk(void* dst, const void* src, size_t bytes, hipStream_t st);

// Many strided 2D word copies in one launch (runtime.hip): rows x width words from src (row
// stride sstride words) to dst (dstride), 16-byte vectors where every copy allows them.
struct Copy2D {
  const uint32_t* src;
  uint32_t* dst;
  size_t sstride, dstride, width, rows;
};
void copy2d_batch(const std::vector<Copy2D>& v, hipStream_t st);

// Per-launch HIP-event timing of one kernel family (the roofline kernel of bench.py):
// when `on`, callers bracket each launch with begin()/end(bytes); collect() resolves the
// events after the stream has drained.  Event creation is host work, so it is only switched
// on for the one instrumented proof.
struct KernelProbe {
  std::atomic<bool> on{false};  // read by every lane's launches, written by timed proofs
  std::vector<std::pair<hipEvent_t, hipEvent_t>> ev;
  std::vector<double> ev_bytes;
  double ms = 0, bytes = 0;
  int launches = 0;
  hipEvent_t begin(hipStream_t st) {
    hipEvent_t e;
    HIP_CHECK(hipEventCreate(&e));
    HIP_CHECK(hipEventRecord(e, st));
    return e;
  }
  std::vector<const char*> ev_tag;
  // BFZ_PROBE_DUMP=1: every timed launch on stderr ("probe <tag> <units> <ms>"), for per-kernel
  // rates (e.g. permutations per second of k_compress against k_hash_leaves)
  bool dump = std::getenv("BFZ_PROBE_DUMP") != nullptr;
  void end(hipEvent_t b, hipStream_t st, double nbytes, const char* tag = "") {
    hipEvent_t e;
    HIP_CHECK(hipEventCreate(&e));
    HIP_CHECK(hipEventRecord(e, st));
    ev.push_back({b, e});
    ev_bytes.push_back(nbytes);
    ev_tag.push_back(tag);
  }
  void collect() {
    for (size_t i = 0; i < ev.size(); i++) {
      HIP_CHECK(hipEventSynchronize(ev[i].second));
      float t = 0;
      HIP_CHECK(hipEventElapsedTime(&t, ev[i].first, ev[i].second));
      if (dump) std::fprintf(stderr, "probe %s %.0f %.5f\n", ev_tag[i], ev_bytes[i], t);
      ms += t;
      bytes += ev_bytes[i];
      launches++;
      HIP_CHECK(hipEventDestroy(ev[i].first));
      HIP_CHECK(hipEventDestroy(ev[i].second));
    }
    ev.clear();
    ev_bytes.clear();
    ev_tag.clear();
  }
  void reset() {
    collect();
    ms = bytes = 0;
    launches = 0;
  }
};
KernelProbe& ntt_probe();  // NTT kernels: k_ntt_r16 (8 B/element), k_lde_mid (12 B/input element)
// Throughput Poseidon2 kernels (k_hash_leaves, k_compress, k_hash_rows8); "bytes" counts
// permutations.
KernelProbe& p2_probe();
KernelProbe& open_probe();    // k_open_partial_batch: algorithmic bytes (fri.hip open_batch)
KernelProbe& reduce_probe();  // k_reduce: algorithmic bytes (fri.hip reduce_range)

}  // namespace bfz
