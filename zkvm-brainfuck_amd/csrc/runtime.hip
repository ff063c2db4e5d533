// Process-wide device state: allocator pool, stream, twiddle tables.
#include <dlfcn.h>

#include "gpu.h"

#include <algorithm>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

namespace bfz {

namespace {
std::mutex g_lanes_mu;
Lane* g_lanes[MAX_LANES] = {};  // intentionally leaked: they live for the process
thread_local Lane* tl_lane = nullptr;
Lane* make_lane(int id) {
  auto* l = new Lane();
  l->id = id;
  HIP_CHECK(hipStreamCreateWithFlags(&l->stream, hipStreamNonBlocking));
  return l;
}
}  // namespace

Lane* lane_at(int i) {
  if (i < 0 || i >= MAX_LANES) throw std::runtime_error("lane index out of range");
  std::lock_guard<std::mutex> lk(g_lanes_mu);
  if (!g_lanes[i]) g_lanes[i] = make_lane(i);
  return g_lanes[i];
}
size_t lane_pool_bytes(int i) {
  if (i < 0 || i >= MAX_LANES) throw std::runtime_error("lane index out of range");
  Lane* l;
  {
    std::lock_guard<std::mutex> lk(g_lanes_mu);
    l = g_lanes[i];
  }
  return l ? l->pool.bytes() : 0;
}
Lane& lane() {
  if (tl_lane) return *tl_lane;
  static Lane* d = lane_at(0);
  return *d;
}
LaneScope::LaneScope(Lane* l) : prev(tl_lane) { tl_lane = l; }
LaneScope::~LaneScope() { tl_lane = prev; }

namespace {
thread_local DevicePool* tl_pool = nullptr;
}
DevicePool& pool() { return tl_pool ? *tl_pool : lane().pool; }
DevicePool& resident_pool() {
  static DevicePool* p = new DevicePool();  // lives for the process
  return *p;
}
ResidentScope::ResidentScope() : prev(tl_pool) { tl_pool = &resident_pool(); }
ResidentScope::~ResidentScope() { tl_pool = prev; }

static std::vector<const void*>& preload_list() {
  static auto* v = new std::vector<const void*>();  // filled by static initialisers
  return *v;
}
void preload_register(const void* kernel) { preload_list().push_back(kernel); }
double preload_kernels() {
  static std::once_flag once;
  double ms = 0;
  std::call_once(once, [&] {
    const char* e = std::getenv("BFZ_PRELOAD");
    if (e && e[0] == '0' && !e[1]) return;
    const auto t0 = std::chrono::steady_clock::now();
    for (const void* k : preload_list()) {
      hipFuncAttributes a;
      HIP_CHECK(hipFuncGetAttributes(&a, k));
    }
    ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  });
  return ms;
}

void run_lanes(int n, const std::function<void(int)>& body) {
  std::exception_ptr err;
  std::mutex mu;
  auto one = [&](int i) {
    try {
      ApiLockScope held;  // the caller holds the API lock for the whole call
      LaneScope ls(lane_at(i));
      body(i);
      HIP_CHECK(hipStreamSynchronize(stream()));
    } catch (...) {
      std::lock_guard<std::mutex> lk(mu);
      if (!err) err = std::current_exception();
    }
  };
  std::vector<std::thread> th;
  for (int i = 1; i < n; i++) th.emplace_back(one, i);
  one(0);
  for (auto& t : th) t.join();
  if (err) std::rethrow_exception(err);
}
hipStream_t stream() { return lane().stream; }

void quiesce() noexcept {
  for (Lane* l : g_lanes)
    if (l && l->stream) (void)hipStreamSynchronize(l->stream);
}

namespace {
struct Roctx {
  int (*push)(const char*) = nullptr;
  int (*pop)() = nullptr;
  Roctx() {
    void* h = dlopen("librocprofiler-sdk-roctx.so", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("/opt/rocm/lib/librocprofiler-sdk-roctx.so", RTLD_NOW | RTLD_LOCAL);
    if (!h) return;
    push = reinterpret_cast<int (*)(const char*)>(dlsym(h, "roctxRangePushA"));
    pop = reinterpret_cast<int (*)()>(dlsym(h, "roctxRangePop"));
    if (!push || !pop) push = nullptr, pop = nullptr;
  }
};
const Roctx& roctx() {
  static const Roctx r;
  return r;
}
}  // namespace
void roctx_push(const char* name) noexcept {
  if (roctx().push) roctx().push(name);
}
void roctx_pop() noexcept {
  if (roctx().pop) roctx().pop();
}

KernelProbe& ntt_probe() {
  static KernelProbe* k = new KernelProbe();
  return *k;
}

KernelProbe& p2_probe() {
  static KernelProbe* k = new KernelProbe();
  return *k;
}

KernelProbe& open_probe() {
  static KernelProbe* k = new KernelProbe();
  return *k;
}

KernelProbe& reduce_probe() {
  static KernelProbe* k = new KernelProbe();
  return *k;
}

// Pinned staging for the small host -> device uploads inside a proof.  A copy from pageable
// memory is staged synchronously by the runtime and leaves the GPU idle until the host catches
// up; from pinned memory it is a plain stream-ordered DMA.  The arena is rewound when a proof
// ends (after its stream synchronize), so a slot is never rewritten while its copy may still
// be pending.
void staging_reset() { lane().stage_off = 0; }

void upload_async(void* dst, const void* src, size_t bytes, hipStream_t st) {
  if (!bytes) return;
  Lane& s = lane();
  if (!s.stage) {
    s.stage_cap = (size_t)8 << 20;
    HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&s.stage), s.stage_cap, hipHostMallocDefault));
  }
  const size_t need = (bytes + 255) & ~(size_t)255;
  if (s.stage_off + need > s.stage_cap) {  // arena full: a synchronous copy is always safe
    HIP_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, st));
    HIP_CHECK(hipStreamSynchronize(st));
    return;
  }
  uint8_t* slot = s.stage + s.stage_off;
  s.stage_off += need;
  std::memcpy(slot, src, bytes);
  HIP_CHECK(hipMemcpyAsync(dst, slot, bytes, hipMemcpyHostToDevice, st));
}

// Bulk host -> device copy of a pageable buffer (host traces, executor events): chunks go
// through two pinned buffers, each filled by several host threads while the DMA of the other
// is in flight, so the copy runs near the PCIe rate instead of the runtime's synchronous
// pageable path.  Returns when the data is on the device.
// Host-to-pinned staging copies split over a persistent set of threads (spawning 8 threads per
// 32 MB chunk cost about as much as the chunk's DMA).  The pool lives for the process; its
// threads sleep between copies.
namespace {
class CopyPool {
 public:
  explicit CopyPool(int nthreads) : nt_(nthreads) {
    for (int i = 1; i < nt_; i++) th_.emplace_back([this, i] { loop(i); });
  }
  // dst[0..n) = src[0..n), the caller's thread taking share 0
  void copy(uint8_t* dst, const uint8_t* src, size_t n) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      dst_ = dst;
      src_ = src;
      n_ = n;
      per_ = (n + nt_ - 1) / nt_;
      pending_ = nt_ - 1;
      gen_++;
    }
    cv_.notify_all();
    part(0);
    std::unique_lock<std::mutex> lk(mu_);
    done_.wait(lk, [this] { return pending_ == 0; });
  }

 private:
  void part(int i) {
    const size_t a = (size_t)i * per_;
    if (a < n_) std::memcpy(dst_ + a, src_ + a, std::min(per_, n_ - a));
  }
  void loop(int i) {
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return gen_ != seen; });
        seen = gen_;
      }
      part(i);
      std::lock_guard<std::mutex> lk(mu_);
      if (--pending_ == 0) done_.notify_all();
    }
  }
  const int nt_;
  std::vector<std::thread> th_;
  std::mutex mu_;
  std::condition_variable cv_, done_;
  uint8_t* dst_ = nullptr;
  const uint8_t* src_ = nullptr;
  size_t n_ = 0, per_ = 0;
  int pending_ = 0;
  uint64_t gen_ = 0;
};
}  // namespace

void upload_bulk(void* dst, const void* src, size_t bytes, hipStream_t st) {
  if (!bytes) return;
  constexpr size_t CHUNK = (size_t)32 << 20;
  constexpr int NTHR = 8;
  struct Bulk {
    uint8_t* buf[2] = {nullptr, nullptr};
    hipEvent_t done[2];
  };
  static Bulk* b = [] {
    auto* x = new Bulk();
    for (int i = 0; i < 2; i++) {
      HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&x->buf[i]), CHUNK, hipHostMallocDefault));
      HIP_CHECK(hipEventCreateWithFlags(&x->done[i], hipEventDisableTiming));
    }
    return x;
  }();
  static CopyPool* pool = new CopyPool(NTHR);  // never destroyed: its threads end with the process
  {  // a page-locked source (bfz_host_alloc, hipHostRegister): one DMA, no staging
    hipPointerAttribute_t a{};
    const hipError_t e = hipPointerGetAttributes(&a, src);
    if (e == hipSuccess && a.type == hipMemoryTypeHost) {
      HIP_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, st));
      HIP_CHECK(hipEventRecord(b->done[0], st));
      HIP_CHECK(hipEventSynchronize(b->done[0]));
      return;
    }
    (void)hipGetLastError();  // pageable memory: the query fails, clear it
  }
  if (bytes <= ((size_t)1 << 20)) {  // small: one staged copy
    const uint8_t* s = static_cast<const uint8_t*>(src);
    HIP_CHECK(hipEventSynchronize(b->done[0]));
    std::memcpy(b->buf[0], s, bytes);
    HIP_CHECK(hipMemcpyAsync(dst, b->buf[0], bytes, hipMemcpyHostToDevice, st));
    HIP_CHECK(hipEventRecord(b->done[0], st));
    HIP_CHECK(hipEventSynchronize(b->done[0]));
    return;
  }
  const uint8_t* s = static_cast<const uint8_t*>(src);
  uint8_t* d = static_cast<uint8_t*>(dst);
  int k = 0;
  for (size_t off = 0; off < bytes; off += CHUNK, k ^= 1) {
    const size_t n = std::min(CHUNK, bytes - off);
    HIP_CHECK(hipEventSynchronize(b->done[k]));  // buffer k's previous DMA has finished
    pool->copy(b->buf[k], s + off, n);
    HIP_CHECK(hipMemcpyAsync(d + off, b->buf[k], n, hipMemcpyHostToDevice, st));
    HIP_CHECK(hipEventRecord(b->done[k], st));
  }
  HIP_CHECK(hipEventSynchronize(b->done[0]));
  HIP_CHECK(hipEventSynchronize(b->done[1]));
}

// Transcript round trips: the host needs a few bytes from the device (a root, the opened
// values, the FRI tail) before it can pick the next challenge, while the GPU idles.  The copy
// goes to a pinned mailbox (a pageable destination makes the runtime stage it), and the host
// spins on an event instead of a stream synchronize that may put the thread to sleep.
void spin_sync(hipStream_t st) {
  Lane& l = lane();
  if (!l.spin) HIP_CHECK(hipEventCreateWithFlags(&l.spin, hipEventDisableTiming));
  const hipEvent_t ev = l.spin;
  HIP_CHECK(hipEventRecord(ev, st));
  for (;;) {
    const hipError_t e = hipEventQuery(ev);
    if (e == hipSuccess) return;
    if (e != hipErrorNotReady) HIP_CHECK(e);
  }
}

void lane_host_reserve() {
  Lane& l = lane();
  if (!l.stage) {
    l.stage_cap = (size_t)8 << 20;
    HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&l.stage), l.stage_cap, hipHostMallocDefault));
  }
  if (!l.box) {
    l.box_cap = (size_t)1 << 16;
    HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&l.box), l.box_cap, hipHostMallocDefault));
  }
  if (!l.spin) HIP_CHECK(hipEventCreateWithFlags(&l.spin, hipEventDisableTiming));
}

void coll_sync(hipStream_t st) {
  static const bool spin = [] {
    const char* e = std::getenv("BFZ_COLL_SPIN");
    return !(e && *e == '0');
  }();
  if (spin) spin_sync(st);
  else HIP_CHECK(hipStreamSynchronize(st));
}

void fetch(void* dst, const void* src, size_t bytes, hipStream_t st) {
  if (!bytes) return;
  Lane& l = lane();
  if (bytes > l.box_cap) {  // no copy into it is pending: every fetch waits for its copy
    if (l.box) HIP_CHECK(hipHostFree(l.box));
    l.box_cap = std::max(bytes, (size_t)1 << 16);
    HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&l.box), l.box_cap, hipHostMallocDefault));
  }
  HIP_CHECK(hipMemcpyAsync(l.box, src, bytes, hipMemcpyDeviceToHost, st));
  spin_sync(st);
  std::memcpy(dst, l.box, bytes);
}

Twiddles& twiddles() {
  static Twiddles* t = new Twiddles();
  return *t;
}

int& api_lock_depth() {
  static thread_local int depth = 0;
  return depth;
}

// Level k of the table (h = 2^k, T[h + j] = w_2h^j) is a strided subset of the powers of
// w_N, N = 2^log_n: w_2h = w_N^(2^(log_n - 1 - k)) (two_adic_gen(b) = g^(2^(24 - b))).  So
// T[h + j] = w_N^e with e = j << (log_n - 1 - k) < N / 2, one product of two short power tables:
// w_N^e = lo[e mod 2^12] * hi[e >> 12].  Field products are exact, so the table is the same
// words as the host's running products (checked by bfz_selftest("twiddles")).
__global__ __launch_bounds__(256) void k_twiddle_table(uint32_t* __restrict__ fwd,
                                                       uint32_t* __restrict__ inv, int log_n,
                                                       const uint32_t* __restrict__ pw, size_t nh) {
  const size_t N = (size_t)1 << log_n;
  for (size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x; idx < N;
       idx += (size_t)gridDim.x * blockDim.x) {
    if (idx == 0) {
      fwd[0] = inv[0] = 0;
      continue;
    }
    const int k = 63 - __clzll((unsigned long long)idx);
    const size_t e = (idx - ((size_t)1 << k)) << (log_n - 1 - k);
    const size_t lo = e & 4095, hi = e >> 12;
    fwd[idx] = kb::mmul(pw[lo], pw[4096 + hi]);
    inv[idx] = kb::mmul(pw[4096 + nh + lo], pw[8192 + nh + hi]);
  }
}

void Twiddles::ensure(int log_n) {
  if (log_n <= logmax) return;
  static std::mutex mu;  // lanes may ask at once; an outgrown table stays allocated (another
  std::lock_guard<std::mutex> lk(mu);  // lane's kernels may still read it)
  if (log_n <= logmax) return;
  if (log_n > 24) throw std::runtime_error("twiddles: KoalaBear's two-adicity is 24");
  // one build covers every transform a proof can ask for (log 24 = an LDE of a 2^23-row trace):
  // 2 x 64 MB of HBM, built on the device in well under a millisecond, so no proof ever grows it
  log_n = std::max(log_n, TWIDDLE_LOG_MAX);
  const size_t N = (size_t)1 << log_n;
  const size_t nh = std::max<size_t>(1, (N / 2) >> 12);
  std::vector<uint32_t> pw(2 * (4096 + nh));
  const uint32_t w = kb::two_adic_gen(log_n), wi = kb::minv(w);
  for (int dir = 0; dir < 2; dir++) {
    uint32_t* lo = pw.data() + dir * (4096 + nh);
    uint32_t* hi = lo + 4096;
    uint32_t a = kb::ONE;
    for (size_t j = 0; j < 4096; j++) { lo[j] = a; a = kb::mmul(a, dir ? wi : w); }
    uint32_t b = kb::ONE;  // a = w^4096 now
    for (size_t j = 0; j < nh; j++) { hi[j] = b; b = kb::mmul(b, a); }
  }
  ResidentScope rs;  // process-lifetime tables, not part of any lane's working set
  DBuf<uint32_t> nf(N), ni(N), dpw(pw.size());
  const hipStream_t st = stream();
  HIP_CHECK(hipMemcpyAsync(dpw.p, pw.data(), pw.size() * 4, hipMemcpyHostToDevice, st));
  hipLaunchKernelGGL(k_twiddle_table, dim3((unsigned)std::min<size_t>(ceil_div(N, 256), 8192)),
                     dim3(256), 0, st, nf.p, ni.p, log_n, (const uint32_t*)dpw.p, nh);
  KCHECK();
  HIP_CHECK(hipStreamSynchronize(st));
  fwd_.store(nf.p, std::memory_order_release);
  inv_.store(ni.p, std::memory_order_release);
  tables_.push_back(std::move(nf));
  tables_.push_back(std::move(ni));
  logmax.store(log_n, std::memory_order_release);
}

// The table the way it was built before the device kernel (running products on the host),
// for bfz_selftest("twiddles").
std::vector<uint32_t> host_twiddles(int log_n, bool inverse) {
  const size_t N = (size_t)1 << log_n;
  std::vector<uint32_t> t(N, 0);
  for (int k = 0; k < log_n; k++) {
    const size_t h = (size_t)1 << k;
    uint32_t w = kb::two_adic_gen(k + 1);
    if (inverse) w = kb::minv(w);
    uint32_t a = kb::ONE;
    for (size_t j = 0; j < h; j++) {
      t[h + j] = a;
      a = kb::mmul(a, w);
    }
  }
  return t;
}

}  // namespace bfz

namespace bfz {
// ------------------------------------------------------------------------ batched 2D copies
constexpr int COPY2D_MAX = 40;  // per launch (kernel-argument space)
struct Copy2DBatch {
  Copy2D c[COPY2D_MAX];
};
template <int V>  // words per access (4: uint4)
__global__ __launch_bounds__(256) void k_copy2d_batch(Copy2DBatch b) {
  const Copy2D c = b.c[blockIdx.y];
  const size_t wv = c.width / V, total = wv * c.rows;
  for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (size_t)gridDim.x * blockDim.x) {
    const size_t r = e / wv, x = (e - r * wv) * V;
    if constexpr (V == 4)
      *reinterpret_cast<uint4*>(c.dst + r * c.dstride + x) =
          *reinterpret_cast<const uint4*>(c.src + r * c.sstride + x);
    else
      c.dst[r * c.dstride + x] = c.src[r * c.sstride + x];
  }
}

void copy2d_batch(const std::vector<Copy2D>& v, hipStream_t st) {
  for (size_t i0 = 0; i0 < v.size(); i0 += COPY2D_MAX) {
    Copy2DBatch b{};
    const int cnt = (int)std::min<size_t>(COPY2D_MAX, v.size() - i0);
    bool vec = true;
    size_t most = 0;
    for (int i = 0; i < cnt; i++) {
      const Copy2D& c = v[i0 + i];
      b.c[i] = c;
      vec = vec && c.width % 4 == 0 && c.sstride % 4 == 0 && c.dstride % 4 == 0 &&
            ((uintptr_t)c.src & 15) == 0 && ((uintptr_t)c.dst & 15) == 0;
      most = std::max(most, c.width * c.rows);
    }
    if (!most) continue;
    const dim3 grid((unsigned)std::min<size_t>(ceil_div(most, (size_t)(vec ? 4 : 1) * 256), 1024),
                    cnt);
    if (vec)
      hipLaunchKernelGGL(k_copy2d_batch<4>, grid, dim3(256), 0, st, b);
    else
      hipLaunchKernelGGL(k_copy2d_batch<1>, grid, dim3(256), 0, st, b);
    KCHECK();
  }
}
}  // namespace bfz

namespace bfz {
// ------------------------------------------------------------------ timed-run helper
// Keeps the stream busy for `us` microseconds (one lane, the constant-rate wall clock), so that
// work the host queues meanwhile then runs back to back: a timed run measures the GPU time of a
// window the way a real run executes it (queued ahead of a blocking collective), without the
// launch gaps the host's probe bookkeeping would leave in it.
__global__ __launch_bounds__(64) void k_delay(long long ticks) {
  const long long t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}

void gpu_delay(double us, hipStream_t st) {
  static const long long khz = [] {
    int dev = 0, r = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&r, hipDeviceAttributeWallClockRate, dev) != hipSuccess || r <= 0)
      r = 100000;  // 100 MHz
    return (long long)r;
  }();
  hipLaunchKernelGGL(k_delay, dim3(1), dim3(64), 0, st, (long long)(us * (double)khz / 1000.0));
  KCHECK();
}
// kernels a proof launches (gpu.h PreloadKernels)
static PreloadKernels preload_runtime{
    (const void*)&k_copy2d_batch<4>,
    (const void*)&k_copy2d_batch<1>};

}  // namespace bfz
