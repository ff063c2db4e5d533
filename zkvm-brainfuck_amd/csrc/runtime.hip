// Process-wide device state: allocator pool, stream, twiddle tables.
#include "gpu.h"

#include <cstring>

namespace bfz {

DevicePool& pool() {
  static DevicePool* p = new DevicePool();  // intentionally leaked: freed by process exit
  return *p;
}

hipStream_t stream() {
  static hipStream_t s = [] {
    hipStream_t st;
    HIP_CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    return st;
  }();
  return s;
}

KernelProbe& ntt_probe() {
  static KernelProbe* k = new KernelProbe();
  return *k;
}

KernelProbe& p2_probe() {
  static KernelProbe* k = new KernelProbe();
  return *k;
}

// Pinned staging for the small host -> device uploads inside a proof.  A copy from pageable
// memory is staged synchronously by the runtime and leaves the GPU idle until the host catches
// up; from pinned memory it is a plain stream-ordered DMA.  The arena is rewound when a proof
// ends (after its stream synchronize), so a slot is never rewritten while its copy may still
// be pending.
namespace {
struct Staging {
  uint8_t* base = nullptr;
  size_t cap = 0, off = 0;
};
Staging& staging() {
  static Staging* s = [] {
    auto* st = new Staging();
    st->cap = (size_t)8 << 20;
    HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&st->base), st->cap, hipHostMallocDefault));
    return st;
  }();
  return *s;
}
}  // namespace

void staging_reset() { staging().off = 0; }

void upload_async(void* dst, const void* src, size_t bytes, hipStream_t st) {
  if (!bytes) return;
  Staging& s = staging();
  const size_t need = (bytes + 255) & ~(size_t)255;
  if (s.off + need > s.cap) {  // arena full: a synchronous copy is always safe
    HIP_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, st));
    HIP_CHECK(hipStreamSynchronize(st));
    return;
  }
  uint8_t* slot = s.base + s.off;
  s.off += need;
  std::memcpy(slot, src, bytes);
  HIP_CHECK(hipMemcpyAsync(dst, slot, bytes, hipMemcpyHostToDevice, st));
}

Twiddles& twiddles() {
  static Twiddles* t = new Twiddles();
  return *t;
}

void Twiddles::ensure(int log_n) {
  if (log_n <= logmax) return;
  size_t N = (size_t)1 << log_n;
  host_fwd.assign(N, 0);
  host_inv.assign(N, 0);
  for (int k = 0; k < log_n; k++) {
    size_t h = (size_t)1 << k;
    uint32_t w = kb::two_adic_gen(k + 1), wi = kb::minv(w);
    uint32_t a = kb::ONE, b = kb::ONE;
    for (size_t j = 0; j < h; j++) {
      host_fwd[h + j] = a;
      host_inv[h + j] = b;
      a = kb::mmul(a, w);
      b = kb::mmul(b, wi);
    }
  }
  // stream-ordered: pooled buffers may still be read by kernels queued on stream()
  fwd.reset(N);
  inv.reset(N);
  HIP_CHECK(hipMemcpyAsync(fwd.p, host_fwd.data(), N * 4, hipMemcpyHostToDevice, stream()));
  HIP_CHECK(hipMemcpyAsync(inv.p, host_inv.data(), N * 4, hipMemcpyHostToDevice, stream()));
  HIP_CHECK(hipStreamSynchronize(stream()));
  logmax = log_n;
}

}  // namespace bfz
