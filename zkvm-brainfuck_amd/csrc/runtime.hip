// Process-wide device state: allocator pool, stream, twiddle tables.
#include "gpu.h"

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
