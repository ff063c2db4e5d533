#!/usr/bin/env python3
"""hipMalloc cost on this part (the first proof's pool fill): one large
allocation against many smaller ones of the same total, then the same sizes again after a free
(does the runtime keep freed memory mapped?).  ctypes over libamdhip64 only; prints JSON."""
import ctypes
import json
import time

hip = ctypes.CDLL("libamdhip64.so")
hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
hip.hipFree.argtypes = [ctypes.c_void_p]
hip.hipMemset.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t]


def ok(e):
    if e != 0:
        raise SystemExit(f"hip error {e}")


def alloc(sizes):
    ps = []
    t0 = time.perf_counter()
    for s in sizes:
        p = ctypes.c_void_p()
        ok(hip.hipMalloc(ctypes.byref(p), s))
        ps.append(p)
    return ps, (time.perf_counter() - t0) * 1e3


def free(ps):
    t0 = time.perf_counter()
    for p in ps:
        ok(hip.hipFree(p))
    return (time.perf_counter() - t0) * 1e3


def main():
    ok(hip.hipSetDevice(0))
    ok(hip.hipFree(None))  # context creation outside the timings
    GiB = 1 << 30
    out = {}
    ps, out["one_9GiB_ms"] = alloc([9 * GiB])
    t0 = time.perf_counter()
    ok(hip.hipMemset(ps[0], 0, 9 * GiB))
    ok(hip.hipDeviceSynchronize())
    out["first_touch_memset_9GiB_ms"] = (time.perf_counter() - t0) * 1e3
    t0 = time.perf_counter()
    ok(hip.hipMemset(ps[0], 0, 9 * GiB))
    ok(hip.hipDeviceSynchronize())
    out["second_memset_9GiB_ms"] = (time.perf_counter() - t0) * 1e3
    out["free_one_ms"] = free(ps)
    ps, _ = alloc([9 * GiB])
    t0 = time.perf_counter()
    ok(hip.hipMemset(ps[0], 0, 9 * GiB))
    ok(hip.hipDeviceSynchronize())
    out["memset_after_free_realloc_9GiB_ms"] = (time.perf_counter() - t0) * 1e3
    free(ps)
    ps, out["288x32MiB_ms"] = alloc([32 << 20] * 288)
    out["free_288_ms"] = free(ps)
    ps, out["one_9GiB_again_ms"] = alloc([9 * GiB])
    free(ps)
    ps, out["4x2304MiB_ms"] = alloc([2304 << 20] * 4)
    free(ps)
    ps, out["one_1GiB_ms"] = alloc([GiB])
    free(ps)
    ps, out["one_64MiB_ms"] = alloc([64 << 20])
    free(ps)
    print(json.dumps({k: round(v, 3) for k, v in out.items()}), flush=True)


if __name__ == "__main__":
    main()
