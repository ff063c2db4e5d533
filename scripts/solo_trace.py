#!/usr/bin/env python3
"""One rank's share of an N-GPU sharded proof (bfz_record_prove_shard_solo) run a few times, for
a rocprofv3 --kernel-trace of the share (scripts/timeline.py reads it: each proof starts at its
k_trace_cpu).  python3 scripts/solo_trace.py WORLD RANK [REPS] [untimed]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zkvm-brainfuck_amd"))


def main():
    world, rank = int(sys.argv[1]), int(sys.argv[2])
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    timed = not (len(sys.argv) > 4 and sys.argv[4] == "untimed")  # untimed: no probes / events
    from bfz import _lib, guests, sdk
    _lib.init(0)
    L = _lib.lib()
    client = sdk.ProverClient()
    pk, _ = client.setup(guests.FIBO_X4)
    rec = ctypes.c_void_p()
    cyc = ctypes.c_uint64()
    buf, n = _lib.u8buf(bytes([255]))
    _lib.check(L.bfz_record_new(ctypes.c_void_p(pk.handle), buf, n, ctypes.byref(rec), ctypes.byref(cyc)))
    import time
    for _ in range(reps):
        tm = _lib.Timings()
        _lib.check(L.bfz_synchronize())
        t0 = time.perf_counter()
        _lib.check(L.bfz_record_prove_shard_solo(ctypes.c_void_p(pk.handle), rec, rank, world,
                                                 ctypes.byref(tm) if timed else None))
        _lib.check(L.bfz_synchronize())
        wall = (time.perf_counter() - t0) * 1e3
        print({"wall_ms": round(wall, 3), **{k: round(v, 3) for k, v in tm.as_dict().items()
                                              if k.endswith("_ms") and v}}, flush=True)
    L.bfz_record_free(rec)


if __name__ == "__main__":
    main()
