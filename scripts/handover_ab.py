"""Chunk-size A/B of the pipelined drop-in hand-over (bench.py compiled_handover): the compiled
CycleArrays::new stand-in converts the headline record's cpu_events in chunks of `chunk` cycles,
pushing each to the device (bfz_cycles_push) as soon as it is written, then bfz_cycles_finish +
bfz_record_prove.  Prints, per chunk size, the pipelined and sequential totals (ms from the Rust-
layout events to the proof) and the time until the last chunk was pushed.

usage (GPU box, repo root): python3 scripts/handover_ab.py
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "zkvm-brainfuck_amd"))

import bench  # noqa: E402
from bfz import _lib, events as _e, guests, sdk  # noqa: E402


def main():
    _lib.init(0)
    client = sdk.ProverClient(device=0)
    prog = guests.FIBO_X4
    pk, _ = client.setup(prog)
    rec = _e.ExecutionRecordArrays.from_executor(prog, bytes([255]))

    def prove(drec):
        ptr = ctypes.POINTER(ctypes.c_uint8)()
        plen = ctypes.c_size_t()
        _lib.check(_lib.lib().bfz_record_prove(ctypes.c_void_p(pk.handle), ctypes.c_void_p(drec.handle),
                                               ctypes.byref(ptr), ctypes.byref(plen), None))
        return _lib.take_bytes(ptr, plen.value)

    import time

    def best(one, steps=4):
        one()
        times, pf = [], None
        for _ in range(steps):
            t0 = time.perf_counter()
            pf = one()
            times.append((time.perf_counter() - t0) * 1e3)
        return min(times), pf

    cyc = _e.cycles_from_record(rec, pinned=True)
    ref_ms, ref = best(lambda: prove(_e.record_from_cycles(pk, cyc, rec.memory)))
    print(f"record_from_cycles (pinned, one DMA) + prove: {ref_ms:.3f} ms", flush=True)
    # the parts: hand-over alone (host time until the record exists) and the proof alone
    sa = _e.CycleArraysStandin()
    rs = _e.rust_cpu_events(rec)
    out = _e.pinned_empty(len(rs), _e.CYCLE)
    threads, _ = bench.host_threads()
    for label, mk in (("record_from_cycles", lambda: _e.record_from_cycles(pk, cyc, rec.memory)),
                      ("ca_handover 32K", lambda: sa.handover(pk, rs, rec.memory, out, threads, 1 << 15)[0]),
                      ("ca_handover 128K", lambda: sa.handover(pk, rs, rec.memory, out, threads, 1 << 17)[0])):
        hs, ps = [], []
        for _ in range(5):
            t0 = time.perf_counter()
            drec = mk()
            t1 = time.perf_counter()
            pf = prove(drec)
            t2 = time.perf_counter()
            assert pf == ref
            hs.append((t1 - t0) * 1e3)
            ps.append((t2 - t1) * 1e3)
        print(f"{label}: hand-over {min(hs):.3f} ms, then prove {min(ps):.3f} ms", flush=True)
    for chunk in [int(c) for c in os.environ.get("CHUNKS", "8192 32768 131072 524288 4194304").split()]:
        r = bench.compiled_handover(pk, rec, prove, best, ref, chunk)
        print(f"chunk {chunk:8d}: pipelined {r['pipelined_ms']:.3f} ms (last push at "
              f"{r['pipelined_last_push_ms']:.3f}), sequential {r['sequential_ms']:.3f}, "
              f"conversion {r['conversion_ms']:.3f}, threads {r['threads']}", flush=True)


if __name__ == "__main__":
    main()
