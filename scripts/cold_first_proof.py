#!/usr/bin/env python3
"""Cold first proof: one fresh process does what a reference user's
`ProverClient::prove().run()` process does -- init, setup, record, ONE prove -- and reports each
phase's wall time, then proves the same record twice more (the warm proofs) for comparison.

Prints one JSON line.  bench.py runs this file as a child process (no profiler, nothing else in
the process) and copies its figures into the bench line as cold_first_proof_ms /
first_prove_after_setup_ms.

  python scripts/cold_first_proof.py [--program fibo_x4|fibo17|hello] [--warm 2]
"""
import argparse
import ctypes
import json
import os
import sys
import time

T_START = time.perf_counter()
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zkvm-brainfuck_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--program", default="fibo_x4")
    ap.add_argument("--warm", type=int, default=2)
    ap.add_argument("--device", type=int, default=0)
    args = ap.parse_args()
    from bfz import _lib, guests, sdk
    prog, stdin = {"fibo_x4": (guests.FIBO_X4, bytes([255])),
                   "fibo17": (guests.FIBO, bytes([17])),
                   "hello": (guests.HELLO, b"")}[args.program]
    L = _lib.lib()
    t = {}
    t0 = time.perf_counter()
    _lib.init(args.device)
    t["init_ms"] = (time.perf_counter() - t0) * 1e3
    t0 = time.perf_counter()
    client = sdk.ProverClient(device=args.device)
    pk, vk = client.setup(prog)
    t["setup_ms"] = (time.perf_counter() - t0) * 1e3
    t0 = time.perf_counter()
    rec = ctypes.c_void_p()
    cycles = ctypes.c_uint64()
    buf, n = _lib.u8buf(stdin)
    _lib.check(L.bfz_record_new(ctypes.c_void_p(pk.handle), buf, n, ctypes.byref(rec),
                                ctypes.byref(cycles)))
    t["record_ms"] = (time.perf_counter() - t0) * 1e3

    def prove():
        ptr = ctypes.POINTER(ctypes.c_uint8)()
        plen = ctypes.c_size_t()
        t1 = time.perf_counter()
        _lib.check(L.bfz_record_prove(ctypes.c_void_p(pk.handle), rec, ctypes.byref(ptr),
                                      ctypes.byref(plen), None))
        ms = (time.perf_counter() - t1) * 1e3
        return ms, _lib.take_bytes(ptr, plen.value)

    t["first_prove_ms"], first = prove()
    warm = []
    for _ in range(args.warm):
        ms, pf = prove()
        warm.append(round(ms, 3))
        if pf != first:
            raise SystemExit("cold_first_proof: warm proof differs from the first proof")
    client.verify(sdk.BfProofWithPublicValues(proof=first, stdin=stdin), vk)
    pool = {}
    for lane in range(4):
        b = ctypes.c_uint64()
        _lib.check(L.bfz_device_pool_bytes(lane, ctypes.byref(b)))
        if b.value:
            pool[str(lane)] = round(b.value / 2**30, 3)
    L.bfz_record_free(rec)
    out = {k: round(v, 3) for k, v in t.items()}
    out.update({"program": args.program, "cycles": cycles.value, "warm_prove_ms": warm,
                "process_to_first_proof_ms": round((time.perf_counter() - T_START) * 1e3
                                                   - sum(warm) - 0.0, 3),
                "pool_gib_by_lane": pool, "proof_bytes": len(first),
                "checked": "host verifier accepted the first proof; warm proofs byte-identical"})
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
