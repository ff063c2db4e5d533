#!/usr/bin/env python3
"""bfz_prove_batch figures alone (bench.py's end_to_end without the rest): per-job executor,
upload and prove times of FIBO_X4 stdin [255] batches, for A/Bs of the pipelined path.
Prints one JSON line.  BFZ_AB_VARIANT=1 lets it load a libbfz built from other sources."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zkvm-brainfuck_amd"))


def main():
    from bfz import _lib, guests, sdk
    _lib.init(0)
    client = sdk.ProverClient()
    pk, _ = client.setup(guests.FIBO_X4)
    stdin = bytes([255])
    client.prove_batch(pk, [stdin] * 8, public_values=False)
    out = []
    for _ in range(2):
        stats = {}
        t0 = time.perf_counter()
        client.prove_batch(pk, [stdin] * 24, public_values=False, stats=stats)
        wall = (time.perf_counter() - t0) * 1e3
        out.append({"ms_per_proof": round(wall / 24, 3),
                    "exec_ms_per_job": round(stats["exec_ms"] / 24, 3),
                    "upload_ms_per_job": round(stats["upload_ms"] / 24, 3),
                    "prove_ms_per_job": round(stats["prove_ms"] / 24, 3)})
    print(json.dumps({"runs": out, "nproc": os.cpu_count(),
                      "affinity": len(os.sched_getaffinity(0))}), flush=True)


if __name__ == "__main__":
    main()
