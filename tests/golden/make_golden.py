#!/usr/bin/env python3
"""Regenerate tests/golden/golden.json from the oracle (oracle/liboracle.so).

The fixtures pin the CPU restatement against itself over time and give the GPU tests a
reference that does not need the oracle at run time:
  * executor known answers — the reference's own value-level goldens
    (crates/core/executor/src/executor.rs:335-416, crates/sdk/src/lib.rs:175-183)
  * Poseidon2KoalaBear<16> outputs on fixed states (canonical u32)
  * sha256 of the main trace of every chip for hello / fibo(17) (normal form)
  * per program: sha256 of the full BFZ1 proof + its three commitments
PCS-level values are "parity unpinned" against the Rust prover (no cargo / Plonky3 here).
"""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(HERE)), "zkvm-brainfuck_amd"))

import numpy as np  # noqa: E402

import oracle_lib as O  # noqa: E402
from bfz import guests  # noqa: E402

CHIPS = ["Cpu", "Program", "AddSub", "Jump", "Memory", "Byte", "MemoryInstrs", "IO"]


def main():
    g = {"known_answers": [], "poseidon2": [], "traces": {}, "proofs": []}
    for name, prog, sin in guests.REFERENCE_PROGRAMS:
        r = O.execute(prog, sin)
        g["known_answers"].append({"name": name, "program": prog, "stdin": list(sin),
                                   "output": list(r["output"]), "cycles": r["cycles"],
                                   "pc": r["pc"], "mp": r["mp"]})
    states = [list(range(16)), [0] * 16, [O.P - 1] * 16,
              [(i * 0x9E3779B1 + 7) % O.P for i in range(16)]]
    outs = O.poseidon2(np.array(states, dtype=np.uint32).reshape(-1))
    for s, o in zip(states, outs.reshape(-1, 16).tolist()):
        g["poseidon2"].append({"in": s, "out": o})
    for name, prog, sin in [("hello", guests.HELLO, []), ("fibo17", guests.FIBO, [17])]:
        d = {}
        for ci, cn in enumerate(CHIPS):
            t = O.trace(prog, sin, ci)
            if t is not None:
                d[cn] = {"shape": list(t.shape), "sha256": hashlib.sha256(t.tobytes()).hexdigest()}
        g["traces"][name] = d
    for name, prog, sin in guests.REFERENCE_PROGRAMS:
        pf = O.prove(prog, sin)
        assert O.verify(prog, pf)
        nc = int.from_bytes(pf[4:8], "little")
        off = 8
        for _ in range(nc):
            off += 4
            ln = int.from_bytes(pf[off:off + 4], "little")
            off += 4 + ln
        roots = [list(np.frombuffer(pf[off + 32 * k: off + 32 * (k + 1)], dtype=np.uint32).tolist())
                 for k in range(3)]
        g["proofs"].append({"name": name, "program": prog, "stdin": list(sin), "len": len(pf),
                            "sha256": hashlib.sha256(pf).hexdigest(), "main_root": roots[0],
                            "perm_root": roots[1], "quotient_root": roots[2],
                            "vk_commit": O.setup_root(prog)})
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(g, f, indent=1)
    print("wrote golden.json")


if __name__ == "__main__":
    main()
