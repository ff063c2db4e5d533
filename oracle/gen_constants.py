#!/usr/bin/env python3
"""Extract the Poseidon2 round-constant TABLE (data, not code) used by the reference.

Source: /root/reference/crates/primitives/src/lib.rs:13-555 (`RC_16_30`, 30 rows x 16
KoalaBear elements built with `KoalaBear::from_wrapped_u32`).  The reference wires
them into Poseidon2KoalaBear<16> in `my_perm()` (crates/stark/src/kb31_poseidon2.rs:35-50):
rows 0..4 = initial external rounds, rows 4..17 element [0] = 13 internal rounds,
rows 17..21 = terminal external rounds (rows 21..29 unused).

This script is run once in the build container (where /root/reference exists) and
writes `oracle/rc_16_30.inc`, a plain list of 480 decimal integers exactly as they
appear in the reference (before reduction mod p).  The generated file is committed so
that the GPU box (which has no /root/reference) can build.
"""
import os
import re
import sys

SRC = "/root/reference/crates/primitives/src/lib.rs"
HERE = os.path.dirname(os.path.abspath(__file__))


def main() -> int:
    text = open(SRC).read()
    start = text.index("pub static ref RC_16_30:")
    end = text.index("pub static ref RC_16_30_U32")
    block = text[start:end]
    vals = [int(v) for v in re.findall(r"from_wrapped_u32\((\d+)\)", block)]
    if len(vals) != 480:
        print(f"expected 480 constants, got {len(vals)}", file=sys.stderr)
        return 1
    outs = [os.path.join(HERE, "rc_16_30.inc"),
            os.path.join(HERE, "..", "zkvm-brainfuck_amd", "csrc", "rc_16_30.inc")]
    for out in outs:
      with open(out, "w") as f:
        f.write("/* Poseidon2 KoalaBear width-16 round constants RC_16_30 (30 x 16, raw u32,\n"
                " * reduce mod p = from_wrapped_u32).  Data extracted by oracle/gen_constants.py\n"
                " * from crates/primitives/src/lib.rs:13-555 of the reference. */\n")
        for r in range(30):
            row = vals[16 * r:16 * r + 16]
            f.write("  " + ", ".join(f"{v}u" for v in row) + ",\n")
      print(f"wrote {out}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
