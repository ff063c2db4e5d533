#!/usr/bin/env python3
"""VALU instruction mix of one kernel in a gfx950 compile of a csrc file, weighted by the
measured issue rates (profiles/r01/ubench_valu*.txt: full rate = 1 unit, half rate = 2).

  python3 scripts/isa_mix.py zkvm-brainfuck_amd/csrc/merkle.hip _ZN3bfz15k_permute_batchEPjm
"""
import collections
import os
import re
import subprocess
import sys
import tempfile

HALF = ("v_min_", "v_max_", "v_cmp", "v_lshlrev", "v_add3", "v_lshl_add", "v_add_co", "v_addc_co",
        "v_sub_co", "v_subb_co", "v_subrev_co", "v_mul_lo", "v_mul_hi", "v_mad_u64", "v_mad_i64",
        "v_cndmask", "v_lshl_or", "v_and_or", "v_or3", "v_bfe", "v_bfi", "v_alignbit", "v_med3",
        "v_min3", "v_mul_u32_u24", "v_mad_u32_u24", "v_cvt_", "v_pk_")


def main():
    src, kernel = sys.argv[1], sys.argv[2]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with tempfile.TemporaryDirectory() as d:
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
                        "--save-temps", "-c", os.path.abspath(src), "-o", "k.o"], cwd=d, check=True,
                       stderr=subprocess.DEVNULL)
        asm = [f for f in os.listdir(d) if f.endswith("gfx950.s")][0]
        txt = open(os.path.join(d, asm)).read()
    m = re.search(r"^" + re.escape(kernel) + r":(.*?)s_endpgm", txt, re.S | re.M)
    if not m:
        sys.exit(f"kernel {kernel} not found")
    mix = collections.Counter()
    full = half = 0
    for line in m.group(1).splitlines():
        t = line.split()
        if not t or not t[0].startswith("v_"):
            continue
        mix[t[0]] += 1
        ops = " ".join(t[1:]).split(",", 1)
        sgpr = len(ops) > 1 and re.search(r"\bs\d+|\bs\[", ops[1]) is not None
        if t[0].startswith(HALF) or sgpr:
            half += 1
        else:
            full += 1
    print(f"{kernel} {sum(mix.values())} VALU instructions")
    for op, k in mix.most_common():
        print(f"{op:28s}{k}")
    print(f"\n# full rate {full} x 1 + half rate (incl. SGPR operand) {half} x 2 = {full + 2 * half} "
          f"full-rate-equivalent lane-ops per thread")


if __name__ == "__main__":
    main()
