#!/usr/bin/env python3
"""VALU instruction mix of kernels in a gfx950 compile of a csrc file, weighted by the
measured issue rates (profiles/r01/ubench_valu*.txt: full rate = 1 unit, half rate = 2).

  python3 scripts/isa_mix.py zkvm-brainfuck_amd/csrc/merkle.hip _ZN3bfz15k_permute_batchEPjm
  python3 scripts/isa_mix.py zkvm-brainfuck_amd/csrc/ntt.hip k_ntt_tile k_lde_mid   (substrings)
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
        "v_min3", "v_mul_u32_u24", "v_mad_u32_u24", "v_cvt_", "v_pk_", "v_perm")
MEM = ("ds_", "global_", "buffer_", "s_barrier", "s_waitcnt")


def compile_asm(src, extra=()):
    """gfx950 assembly text of one source file (hipcc --save-temps)."""
    csrc = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                        "zkvm-brainfuck_amd", "csrc")
    with tempfile.TemporaryDirectory() as d:
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
                        "--save-temps", "-I", csrc, *extra, "-c", os.path.abspath(src), "-o", "k.o"], cwd=d,
                       check=True, stderr=subprocess.DEVNULL)
        asm = [f for f in os.listdir(d) if f.endswith("gfx950.s")][0]
        return open(os.path.join(d, asm)).read()


def kernels(txt):
    return re.findall(r"^(_Z\w+):\s*;", txt, re.M)


def mix_of(txt, kernel):
    """(VALU mnemonic counts, full-rate count, half-rate count, memory/barrier counts, vgprs)."""
    m = re.search(r"^" + re.escape(kernel) + r":(.*?)s_endpgm", txt, re.S | re.M)
    if not m:
        sys.exit(f"kernel {kernel} not found")
    mix, mem = collections.Counter(), collections.Counter()
    full = half = 0
    for line in m.group(1).splitlines():
        t = line.split()
        if not t:
            continue
        if t[0].startswith(MEM):
            mem[t[0]] += 1
        if not t[0].startswith("v_"):
            continue
        mix[t[0]] += 1
        ops = " ".join(t[1:]).split(",", 1)
        sgpr = len(ops) > 1 and re.search(r"\bs\d+|\bs\[", ops[1]) is not None
        if t[0].startswith(HALF) or sgpr:
            half += 1
        else:
            full += 1
    v = re.search(r"\.name:\s+" + re.escape(kernel) + r"\s.*?\.vgpr_count:\s+(\d+)", txt, re.S)
    return mix, full, half, mem, int(v.group(1)) if v else None


def main():
    src, wanted = sys.argv[1], sys.argv[2:]
    txt = compile_asm(src)
    names = [k for k in kernels(txt) if any(w == k or w in k for w in wanted)]
    for kernel in names:
        mix, full, half, mem, vgpr = mix_of(txt, kernel)
        print(f"{kernel} {sum(mix.values())} VALU instructions, {vgpr} VGPRs")
        for op, k in mix.most_common():
            print(f"  {op:28s}{k}")
        print(f"  memory/barrier: {dict(mem)}")
        print(f"  # full rate {full} x 1 + half rate (incl. SGPR operand) {half} x 2 = "
              f"{full + 2 * half} full-rate-equivalent lane-ops per thread\n")


if __name__ == "__main__":
    main()
