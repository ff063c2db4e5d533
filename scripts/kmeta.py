#!/usr/bin/env python3
"""Register / LDS / scratch metadata of the kernels of a gfx950 compile of a csrc file.
  python3 scripts/kmeta.py zkvm-brainfuck_amd/csrc/fri.hip open_mfma [-DFLAG=1 ...]"""
import re
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
import isa_mix  # noqa: E402


def main():
    src, pat = sys.argv[1], sys.argv[2]
    txt = isa_mix.compile_asm(src, sys.argv[3:])
    sec = txt[txt.index("amdhsa.kernels:"):]
    for ent in re.split(r"\n  - ", sec)[1:]:
        name = re.search(r"\.name:\s+(\S+)", ent)
        if not name or pat not in name.group(1):
            continue
        f = {k: re.search(r"\." + k + r":\s+(\d+)", ent) for k in
             ("vgpr_count", "agpr_count", "sgpr_count", "vgpr_spill_count", "group_segment_fixed_size",
              "private_segment_fixed_size")}
        print(name.group(1)[:60], {k: int(v.group(1)) for k, v in f.items() if v})


if __name__ == "__main__":
    main()
