#!/usr/bin/env python3
"""VALU cost of a 2^L coset LDE per radix-2 element-stage, from the gfx950 ISA of the three
kernels one LDE launches (ntt.hip coset_lde, L > 14):
  k_ntt_tile<false,14,true>  iDFT stages 0..13 over n elements     (16 elements / thread)
  k_lde_mid<L>          iDFT stages 14..L-1, coset scale, DFT stages L-1..14 of both halves
                        (16 input elements / thread, 32 outputs)
  k_ntt_tile<true,14>   DFT stages 13..0 over the 2n outputs        (16 elements / thread)
An LDE of n x w does 3*n*log2(n)*w element-stages (iDFT n + DFT n on each coset half).
Prints units (full-rate VALU lane-ops) per element-stage: bench.py multiplies this by the
proof's element-stages and divides by the NTT kernel time to get the VALU-issue fraction.

  python3 scripts/ntt_isa.py 22 > profiles/r02/ntt_isa_mix.txt
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import isa_mix  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    L = int(sys.argv[1]) if len(sys.argv) > 1 else 22
    txt = isa_mix.compile_asm(os.path.join(ROOT, "zkvm-brainfuck_amd", "csrc", "ntt.hip"))
    names = isa_mix.kernels(txt)
    # the DIT pass the LDE launches reads its first window straight from HBM (DIN = true)
    dit = [k for k in names if k.startswith("_ZN3bfz10k_ntt_tileILb0ELi14ELb1E")]
    tile_dit = (dit or [k for k in names if k.startswith("_ZN3bfz10k_ntt_tileILb0ELi14E")])[0]
    tile_dif = [k for k in names if k.startswith("_ZN3bfz10k_ntt_tileILb1ELi14E")][0]
    mid = [k for k in names if k.startswith(f"_ZN3bfz9k_lde_midILi{L}E")][0]
    b2 = L - 14
    # (kernel, element-stages per thread, input elements per thread)
    rows = [(tile_dit, 16 * 14, 16), (mid, 16 * 3 * b2, 16), (tile_dif, 16 * 14, 16)]
    total_units = total_stages = 0.0
    print(f"# coset LDE 2^{L}: VALU units per element-stage (scripts/ntt_isa.py; full rate = 1, "
          "half rate = 2, weights from profiles/r01/ubench_valu*.txt)")
    for k, stages, inputs in rows:
        mix, full, half, mem, vgpr = isa_mix.mix_of(txt, k)
        units = full + 2 * half
        # the DIF tile runs over the 2n outputs: twice per input element
        reps = 2 if k == tile_dif else 1
        total_units += reps * units / inputs
        total_stages += reps * stages / inputs
        print(f"{k}: {sum(mix.values())} VALU instr, {units} units, {vgpr} VGPRs, "
              f"{stages} element-stages / thread -> {units / stages:.3f} units / element-stage; "
              f"memory/barrier {dict(mem)}")
    print(f"per input element: {total_units:.1f} units over {total_stages:.0f} element-stages "
          f"(3 * log2 n = {3 * L})")
    print(f"UNITS_PER_ELEMENT_STAGE {total_units / total_stages:.3f}")


if __name__ == "__main__":
    main()
