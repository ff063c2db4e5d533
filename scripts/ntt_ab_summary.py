"""Summary of scripts/gpu_ntt_variants.sh: per variant and rep, the coset-LDE time the microbenchmark
printed and the average duration (us) of the DIT tile, k_lde_mid<22> and the DIF tile from the
rocprofv3 --stats CSV, plus the output hash (identical for every variant that computes the same
transform).

usage: python3 scripts/ntt_ab_summary.py gpurun_out/ntt_ab
"""
import csv
import os
import re
import sys


def kernel_us(path):
    out = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r["Name"]
            us = float(r["AverageNs"]) / 1e3
            if "k_lde_mid<22>" in name:
                out["mid"] = us
            elif "k_ntt_tile<false, 14" in name:
                out["DIT"] = us
            elif "k_ntt_tile<true, 14" in name:
                out["DIF"] = us
    return out


def main():
    d = sys.argv[1]
    rows = []
    for fn in sorted(os.listdir(d)):
        m = re.match(r"(.+)_(\d+)\.log$", fn)
        if not m:
            continue
        v, rep = m.group(1), m.group(2)
        log = open(os.path.join(d, fn)).read()
        lde = re.search(r"coset LDE 2\^22 x 8:\s+([\d.]+) us", log)
        h = re.search(r"out ([0-9a-f]+)", log)
        k = kernel_us(os.path.join(d, f"{v}_{rep}_kernel_stats.csv"))
        rows.append((v, rep, float(lde.group(1)) if lde else float("nan"), k, h.group(1) if h else "-"))
    for v, rep, lde, k, h in sorted(rows, key=lambda r: (r[0] != "base", r[0], r[1])):
        print(f"  {v + '_' + rep:14s} LDE {lde:7.1f} us  DIT {k.get('DIT', 0):6.1f}  mid {k.get('mid', 0):6.1f}  "
              f"DIF {k.get('DIF', 0):6.1f}  out {h}")


if __name__ == "__main__":
    main()
