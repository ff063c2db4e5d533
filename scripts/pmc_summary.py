"""Summarize rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes per kernel.

For the NTT kernels (the bench roofline kernels) it reports, per launch, the algorithmic
bytes next to the counted traffic: k_ntt_tile / k_ntt_r16 8 B per element (one read + one write),
k_lde_mid 12 B per input element (read n, write the 2n LDE); a launch covers Grid_Size * 16
input elements.
MI355X_MICROARCH.md: FETCH_SIZE under-reports wide coalesced reads by exactly 2x on gfx950;
both the raw and the x2-corrected fetch figures are written.  Counter units are kB.
"""
import collections
import csv
import glob
import json
import os
import sys


def load(root, counter):
    rows = []
    for f in glob.glob(os.path.join(root, f"pmc_{counter}", "**", "*counter_collection*.csv"),
                       recursive=True):
        rows += list(csv.DictReader(open(f)))
    return rows


def per_kernel(rows):
    agg = collections.defaultdict(lambda: {"launches": 0, "value": 0.0, "grid": 0})
    for r in rows:
        name = r.get("Kernel_Name", "?")
        # template arguments kept (k_ntt_tile<true, 14>); "(anonymous namespace)::" is dropped
        # before cutting the parameter list, or every tracegen kernel collapses into "bfz::"
        key = name.replace("(anonymous namespace)::", "").split("(")[0]
        a = agg[key]
        a["launches"] += 1
        a["value"] += float(r.get("Counter_Value", 0) or 0)
        a["grid"] += int(float(r.get("Grid_Size", 0) or 0))
    return agg


def durations(root):
    """{kernel: (launches, mean us, max us)} from the kernel traces the --pmc passes wrote beside
    their counters (outliers must show up in review, not be averaged away)."""
    d = collections.defaultdict(list)
    for f in glob.glob(os.path.join(root, "pmc_*", "**", "*kernel_trace*.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            key = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
            d[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    return {k: (len(v), sum(v) / len(v), max(v)) for k, v in d.items()}


def main(root):
    fetch = per_kernel(load(root, "FETCH_SIZE"))
    write = per_kernel(load(root, "WRITE_SIZE"))
    dur = durations(root)
    out = {"unit": "kB per launch (rocprofv3 FETCH_SIZE / WRITE_SIZE); durations in us from the same "
                   "passes' kernel traces (counter passes run slower than plain runs)", "kernels": {}}
    for k in sorted(set(fetch) | set(write)):
        f, w = fetch.get(k), write.get(k)
        n = max((f or w)["launches"], 1)
        e = {"launches": n,
             "fetch_kB": round(f["value"] / f["launches"], 1) if f else None,
             "write_kB": round(w["value"] / w["launches"], 1) if w else None}
        per_elem = 8 if ("k_ntt_r16" in k or "k_ntt_tile" in k) else 12 if "k_lde_mid" in k else 0
        if per_elem and f and w:  # NTT kernels: a launch covers Grid_Size * 16 input elements
            elems = f["grid"] / f["launches"] * 16
            e["algorithmic_kB"] = round(per_elem * elems / 1024, 1)
            e["traffic_kB_fetch_x2_plus_write"] = round(2 * e["fetch_kB"] + e["write_kB"], 1)
            e["traffic_kB_raw"] = round(e["fetch_kB"] + e["write_kB"], 1)
        if k in dur:
            e["duration_us_mean"] = round(dur[k][1], 2)
            e["duration_us_max"] = round(dur[k][2], 2)
        out["kernels"][k] = e
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out")
