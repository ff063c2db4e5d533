"""Per-launch outliers of a rocprofv3 --kernel-trace CSV: for each hot kernel
the launch count, mean and maximum duration, and for the longest launches overall their dispatch
index, grid, start time, the launches around them and the phase they belong to (setup = before the
first k_trace_cpu dispatch, proof k = from the k-th k_trace_cpu on).

usage: python3 scripts/kernel_outliers.py run_kernel_trace.csv [top_n]
"""
import csv
import re
import statistics
import sys
from collections import defaultdict


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"\(.*", "", name)
    return name.replace("void ", "").replace("bfz::", "")


def load(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            wg = int(r["Workgroup_Size_X"]) * int(r["Workgroup_Size_Y"]) * int(r["Workgroup_Size_Z"])
            grid = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
            rows.append({"start": int(r["Start_Timestamp"]), "end": int(r["End_Timestamp"]),
                         "name": short(r["Kernel_Name"]), "wgs": grid // max(wg, 1), "wg": wg,
                         "dispatch": int(r.get("Dispatch_Id", 0) or 0)})
    rows.sort(key=lambda r: r["start"])
    return rows


def per_kernel_stats(rows):
    """{name: {"launches", "mean_us", "max_us", "max_index"}}; index = position in start order."""
    by = defaultdict(list)
    for i, r in enumerate(rows):
        by[r["name"]].append((r["end"] - r["start"], i))
    out = {}
    for k, v in by.items():
        d = [x[0] for x in v]
        mx = max(v)
        out[k] = {"launches": len(v), "mean_us": round(statistics.mean(d) / 1e3, 2),
                  "max_us": round(mx[0] / 1e3, 2), "max_index": mx[1]}
    return out


def phase_of(rows, i):
    starts = [j for j, r in enumerate(rows) if r["name"].endswith("k_trace_cpu")]
    k = sum(1 for j in starts if j <= i)
    return "setup / before the first proof" if k == 0 else f"proof {k - 1}"


def main():
    rows = load(sys.argv[1])
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    t0 = rows[0]["start"]
    st = per_kernel_stats(rows)
    print("kernel: launches, mean us, max us (launch index)")
    for k, v in sorted(st.items(), key=lambda kv: -kv[1]["mean_us"] * kv[1]["launches"])[:20]:
        print(f"  {k}: {v['launches']}, {v['mean_us']}, {v['max_us']} (#{v['max_index']})")
    print(f"longest {top} launches:")
    order = sorted(range(len(rows)), key=lambda i: rows[i]["start"] - rows[i]["end"])[:top]
    for i in order:
        r = rows[i]
        prev = rows[i - 1]["name"] if i else "-"
        nxt = rows[i + 1]["name"] if i + 1 < len(rows) else "-"
        gap = (r["start"] - rows[i - 1]["end"]) / 1e3 if i else 0.0
        print(f"  #{i} {r['name']} {(r['end'] - r['start']) / 1e3:.1f} us, {r['wgs']} workgroups x "
              f"{r['wg']}, at {(r['start'] - t0) / 1e6:.3f} ms ({phase_of(rows, i)}); "
              f"after {prev} (gap {gap:.1f} us), before {nxt}")


if __name__ == "__main__":
    main()
