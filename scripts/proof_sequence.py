#!/usr/bin/env python3
"""The last proof of a rocprofv3 --kernel-trace CSV as a launch sequence (a proof starts at its
k_trace_cpu): start offset (us), kernel, run length of consecutive same-name launches, summed
duration (us), and the idle time before the run.
  python3 scripts/proof_sequence.py run_kernel_trace.csv > sequence.txt"""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if "k_trace_cpu" in r["Kernel_Name"]]
    last = rows[starts[-1]:] if starts else rows
    t0 = int(last[0]["Start_Timestamp"])
    runs = []
    prev_end = t0
    for r in last:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        name = r["Kernel_Name"].replace("bfz::", "").split("(")[0][:56]
        gap = max(0, s - prev_end)
        if runs and runs[-1][1] == name:
            runs[-1][2] += 1
            runs[-1][3] += e - s
            runs[-1][4] += gap
        else:
            runs.append([s - t0, name, 1, e - s, gap])
        prev_end = max(prev_end, e)
    busy = sum(r[3] for r in runs)
    idle = sum(r[4] for r in runs)
    print(f"launches {len(last)}, span {(prev_end - t0) / 1e3:.1f} us, busy {busy / 1e3:.1f} us, "
          f"idle {idle / 1e3:.1f} us")
    for off, name, cnt, dur, gap in runs:
        print(f"{off / 1e3:9.1f} {name:56s} x{cnt:<3d} {dur / 1e3:8.1f} idle {gap / 1e3:6.1f}")


if __name__ == "__main__":
    main()
