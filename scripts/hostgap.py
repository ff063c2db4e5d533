"""Host marks (BFZ_HOST_TRACE=1 stderr: 'host <rel us> <what> (abs <steady_clock us>)') against a
rocprofv3 --kernel-trace CSV of the same run: for every GPU idle gap longer than a threshold,
the host marks that fall inside it (times relative to the gap's start), so each gap splits into
host work and launch latency.  Assumes both clocks are CLOCK_MONOTONIC (checked: the marks must
land between kernel launches and their starts).

usage: python3 scripts/hostgap.py gpurun_out/kt/run_kernel_trace.csv gpurun_out/kt.log [min_gap_us]
"""
import csv
import re
import sys


def main():
    kt, log = sys.argv[1], sys.argv[2]
    min_gap = float(sys.argv[3]) if len(sys.argv) > 3 else 15.0
    ks = []
    with open(kt) as f:
        for r in csv.DictReader(f):
            name = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "")
            ks.append((int(r["Start_Timestamp"]) / 1e3, int(r["End_Timestamp"]) / 1e3, name))
    ks.sort()
    marks = []
    pat = re.compile(r"^host\s+\S+\s+(.*) \(abs ([0-9.]+)\)")
    with open(log) as f:
        for line in f:
            m = pat.match(line.strip())
            if m:
                marks.append((float(m.group(2)), m.group(1)))
    marks.sort()
    if not marks or not ks:
        print("no marks or kernels")
        return
    print(f"kernels {ks[0][0]:.1f} .. {ks[-1][1]:.1f} us; marks {marks[0][0]:.1f} .. {marks[-1][0]:.1f} us")
    end = ks[0][1]
    mi = 0
    total = 0.0
    for s, e, name in ks[1:]:
        if s - end >= min_gap:
            total += s - end
            inside = []
            while mi < len(marks) and marks[mi][0] < s:
                if marks[mi][0] >= end - 200:
                    inside.append(f"{marks[mi][1]}@{marks[mi][0] - end:+.0f}")
                mi += 1
            print(f"gap {s - end:7.1f} us before {name[:40]:40s} | " + ", ".join(inside))
        end = max(end, e)
    print(f"gaps >= {min_gap} us: {total:.1f} us in all")


if __name__ == "__main__":
    main()
