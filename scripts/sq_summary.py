"""Summarize the SQ wave-state pass of scripts/gpu_sq.sh (rocprofv3 --pmc, counters only):
per kernel, the fractions of SQ_WAVE_CYCLES spent parked at s_waitcnt / barriers (wait_any),
ready but not issued (wait_inst), issuing anything (active) and issuing VALU (valu), summed
over the kernel's launches.  Usage: python3 scripts/sq_summary.py gpurun_out > profiles/rNN/sq_summary.txt
"""
import collections
import csv
import glob
import os
import sys

COUNTERS = ("SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
            "SQ_ACTIVE_INST_VALU")


def main(root):
    agg = collections.defaultdict(lambda: collections.Counter())
    for f in glob.glob(os.path.join(root, "pmc_sq", "**", "*counter_collection*.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r.get("Kernel_Name", "?").replace("(anonymous namespace)::", "").split("(")[0]
            agg[name][r.get("Counter_Name", "?")] += float(r.get("Counter_Value", 0) or 0)
    rows = sorted(agg.items(), key=lambda kv: -kv[1]["SQ_WAVE_CYCLES"])
    print("# SQ wave-state counters (scripts/gpu_sq.sh + scripts/sq_summary.py; fractions of "
          "SQ_WAVE_CYCLES per kernel, summed over launches)")
    print("# wait_any = parked at s_waitcnt/barrier; wait_inst = ready but not issued; "
          "active = issuing; valu = issuing VALU")
    print(f"{'kernel':60s} {'wait_any':>8s} {'wait_inst':>9s} {'active':>7s} {'valu':>6s}")
    for name, c in rows[:28]:
        w = c["SQ_WAVE_CYCLES"] or 1.0
        print(f"{name[:60]:60s} {c['SQ_WAIT_ANY'] / w:8.2f} {c['SQ_WAIT_INST_ANY'] / w:9.2f} "
              f"{c['SQ_ACTIVE_INST_ANY'] / w:7.2f} {c['SQ_ACTIVE_INST_VALU'] / w:6.2f}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out")
