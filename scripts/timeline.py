"""Per-proof GPU timeline from a rocprofv3 --kernel-trace CSV: wall span, busy time, idle gaps
(largest, with the kernels around them) and time in under-filled launches (fewer workgroups than
CUs).  A proof starts at each k_trace_cpu dispatch.

usage: python3 scripts/timeline.py gpurun_out/kt/run_kernel_trace.csv [n_cus]
"""
import csv
import re
import sys
from collections import defaultdict


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"\(.*", "", name)
    return name.replace("void ", "")


def main():
    path = sys.argv[1]
    ncu = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            wg = int(r["Workgroup_Size_X"]) * int(r["Workgroup_Size_Y"]) * int(r["Workgroup_Size_Z"])
            grid = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
                         grid // max(wg, 1)))
    rows.sort()
    starts = [i for i, r in enumerate(rows) if r[2].endswith("k_trace_cpu")]
    proofs = []
    for a, b in zip(starts, starts[1:] + [len(rows)]):
        proofs.append(rows[a:b])
    for pi, pr in enumerate(proofs):
        t0, t1 = pr[0][0], max(r[1] for r in pr)
        busy = 0
        cur_s, cur_e = pr[0][0], pr[0][1]
        gaps = []
        for i, (s, e, n, g) in enumerate(pr[1:], 1):
            if s > cur_e:
                busy += cur_e - cur_s
                gaps.append((s - cur_e, pr[i - 1][2], n))
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
        busy += cur_e - cur_s
        small = defaultdict(float)
        for s, e, n, g in pr:
            if g < ncu:
                small[n] += (e - s) / 1e6
        print(f"proof {pi}: {len(pr)} dispatches, span {(t1 - t0) / 1e6:.3f} ms, busy {busy / 1e6:.3f} ms,"
              f" idle {(t1 - t0 - busy) / 1e6:.3f} ms in {len(gaps)} gaps;"
              f" under-filled launches {sum(small.values()):.3f} ms")
        if pi == len(proofs) - 1:
            gaps.sort(reverse=True)
            print("  largest gaps (us): " + "; ".join(f"{g / 1e3:.0f} {a} -> {b}" for g, a, b in gaps[:12]))
            tot = defaultdict(float)
            for g, a, b in gaps:
                tot[b] += g / 1e6
            print("  idle before (ms): " + "; ".join(f"{k} {v:.3f}" for k, v in sorted(tot.items(), key=lambda x: -x[1])[:10]))
            print("  under-filled (ms): " + "; ".join(f"{k} {v:.3f}" for k, v in sorted(small.items(), key=lambda x: -x[1])[:14]))


if __name__ == "__main__":
    main()
