"""The launch sequence of one proof from a rocprofv3 --kernel-trace CSV: every dispatch of the
chosen proof (the k-th k_trace_cpu starts proof k) with its start offset, duration, idle gap before
it and grid size, then the kernels' summed time per phase (runs of launches between transcript
points: the phases are cut at the challenge kernels).

usage: python3 scripts/proof_sequence.py run_kernel_trace.csv [proof_index]
"""
import sys

from kernel_outliers import load

CUT = ("k_challenge_perm", "k_challenge_quot", "k_challenge_zeta", "k_inv_denoms", "k_fri_finish")


def main():
    rows = load(sys.argv[1])
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    starts = [i for i, r in enumerate(rows) if r["name"].endswith("k_trace_cpu")]
    a = starts[k]
    b = starts[k + 1] if k + 1 < len(starts) else len(rows)
    t0 = rows[a]["start"]
    phase, phases, acc = "tracegen", [], {}
    prev_end = rows[a]["start"]
    for i in range(a, b):
        r = rows[i]
        name = r["name"]
        if any(c in name for c in CUT):
            phases.append((phase, acc))
            phase, acc = name, {}
        d = (r["end"] - r["start"]) / 1e3
        gap = (r["start"] - prev_end) / 1e3
        prev_end = max(prev_end, r["end"])
        acc[name] = acc.get(name, 0.0) + d
        print(f"{(r['start'] - t0) / 1e3:9.1f} us  {d:8.1f} us  gap {gap:6.1f}  {r['wgs']:7d} x {r['wg']:4d}  {name}")
    phases.append((phase, acc))
    print("\nper phase (kernel us):")
    for name, acc in phases:
        tot = sum(acc.values())
        top = sorted(acc.items(), key=lambda kv: -kv[1])[:6]
        print(f"  {name}: {tot:.1f} us; " + ", ".join(f"{n} {v:.0f}" for n, v in top))


if __name__ == "__main__":
    main()
