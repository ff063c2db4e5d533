"""Per-kernel dynamic counters of the coset LDE (scripts/gpu_ntt_counters.sh) at a known
element-stage count: a coset LDE of an n x w matrix (n = 2^L) runs
    k_ntt_tile<false,14> (iDFT stages 0-13 of n):        14 n w element-stages
    k_lde_mid<L>          (iDFT stages 14.., DFT of both halves' stages 14..): 3 (L - 14) n w
    k_ntt_tile<true,14>  (DFT stages 13-0 of 2n):         28 n w
A launch of each covers one matrix, so per-launch counters divide by these.  Reported per kernel:
VALU / SALU / LDS / VMEM wave-instructions x 64 lanes per element-stage (lane-instructions), the
VALU issue rate against the 256 CU x 4 SIMD x 32 lanes x 2.4 GHz peak (a full-rate wave64
instruction = 64 lane-ops = 2 SIMD cycles), the fraction of wave-cycles with a VALU instruction
in flight (SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES, both quad-cycle units), L2 hit rate and the
FETCH_SIZE (x2, MI355X_MICROARCH.md) + WRITE_SIZE traffic against the algorithmic bytes.
Usage: python3 scripts/ntt_counters.py gpurun_out > profiles/rNN/ntt_counters.json
"""
import collections
import csv
import glob
import json
import os
import re
import sys

L, W = 22, 8
N = 1 << L
PEAK_LANE_OPS = 256 * 4 * 32 * 2.4e9  # 78.6 T full-rate lane-ops/s


def kernel_key(name):
    name = name.replace("(anonymous namespace)::", "")
    m = re.match(r"(?:void )?bfz::(k_\w+)(<[^(]*>)?", name)
    return (m.group(1) + (m.group(2) or "")).replace(" ", "") if m else name.split("(")[0]


def family(key):
    if key.startswith("k_ntt_tile<false,14"):
        return "dit_tile", 14.0 * N * W, 8.0 * N * W
    if key.startswith("k_ntt_tile<true,14"):
        return "dif_tile", 28.0 * N * W, 16.0 * N * W
    if key.startswith(f"k_lde_mid<{L}>"):
        return "lde_mid", 3.0 * (L - 14) * N * W, 12.0 * N * W
    return None, 0.0, 0.0


def load(root, name):
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(root, f"ntt_pmc_{name}", "**", "*counter_collection*.csv"),
                       recursive=True):
        for r in csv.DictReader(open(f)):
            k = kernel_key(r.get("Kernel_Name", "?"))
            per[k][r["Counter_Name"]].append(float(r.get("Counter_Value", 0) or 0))
    return per


def times(root):
    out = {}
    for f in glob.glob(os.path.join(root, "ntt_pmc_stats", "**", "*kernel_stats*.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            out[kernel_key(r["Name"])] = float(r["AverageNs"]) * 1e-9
    return out


def main(root):
    groups = {n: load(root, n) for n in ("inst", "busy", "l2", "fetch", "write")}
    avg_s = times(root)
    res = {"workload": f"scripts/ubench_ntt lde {L} {W}: coset LDE of a 2^{L} x {W} matrix",
           "units": "lane-instructions (wave-instructions x 64) per element-stage", "kernels": {}}
    keys = set()
    for g in groups.values():
        keys |= set(g)
    for k in sorted(keys):
        fam, es, alg = family(k)
        if not fam:
            continue
        def avg(group, c):
            v = groups[group].get(k, {}).get(c)
            return sum(v) / len(v) if v else None
        e = {"family": fam, "element_stages_per_launch": es, "algorithmic_bytes_per_launch": alg}
        for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD",
                  "SQ_INSTS_VMEM_WR", "SQ_INSTS_SMEM"):
            v = avg("inst", c)
            if v is not None:
                e[c.lower().replace("sq_insts_", "") + "_per_elem_stage"] = round(v * 64 / es, 3)
        t = avg_s.get(k)
        if t:
            e["avg_launch_us"] = round(t * 1e6, 1)
            v = avg("inst", "SQ_INSTS_VALU")
            if v is not None:
                e["valu_issue_frac"] = round(v * 64 / t / PEAK_LANE_OPS, 3)
            e["hbm_gbs_algorithmic"] = round(alg / t / 1e9, 1)
        act, wc = avg("busy", "SQ_ACTIVE_INST_VALU"), avg("inst", "SQ_WAVE_CYCLES")
        if act is not None and wc:
            e["valu_active_per_wave_cycle"] = round(act / wc, 3)
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_LDS"):
            v = avg("busy", c)
            if v is not None and wc:
                e[c.lower().replace("sq_", "") + "_per_wave_cycle"] = round(v / wc, 3)
        hit, miss = avg("l2", "TCC_HIT_sum"), avg("l2", "TCC_MISS_sum")
        if hit is not None and miss is not None and hit + miss > 0:
            e["l2_hit_rate"] = round(hit / (hit + miss), 3)
        f, w = avg("fetch", "FETCH_SIZE"), avg("write", "WRITE_SIZE")
        if f is not None and w is not None:
            e["fetch_MB_raw"] = round(f * 1024 / 1e6, 1)
            e["write_MB"] = round(w * 1024 / 1e6, 1)
            e["traffic_over_algorithmic_fetch_x2"] = round((2 * f + w) * 1024 / alg, 3)
            e["traffic_over_algorithmic_raw"] = round((f + w) * 1024 / alg, 3)
        res["kernels"][k] = e
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out")
