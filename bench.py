#!/usr/bin/env python3
"""Headline benchmark: core-proof wall time for a fibonacci trace of 2^22 rows on MI355X.

Workload (BASELINE.json metric "core-proof wall-time (ms) + NTT HBM GB/s, fibonacci trace
2^22 rows"): the FIBO_X4 guest (the reference fibonacci guest run 4x, stdin [255]) executes
3,767,729 cycles -> Cpu 2^22 x 31, MemoryInstrs 2^21 x 41, AddSub 2^20 x 7, Jump 2^20 x 45 ...
A "step" is one full core proof from the executor's events already resident in HBM:
device trace generation (generate_dependencies + generate_traces), main commit, LogUp,
quotient, FRI open and proof assembly.  The executor and the event upload run before the
timed region.  Every rank proves its own replica (no data-path collective: replicas only), so
the job is weak-scaled; `value` is the wall time of one step (max over ranks).

Also reported: the HBM roofline of the coset-LDE (NTT) kernels on SURVEY 8(d)'s basis
(12*n*w B per LDE / NTT kernel time, per-launch HIP events on the prover's stream), their
VALU-issue fraction, the Poseidon2 kernels' VALU fraction, and the oracle (CPU restatement)
proving the same headline workload on the host cores.
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "zkvm-brainfuck_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
# VALU issue peak: 256 CUs x 4 SIMDs x 32 lanes/cycle (a wave64 VALU op issues over 2 cycles,
# MI355X_MICROARCH.md) x 2.4 GHz, in full-rate lane-ops/s; half-rate ops (mul_lo/hi, mad_u64,
# min, 64-bit adds) count as 2.  scripts/ubench_valu.hip measures 75 T for v_sub/v_xor.
VALU_PEAK_TOPS = 256 * 4 * 32 * 2.4e9 / 1e12
# Full-rate-equivalent VALU lane-ops of one Poseidon2 permutation in k_permute_batch
# (gfx950 ISA instruction mix, profiles/r02/poseidon2_isa_mix.txt).
P2_UNITS_PER_PERM = 5133
PMC_SUMMARY = os.path.join(ROOT, "profiles", "r06", "profile_round_pmc_summary.json")


# VALU units (full-rate lane-ops) per radix-2 element-stage of a 2^22 coset LDE, from the gfx950
# ISA of k_ntt_tile<false,14,true> + k_lde_mid<22> + k_ntt_tile<true,14> (scripts/ntt_isa.py ->
# profiles/r02/ntt_isa_mix.txt).  Smaller chips' LDEs use the same kernels' shapes within ~5%.
NTT_UNITS_PER_ELEM_STAGE = 7.023
# Dynamic counters of the same kernels at a known element-stage count (scripts/gpu_ntt_counters.sh
# -> scripts/ntt_counters.py): SQ_INSTS_VALU x 64 per element-stage, SQ wave-state fractions.
NTT_COUNTERS = os.path.join(ROOT, "profiles", "r05", "ntt_counters.json")
# element-stage shares of a 2^22 coset LDE: DIT tile 14, k_lde_mid<22> 3 x 8, DIF tile 2 x 14 (of 66)
NTT_FAMILY_SHARE = {"dit_tile": 14 / 66, "lde_mid": 24 / 66, "dif_tile": 28 / 66}


def ntt_traffic():
    """(HBM bytes per NTT launch, traffic / per-pass algorithmic bytes) from the committed
    rocprofv3 PMC passes (scripts/gpu_pmc.sh: FETCH_SIZE x2 per MI355X_MICROARCH.md +
    WRITE_SIZE, separate runs); per-pass algorithmic = 8 B per element per tile pass, 12 B per
    input element per k_lde_mid launch."""
    try:
        k = json.load(open(PMC_SUMMARY))["kernels"]
        rows = [v for n, v in k.items() if any(x in n for x in ("k_ntt_r16", "k_ntt_tile", "k_lde_mid"))]
        launches = sum(v["launches"] for v in rows)
        traffic = sum(v["traffic_kB_fetch_x2_plus_write"] * v["launches"] for v in rows) * 1024
        alg = sum(v["algorithmic_kB"] * v["launches"] for v in rows) * 1024
        return traffic / launches, traffic / alg
    except (OSError, KeyError, ValueError, ZeroDivisionError):
        return None, None


def ntt_roofline(tm):
    """HBM roofline of the NTT kernels on SURVEY §8(d)'s basis: 12*n*w algorithmic bytes per
    coset LDE of an n x w matrix (read n, write 2n), summed over the proof, divided by the
    summed per-launch HIP-event time of the NTT kernels (k_ntt_tile, k_lde_mid, k_ntt_r16; one
    LDE = 3 launches = 3 HBM passes).  The per-pass figure (each launch's own read + write) is
    kept as a secondary field."""
    if tm.ntt_kernel_ms <= 0:
        return None
    launches = max(tm.ntt_kernel_launches, 1)
    achieved = tm.lde_bytes / (tm.ntt_kernel_ms * 1e-3) / 1e9
    per_pass = tm.ntt_kernel_bytes / (tm.ntt_kernel_ms * 1e-3) / 1e9
    alg_per_launch = tm.lde_bytes / launches
    _, ratio_pass = ntt_traffic()
    traffic = None
    if ratio_pass:  # PMC bytes per launch, scaled to this proof's per-pass byte count
        traffic = ratio_pass * tm.ntt_kernel_bytes / launches
    return {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": round(traffic) if traffic else None,
            "algorithmic_per_launch": round(alg_per_launch),
            "traffic_over_algorithmic": round(traffic / alg_per_launch, 3) if traffic else None,
            "traffic_source": "profiles/r06/profile_round_pmc_summary.json (FETCH_SIZE x2 + WRITE_SIZE per "
                              "launch, scaled to this proof's launches)",
            "basis": "SURVEY 8(d): 12*n*w B per coset LDE (read n, write 2n) / NTT kernel time",
            "kernel": "coset LDE = k_ntt_tile<false,14> (iDFT stages 0-13) + k_lde_mid<L> (iDFT "
                      "stages 14.., coset scale, DFT of both halves) + k_ntt_tile<true,14> (DFT "
                      "stages 13-0 of the 2n outputs)",
            "launches": tm.ntt_kernel_launches,
            "avg_launch_us": round(tm.ntt_kernel_ms * 1e3 / launches, 2),
            "kernel_ms": round(tm.ntt_kernel_ms, 3),
            "per_pass_gbs": round(per_pass, 1),
            "per_pass_frac": round(per_pass / HBM_PEAK_GBS, 4),
            "per_pass_note": "each launch's own read + write (8 B/elem tile pass, 12 B/input "
                             "elem middle): 3 HBM passes per LDE"}


def ntt_valu(tm):
    """VALU issue of the same NTT kernels FROM COUNTERS: the measured VALU
    wave-instructions per element-stage of each kernel (profiles/r05/ntt_counters.json, rocprofv3
    SQ_INSTS_VALU at a known element-stage count), weighted by its share of a 2^22 coset LDE, x the
    proof's element-stages / NTT kernel time = lane-instructions/s, against the 78.6 T lane-ops/s
    issue peak.  frac_units weights the instructions by the ISA's half-rate share (units per
    instruction, profiles/r02/ntt_isa_mix.txt); wait_any / wait_inst / valu_active are the SQ
    wave-state fractions of the same run: where the other cycles go."""
    if tm.ntt_kernel_ms <= 0 or tm.lde_elem_stages <= 0:
        return None
    try:
        ks = json.load(open(NTT_COUNTERS))["kernels"].values()
        fam = {k["family"]: k for k in ks}
        w = NTT_FAMILY_SHARE
        instr = sum(w[f] * fam[f]["valu_per_elem_stage"] for f in w)
        sq = {key: round(sum(w[f] * fam[f][key + "_per_wave_cycle"] for f in w), 3)
              for key in ("wait_any", "wait_inst_any", "active_inst_any", "valu_active")}
        per_kernel = {f: {"valu_instr_per_elem_stage": fam[f]["valu_per_elem_stage"],
                          "lds_instr_per_elem_stage": fam[f]["lds_per_elem_stage"],
                          "salu_instr_per_elem_stage": fam[f]["salu_per_elem_stage"],
                          "valu_issue_frac": fam[f]["valu_issue_frac"]} for f in w}
    except (OSError, KeyError, ValueError):
        return None
    lane_instr_s = instr * tm.lde_elem_stages / (tm.ntt_kernel_ms * 1e-3)
    units_per_instr = NTT_UNITS_PER_ELEM_STAGE / instr
    frac = lane_instr_s / (VALU_PEAK_TOPS * 1e12)
    return {"bound": "valu (latency / barrier-limited: see wait fractions)",
            "valu_instr_per_element_stage": round(instr, 3),
            "element_stages_per_proof": int(tm.lde_elem_stages),
            "achieved": round(lane_instr_s / 1e12, 1), "peak": round(VALU_PEAK_TOPS, 1),
            "unit": "T VALU lane-instructions/s", "frac": round(frac, 4),
            "frac_units": round(frac * units_per_instr, 4),
            "units_per_instruction_isa": round(units_per_instr, 3),
            "sq_fractions_of_wave_cycles": sq, "per_kernel": per_kernel,
            "source": "profiles/r05/ntt_counters.json (scripts/gpu_ntt_counters.sh: ubench_ntt "
                      "lde 22 8 under rocprofv3 --pmc)"}


def poseidon2_roofline(tm):
    """VALU roofline of the Merkle hashing kernels (k_hash_leaves, k_compress, k_hash_rows8),
    timed per launch with HIP events; these are integer-VALU bound, not HBM or MFMA."""
    if tm.p2_kernel_ms <= 0:
        return None
    gps = tm.p2_perms / (tm.p2_kernel_ms * 1e-3) / 1e9
    tops = gps * P2_UNITS_PER_PERM / 1e3
    return {"bound": "valu", "kernels": "k_hash_leaves + k_compress + k_hash_rows8",
            "perms_per_proof": int(tm.p2_perms), "kernel_ms": round(tm.p2_kernel_ms, 3),
            "launches": tm.p2_launches, "achieved_gperms_s": round(gps, 2),
            "units_per_perm": P2_UNITS_PER_PERM, "achieved": round(tops, 1),
            "peak": round(VALU_PEAK_TOPS, 1), "unit": "T full-rate VALU lane-ops/s",
            "frac": round(tops / VALU_PEAK_TOPS, 4)}


def openings_roofline(tm):
    """HBM roofline of the opening kernels, timed per launch with HIP events on the prover
    stream: k_open_partial_batch (barycentric sums over each matrix's low coset: 4 B per word +
    16 B per row and point for one weight table per LDE height) and k_reduce (FRI reduced
    openings over the whole LDE: 4 B per word + 16 B per row for each denominator table read
    and for ro written)."""
    out = {}
    for key, ms, nbytes, launches, kernel in (
            ("partial", tm.open_kernel_ms, tm.open_kernel_bytes, tm.open_kernel_launches,
             "k_open_partial_batch<NP>"),
            ("reduce", tm.reduce_kernel_ms, tm.reduce_kernel_bytes, tm.reduce_kernel_launches,
             "k_reduce")):
        if ms <= 0:
            continue
        gbs = nbytes / (ms * 1e-3) / 1e9
        out[key] = {"kernel": kernel, "bytes_per_proof": int(nbytes), "kernel_ms": round(ms, 3),
                    "launches": launches, "achieved": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4)}
    if not out:
        return None
    ms = sum(v["kernel_ms"] for v in out.values())
    nb = sum(v["bytes_per_proof"] for v in out.values())
    gbs = nb / (ms * 1e-3) / 1e9
    out.update({"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(gbs / HBM_PEAK_GBS, 4)})
    return out


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline():
    """The oracle (C restatement of the reference prover, OpenMP) proving the headline workload
    itself -- FIBO_X4 with stdin [255], Cpu trace 2^22 rows, executor included as in the
    reference's utils/prove.rs:23-66 -- on the host cores this process may use (its CPU
    affinity, capped by OMP_NUM_THREADS: the GPU box gives a one-GPU job a 16-core share).
    Runs in a child process so its OpenMP pool does not perturb the GPU process."""
    code = (
        "import sys,time; sys.path.insert(0,%r); sys.path.insert(0,%r);"
        "import oracle_lib as O; from bfz import guests;"
        "t=time.time(); O.prove(guests.FIBO_X4,[255]); print(time.time()-t)"
    ) % (os.path.join(ROOT, "tests"), os.path.join(ROOT, "zkvm-brainfuck_amd"))
    threads, avail = host_threads()
    env = dict(os.environ, OMP_NUM_THREADS=str(threads))
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                         timeout=900)
    secs = float(out.stdout.strip().splitlines()[-1])
    return {"value": round(secs * 1000.0, 1), "unit": "ms per 2^22-row core proof",
            "cores": threads, "kind": "port",
            "nproc": os.cpu_count(), "affinity_cpus": avail, "cpu_model": cpu_model(),
            "threads_note": ("OMP_NUM_THREADS caps the pool: the GPU pool sets it to this job's "
                             "CPU share (16 cores per GPU) although nproc shows the whole host"
                             if threads < avail else "every CPU this process may use"),
            "sample": f"whole headline workload: oracle prove of FIBO_X4 stdin [255] (3,767,729 "
                      f"cycles, Cpu 2^22 rows, executor included) = {secs:.2f} s on {threads} "
                      f"OpenMP threads"}


def end_to_end(client, pk, prog, stdin, jobs=24):
    """Proofs from (program, stdin) with execution and upload included: the reference's
    utils/prove.rs:23-66 loop (execute, then prove) as bfz_prove_batch pipelines it -- executor
    threads into pinned memory, a copy stream for the events, the GPU proving job k while job
    k+1 executes and uploads -- next to one unpipelined bfz_prove (execute + upload + prove)."""
    import time as _t
    # warm-up batch: every pinned host buffer reaches its steady size (growth pins fresh pages)
    client.prove_batch(pk, [stdin] * 8, public_values=False)
    stats = {}
    t0 = _t.perf_counter()
    proofs = client.prove_batch(pk, [stdin] * jobs, public_values=False, stats=stats)
    wall = (_t.perf_counter() - t0) * 1e3
    import ctypes
    from bfz import _lib as _l
    buf, n = _l.u8buf(stdin)
    singles = []
    for _ in range(3):
        t1 = _t.perf_counter()
        ptr = ctypes.POINTER(ctypes.c_uint8)()
        plen = ctypes.c_size_t()
        _l.check(_l.lib().bfz_prove(ctypes.c_void_p(pk.handle), buf, n, ctypes.byref(ptr),
                                    ctypes.byref(plen)))
        singles.append((_t.perf_counter() - t1) * 1e3)
        one = _l.take_bytes(ptr, plen.value)
    assert all(p.proof == one for p in proofs), "batch proofs differ from bfz_prove"
    return {"jobs": jobs, "ms_per_proof": round(wall / jobs, 3),
            "proofs_per_s": round(jobs * 1e3 / wall, 3),
            "exec_threads": stats["exec_threads"],
            "exec_ms_per_job": round(stats["exec_ms"] / jobs, 3),
            "upload_ms_per_job": round(stats["upload_ms"] / jobs, 3),
            "prove_ms_per_job": round(stats["prove_ms"] / jobs, 3),
            "unpipelined_bfz_prove_ms": round(min(singles), 3),
            "what": "bfz_prove_batch of FIBO_X4 stdin [255] from the program text: execution "
                    "(host threads), event upload (copy stream) and proving overlapped; "
                    "unpipelined = one bfz_prove (execute, upload, prove in sequence)"}


def drop_in_path(pk, prog, stdin, ref_proof, steps=3):
    """bfz_prove_traces -- the entry a Rust MachineProver::prove would call -- from host
    row-major traces (the reference's generate_traces output, prover.rs:58-81): pinned
    double-buffered upload, transpose to the device layout, proof.  Traces are generated on
    the host before the timed region."""
    import time as _t
    from bfz import sdk as _s
    traces = _s.generate_traces(prog, stdin)
    prover = _s.CoreProver()
    prover.prove(pk, traces)  # warm
    times = []
    for _ in range(steps):
        t0 = _t.perf_counter()
        pf = prover.prove(pk, traces)
        times.append((_t.perf_counter() - t0) * 1e3)
    assert pf == ref_proof, "host-trace proof differs from the record path"
    nbytes = sum(int(t.nbytes) for _, _, t in traces)
    return {"ms": round(min(times), 3), "trace_bytes": nbytes,
            "what": "bfz_prove_traces from host row-major traces (all 8 chips, "
                    f"{nbytes / 1e9:.2f} GB) incl. upload + transpose + proof"}


def events_path(pk, prog, stdin, ref_proof, steps=3):
    """The Rust HipProver::prove path: the reference record (Executor::run's ExecutionRecord) ->
    the compact hand-over (CycleArrays::new: one 16-byte bfz_cycle per CpuEvent + the memory
    events, pageable host memory) -> bfz_record_from_cycles (upload, device rebuild of every
    event, validation) -> bfz_record_prove (device trace generation + proof).  The executor runs
    before the timed region, as it does before MachineProver::prove (utils/prove.rs:38-44); the
    host conversion is timed on its own (numpy here; rayon over cpu_events in the Rust crate).
    The full-event hand-over (bfz_record_from_events, ~64 B per cycle) is timed beside it."""
    import ctypes
    import time as _t
    from bfz import _lib as _l, events as _e
    rec = _e.ExecutionRecordArrays.from_executor(prog, stdin)

    def prove(drec):
        ptr = ctypes.POINTER(ctypes.c_uint8)()
        plen = ctypes.c_size_t()
        _l.check(_l.lib().bfz_record_prove(ctypes.c_void_p(pk.handle), ctypes.c_void_p(drec.handle),
                                           ctypes.byref(ptr), ctypes.byref(plen), None))
        return _l.take_bytes(ptr, plen.value)

    conv = []
    for _ in range(3):
        t0 = _t.perf_counter()
        cyc = _e.cycles_from_record(rec, pinned=True)
        conv.append((_t.perf_counter() - t0) * 1e3)
    cyc_pageable = _e.cycles_from_record(rec)

    def best(one):
        one()  # warm
        times, pf = [], None
        for _ in range(steps):
            t0 = _t.perf_counter()
            pf = one()
            times.append((_t.perf_counter() - t0) * 1e3)
        return min(times), pf

    ms, pf = best(lambda: prove(_e.record_from_cycles(pk, cyc, rec.memory)))
    assert pf == ref_proof, "compact-cycle proof differs from the record path"
    compiled = compiled_handover(pk, rec, prove, best, ref_proof)
    ms_pageable, pf = best(lambda: prove(_e.record_from_cycles(pk, cyc_pageable, rec.memory)))
    assert pf == ref_proof, "compact-cycle proof (pageable hand-over) differs from the record path"
    ms_full, pf = best(lambda: prove(_e.record_from_events(pk, rec)))
    assert pf == ref_proof, "events-path proof differs from the record path"
    nbytes = int(cyc.nbytes + rec.memory.nbytes)
    full = sum(int(getattr(rec, k).nbytes) for k in ("cpu", "add", "sub", "jump", "io",
                                                     "memory_instr", "memory"))
    return {"ms": round(ms, 3), "compiled": compiled, "handover_bytes": nbytes,
            "bytes_per_cycle": round(nbytes / len(rec.cpu), 2),
            "host_conversion_ms": round(min(conv), 3),
            "host_conversion_what": "cycles_from_record (numpy, one thread) over the record's "
                                    f"{len(rec.cpu)} cpu_events, into bfz_host_alloc memory",
            "pageable_ms": round(ms_pageable, 3),
            "full_events_ms": round(ms_full, 3), "full_event_bytes": full,
            "what": "bfz_record_from_cycles (16 B per cycle in page-locked bfz_host_alloc memory, "
                    f"as the Rust CycleArrays builds it, + memory events; {nbytes / 1e6:.0f} MB) + "
                    "bfz_record_prove: the Rust HipProver::prove path, upload and device event "
                    "rebuild included; pageable_ms = the same hand-over from pageable memory "
                    "(staged through the library's pinned chunks); full_events_ms = the full "
                    f"events through bfz_record_from_events ({full / 1e6:.0f} MB, pageable)"}


def host_threads():
    """The CPU threads this process may use: its affinity, capped by OMP_NUM_THREADS (the GPU
    pool sets it to a one-GPU job's share, 16, although nproc shows the whole host)."""
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    return min(avail, int(os.environ.get("OMP_NUM_THREADS") or avail)), avail


def compiled_handover(pk, rec, prove, best, ref_proof, chunk=1 << 17):
    """The Rust HipProver::prove path with its host conversion in compiled code (VERDICT r4 item
    2): crates/bf-hip-prover/standin/libcycle_arrays.so converts record.cpu_events -- laid out as
    rustc lays out Vec<CpuEvent>, 48 B each -- on the job's threads straight into page-locked
    memory, as CycleArrays::new does with rayon.  Three timings, each from the Rust-layout events
    to the finished proof:
      conversion_ms  the conversion alone (CycleArrays::new)
      sequential_ms  conversion, then one bfz_record_from_cycles, then bfz_record_prove
      pipelined_ms   conversion in chunks of `chunk` cycles, each pushed (bfz_cycles_push) as soon
                     as it is written so its DMA overlaps the next chunk's conversion; then
                     bfz_cycles_finish and bfz_record_prove"""
    import time as _t
    from bfz import events as _e
    threads, _ = host_threads()
    rs = _e.rust_cpu_events(rec)
    out = _e.pinned_empty(len(rs), _e.CYCLE)
    sa = _e.CycleArraysStandin()
    conv = []
    for _ in range(5):
        t0 = _t.perf_counter()
        sa.convert(rs, out, threads)
        conv.append((_t.perf_counter() - t0) * 1e3)
    seq_ms, pf = best(lambda: (sa.convert(rs, out, threads),
                               prove(_e.record_from_cycles(pk, out, rec.memory)))[1])
    assert pf == ref_proof, "compiled-conversion proof differs from the record path"
    pushed = []

    def piped():
        drec, cms = sa.handover(pk, rs, rec.memory, out, threads, chunk)
        pushed.append(cms)
        return prove(drec)
    pipe_ms, pf = best(piped)
    assert pf == ref_proof, "pipelined hand-over proof differs from the record path"
    return {"conversion_ms": round(min(conv), 3), "sequential_ms": round(seq_ms, 3),
            "pipelined_ms": round(pipe_ms, 3), "pipelined_last_push_ms": round(min(pushed), 3),
            "threads": threads, "chunk_cycles": chunk, "rust_event_bytes": int(rs.nbytes),
            "what": "crates/bf-hip-prover/standin/cycle_arrays.cpp: CycleArrays::new compiled "
                    "(C++ stand-in of the Rust crate, no Rust toolchain here) over cpu_events in "
                    "the rustc layout (48 B per event) into bfz_host_alloc memory on the job's "
                    "threads; sequential = convert + bfz_record_from_cycles + prove, pipelined = "
                    "chunked conversion with each chunk's DMA overlapping the next "
                    "(bfz_cycles_push) + bfz_cycles_finish + prove; the proof is checked"}


SHARDED_EXTRA_LIMIT_S = 150


def run_with_limit(fn, seconds):
    """fn() in a daemon thread; its result, or None if it has not returned within `seconds`."""
    import threading
    box = {}

    def body():
        try:
            box["r"] = fn()
        except Exception as e:  # noqa: BLE001 - reported in the bench line
            box["r"] = {"error": f"{type(e).__name__}: {e}"}

    th = threading.Thread(target=body, daemon=True)
    th.start()
    th.join(seconds)
    return None if th.is_alive() else box.get("r")


def sharded_latency(dist, pk, rec, rank, world, device, ref_proof, steps=3):
    """Latency of ONE proof split over all ranks (bfz_record_prove_sharded: every rank hashes
    its subtree of each large Merkle tree; the subtree roots are all-gathered and the query
    openings sum-all-reduced over RCCL on device buffers), measured after the replica timing
    on the same record and checked byte for byte against the single-GPU proof.  Needs one GPU
    per rank; guarded by a 120 s collective timeout so a failure cannot hang the bench."""
    import datetime
    import torch
    from bfz import _lib as _l, shard as _sh
    if "BFZ_DEVICE" in os.environ or torch.cuda.device_count() < world:
        return {"skipped": "ranks share a GPU (RCCL needs one GPU per rank)"}
    try:
        torch.cuda.set_device(device)
        grp = dist.new_group(backend="nccl", timeout=datetime.timedelta(seconds=120))
        coll = _sh.Collectives(dist, group=grp, device=device)
        pf = _sh.prove_record_sharded(pk.handle, rec, coll, rank)
        exact = pf == ref_proof
        ms = timed_steps(lambda: _sh.prove_record_sharded(pk.handle, rec, coll, rank), steps, dist,
                         sync=lambda: _l.check(_l.lib().bfz_synchronize()))
        return {"ms_per_proof": round(ms, 3), "steps": steps, "bit_exact_vs_single_gpu": exact,
                "ranks": world, "scaling": "strong (one proof over all ranks)",
                "collectives": "RCCL (torch nccl backend): subtree-root all-gather + query-word "
                               "all-reduce on HBM buffers"}
    except Exception as e:  # keep the replica line if the sharded path fails
        return {"error": f"{type(e).__name__}: {e}"}


# Collective-time model of the N-GPU sharded proof.  Inputs, stated as
# assumptions because this pool has no multi-GPU box to measure RCCL on:
#  - xGMI: 7 links per MI355X, ~153 GB/s each (the build brief's figure, taken as bidirectional),
#    so 76.8 GB/s per direction per link; every pair of GPUs of the node has its own link;
#  - RCCL reaches XGMI_EFF of a link's rate on large messages and costs XGMI_ALPHA_US per
#    collective (launch + synchronisation) on small ones.
XGMI_LINK_GBS = 153.6 / 2
XGMI_EFF = 0.7
XGMI_ALPHA_US = 20.0


def collective_ms(kind, nbytes, world):
    """One collective on a fully connected node: an all-gather of `nbytes` per rank sends it to
    each of the N-1 peers over their own links in parallel; a sum all-reduce of an `nbytes`
    vector is a reduce-scatter plus an all-gather of nbytes/N per peer link."""
    bw = XGMI_LINK_GBS * XGMI_EFF * 1e9
    if kind == 0:
        return (XGMI_ALPHA_US * 1e-6 + nbytes / bw) * 1e3
    return (2 * XGMI_ALPHA_US * 1e-6 + 2 * (nbytes / world) / bw) * 1e3


def collective_model(exchanges, world, overlaps=None):
    """Per-rank bytes and modeled time of the logged collectives of one rank's share.  overlaps[i]
    (bfz_shard_solo_overlaps, from the instrumented run): GPU milliseconds the rank has queued to
    run while collective i is in flight -- already inside the share's compute time, so collective
    i adds max(0, its time - overlaps[i])."""
    ov = list(overlaps or []) + [0.0] * max(0, len(exchanges) - len(overlaps or []))
    full = [collective_ms(k, b, world) for k, b in exchanges]
    ms = sum(max(0.0, t - o) for t, o in zip(full, ov))
    recv = sum((world - 1) * b if k == 0 else 2 * (world - 1) * b / world for k, b in exchanges)
    big = sorted(((b, k) for k, b in exchanges), reverse=True)[:4]
    return {"collectives": len(exchanges),
            "unoverlapped_ms": round(sum(full), 3),
            "overlapped_ms": round(sum(min(t, o) for t, o in zip(full, ov)), 3),
            "allgathers": sum(1 for k, _ in exchanges if k == 0),
            "allreduces": sum(1 for k, _ in exchanges if k == 1),
            "recv_bytes_per_rank": int(recv),
            "largest": [{"kind": "all-gather" if k == 0 else "all-reduce", "bytes_per_rank": int(b),
                         "ms": round(collective_ms(k, b, world), 3)} for b, k in big],
            "modeled_ms": round(ms, 3)}


def replication_tradeoff(stages, cells_main, cells_perm, world):
    """The work every rank repeats at N GPUs (main + permutation iDFTs, LogUp rows: measured on
    the slowest rank's share) against the column-sharded alternative: each rank runs the iDFT and
    the full coset LDE of 1/N of the columns, then one all-to-all turns column shards into the
    row shards the Merkle subtrees need (each rank sends (N-1)/N of its 2n x w/N LDE words, over
    N-1 links in parallel); the LogUp rows need whole rows of the main trace, so sharding them
    would add an all-gather of the main trace (modeled the same way)."""
    replicated = stages.get("main_idft_ms", 0) + stages.get("perm_idft_ms", 0) + stages.get("perm_rows_ms", 0)
    lde_words = 2 * (cells_main + cells_perm)
    a2a_bytes_per_link = 4 * lde_words / world / world
    a2a = collective_ms(0, a2a_bytes_per_link, world)
    gather_main = collective_ms(0, 4 * cells_main / world, world)
    alt = ((stages.get("main_idft_ms", 0) + stages.get("perm_idft_ms", 0)) / world
           + stages.get("perm_rows_ms", 0) / world + a2a + gather_main)
    return {"replicated_ms": round(replicated, 3), "column_sharded_ms": round(alt, 3),
            "all_to_all_ms": round(a2a, 3), "main_trace_allgather_ms": round(gather_main, 3),
            "choice": "replicate" if replicated <= alt else "column-shard"}


def shard_solo(pk, rec, world, steps=3):
    """Per-rank work of a `world`-GPU sharded proof measured on ONE GPU (VERDICT r2 Next 6):
    bfz_record_prove_shard_solo runs rank k's share -- the same kernels and sizes as
    bfz_record_prove_sharded on rank k -- with the exchanges as no-ops, for every k; the slowest
    rank is the predicted per-proof latency of the N-GPU proof before collective time."""
    import ctypes
    from bfz import _lib as _l
    L = _l.lib()
    ranks = []
    exchanges = None
    for k in range(world):
        # stage breakdown from one instrumented run (stage events + per-launch kernel probes: the
        # probes' host work stretches a many-launch share), the share's time from uninstrumented
        # runs on the wall clock, as the single-GPU headline is timed
        best = _l.Timings()
        _l.check(L.bfz_record_prove_shard_solo(ctypes.c_void_p(pk.handle), rec, k, world,
                                               ctypes.byref(best)))
        n = ctypes.c_size_t()  # the GPU work beside each collective, from this timed run
        _l.check(L.bfz_shard_solo_overlaps(None, 0, ctypes.byref(n)))
        ovl = (ctypes.c_double * max(n.value, 1))()
        _l.check(L.bfz_shard_solo_overlaps(ovl, n.value, ctypes.byref(n)))
        overlaps = [round(ovl[i], 4) for i in range(n.value)]
        wall = []
        for _ in range(steps):
            _l.check(L.bfz_synchronize())
            t0 = time.perf_counter()
            _l.check(L.bfz_record_prove_shard_solo(ctypes.c_void_p(pk.handle), rec, k, world, None))
            _l.check(L.bfz_synchronize())
            wall.append((time.perf_counter() - t0) * 1e3)
        if exchanges is None:  # every rank takes part in the same collectives
            n = ctypes.c_size_t()
            _l.check(L.bfz_shard_solo_exchanges(None, None, 0, ctypes.byref(n)))
            kinds = (ctypes.c_int * max(n.value, 1))()
            sizes = (ctypes.c_uint64 * max(n.value, 1))()
            _l.check(L.bfz_shard_solo_exchanges(kinds, sizes, n.value, ctypes.byref(n)))
            exchanges = [(kinds[i], sizes[i]) for i in range(n.value)]
            cells = (best.main_cells, best.perm_cells)
        ranks.append({"rank": k, "total_ms": round(min(wall), 3),
                      "instrumented_total_ms": round(best.total_ms, 3),
                      "collective_overlap_ms": overlaps,
                      "stages_ms": {n: round(v, 3) for n, v in best.as_dict().items()
                                    if n.endswith("_ms") and n not in ("total_ms", "lde_ms", "ntt_kernel_ms", "p2_kernel_ms")}})
    worst = max(r["total_ms"] for r in ranks)
    slow = max(ranks, key=lambda r: r["total_ms"])
    # the overlap a collective gets is the least any rank queues beside it (every rank waits)
    ovs = [r["collective_overlap_ms"] for r in ranks]
    overlap = [min(o[i] if i < len(o) else 0.0 for o in ovs) for i in range(len(exchanges))]
    return {"world": world, "max_rank_ms": worst, "ranks": ranks,
            "collectives": collective_model(exchanges, world, overlap),
            "replication": replication_tradeoff(slow["stages_ms"], cells[0], cells[1], world),
            "what": f"each rank's share of a {world}-GPU sharded proof run alone on one GPU with "
                    "no-op exchanges (bfz_record_prove_shard_solo); total_ms = best wall time of "
                    f"{steps} uninstrumented runs, stages from one instrumented run; excludes "
                    "collective time"}


def sustained(step, seconds, sync):
    """Proofs back to back for about `seconds` after the timed steps (same record, same
    stream): the steady-state rate over many proofs, and a GPU phase long enough for a
    utilisation sampler polling every few seconds to see the device busy."""
    sync()
    t0 = time.perf_counter()
    k = 0
    while time.perf_counter() - t0 < seconds:
        step()
        k += 1
    sync()
    wall = time.perf_counter() - t0
    return {"proofs": k, "seconds": round(wall, 3), "ms_per_proof": round(wall * 1e3 / max(k, 1), 3),
            "what": "back-to-back proofs of the same record after the timed steps (one rank)"}


def sustained_lanes(pk, rec, ms_one, seconds, ref_proof):
    """The same steady state through bfz_record_prove_repeat with 1, 2 and 3 proofs in flight
    (VERDICT r4 item 5): two lanes (streams, pools, pinned mailboxes, one host thread each) let
    one proof's latency-bound launches run beside the other's bulk kernels.  Every proof is
    compared with the first inside the library; the first is checked here."""
    import ctypes
    from bfz import _lib as _l
    L = _l.lib()
    out = {}
    count = max(4, int(seconds * 1e3 / max(ms_one, 1.0)))
    for inflight in (1, 2, 3):
        ptr = ctypes.POINTER(ctypes.c_uint8)()
        n = ctypes.c_size_t()
        wall = ctypes.c_double()
        _l.check(L.bfz_record_prove_repeat(ctypes.c_void_p(pk.handle), rec, count, inflight,
                                           ctypes.byref(ptr), ctypes.byref(n), ctypes.byref(wall)))
        if _l.take_bytes(ptr, n.value) != ref_proof:
            raise SystemExit("bench: bfz_record_prove_repeat proof differs from the verified proof")
        out[str(inflight)] = round(wall.value / count, 3)
    pool = {}  # each lane's buffer pool after the runs: the device resident set of one proof in flight
    for lane in range(4):
        b = ctypes.c_uint64()
        _l.check(L.bfz_device_pool_bytes(lane, ctypes.byref(b)))
        if b.value:
            pool[str(lane)] = round(b.value / 2**30, 2)
    return {"proofs": count, "ms_per_proof_by_inflight": out, "pool_gib_by_lane": pool,
            "what": "bfz_record_prove_repeat: `proofs` proofs of the record back to back with 1, 2 or "
                    "3 in flight (one lane = stream + buffer pool + pinned mailboxes + host thread); "
                    "all byte-identical, the first checked against the verified proof; the "
                    "headline `value` stays the single-proof latency; pool_gib_by_lane = device "
                    "memory each lane's buffer pool holds afterwards (bfz_device_pool_bytes; "
                    "process-wide tables, keys and record events not included: they "
                    "live in a separate resident pool)"}


def timed_steps(step, steps, dist=None, sync=lambda: None):
    """Runs `step` exactly `steps` times between barrier + device synchronize on both sides
    and returns ms per step, the max over ranks (every rank proves its own replica; the
    slowest sets the job's pace)."""
    if dist:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    t1 = time.perf_counter()
    if dist:
        dist.barrier()
    ms = (t1 - t0) * 1000.0 / steps
    if dist:
        import torch
        t = torch.tensor([ms], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ms = float(t.item())
    return ms


def cold_first_proof():
    """The first proof of a fresh process: scripts/cold_first_proof.py in a
    child process -- init, setup, record, ONE prove (timed), host-verified, then two warm proofs
    of the same record -- with nothing else on the GPU (it runs before this process initialises
    the device).  The reference's `e2e=` timer brackets exactly such a single prove call
    (crates/core/machine/src/utils/prove.rs:44-56)."""
    out = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "cold_first_proof.py")],
                         capture_output=True, text=True, timeout=300)
    if out.returncode != 0:
        return {"error": (out.stderr or out.stdout).strip().splitlines()[-1:]}
    r = json.loads(out.stdout.strip().splitlines()[-1])
    r["what"] = ("fresh child process: bfz_init, setup (ProverClient::setup), bfz_record_new "
                 "(execute + event upload + the tables for the record's heights), then ONE "
                 "bfz_record_prove = first_prove_ms; warm_prove_ms = the next proofs of the record")
    return r


def run_pcs(args, rank, world, device, dist, coll):
    """Column-sharded commit + FRI commit phase of a synthetic 2^log_n x cols trace (uniform
    random Montgomery words, seeded per rank); one step = bfz_commit_fri_sharded on every rank:
    LDE of the rank's columns, the all-to-all, the Merkle commit and the FRI rounds."""
    import torch
    from bfz import shard as bfz_shard
    P = 0x7F000001
    log_n, W = args.log_n, args.cols
    if W % world:
        raise SystemExit(f"--cols {W} is not divisible by {world} ranks")
    wl = W // world
    dev = torch.device("cuda", device)
    torch.cuda.set_device(dev)

    def rank_cols(r):  # rank r's columns: uniform words, seeded per rank
        g = torch.Generator(device=dev)
        g.manual_seed(0x5EED + r)
        return torch.randint(0, P, (wl, 1 << log_n), dtype=torch.int32, device=dev, generator=g)

    cols = rank_cols(rank)
    send = recv = None
    if world > 1:
        send = torch.empty((wl * (2 << log_n),), dtype=torch.int32, device=dev)
        recv = torch.empty_like(send)

    def step():
        return bfz_shard.commit_fri_sharded(cols, log_n, coll, rank, send, recv)

    for _ in range(args.warmup):
        root, fri, fin = step()
    ms = timed_steps(step, args.steps, dist, sync=torch.cuda.synchronize)
    root, fri, fin = step()  # collective: every rank takes part
    exact = None
    if world > 1 and rank == 0:
        # the same trace committed by one rank alone (world = 1): the sharded root, FRI roots and
        # final value must be identical
        full = torch.cat([rank_cols(r) for r in range(world)])
        r1, f1, fin1 = bfz_shard.commit_fri_sharded(full, log_n, None, 0)
        exact = bool((r1 == root).all() and f1.shape == fri.shape and (f1 == fri).all()
                     and (fin1 == fin).all())
        del full
    if rank == 0:
        n = 1 << log_n
        lde_bytes = 12.0 * n * W  # coset LDE algorithmic bytes of the whole trace
        line = {
            "metric": f"column-sharded commit + FRI commit phase, synthetic 2^{log_n} x {W} trace",
            "value": round(ms, 3), "unit": "ms", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms, 3), "higher_is_better": False,
            "scaling": "strong", "vs_baseline": None, "dtype": "u32 (KoalaBear mod-p)",
            "data": "synthetic: uniform random field words, seeded per rank",
            "config": {"workload": f"trace 2^{log_n} rows x {W} columns, {wl} per rank; LDE x2, "
                                   "Merkle commit, FRI fold to a constant",
                       "parallelism": f"column shards x{world} -> all-to-all -> row shards"},
            "trace_cells_per_s": round(n * W / (ms * 1e-3), 1),
            "lde_equiv_gbs": round(lde_bytes / (ms * 1e-3) / 1e9, 1),
            "fri_rounds": int(len(fri)),
            "bit_exact_vs_world1": exact,
            "root": [int(x) for x in root],
        }
        print(json.dumps(line), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-cold", action="store_true",
                    help="skip the fresh-process first-proof measurement (cold_first_proof_ms)")
    ap.add_argument("--rccl-sharded", action="store_true",
                    help="replicas mode at N > 1: also time one proof split over all ranks over RCCL "
                         "(sharded_proof; never run on hardware with more than one rank -- opt-in "
                         "so a hang in an unvalidated collective cannot cost the replica line)")
    ap.add_argument("--no-extra", action="store_true",
                    help="skip the end-to-end batch and drop-in-path figures")
    ap.add_argument("--mode", choices=("replicas", "sharded", "pcs"), default="replicas",
                    help="replicas: one independent proof per rank (weak scaling, default); "
                         "sharded: one proof split across all ranks (strong scaling); "
                         "pcs: column-sharded commit + FRI of a synthetic trace (BASELINE "
                         "configs 4/5, strong scaling)")
    ap.add_argument("--sustain-s", type=float, default=8.0,
                    help="replicas mode: seconds of back-to-back proofs after the timed steps "
                         "(0 = skip)")
    ap.add_argument("--solo-world", default="2,4,8",
                    help="replicas mode at N=1: also time each rank's share of an N-GPU sharded "
                         "proof alone (bfz_record_prove_shard_solo) for each N of this "
                         "comma-separated list -- the predicted strong-scaling curve of one proof "
                         "before collective time ('' or 0 = skip)")
    ap.add_argument("--log-n", type=int, default=24, help="pcs mode: trace rows = 2^log_n")
    ap.add_argument("--cols", type=int, default=64, help="pcs mode: trace columns")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    sharded = args.mode in ("sharded", "pcs") and world > 1
    # gloo prints its connection banner on stdout during init: keep stdout for the JSON line
    sys.stdout.flush()
    saved_stdout = os.dup(1)
    os.dup2(2, 1)
    if world > 1:
        # a failed RCCL collective raises after its timeout instead of hanging (sharded_latency)
        os.environ.setdefault("TORCH_NCCL_BLOCKING_WAIT", "1")
        import torch.distributed as dist
        if sharded:
            import torch
            own_gpu = ("BFZ_DEVICE" not in os.environ and torch.cuda.is_available()
                       and local_rank < torch.cuda.device_count())
            if own_gpu:  # exchanges over RCCL (xGMI), CPU tensors (timing) over gloo
                torch.cuda.set_device(local_rank)
                dist.init_process_group("cpu:gloo,cuda:nccl")
            else:  # several ranks on one GPU (testing)
                dist.init_process_group("gloo")
        else:
            dist.init_process_group("gloo")
        dist.barrier()  # every rank connected before stdout is restored
    os.dup2(saved_stdout, 1)
    os.close(saved_stdout)

    cold = None
    if world == 1 and args.mode == "replicas" and not args.no_cold:
        cold = cold_first_proof()  # before this process touches the GPU

    from bfz import _lib, guests, sdk
    import ctypes

    from bfz import shard as bfz_shard
    # BFZ_DEVICE pins every rank to one GPU (rehearsing --mode sharded on a one-GPU box)
    device = int(os.environ.get("BFZ_DEVICE", local_rank))
    _lib.init(device)
    if args.mode == "pcs":
        run_pcs(args, rank, world, device, dist,
                bfz_shard.Collectives(dist, device=device) if world > 1 else None)
        if dist:
            dist.destroy_process_group()
        return
    L = _lib.lib()
    client = sdk.ProverClient(device=device)
    prog, stdin = guests.FIBO_X4, bytes([255])
    pk, vk = client.setup(prog)
    rec = ctypes.c_void_p()
    cycles = ctypes.c_uint64()
    buf, n = _lib.u8buf(stdin)
    _lib.check(L.bfz_record_new(ctypes.c_void_p(pk.handle), buf, n, ctypes.byref(rec),
                                ctypes.byref(cycles)))

    coll = bfz_shard.Collectives(dist, device=device) if sharded else None

    def one(timings=None):
        if sharded:
            return bfz_shard.prove_record_sharded(pk.handle, rec, coll, rank, timings)
        ptr = ctypes.POINTER(ctypes.c_uint8)()
        plen = ctypes.c_size_t()
        _lib.check(L.bfz_record_prove(ctypes.c_void_p(pk.handle), rec, ctypes.byref(ptr),
                                      ctypes.byref(plen), ctypes.byref(timings) if timings else None))
        return _lib.take_bytes(ptr, plen.value)

    t_first = time.perf_counter()
    first_proof = one()  # the first prove after setup in this process (counts as a warmup step)
    first_ms = (time.perf_counter() - t_first) * 1e3
    for _ in range(args.warmup - 1):  # the lane's buffer pool fills during the first proofs
        one()
    # one timed-with-events proof for the roofline (kept out of the headline timing), verified on
    # the host; the warmup is repeated after it, right before the timed steps, so the GPU is not
    # coming out of the idle (clocked-down) phase of the host verification when timing starts
    tm = _lib.Timings()
    proof = one(tm)
    client.verify(sdk.BfProofWithPublicValues(proof=proof, stdin=stdin), vk)
    for _ in range(args.warmup):
        one()

    last = {}

    def kept():  # the proof stays referenced; it is compared after the timed region
        last["proof"] = one()

    ms = timed_steps(kept, args.steps, dist, sync=lambda: _lib.check(L.bfz_synchronize()))
    # every timed step proves the same record: the last one must be the verified proof's bytes
    if last["proof"] != proof:
        raise SystemExit("bench: the last timed proof differs from the verified proof")
    if first_proof != proof:
        raise SystemExit("bench: the first proof differs from the verified proof")
    extra = {}
    if not sharded and args.sustain_s > 0:
        last.clear()
        extra["sustained"] = sustained(kept, args.sustain_s,
                                       sync=lambda: _lib.check(L.bfz_synchronize()))
        if last["proof"] != proof:
            raise SystemExit("bench: the last sustained proof differs from the verified proof")
        extra["sustained"]["last_proof_checked"] = True
        extra["sustained"]["lanes"] = sustained_lanes(pk, rec, ms, args.sustain_s, proof)
    hung = False
    if world > 1 and not sharded and args.rccl_sharded:  # every rank takes part
        # RCCL has no run on this pool's one-GPU boxes: a hang in it must not cost the replica
        # line, so the attempt runs in a thread with a wall-clock limit of its own
        res = run_with_limit(lambda: sharded_latency(dist, pk, rec, rank, world, device, proof),
                             SHARDED_EXTRA_LIMIT_S)
        # a failed or abandoned RCCL attempt may leave a communicator blocked: skip teardown
        hung = res is None or "error" in res
        extra["sharded_proof"] = res if res is not None else {
            "error": f"no result within {SHARDED_EXTRA_LIMIT_S} s (abandoned)"}

    if rank == 0:
        lde_gbs = tm.lde_bytes / (tm.lde_ms * 1e-3) / 1e9 if tm.lde_ms > 0 else 0.0
        # whole job: replicas finish `world` proofs every `ms`; sharded ranks finish one
        job_ms = ms if sharded else ms / world
        line = {
            "metric": "core-proof wall-time (ms) + NTT HBM GB/s, fibonacci trace 2^22 rows",
            "value": round(job_ms, 3),
            "unit": "ms",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": False,
            "scaling": "strong" if sharded else "weak",
            "vs_baseline": None,
            "dtype": "u32 (KoalaBear mod-p)",
            "data": "real execution trace of the FIBO_X4 guest, stdin [255] (no synthetic fill)",
            "config": {"workload": "fibo_x4 stdin[255]: 3,767,729 cycles, Cpu trace 2^22 rows, "
                                   "full core proof (84 FRI queries, 16 PoW bits)",
                       "cycles": cycles.value,
                       "parallelism": f"sharded x{world}" if sharded else f"replicas x{world}",
                       "value_is": ("ms per proof, one proof sharded over all ranks" if sharded
                                    else "ms per proof for the whole job = step time / ranks")},
            "aggregate_proofs_per_s": round((1 if sharded else world) * 1000.0 / ms, 4),
            "ntt_hbm_gbs": round(lde_gbs, 1),
            "stages_ms": {k: round(v, 3) for k, v in tm.as_dict().items() if k.endswith("_ms")},
            "roofline": ntt_roofline(tm),
            "ntt_valu": ntt_valu(tm),
            "poseidon2": poseidon2_roofline(tm),
            "openings": openings_roofline(tm),
            "first_prove_after_setup_ms": round(first_ms, 3),
            "cold_first_proof_ms": cold.get("first_prove_ms") if cold else None,
            "cold_first_proof": cold,
            "proof_bytes": len(proof),
            "proof_check": "host verifier accepted the proof; the last timed proof (and the last "
                           "sustained one) are byte-identical to it",
        }
        if "sustained" in extra:
            line["sustained"] = extra["sustained"]
        if world > 1 and not sharded and "sharded_proof" in extra:
            line["sharded_proof"] = extra["sharded_proof"]
        solo = [int(x) for x in str(args.solo_world).split(",") if x.strip() and int(x) > 1]
        if world == 1 and solo:
            runs = {n: shard_solo(pk, rec, n) for n in solo}
            curve = {"1": round(ms, 3)}
            curve.update({str(n): runs[n]["max_rank_ms"] for n in solo})
            modeled = {str(n): runs[n]["collectives"]["modeled_ms"] for n in solo}
            with_coll = {"1": round(ms, 3)}
            with_coll.update({str(n): round(runs[n]["max_rank_ms"] + runs[n]["collectives"]["modeled_ms"], 3)
                              for n in solo})
            line["shard_solo_curve"] = {
                "ms_per_proof_by_gpus": curve,
                "speedup_by_gpus": {k: round(ms / v, 2) for k, v in curve.items()},
                "modeled_collective_ms": modeled,
                "ms_per_proof_with_collectives": with_coll,
                "speedup_with_collectives": {k: round(ms / v, 2) for k, v in with_coll.items()},
                "collectives_by_gpus": {str(n): runs[n]["collectives"] for n in solo},
                "replication_by_gpus": {str(n): runs[n]["replication"] for n in solo},
                "collective_model": {
                    "xgmi_link_gbs_per_direction": XGMI_LINK_GBS, "efficiency": XGMI_EFF,
                    "latency_us_per_collective": XGMI_ALPHA_US,
                    "source": "build brief: 7 xGMI links x ~153 GB/s per MI355X (bidirectional "
                              "assumed); efficiency and latency assumed, not measured (no "
                              "multi-GPU box on this pool); a collective is a blocking host call "
                              "while the GPU runs what the prover queued before it: the quotient "
                              "exchange is two all-gathers, the first beside the tallest chip's "
                              "quotient kernel, the second beside the other chips' chunk LDEs, "
                              "and each is charged max(0, its time - that GPU time measured in "
                              "the rank's timed run); every other collective is charged in full "
                              "(the stream is drained before it)"},
                "what": "one proof split over N GPUs, predicted: N = 1 is the timed single-GPU "
                        "proof; N > 1 is the slowest rank's share run alone on this GPU with "
                        "no-op exchanges (bfz_record_prove_shard_solo), before collective time",
                "ranks": {str(n): runs[n]["ranks"] for n in solo},
                "logup_stage_parts": {
                    "replicated": ["perm_rows_ms (permutation rows + cumulative-sum scan: whole "
                                   "rows of the trace domain)",
                                   "perm_idft_ms (iDFT of every permutation column; since "
                                   "round 6 with the residue folds and, at N = 2 / 4 / 8, the "
                                   "strided stages of the forward DFT fused into its second pass "
                                   "-- k_lde_mid / k_coef_fold)"],
                    "split": ["perm_dft_ms (the contiguous tile pass of the size-2n/N forward "
                              "DFT, for the next-residue shards too at N >= 4)",
                              "perm_hash_ms (this rank's Merkle subtree)"]}}
        if world == 1 and not args.no_extra:
            line["end_to_end"] = end_to_end(client, pk, prog, stdin)
            line["events_path"] = events_path(pk, prog, stdin, proof)
            line["drop_in_path"] = drop_in_path(pk, prog, stdin, proof)
        if not args.no_cpu_baseline and world == 1:  # the CPU baseline is timed at N=1 only
            try:
                line["cpu_baseline"] = cpu_baseline()
            except Exception as e:  # keep the GPU line even if the baseline fails
                line["cpu_baseline"] = {"error": str(e)}
        print(json.dumps(line), flush=True)
    if hung:  # a collective may still be blocked: skip teardown that would wait for it
        sys.stdout.flush()
        sys.stderr.flush()
        # the replica line is printed; an abandoned attempt (a thread still blocked inside libbfz)
        # is not a clean run, so the status says so; a collective that failed with an
        # error has returned and leaves a clean exit
        os._exit(3 if extra.get("sharded_proof", {}).get("error", "").startswith("no result") else 0)
    L.bfz_record_free(rec)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
