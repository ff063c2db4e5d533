"""CPU tests of the C ABI (libbfz.so): loads, exports every declared symbol, host paths work,
and the product's host verifier accepts oracle proofs (an independent implementation)."""
import json
import os
import re

import pytest

import oracle_lib as O
from bfz import _lib, guests, sdk

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = json.load(open(os.path.join(ROOT, "tests", "golden", "golden.json")))


def declared_symbols():
    hdr = open(os.path.join(ROOT, "include", "bfz.h")).read()
    return sorted(set(re.findall(r"\b(bfz_[a-z0-9_]+)\s*\(", hdr)))


def test_library_exports_every_declared_symbol():
    L = _lib.lib()
    syms = declared_symbols()
    assert len(syms) >= 16
    for s in syms:
        assert hasattr(L, s), s
    assert {s for s, _, _ in _lib.SIGNATURES} == set(syms)


@pytest.mark.parametrize("ka", GOLDEN["known_answers"], ids=lambda k: k["name"])
def test_execute_known_answers_through_abi(ka):
    out = sdk.ProverClient().execute(ka["program"], ka["stdin"]).run()
    assert list(out) == ka["output"]


def test_execute_errors_are_reported():
    with pytest.raises(_lib.BfzError, match="unmatched"):
        sdk.ProverClient().execute("]", []).run()
    with pytest.raises(_lib.BfzError, match="input"):
        sdk.ProverClient().execute(",", []).run()


def _vk(prog):
    return sdk.BfVerifyingKey(commit=[O.to_mont(x) for x in O.setup_root(prog)], elf=prog)


@pytest.mark.parametrize("name,prog,stdin", guests.REFERENCE_PROGRAMS)
def test_host_verifier_accepts_oracle_proofs(name, prog, stdin):
    pf = O.prove(prog, stdin)
    sdk.ProverClient().verify(sdk.BfProofWithPublicValues(proof=pf, stdin=bytes(stdin)), _vk(prog))


def test_host_verifier_rejects_tampering_and_wrong_vk():
    prog = guests.HELLO
    pf = O.prove(prog, [])
    c = sdk.ProverClient()
    vk = _vk(prog)
    for frac in (0.002, 0.02, 0.2, 0.5, 0.9, 0.9999):
        bad = bytearray(pf)
        bad[int(len(bad) * frac)] ^= 0x10
        with pytest.raises(_lib.BfzError, match="verification failed"):
            c.verify(sdk.BfProofWithPublicValues(proof=bytes(bad), stdin=b""), vk)
    wrong = _vk(guests.LOOP)
    wrong.elf = prog
    with pytest.raises(_lib.BfzError):
        c.verify(sdk.BfProofWithPublicValues(proof=pf, stdin=b""), wrong)


# ---------------------------------------------------------------- proof byte forms (bincode)
import struct  # noqa: E402

import bincode_ref as BR  # noqa: E402


@pytest.mark.parametrize("name,prog,stdin", guests.REFERENCE_PROGRAMS[:4] +
                         [("hello", guests.HELLO, [])])
def test_bincode_encoder_matches_independent_model(name, prog, stdin):
    """csrc/proof.cpp's bincode ShardProof == the separately written Python model, in both
    field representations; bincode -> BFZ1 is the exact inverse; the decoded model re-encodes
    to the same BFZ1 bytes."""
    pf = O.prove(prog, stdin)
    model = BR.parse_bfz1(pf)
    assert BR.encode_bfz1(model) == pf
    for repr_, mont in ((sdk.FIELD_MONTGOMERY, True), (sdk.FIELD_CANONICAL, False)):
        bc = sdk.proof_to_bincode(pf, repr_)
        assert bc == BR.encode_bincode(model, montgomery=mont)
        assert sdk.proof_from_bincode(bc, repr_) == pf


def test_bincode_layout_landmarks():
    """Spot-check the serde layout: 3 digests, then u64 chip count, chip_ordering at the end
    as (u64 len, name, u64 index) in proof order."""
    pf = O.prove(guests.HELLO, [])
    model = BR.parse_bfz1(pf)
    bc = sdk.proof_to_bincode(pf, sdk.FIELD_CANONICAL)
    assert list(struct.unpack_from("<8I", bc, 0)) == model["roots"][0]
    assert struct.unpack_from("<Q", bc, 96)[0] == len(model["chips"])
    tail = b"".join(struct.pack("<Q", len(BR.CHIPS[c])) + BR.CHIPS[c].encode() + struct.pack("<Q", i)
                    for i, c in enumerate(model["chips"]))
    assert bc.endswith(struct.pack("<Q", len(model["chips"])) + tail)


def test_verify_bincode_and_proof_with_public_values():
    prog = guests.FIBO
    pf = O.prove(prog, [17])
    vk = _vk(prog)
    c = sdk.ProverClient()
    bc = sdk.proof_to_bincode(pf)
    c.verify_bincode(bc, vk)
    c.verify_bincode(sdk.proof_to_bincode(pf, sdk.FIELD_CANONICAL), vk, sdk.FIELD_CANONICAL)
    with pytest.raises(_lib.BfzError, match="verification failed"):  # wrong representation
        c.verify_bincode(bc, vk, sdk.FIELD_CANONICAL)
    bad = bytearray(bc)
    bad[len(bad) // 2] ^= 1
    with pytest.raises(_lib.BfzError, match="verification failed"):
        c.verify_bincode(bytes(bad), vk)
    wp = sdk.BfProofWithPublicValues(proof=pf, stdin=bytes([17]))
    ser = wp.to_bincode()
    assert ser == bc + struct.pack("<Q", 1) + bytes([17])
    back = sdk.BfProofWithPublicValues.from_bincode(ser)
    assert back.proof == pf and back.stdin == bytes([17])


def _tampered(pf, fn):
    m = BR.parse_bfz1(pf)
    fn(m)
    return BR.encode_bfz1(m)


def test_verifier_rejects_out_of_range_log_degree_and_round_count():
    """a log degree word >= 2^31 (a negative int) or above 23, and a commit phase
    shorter than the tallest matrix, are rejected before any shift by them.  Log degree 0 is a
    legal 1-row trace: claimed for a taller chip it fails the Merkle openings."""
    prog = guests.HELLO
    pf = O.prove(prog, [])
    vk = _vk(prog)
    c = sdk.ProverClient()

    def set_logdeg(v):
        return lambda m: m["opened"][0].__setitem__("log_degree", v)

    for v in (0x80000000, 0xFFFFFFFF, 24):
        with pytest.raises(_lib.BfzError, match="log degree out of range"):
            c.verify(sdk.BfProofWithPublicValues(proof=_tampered(pf, set_logdeg(v)), stdin=b""), vk)
    with pytest.raises(_lib.BfzError, match="path length"):
        c.verify(sdk.BfProofWithPublicValues(proof=_tampered(pf, set_logdeg(0)), stdin=b""), vk)

    def short_commit(m):
        m["commit_roots"].pop()
        for q in m["queries"]:
            q["steps"].pop()

    with pytest.raises(_lib.BfzError, match="FRI round count"):
        c.verify(sdk.BfProofWithPublicValues(proof=_tampered(pf, short_commit), stdin=b""), vk)


def test_verifier_fuzz_rejects_every_mutation():
    """(f)3 as a fuzz target: 300 seeded mutations of a valid proof (bit flips, words set to
    0 / 1 / p-1 / p / 2^31 / 2^32-1 / random, inserted words, truncations, header words) are
    each rejected with an error -- no crash, no accepted variant (the local-only chips' unopened
    next values included, see verifier.cpp)."""
    import random
    prog = guests.HELLO
    pf = O.prove(prog, [])
    vk = _vk(prog)
    c = sdk.ProverClient()
    rng = random.Random(2024)
    specials = [0, 1, 0x7F000000, 0x7F000001, 0x80000000, 0xFFFFFFFF]
    tried = 0
    while tried < 300:
        b = bytearray(pf)
        kind = rng.randrange(5)
        if kind == 0:
            b[rng.randrange(len(b))] ^= 1 << rng.randrange(8)
        elif kind == 1:
            o = rng.randrange(len(b) // 4) * 4
            b[o:o + 4] = struct.pack("<I", rng.choice(specials + [rng.getrandbits(32)]))
        elif kind == 2:
            b = b[:rng.randrange(len(b))]
        elif kind == 3:
            o = rng.randrange(len(b) // 4) * 4
            b[o:o] = struct.pack("<I", rng.getrandbits(32))
        else:
            o = rng.randrange(min(len(b) // 4, 256)) * 4
            b[o:o + 4] = struct.pack("<I", rng.choice(specials + [2, 0x10000, rng.getrandbits(32)]))
        if bytes(b) == pf:
            continue
        tried += 1
        with pytest.raises(_lib.BfzError):
            c.verify(sdk.BfProofWithPublicValues(proof=bytes(b), stdin=b""), vk)


def test_verifier_rejects_nonzero_next_of_local_only_chips():
    """Normal form: the reference prover writes zero next values for local-only chips
    (prover.rs:484-487); they are not opened, so only the normal-form check catches them."""
    prog = guests.HELLO
    pf = O.prove(prog, [])
    m = BR.parse_bfz1(pf)
    local = [i for i, o in enumerate(m["opened"]) if not any(any(x) for x in o["main_next"])]
    assert local, "hello has local-only chips (AddSub, Jump, IO)"

    def poke(mm):
        mm["opened"][local[0]]["main_next"][0][0] = 1

    with pytest.raises(_lib.BfzError, match="local-only chip"):
        sdk.ProverClient().verify(
            sdk.BfProofWithPublicValues(proof=_tampered(pf, poke), stdin=b""), _vk(prog))


def test_pcs_variant_switch_is_consistent():
    """Decision D1: with the opened values kept out of the transcript, the
    oracle's proof differs, and each verifier accepts exactly the proofs of its own variant."""
    prog = guests.LOOP if hasattr(guests, "LOOP") else guests.HELLO
    a = O.prove(prog, [], observe_openings=True)
    b = O.prove(prog, [], observe_openings=False)
    assert a != b
    vk = _vk(prog)
    c = sdk.ProverClient()
    try:
        sdk.set_pcs_variant(0)
        c.verify(sdk.BfProofWithPublicValues(proof=b, stdin=b""), vk)
        with pytest.raises(_lib.BfzError, match="verification failed"):
            c.verify(sdk.BfProofWithPublicValues(proof=a, stdin=b""), vk)
        assert O.verify(prog, b, observe_openings=False)
        assert not O.verify(prog, a, observe_openings=False)
    finally:
        sdk.set_pcs_variant(-1)
    c.verify(sdk.BfProofWithPublicValues(proof=a, stdin=b""), vk)
    with pytest.raises(_lib.BfzError, match="verification failed"):
        c.verify(sdk.BfProofWithPublicValues(proof=b, stdin=b""), vk)


def test_query_count_validation():
    """FRI_QUERIES-style overrides must be positive."""
    with pytest.raises(_lib.BfzError, match="num_queries"):
        sdk.set_num_queries(-3)
    sdk.set_num_queries(0)


def _events(elf, stdin, executor):
    import ctypes
    buf, n = _lib.u8buf(bytes(stdin))
    p = ctypes.POINTER(ctypes.c_uint8)()
    ln = ctypes.c_size_t()
    _lib.check(_lib.lib().bfz_execute_events(elf.encode(), buf, n, executor, ctypes.byref(p),
                                             ctypes.byref(ln)))
    return _lib.take_bytes(p, ln.value)


from bfgen import random_program as _random_program  # noqa: E402


@pytest.mark.parametrize("prog,stdin", [(p, s) for _, p, s in guests.REFERENCE_PROGRAMS]
                         + [(guests.FIBO, [17]), (guests.FIBO, [60])])
def test_pipeline_executor_matches_record_executor(prog, stdin):
    """The prover pipeline's executor (pinned arrays, dense cells, address-ordered memory events
    without a sort) emits the record executor's event stream field for field."""
    assert _events(prog, stdin, 1) == _events(prog, stdin, 0)


def test_pipeline_executor_random_programs_and_tape_wrap():
    import numpy as np
    rng = np.random.default_rng(7)
    progs = [_random_program(rng, int(rng.integers(5, 60))) for _ in range(60)]
    progs += ["<<<+.>>>>>-.<<", "<" * 5000 + "+" + ">" * 9000 + "-.", ">>+<<<<<<-."]
    for p in progs:
        a, b = _events(p, [3], 0), _events(p, [3], 1)
        assert a == b, p
    with pytest.raises(_lib.BfzError, match="input"):
        _events(",", [], 1)


def _arity(params: str) -> int:
    params = re.sub(r"\([^()]*\)", "", params)  # function-pointer types
    params = params.strip()
    return 0 if params in ("", "void") else params.count(",") + 1


def test_rust_ffi_matches_header():
    """crates/bfz-sys (the Rust binding a maintainer adds; not compiled here) declares every
    entry point of include/bfz.h with the same number of arguments."""
    hdr = open(os.path.join(ROOT, "include", "bfz.h")).read()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    c = {m.group(1): _arity(m.group(2))
         for m in re.finditer(r"\b(bfz_[a-z0-9_]+)\s*\(((?:[^()]|\([^()]*\))*)\)\s*;", hdr)}
    rs = open(os.path.join(ROOT, "crates", "bfz-sys", "src", "lib.rs")).read()
    r = {m.group(1): _arity(re.sub(r"\w+\s*:", "", m.group(2)))
         for m in re.finditer(r"pub fn (bfz_[a-z0-9_]+)\(((?:[^()]|\([^()]*\))*)\)", rs)}
    assert set(c) == set(declared_symbols())
    assert c == r


@pytest.mark.parametrize("prog,stdin", [("+", []), (".", []), (">", []), (",", [9]), ("-", [])])
def test_one_cycle_programs_prove_and_verify(prog, stdin):
    """A one-cycle program has a 1-row Cpu trace (cpu/trace.rs:33: next_power_of_two, no
    minimum): its 2-row LDE's reduced opening joins the FRI layer after the last fold
    (decision D11), and both verifiers accept the proof (log degree 0 is legal)."""
    pf = O.prove(prog, stdin)
    assert O.verify(prog, pf)
    sdk.ProverClient().verify(sdk.BfProofWithPublicValues(proof=pf, stdin=bytes(stdin)), _vk(prog))
    # the Cpu chip's opened log degree is 0
    assert sdk.proof_to_bincode(pf)  # and the wire format encodes it


def test_event_struct_layouts_match_header(tmp_path):
    """bfz.h's bfz_*_event structs (compiled with gcc) have exactly the numpy layouts bfz/events.py
    hands to bfz_record_from_events and the field order of crates/bfz-sys."""
    import subprocess
    from bfz import events as E
    checks = {"bfz_cpu_event": E.CPU, "bfz_alu_event": E.ALU, "bfz_jump_event": E.JUMP,
              "bfz_mem_instr_event": E.MEM_INSTR, "bfz_io_event": E.IO, "bfz_memory_event": E.MEMORY,
              "bfz_cycle": E.CYCLE}
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{ROOT}/include/bfz.h"',
             "int main(void) {"]
    for st, dt in checks.items():
        lines.append(f'printf("{st} size %zu\\n", sizeof({st}));')
        for name in dt.names:
            field = name
            for acc in ("mv_access_", "next_mv_access_"):
                if name.startswith(acc):
                    field = acc[:-1] + "." + name[len(acc):]
            lines.append(f'printf("{st} {name} %zu\\n", offsetof({st}, {field}));')
    lines.append("return 0; }")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c11", "-o", str(exe), str(src)], check=True)
    got = {}
    for ln in subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split("\n"):
        if ln:
            st, name, v = ln.split()
            got[(st, name)] = int(v)
    for st, dt in checks.items():
        assert got[(st, "size")] == dt.itemsize, st
        for name in dt.names:
            assert got[(st, name)] == dt.fields[name][1], (st, name)
    # crates/bfz-sys declares the same fields in the same order
    rs = open(os.path.join(ROOT, "crates", "bfz-sys", "src", "lib.rs")).read()
    hdr = open(os.path.join(ROOT, "include", "bfz.h")).read()
    for st in list(checks) + ["bfz_memory_access", "bfz_events"]:
        m = re.search(r"typedef struct \{[^{}]*?\}\s*" + st + ";", hdr, re.S)
        cfields = re.findall(r"(\w+)(?:\[\d+\])?\s*[,;]", re.sub(r"/\*.*?\*/", "", m.group(0).split("{", 1)[1].rsplit("}", 1)[0]))
        r = re.search(r"pub struct " + st + r" \{(.*?)\n\}", rs, re.S)
        rfields = re.findall(r"pub (\w+):", r.group(1))
        assert cfields == rfields, st


def _prep_host_key(prog):
    import ctypes as ct
    import numpy as np
    out = []
    for c in (5, 1):  # Byte (2^16 rows) sorts before Program
        p = ct.POINTER(ct.c_uint32)()
        h, w = ct.c_size_t(), ct.c_size_t()
        buf, n = _lib.u8buf(b"")
        _lib.check(_lib.lib().bfz_trace(prog.encode(), buf, n, c, 1, ct.byref(p), ct.byref(h),
                                        ct.byref(w)))
        arr = np.ctypeslib.as_array(p, shape=(h.value * w.value,)).copy().reshape(h.value, w.value)
        _lib.lib().bfz_free(p)
        out.append((c, sdk.CHIPS[c], arr))
    commit = [O.to_mont(x) for x in O.setup_root(prog)]
    return sdk.StarkProvingKey(commit=commit, traces=out,
                               chip_ordering={"Byte": 0, "Program": 1}, local_only=[False, False])


def test_pk_from_host_refuses_traces_that_are_not_the_programs():
    """bfz_pk_from_host (MachineProver::pk_to_device) checks the host key before any device
    work: a tampered Byte or Program preprocessed trace, a missing chip or a wrong width is an
    error (the commit check needs the device and is in tests/test_gpu.py)."""
    import numpy as np
    hpk = _prep_host_key(guests.HELLO)
    bad = [(c, n, t.copy()) for c, n, t in hpk.traces]
    bad[0][2][5, 1] ^= 1  # Byte multiplicand column
    with pytest.raises(_lib.BfzError, match="Byte is not the program's"):
        sdk.CoreProver.pk_to_device(sdk.StarkProvingKey(hpk.commit, bad, hpk.chip_ordering, hpk.local_only))
    bad = [(c, n, t.copy()) for c, n, t in hpk.traces]
    bad[1][2][3, 4] = O.to_mont(7)  # an op_a byte of instruction 3
    with pytest.raises(_lib.BfzError, match="Program is not the program's"):
        sdk.CoreProver.pk_to_device(sdk.StarkProvingKey(hpk.commit, bad, hpk.chip_ordering, hpk.local_only))
    with pytest.raises(_lib.BfzError, match="Program and Byte"):
        sdk.CoreProver.pk_to_device(sdk.StarkProvingKey(hpk.commit, hpk.traces[:1], {}, []))
    with pytest.raises(_lib.BfzError, match="bad shape"):
        sdk.CoreProver.pk_to_device(sdk.StarkProvingKey(
            hpk.commit, [hpk.traces[0], (1, "Program", np.ascontiguousarray(hpk.traces[1][2][:, :5]))],
            hpk.chip_ordering, hpk.local_only))
    bad = [(c, n, t.copy()) for c, n, t in hpk.traces]
    bad[1][2][0, 1] = O.to_mont(9)  # opcode 9 does not exist
    with pytest.raises(_lib.BfzError, match="opcode"):
        sdk.CoreProver.pk_to_device(sdk.StarkProvingKey(hpk.commit, bad, hpk.chip_ordering, hpk.local_only))


def test_rust_crates_have_no_stubs_and_declare_their_dependencies():
    """The Rust drop-in (crates/; not compiled here) has no unimplemented!/todo! bodies, every
    external crate bf-hip-prover uses is a dependency in its Cargo.toml, and it does not depend
    on bf-prover (which depends on it behind the `hip` feature: no cycle)."""
    for d, _, files in os.walk(os.path.join(ROOT, "crates")):
        for f in files:
            if f.endswith(".rs"):
                src = open(os.path.join(d, f)).read()
                assert not re.search(r"\b(unimplemented|todo)!\s*\(", src), f
    src = open(os.path.join(ROOT, "crates", "bf-hip-prover", "src", "lib.rs")).read()
    toml = open(os.path.join(ROOT, "crates", "bf-hip-prover", "Cargo.toml")).read()
    deps = set(re.findall(r"^([a-z0-9-]+)\s*=", toml.split("[dependencies]")[1].split("\n[")[0], re.M))
    used = set(re.findall(r"(?<![\w:])((?:p3|bf|bfz)_[a-z0-9_]+)::", src)) | set(
        re.findall(r"^use ((?:p3|bf|bfz)_[a-z0-9_]+)", src, re.M))
    used |= {"bincode"} if "bincode::" in src else set()
    used |= {"hashbrown"} if "hashbrown::" in src else set()
    for crate in used:
        assert crate.replace("_", "-") in deps, crate
    assert "bf-prover" not in deps
    # the workspace patch makes bf-prover select it (components.rs) behind `hip`
    patch = open(os.path.join(ROOT, "crates", "reference-patch", "0001-hip-core-prover.patch")).read()
    assert 'type CoreProver = bf_hip_prover::HipProver;' in patch
    assert 'hip = ["dep:bf-hip-prover"]' in patch and 'hip = ["bf-prover/hip"]' in patch


@pytest.mark.skipif(not os.path.isdir("/root/reference/crates"), reason="reference checkout absent")
def test_reference_patch_applies():
    """crates/reference-patch applies cleanly to the reference workspace (dry run, nothing
    written)."""
    import subprocess
    r = subprocess.run(["patch", "--dry-run", "-p1", "-d", "/root/reference", "-i",
                        os.path.join(ROOT, "crates", "reference-patch", "0001-hip-core-prover.patch")],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr


def test_batch_handover_failure_releases_emitted_proofs():
    """a bfz_prove_batch hand-over that fails part-way releases the proofs it already
    handed out through bfz_free (they are library-owned vectors, not malloc'd) and clears every
    slot; host-only, so it runs without a GPU."""
    from bfz import _lib
    assert _lib.lib().bfz_selftest(b"emit_rollback") == 0, _lib.lib().bfz_last_error()
    assert _lib.lib().bfz_selftest(b"no_such_test") != 0


@pytest.mark.parametrize("name,prog,stdin", guests.REFERENCE_PROGRAMS[:4] + [("fibo17", guests.FIBO, [17])])
def test_cycle_arrays_standin_matches_python_conversion(name, prog, stdin):
    """The compiled stand-in of the Rust CycleArrays::new (crates/bf-hip-prover/standin, over
    cpu_events laid out as rustc lays out CpuEvent) writes the same 16-byte cycles as the numpy
    mirror cycles_from_record, on 1, 3 and 8 threads (no device needed)."""
    import numpy as np
    from bfz import events
    rec = events.ExecutionRecordArrays.from_executor(prog, stdin)
    want = events.cycles_from_record(rec)
    rs = events.rust_cpu_events(rec)
    sa = events.CycleArraysStandin()
    for threads in (1, 3, 8):
        got = np.zeros(len(want), dtype=events.CYCLE)
        got.view(np.uint8)[:] = 0xAB  # every byte must be written
        sa.convert(rs, got, threads)
        assert got.tobytes() == want.tobytes(), (name, threads)
