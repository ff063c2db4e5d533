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
    """a log degree word >= 2^31 (a negative int) or 0, and a commit phase shorter
    than the tallest matrix, are rejected before any shift by them."""
    prog = guests.HELLO
    pf = O.prove(prog, [])
    vk = _vk(prog)
    c = sdk.ProverClient()

    def set_logdeg(v):
        return lambda m: m["opened"][0].__setitem__("log_degree", v)

    for v in (0x80000000, 0xFFFFFFFF, 0, 24):
        with pytest.raises(_lib.BfzError, match="log degree out of range"):
            c.verify(sdk.BfProofWithPublicValues(proof=_tampered(pf, set_logdeg(v)), stdin=b""), vk)

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
