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
