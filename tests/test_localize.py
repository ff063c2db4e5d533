"""scripts/localize_parity.py: a reference proof made under any one of the
[p3-recalled] alternatives D1-D10 -- here stood in for by the oracle with that
switch flipped -- is named back exactly, and the default proof is reproduced byte for byte.
CPU only (oracle + the independent bincode model)."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))

import bincode_ref as B  # noqa: E402
import localize_parity as LP  # noqa: E402
import oracle_lib as O  # noqa: E402
from bfz import guests  # noqa: E402

NAME, PROG, STDIN = guests.REFERENCE_PROGRAMS[1]  # add_sub: the cheapest oracle proof
CASES = [  # (oracle switches, D1 observe_openings, bincode Montgomery?, expected non-defaults)
    ({}, True, True, {}),
    ({}, True, False, {"D10": "canonical"}),
    ({}, False, True, {"D1": "observe_openings=0"}),
    ({"diag_alt": 1}, True, True, {"D2": "diag_alt=1"}),
    ({"m4_horizen": 1}, True, True, {"D3a": "m4_horizen=1"}),
    ({"no_initial_mds": 1}, True, True, {"D3b": "no_initial_mds=1"}),
    ({"inject_first": 1}, True, True, {"D4": "inject_first=1"}),
    ({"fri_coeff_major": 1}, True, True, {"D5": "fri_coeff_major=1"}),
    ({"query_extra_bits": 1}, True, True, {"D6": "query_extra_bits=1"}),
    ({"sample_front": 1}, True, True, {"D7": "sample_front=1"}),
    ({"selectors_normalized": 1}, True, True, {"D8": "selectors_normalized=1"}),
    ({"force_witness": 2}, True, True, {"D9": "witness"}),
    ({"sample_front": 1, "fri_coeff_major": 1, "m4_horizen": 1}, False, False,
     {"D7": "sample_front=1", "D5": "fri_coeff_major=1", "D3a": "m4_horizen=1",
      "D1": "observe_openings=0", "D10": "canonical"}),
]


@pytest.fixture(scope="module")
def loc():
    return LP.Localizer(PROG, STDIN)


@pytest.mark.parametrize("switches,observe,mont,expect", CASES)
def test_localize_names_the_alternative(loc, switches, observe, mont, expect):
    O.set_variant(**switches)
    try:
        ref = B.encode_bincode(B.parse_bfz1(O.prove(PROG, STDIN, observe_openings=observe)), mont)
    finally:
        O.reset_variant()
    res = loc.localize(ref)
    assert res["match"], res
    got = {k: v for k, v in res["decisions"].items()
           if v not in ("default", "smallest witness", "montgomery")}
    if "D9" in expect:  # the witness value itself is not known in advance
        assert got.pop("D9").startswith("witness=")
        expect = {k: v for k, v in expect.items() if k != "D9"}
    assert got == expect


def test_localize_reports_the_first_differing_section(loc):
    """A proof whose opened values were tampered with is not reproduced by any switch: the
    report names section D (opened values), after A-C matched."""
    pf = B.parse_bfz1(O.prove(PROG, STDIN))
    pf["opened"][0]["main_local"][0] = [(pf["opened"][0]["main_local"][0][0] + 1) % B.P, 0, 0, 0]
    res = loc.localize(B.encode_bincode(pf, True))
    assert not res["match"] and res["stage"] == "D opened values", res
