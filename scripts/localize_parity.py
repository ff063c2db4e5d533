"""Localize a byte mismatch against a reference proof to the [p3-recalled] decisions D1-D10.

    python scripts/localize_parity.py --program hello --proof ref_hello.bin
    python scripts/localize_parity.py --program fibo --stdin 17 --proof ref_fibo17.bin

`ref_*.bin` is `bincode::serialize(&ShardProof)` of the reference prover's core proof of that
program (what `bf_core_machine::utils::prove` returns, utils/prove.rs:46), made wherever cargo
and the zkMIPS Plonky3 fork exist.  The oracle (oracle/, test infrastructure) carries every
unpinned decision of DESIGN.md §2 behind a switch (oracle/or_hash.h or_variant_t); this script
walks the proof in transcript order and, at each section, finds the switch settings that
reproduce the reference's bytes:

  A  main commitment        D2 internal diagonal, D3a M4, D3b initial layer, D4 injection order,
                            D10 field words (Montgomery / canonical)
  B  permutation commitment D7 challenger sample order
  C  quotient commitment    D8 selector normalization
  D  opened values          (no switch: a difference here is outside D1-D10)
  E  FRI commitments        D1 openings observed before alpha, D5 leaf flattening
  F  final value, PoW       D9 witness (the reference's rayon find_any: forced to its value)
  G  query openings         D6 query index bits

Prints one JSON object: the decisions that reproduce the proof byte for byte (or the first
section no combination reproduces).  Oracle only: nothing here touches the product.
"""
import argparse
import itertools
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "tests"), os.path.join(ROOT, "zkvm-brainfuck_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import bincode_ref as B  # noqa: E402
import oracle_lib as O  # noqa: E402

# decision -> (oracle switch, default, alternatives); D1 is prove()'s observe_openings
DECISIONS = {
    "D1": ("observe_openings", 1, [0]),
    "D2": ("diag_alt", 0, [1]),
    "D3a": ("m4_horizen", 0, [1]),
    "D3b": ("no_initial_mds", 0, [1]),
    "D4": ("inject_first", 0, [1]),
    "D5": ("fri_coeff_major", 0, [1]),
    "D6": ("query_extra_bits", 0, [1, 2]),
    "D7": ("sample_front", 0, [1]),
    "D8": ("selectors_normalized", 0, [1]),
}
STAGES = [  # (name, decisions searched, section predicate)
    ("A main commitment", ["D2", "D3a", "D3b", "D4"], lambda a, b: a["roots"][0] == b["roots"][0]),
    ("B permutation commitment", ["D7"], lambda a, b: a["roots"][1] == b["roots"][1]),
    ("C quotient commitment", ["D8"], lambda a, b: a["roots"][2] == b["roots"][2]),
    ("D opened values", [], lambda a, b: a["opened"] == b["opened"] and a["chips"] == b["chips"]),
    ("E FRI commitments", ["D1", "D5"], lambda a, b: a["commit_roots"] == b["commit_roots"]),
    ("F final value", [], lambda a, b: a["final_poly"] == b["final_poly"]),
    ("G query openings", ["D6"], lambda a, b: a["queries"] == b["queries"]),
]


class Localizer:
    def __init__(self, program: str, stdin, num_queries: int = 84):
        self.program, self.stdin, self.nq = program, list(stdin), num_queries
        self.cache = {}

    def proof(self, cfg: dict) -> dict:
        key = tuple(sorted(cfg.items()))
        if key not in self.cache:
            sw = {DECISIONS[d][0]: v for d, v in cfg.items() if d.startswith("D") and d != "D1"}
            if cfg.get("witness") is not None:
                sw.update(force_witness=1, witness=cfg["witness"])
            O.set_variant(**sw)
            try:
                raw = O.prove(self.program, self.stdin, num_queries=self.nq,
                              observe_openings=bool(cfg.get("D1", 1)))
            finally:
                O.reset_variant()
            self.cache[key] = B.parse_bfz1(raw)
        return self.cache[key]

    def localize(self, ref: bytes) -> dict:
        refs = {}
        for mont in (True, False):
            try:
                refs[mont] = B.decode_bincode(ref, mont)
            except (ValueError, KeyError, IndexError, Exception):  # noqa: BLE001 - not this form
                pass
        if not refs:
            return {"match": False, "stage": "decode", "detail": "not a bincode ShardProof"}
        cfg = {d: DECISIONS[d][1] for d in DECISIONS}
        cfg["witness"] = None
        mont = None
        for name, decs, same in STAGES:
            combos = _combos(decs)  # default first, then 1, 2, ... deviations
            reprs = [True, False] if mont is None else [mont]
            hit = None
            for combo in combos:
                trial = dict(cfg, **combo)
                pf = self.proof(trial)
                for m in reprs:
                    if m in refs and same(pf, refs[m]):
                        hit = (trial, m)
                        break
                if hit:
                    break
            if not hit:
                return {"match": False, "stage": name, "decisions": _report(cfg, mont),
                        "detail": "no combination of " + (", ".join(decs) or "(no switch)") +
                                  " reproduces this section"}
            cfg, mont = hit
            if name.startswith("F"):  # D9: the reference witness decides the query indices
                ref_w = refs[mont]["pow_witness"]
                if self.proof(cfg)["pow_witness"] != ref_w:
                    cfg = dict(cfg, witness=ref_w)
        pf = self.proof(cfg)
        exact = B.encode_bincode(pf, mont) == ref
        return {"match": exact, "stage": "all" if exact else "bytes", "decisions": _report(cfg, mont)}


def _combos(decs):
    out = []
    for k in range(len(decs) + 1):
        for chosen in itertools.combinations(decs, k):
            for vals in itertools.product(*[DECISIONS[d][2] for d in chosen]):
                out.append(dict(zip(chosen, vals)))
    return out


def _report(cfg, mont):
    rep = {}
    for d, (sw, default, _) in DECISIONS.items():
        v = cfg.get(d, default)
        rep[d] = "default" if v == default else f"{sw}={v}"
    rep["D9"] = "smallest witness" if cfg.get("witness") is None else f"witness={cfg['witness']}"
    rep["D10"] = "unknown" if mont is None else ("montgomery" if mont else "canonical")
    return rep


def main():
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--program", required=True,
                    help="a guest name from bfz/guests.py (hello, fibo, ...) or a .bf file")
    ap.add_argument("--stdin", type=int, nargs="*", default=[])
    ap.add_argument("--proof", required=True, help="bincode ShardProof bytes of the reference")
    ap.add_argument("--queries", type=int, default=84)
    a = ap.parse_args()
    from bfz import guests
    prog = getattr(guests, a.program.upper(), None)
    if prog is None:
        prog = open(a.program).read()
    res = Localizer(prog, a.stdin, a.queries).localize(open(a.proof, "rb").read())
    print(json.dumps(res, indent=1))
    sys.exit(0 if res["match"] else 1)


if __name__ == "__main__":
    main()
