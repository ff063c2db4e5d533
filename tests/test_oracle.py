"""CPU tests of the oracle (the checker) against the reference's own goldens and properties."""
import hashlib
import json
import os

import numpy as np
import pytest

import oracle_lib as O
from bfz import guests

GOLDEN = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "golden.json")))
P = O.P


# --- the reference's value-level known answers (executor.rs:335-416, sdk/src/lib.rs:175-183)
@pytest.mark.parametrize("prog,stdin,check", [
    ("++-.", [], lambda r: r["output"][0] == 1),                     # test_add_sub_run
    (">><", [], lambda r: r["mp"] == 1),                              # test_mem_run
    ("[----]", [1], lambda r: r["cycles"] == 2),                      # test_jmp_run
    (",.", [1], lambda r: r["output"][0] == 1),                       # test_io_run
    (guests.PRINTA, [], lambda r: r["output"][0] == ord("A")),        # test_printa_run
    (guests.MOVE, [], lambda r: list(r["output"][:2]) == [2, 0]),     # test_move_run
    (guests.LOOP, [], lambda r: r["pc"] == 9 and r["output"][0] == 0),  # test_loop_run
    (guests.HELLO, [], lambda r: r["output"][:5] == b"Hello"),        # test_hello_run
    (guests.FIBO, [17], lambda r: r["output"][0] == 85),              # test_fibo_run / test_execute
])
def test_executor_known_answers(prog, stdin, check):
    assert check(O.execute(prog, stdin))


def test_known_answer_fixture():
    for ka in GOLDEN["known_answers"]:
        r = O.execute(ka["program"], ka["stdin"])
        assert list(r["output"]) == ka["output"] and r["cycles"] == ka["cycles"]


def test_two_adic_generators():
    g24 = O.two_adic_gen(24)
    assert g24 == pow(3, 127, P) == 1791270792
    for k in range(1, 25):
        g = O.two_adic_gen(k)
        assert pow(g, 1 << k, P) == 1 and pow(g, 1 << (k - 1), P) != 1
        if k > 1:
            assert O.two_adic_gen(k - 1) == g * g % P
    # entries recalled from p3-koala-bear TWO_ADIC_GENERATORS
    assert [O.two_adic_gen(k) for k in (1, 2, 3, 4)] == [0x7F000000, 0x7E010002, 0x6832FE4A, 0x08DBD69C]


def _naive_lde(col, shift):
    n = len(col)
    w = O.two_adic_gen(n.bit_length() - 1)
    winv = pow(w, P - 2, P)
    ninv = pow(n, P - 2, P)
    coeffs = [sum(col[j] * pow(winv, j * k, P) for j in range(n)) * ninv % P for k in range(n)]
    N = 2 * n
    wN = O.two_adic_gen(N.bit_length() - 1)
    out = []
    for i in range(N):
        x = shift * pow(wN, i, P) % P
        out.append(sum(c * pow(x, k, P) for k, c in enumerate(coeffs)) % P)
    lg = N.bit_length() - 1
    rev = [int(format(i, f"0{lg}b")[::-1], 2) if lg else 0 for i in range(N)]
    return [out[rev[i]] for i in range(N)]


@pytest.mark.parametrize("n", [1, 2, 4, 8, 16])
def test_oracle_lde_matches_naive_dft(n):
    rng = np.random.default_rng(n)
    m = rng.integers(0, P, size=(n, 3), dtype=np.uint64).astype(np.uint32)
    got = O.coset_lde(m, 3)
    for c in range(3):
        assert got[:, c].tolist() == _naive_lde(m[:, c].tolist(), 3)


def test_poseidon2_fixture():
    for kat in GOLDEN["poseidon2"]:
        out = O.poseidon2(np.array(kat["in"], dtype=np.uint32))
        assert out.tolist() == kat["out"]


def test_trace_fixture():
    chips = ["Cpu", "Program", "AddSub", "Jump", "Memory", "Byte", "MemoryInstrs", "IO"]
    for name, prog, sin in [("hello", guests.HELLO, []), ("fibo17", guests.FIBO, [17])]:
        for ci, cn in enumerate(chips):
            t = O.trace(prog, sin, ci)
            exp = GOLDEN["traces"][name].get(cn)
            if exp is None:
                assert t is None
            else:
                assert list(t.shape) == exp["shape"]
                assert hashlib.sha256(t.tobytes()).hexdigest() == exp["sha256"]


def test_trace_shapes_match_reference_widths():
    widths = {0: 31, 1: 1, 2: 7, 3: 45, 4: 12, 5: 2, 6: 41, 7: 5}
    for ci, w in widths.items():
        t = O.trace(guests.FIBO, [17], ci)
        assert t.shape[1] == w
    assert O.trace(guests.FIBO, [17], 0).shape[0] == 1 << 16   # 33,341 cycles -> 2^16 rows
    assert O.trace(guests.FIBO, [17], 5).shape[0] == 1 << 16   # Byte: fixed 2^16


@pytest.mark.parametrize("name,prog,stdin", guests.REFERENCE_PROGRAMS)
def test_prove_verify_reference_programs(name, prog, stdin):
    """run_test (crates/core/machine/src/utils/prove.rs:68-95): prove, then verify with a
    freshly built machine.  Also pins the proof bytes (normal form) to the fixture."""
    pf = O.prove(prog, stdin)
    assert O.verify(prog, pf)
    g = [x for x in GOLDEN["proofs"] if x["name"] == name][0]
    assert hashlib.sha256(pf).hexdigest() == g["sha256"]


def test_proof_is_deterministic():
    a = O.prove(guests.HELLO, [])
    b = O.prove(guests.HELLO, [])
    assert a == b


@pytest.mark.parametrize("offset_frac", [0.001, 0.01, 0.05, 0.3, 0.7, 0.999])
def test_tampered_proof_rejected(offset_frac):
    pf = bytearray(O.prove(guests.LOOP, []))
    i = int(len(pf) * offset_frac)
    pf[i] ^= 0x01
    assert not O.verify(guests.LOOP, bytes(pf))


def test_wrong_program_rejected():
    pf = O.prove(guests.LOOP, [])
    assert not O.verify(guests.LOOP + "+", pf)


def test_challenger_duplex_semantics():
    # sampling with nothing observed duplexes the zero state; samples pop from the END
    s = O.challenger([], 8)
    st = O.poseidon2(np.zeros(16, dtype=np.uint32)).tolist()
    assert s == st[:8][::-1]
    # after 8 observations the sponge has already absorbed them
    obs = list(range(1, 9))
    s2 = O.challenger(obs, 1)
    st2 = O.poseidon2(np.array(obs + [0] * 8, dtype=np.uint32)).tolist()
    assert s2 == [st2[7]]


def _ef_mul(a, b):
    """EF = F[x]/(x^4 - 3) (kb31: W = 3), canonical coefficient lists"""
    r = [0] * 7
    for i in range(4):
        for j in range(4):
            r[i + j] += a[i] * b[j]
    return [(r[k] + 3 * (r[k + 4] if k + 4 < 7 else 0)) % P for k in range(4)]


@pytest.mark.parametrize("logn,w", [(1, 1), (3, 2), (5, 3), (6, 5)])
def test_oracle_pcs_commit_fri_closed_form(logn, w):
    """The column-sharded PCS restatement (oracle/or_pcs.c, the checker of bfz_commit_fri_sharded)
    pinned by an independent closed form: its root is the MerkleTreeMmcs root of the coset LDE
    (O.merkle_root), it folds to a constant, and the constant is what FRI's fold does to the
    batched polynomial f = sum_c alpha^c P_c (P_c interpolates column c over H, naive DFT here):
    each fold keeps f_even + beta f_odd of f(3 y) -- the fold ignores the coset shift -- so
    final = sum_j F_j 3^j prod_(r: bit r of j) beta_r."""
    n = 1 << logn
    rng = np.random.default_rng(1000 + logn)
    m = rng.integers(0, P, size=(n, w), dtype=np.uint64).astype(np.uint32)
    root, fri, fin, constant, (alpha, betas) = O.pcs_commit_fri(m, challenges=True)
    assert constant
    assert root == O.merkle_root([O.coset_lde(m, 3)])
    assert len(fri) == len(betas) == logn
    wn_inv = pow(O.two_adic_gen(logn), P - 2, P)
    ninv = pow(n, P - 2, P)
    F = [[0, 0, 0, 0] for _ in range(n)]
    ap = [1, 0, 0, 0]
    for c in range(w):
        col = [int(v) for v in m[:, c]]
        for k in range(n):
            ck = sum(col[j] * pow(wn_inv, j * k, P) for j in range(n)) * ninv % P
            F[k] = [(F[k][e] + ap[e] * ck) % P for e in range(4)]
        ap = _ef_mul(ap, alpha)
    want = [0, 0, 0, 0]
    for j in range(n):
        t = [F[j][e] * pow(3, j, P) % P for e in range(4)]
        for r in range(logn):
            if (j >> r) & 1:
                t = _ef_mul(t, betas[r])
        want = [(want[e] + t[e]) % P for e in range(4)]
    assert fin == want
