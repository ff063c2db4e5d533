"""The index and coset algebra of the sharded proof, checked in plain Python.

A rank of a G-way sharded proof holds bit-reversed LDE positions [k m, (k+1) m), m = 2n / G.
Those are the natural points i = G t + r (r = bitrev_G(k)) of shift * H_2n, i.e. the coset
a <w_m> with a = shift * w_2n^r, so the shard is a size-m forward DIF (bit-reversed output) of
the folded coefficients d_u = sum_l c_(u + l m) a^(u + l m) -- what ntt.hip's coset_residue
computes.  The quotient's next row (i + 2) of every point of a shard lies in the one residue
class (r + 2) mod G, owned by rank bitrev_G(r + 2 mod G).
"""
import random

import pytest

P = 0x7F000001


def _gen(bits):
    return pow(pow(3, 127, P), 1 << (24 - bits), P)


def _brev(x, b):
    return int(format(x, f"0{b}b")[::-1], 2) if b else 0


@pytest.mark.parametrize("logn", [4, 5, 6])
def test_residue_shards_are_the_bitreversed_coset_lde(logn):
    rng = random.Random(logn)
    n = 1 << logn
    c = [rng.randrange(P) for _ in range(n)]
    shift = 3
    w2n = _gen(logn + 1)
    lde = [0] * (2 * n)
    for i in range(2 * n):
        x = shift * pow(w2n, i, P) % P
        lde[_brev(i, logn + 1)] = sum(cj * pow(x, j, P) for j, cj in enumerate(c)) % P
    for lg in (1, 2, 3):
        G = 1 << lg
        m = 2 * n // G
        zeta = _gen(logn + 1 - lg)
        for k in range(G):
            r = _brev(k, lg)
            a = shift * pow(w2n, r, P) % P
            d = [sum(c[j] * pow(a, j, P) for j in range(u, n, m)) % P for u in range(m)]
            shard = [sum(d[u] * pow(zeta, u * _brev(t, logn + 1 - lg), P) for u in range(m)) % P
                     for t in range(m)]
            assert shard == lde[k * m:(k + 1) * m]
            k2 = _brev((r + 2) % G, lg)
            for t in range(m):
                i = _brev(k * m + t, logn + 1)
                assert _brev((i + 2) % (2 * n), logn + 1) // m == k2


def test_coefficient_slices_sum_to_the_opening():
    """sum over ranks of the slice sum_(j in [k n/G, (k+1) n/G)) c_j z^j is p(z)."""
    rng = random.Random(7)
    n, G = 64, 4
    c = [rng.randrange(P) for _ in range(n)]
    z = rng.randrange(P)
    full = sum(cj * pow(z, j, P) for j, cj in enumerate(c)) % P
    parts = [sum(c[j] * pow(z, j, P) for j in range(k * n // G, (k + 1) * n // G)) % P
             for k in range(G)]
    assert sum(parts) % P == full


@pytest.mark.parametrize("logh", [1, 2, 3, 5])
def test_second_point_denominators_from_the_zeta_table(logh):
    """fri.hip prev2_pos: on an LDE of height H = 2n over 3 H_2n (bit-reversed positions),
    1 / (x_t - z w_n) = w_n^-1 / (x_t' - z) where t' holds natural index bitrev(t) - 2."""
    H = 1 << logh
    wH = _gen(logh)
    wn = pow(wH, 2, P)
    z = 123456789
    for t in range(H):
        i = _brev(t, logh)
        x = 3 * pow(wH, i, P) % P
        t2 = _brev((i - 2) % H, logh)
        x2 = 3 * pow(wH, _brev(t2, logh), P) % P
        lhs = pow((x - z * wn) % P, P - 2, P)
        rhs = pow(wn, P - 2, P) * pow((x2 - z) % P, P - 2, P) % P
        assert lhs == rhs


@pytest.mark.parametrize("lg", [1, 2, 3, 4])
def test_register_fold_halving_steps(lg):
    """ntt.hip k_coef_fold: a thread of the iDFT's second pass holds the 16 coefficients
    c_(k0 + i D), D = n / 16.  For G = 2^lg ranks (m = 2n / G = S D, S = 2^(5 - lg) outputs per
    thread) the fold d_u = a^u sum_l c_(u + l m) (a^m)^l of u = k0 + i0 D, i0 < S, uses exactly the
    thread's terms i0 + l S, and the halving steps y_i += y_(i + h) (a^m)^(h / S), h = 8 .. S,
    compute the sums sum_l x_(i0 + l S) (a^m)^l."""
    rng = random.Random(lg)
    logn = 8
    n = 1 << logn
    D = n // 16
    m = 2 * n >> lg
    S = m // D
    assert S == 1 << (5 - lg)
    c = [rng.randrange(P) for _ in range(n)]
    a = rng.randrange(1, P)
    am = pow(a, m, P)
    ref = [sum(c[j] * pow(a, j, P) for j in range(u, n, m)) % P for u in range(m)]
    got = [None] * m
    for k0 in range(D):
        x = [c[k0 + i * D] for i in range(16)]
        y = list(x)
        h = 8
        while h >= S:
            f = pow(am, h // S, P)
            for i in range(h):
                y[i] = (y[i] + y[i + h] * f) % P
            h //= 2
        for i0 in range(S):
            u = k0 + i0 * D
            got[u] = y[i0] * pow(a, u, P) % P
    assert got == ref


@pytest.mark.parametrize("logn", [11, 12, 14])
def test_logup_running_sum_tiles_cover_natural_rows_in_order(logn):
    """logup.hip k_phi_sums / k_phi_write: natural row i = x 2^(L-5) + z is stored at
    t = rev(z) 32 + rev5(x); a tile (all 32 x, 64 consecutive z) reads whole 32-row storage runs,
    and tile rows (x, b) taken row-major are consecutive natural ranges -- so a flat scan of the
    tile sums in that order gives every tile row's natural-order prefix."""
    n = 1 << logn
    Z = n >> 5
    nt = Z // 64
    seen = set()
    for b in range(nt):
        for zl in range(64):
            run = [(_brev(b * 64 + zl, logn - 5) << 5) | xr for xr in range(32)]
            assert run == list(range(run[0], run[0] + 32))  # one contiguous storage run
            for xr in range(32):
                x = _brev(xr, 5)
                i = x * Z + b * 64 + zl
                assert _brev(i, logn) == run[xr]
                seen.add(run[xr])
    assert len(seen) == n
    order = []  # tile rows row-major: natural ranges [x Z + 64 b, + 64)
    for x in range(32):
        for b in range(nt):
            order.append(x * Z + 64 * b)
    assert order == list(range(0, n, 64))
