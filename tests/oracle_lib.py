"""ctypes wrapper of oracle/liboracle.so — TEST INFRASTRUCTURE ONLY (the checker).

Canonical u32 field values everywhere (the product uses Montgomery form at its ABI).
"""
from __future__ import annotations

import ctypes
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.path.join(ROOT, "oracle", "liboracle.so")
P = 0x7F000001

_L = None


def lib():
    global _L
    if _L is None:
        if not os.path.exists(ORACLE_SO):
            import subprocess
            subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True,
                           stdout=subprocess.DEVNULL)
        L = ctypes.CDLL(ORACLE_SO)
        P8 = ctypes.POINTER(ctypes.c_uint8)
        P32 = ctypes.POINTER(ctypes.c_uint32)
        L.or_api_execute.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t, P8,
                                     ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t),
                                     ctypes.POINTER(ctypes.c_uint64), P32, P32]
        L.or_api_prove.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t,
                                   ctypes.POINTER(P8), ctypes.POINTER(ctypes.c_size_t)]
        L.or_api_verify.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t]
        L.or_api_free.argtypes = [ctypes.c_void_p]
        L.or_api_trace.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int,
                                   ctypes.c_int, ctypes.POINTER(P32),
                                   ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_size_t)]
        L.or_api_poseidon2.argtypes = [P32, ctypes.c_size_t]
        L.or_api_hash.argtypes = [P32, ctypes.c_size_t, P32]
        L.or_api_coset_lde.argtypes = [P32, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_uint32, P32]
        L.or_api_merkle_root.argtypes = [ctypes.POINTER(P32), ctypes.POINTER(ctypes.c_size_t),
                                         ctypes.POINTER(ctypes.c_size_t), ctypes.c_int, P32]
        L.or_api_two_adic_gen.restype = ctypes.c_uint32
        L.or_api_challenger.argtypes = [P32, ctypes.c_size_t, P32, ctypes.c_size_t]
        L.or_api_pcs_commit_fri.argtypes = [P32, ctypes.c_size_t, ctypes.c_size_t, P32, P32,
                                            ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t), P32,
                                            P32]
        L.or_api_setup_root.argtypes = [ctypes.c_char_p, P32]
        L.or_api_perm_trace.argtypes = [ctypes.c_int, P32, P32, ctypes.c_size_t, P32, P32, P32, P32]
        L.or_set_num_queries.argtypes = [ctypes.c_int]
        L.or_set_pcs_variant.argtypes = [ctypes.c_int]
        L.or_variant_set.argtypes = [ctypes.c_char_p, ctypes.c_uint32]
        L.or_variant_reset.argtypes = []
        _L = L
    return _L


VARIANT_NAMES = ("diag_alt", "m4_horizen", "no_initial_mds", "inject_first", "fri_coeff_major",
                 "query_extra_bits", "sample_front", "selectors_normalized", "force_witness",
                 "witness")


def set_variant(**kw):
    """The oracle's [p3-recalled] switches D2-D9 (oracle/or_hash.h or_variant_t); D1 is the
    observe_openings argument of prove / verify.  Unnamed switches are reset to the default."""
    L = lib()
    L.or_variant_reset()
    for k, v in kw.items():
        if L.or_variant_set(k.encode(), int(v)) != 0:
            raise KeyError(k)


def reset_variant():
    lib().or_variant_reset()


def execute(prog: str, stdin):
    L = lib()
    out = (ctypes.c_uint8 * 65536)()
    n = ctypes.c_size_t()
    cyc = ctypes.c_uint64()
    pc = ctypes.c_uint32()
    mp = ctypes.c_uint32()
    inb = bytes(stdin)
    r = L.or_api_execute(prog.encode(), inb, len(inb), out, 65536, ctypes.byref(n),
                         ctypes.byref(cyc), ctypes.byref(pc), ctypes.byref(mp))
    if r:
        raise RuntimeError(f"oracle execute failed: {r}")
    return {"output": bytes(out[: n.value]), "cycles": cyc.value, "pc": pc.value, "mp": mp.value}


def prove(prog: str, stdin, num_queries: int = 84, observe_openings: bool = True) -> bytes:
    L = lib()
    L.or_set_num_queries(num_queries)
    L.or_set_pcs_variant(int(observe_openings))
    p = ctypes.POINTER(ctypes.c_uint8)()
    n = ctypes.c_size_t()
    inb = bytes(stdin)
    r = L.or_api_prove(prog.encode(), inb, len(inb), ctypes.byref(p), ctypes.byref(n))
    if r:
        raise RuntimeError(f"oracle prove failed: {r}")
    b = ctypes.string_at(p, n.value)
    L.or_api_free(p)
    return b


def verify(prog: str, proof: bytes, num_queries: int = 84, observe_openings: bool = True) -> bool:
    L = lib()
    L.or_set_num_queries(num_queries)
    L.or_set_pcs_variant(int(observe_openings))
    return L.or_api_verify(prog.encode(), proof, len(proof)) == 0


def trace(prog: str, stdin, chip: int, prep: bool = False):
    import numpy as np
    L = lib()
    p = ctypes.POINTER(ctypes.c_uint32)()
    h = ctypes.c_size_t()
    w = ctypes.c_size_t()
    inb = bytes(stdin)
    r = L.or_api_trace(prog.encode(), inb, len(inb), chip, int(prep), ctypes.byref(p),
                       ctypes.byref(h), ctypes.byref(w))
    if r:
        return None
    arr = np.ctypeslib.as_array(p, shape=(h.value * w.value,)).copy().reshape(h.value, w.value)
    L.or_api_free(p)
    return arr


def poseidon2(states):
    import numpy as np
    a = np.ascontiguousarray(states, dtype=np.uint32).copy()
    lib().or_api_poseidon2(a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), a.size // 16)
    return a


def coset_lde(evals, shift: int):
    import numpy as np
    a = np.ascontiguousarray(evals, dtype=np.uint32)
    n, w = a.shape
    out = np.zeros((2 * n, w), dtype=np.uint32)
    lib().or_api_coset_lde(a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), n, w, shift,
                           out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)))
    return out


def merkle_root(mats):
    import numpy as np
    mats = [np.ascontiguousarray(m, dtype=np.uint32) for m in mats]
    ptrs = (ctypes.POINTER(ctypes.c_uint32) * len(mats))(
        *[m.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)) for m in mats])
    hs = (ctypes.c_size_t * len(mats))(*[m.shape[0] for m in mats])
    ws = (ctypes.c_size_t * len(mats))(*[m.shape[1] for m in mats])
    root = (ctypes.c_uint32 * 8)()
    lib().or_api_merkle_root(ptrs, hs, ws, len(mats), root)
    return list(root)


def pcs_commit_fri(m, challenges=False):
    """Column-sharded PCS restatement (oracle/or_pcs.c): commitment root of the coset LDE of the
    n x w matrix m (canonical words, natural row order), the FRI commit-phase roots of the
    batched column sum_c alpha^c col_c, and the final constant -- canonical words.  With
    challenges=True also (alpha, [beta per round]) as EF word lists."""
    import numpy as np
    a = np.ascontiguousarray(m, dtype=np.uint32)
    n, w = a.shape
    cap = n.bit_length() + 1
    root = (ctypes.c_uint32 * 8)()
    fri = (ctypes.c_uint32 * (8 * cap))()
    nr = ctypes.c_size_t()
    fin = (ctypes.c_uint32 * 4)()
    ch = (ctypes.c_uint32 * (4 + 4 * cap))()
    rc = lib().or_api_pcs_commit_fri(a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), n, w, root,
                                     fri, cap, ctypes.byref(nr), fin, ch)
    if rc == -2:
        raise MemoryError("oracle pcs: LDE allocation failed")
    rounds = [list(fri[8 * i: 8 * i + 8]) for i in range(nr.value)]
    out = (list(root), rounds, list(fin), rc == 0)
    if challenges:
        out += ((list(ch[:4]), [list(ch[4 + 4 * i: 8 + 4 * i]) for i in range(nr.value)]),)
    return out


def setup_root(prog: str):
    root = (ctypes.c_uint32 * 8)()
    lib().or_api_setup_root(prog.encode(), root)
    return list(root)


def two_adic_gen(bits: int) -> int:
    return lib().or_api_two_adic_gen(bits)


def challenger(obs, m):
    arr = (ctypes.c_uint32 * max(1, len(obs)))(*obs)
    out = (ctypes.c_uint32 * m)()
    lib().or_api_challenger(arr, len(obs), out, m)
    return list(out)


def to_mont(x: int) -> int:
    return (x << 32) % P


def from_mont(x: int) -> int:
    return (x * pow(2, -32, P)) % P


def perm_trace(chip: int, main, prep, alpha, beta):
    """generate_permutation_trace (permutation.rs:75-148) of one chip: (n x 4 pw flattened
    permutation trace, cumulative sum), canonical values."""
    import numpy as np
    P32 = ctypes.POINTER(ctypes.c_uint32)
    m = np.ascontiguousarray(main, dtype=np.uint32)
    n = m.shape[0]
    pr = None if prep is None else np.ascontiguousarray(prep, dtype=np.uint32)
    out = np.zeros((n, 4 * 9), dtype=np.uint32)  # widest chip: Cpu, 9 EF columns
    cs = (ctypes.c_uint32 * 4)()
    a = (ctypes.c_uint32 * 4)(*alpha)
    b = (ctypes.c_uint32 * 4)(*beta)
    pw = lib().or_api_perm_trace(chip, m.ctypes.data_as(P32),
                                 pr.ctypes.data_as(P32) if pr is not None else None, n, a, b,
                                 out.ctypes.data_as(P32), cs)
    flat = out.reshape(-1)[: n * 4 * pw].reshape(n, 4 * pw)
    return flat, list(cs)
