"""GPU parity tests: the HIP path (through the C ABI) against the oracle, bit for bit."""
import ctypes
import hashlib
import json
import os

import numpy as np
import pytest

import oracle_lib as O
from bfz import _lib, guests, sdk

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = json.load(open(os.path.join(ROOT, "tests", "golden", "golden.json")))
P = O.P
P32 = ctypes.POINTER(ctypes.c_uint32)


def mont(a):
    return ((np.asarray(a, dtype=np.uint64) << np.uint64(32)) % np.uint64(P)).astype(np.uint32)


def unmont(a):
    inv = pow(2, -32, P)
    return ((np.asarray(a, dtype=np.uint64) * np.uint64(inv)) % np.uint64(P)).astype(np.uint32)


@pytest.fixture(scope="module", autouse=True)
def gpu():
    _lib.init(0)
    yield


def test_poseidon2_batch_parity():
    rng = np.random.default_rng(1)
    st = rng.integers(0, P, size=(4096, 16), dtype=np.uint64).astype(np.uint32)
    for kat in GOLDEN["poseidon2"]:
        st[: 1] = np.array(kat["in"], dtype=np.uint32)
        dev = mont(st).reshape(-1).copy()
        _lib.check(_lib.lib().bfz_poseidon2_permute(dev.ctypes.data_as(P32), len(st)))
        got = unmont(dev).reshape(-1, 16)
        assert got[0].tolist() == kat["out"]
        exp = O.poseidon2(st.reshape(-1)).reshape(-1, 16)
        assert np.array_equal(got, exp)


def test_poseidon2_extreme_states_parity():
    """The lazy forms' bounds (signed state, unreduced 64-bit internal diagonal elements,
    poseidon2.h) at the edges: device words (Montgomery form) 0, 1, p - 1, (p +- 1)/2 and
    alternating extremes, then 2^18 random states."""
    edge = [np.zeros(16), np.full(16, P - 1), np.ones(16), np.tile([P - 1, 0], 8),
            np.tile([0, P - 1], 8), np.full(16, (P - 1) // 2), np.full(16, (P + 1) // 2),
            np.arange(P - 16, P), np.tile([P - 1, 1], 8)]
    rng = np.random.default_rng(7)
    words = np.concatenate([np.array(edge, dtype=np.uint64),
                            rng.integers(0, P, size=(1 << 18, 16), dtype=np.uint64)]).astype(np.uint32)
    dev = words.reshape(-1).copy()
    _lib.check(_lib.lib().bfz_poseidon2_permute(dev.ctypes.data_as(P32), len(words)))
    exp = O.poseidon2(unmont(words).reshape(-1)).reshape(-1, 16)
    assert np.array_equal(unmont(dev).reshape(-1, 16), exp)


def test_poseidon2_lane_mode_parity():
    """16-lanes-per-state permutation (DPP cross-lane MDS) == oracle."""
    rng = np.random.default_rng(3)
    st = rng.integers(0, P, size=(100, 16), dtype=np.uint64).astype(np.uint32)
    st[0] = GOLDEN["poseidon2"][0]["in"]
    dev = mont(st).reshape(-1).copy()
    _lib.check(_lib.lib().bfz_poseidon2_permute_small(dev.ctypes.data_as(P32), len(st)))
    got = unmont(dev).reshape(-1, 16)
    assert got[0].tolist() == GOLDEN["poseidon2"][0]["out"]
    assert np.array_equal(got, O.poseidon2(st.reshape(-1)).reshape(-1, 16))


@pytest.mark.parametrize("logn,w", [(0, 3), (1, 2), (4, 31), (5, 1), (10, 45), (13, 7), (16, 4),
                                    (17, 9), (20, 2)])
def test_coset_lde_parity(logn, w):
    rng = np.random.default_rng(logn * 100 + w)
    n = 1 << logn
    m = rng.integers(0, P, size=(n, w), dtype=np.uint64).astype(np.uint32)
    out = np.zeros((2 * n, w), dtype=np.uint32)
    src = mont(m).copy()
    _lib.check(_lib.lib().bfz_coset_lde(src.ctypes.data_as(P32), n, w, int(mont([3])[0]),
                                        out.ctypes.data_as(P32)))
    exp = O.coset_lde(m, 3)
    assert np.array_equal(unmont(out), exp)


def test_commit_root_parity():
    rng = np.random.default_rng(7)
    shapes = [(1 << 12, 31), (1 << 12, 41), (1 << 11, 7), (1 << 9, 45), (16, 5), (16, 12)]
    mats = [rng.integers(0, P, size=s, dtype=np.uint64).astype(np.uint32) for s in shapes]
    ldes = [O.coset_lde(m, 3) for m in mats]
    exp = O.merkle_root(ldes)
    dev = [mont(m).copy() for m in mats]
    ptrs = (P32 * len(dev))(*[d.ctypes.data_as(P32) for d in dev])
    hs = (ctypes.c_size_t * len(dev))(*[s[0] for s in shapes])
    ws = (ctypes.c_size_t * len(dev))(*[s[1] for s in shapes])
    root = (ctypes.c_uint32 * 8)()
    _lib.check(_lib.lib().bfz_commit(ptrs, hs, ws, len(dev), root))
    assert unmont(list(root)).tolist() == exp


@pytest.fixture(scope="module")
def client():
    return sdk.ProverClient()


@pytest.mark.parametrize("name,prog,stdin", guests.REFERENCE_PROGRAMS)
def test_proof_bytes_match_oracle(client, name, prog, stdin):
    pk, vk = client.setup(prog)
    g = [x for x in GOLDEN["proofs"] if x["name"] == name][0]
    assert unmont(vk.commit).tolist() == g["vk_commit"]
    pf = client.prove(pk, stdin).run()
    assert hashlib.sha256(pf.proof).hexdigest() == g["sha256"], "differs from the oracle fixture"
    assert pf.proof == O.prove(prog, stdin)
    client.verify(pf, vk)                      # product host verifier
    assert O.verify(prog, pf.proof)            # oracle verifier


def _device_trace(prog, stdin, chip):
    p = ctypes.POINTER(ctypes.c_uint32)()
    h, w = ctypes.c_size_t(), ctypes.c_size_t()
    inb = bytes(stdin)
    buf = (ctypes.c_uint8 * max(len(inb), 1))(*inb)
    rc = _lib.lib().bfz_trace_device(prog.encode(), buf, len(inb), chip, ctypes.byref(p),
                                     ctypes.byref(h), ctypes.byref(w))
    if rc == 1:
        return None
    _lib.check(rc)
    arr = np.ctypeslib.as_array(p, shape=(h.value * w.value,)).copy().reshape(h.value, w.value)
    _lib.lib().bfz_free(p)
    return arr


@pytest.mark.parametrize("name,prog,stdin", guests.REFERENCE_PROGRAMS +
                         [("fibo255", guests.FIBO, [255])])
def test_device_traces_match_oracle(name, prog, stdin):
    """generate_dependencies + generate_traces on the device (tracegen.hip) == the oracle's
    host traces, every chip, including the Byte/Program multiplicity histograms."""
    for chip in range(8):
        exp = O.trace(prog, stdin, chip)
        got = _device_trace(prog, stdin, chip)
        assert (got is None) == (exp is None), (name, chip)
        if exp is not None:
            assert np.array_equal(unmont(got), exp), (name, sdk.CHIPS[chip])


def test_prove_from_host_traces_matches(client):
    """MachineProver boundary: traces produced on the host (generate_traces) proved through
    bfz_prove_traces give the same bytes as the record path and the oracle."""
    pk, vk = client.setup(guests.FIBO)
    traces = sdk.generate_traces(guests.FIBO, [17])
    assert [name for _, name, _ in traces][0] == "Cpu"
    for c, name, t in traces:  # the same traces the oracle generates (canonical form)
        assert np.array_equal(unmont(t), O.trace(guests.FIBO, [17], c)), name
    pf = sdk.CoreProver().prove(pk, traces)
    assert pf == client.prove(pk, [17]).run().proof
    assert pf == O.prove(guests.FIBO, [17])
    client.verify(sdk.BfProofWithPublicValues(proof=pf, stdin=bytes([17])), vk)


def test_split_commit_open_matches_prove(client):
    """MachineProver::commit + observe_into + open (prover.rs:209-236, 595-601, 242-553) through
    the split C ABI give the bytes of the one-call prove; open leaves the challenger unchanged
    (the reference opens on a clone, prover.rs:578) and the main data can be opened again."""
    pk, vk = client.setup(guests.FIBO)
    traces = sdk.generate_traces(guests.FIBO, [17])
    prover = sdk.CoreProver()
    data = prover.commit(pk, traces)
    ch = prover.new_challenger()
    prover.observe_into(pk, ch)
    before = bytes(ch)
    pf = prover.open(pk, data, ch)
    assert bytes(ch) == before
    assert pf == client.prove(pk, [17]).run().proof
    assert pf == O.prove(guests.FIBO, [17])
    assert prover.open(pk, data, ch) == pf
    # the record path (device-generated traces) commits to the same root
    rec = ctypes.c_void_p()
    buf, n = _lib.u8buf(bytes([17]))
    _lib.check(_lib.lib().bfz_record_new(ctypes.c_void_p(pk.handle), buf, n, ctypes.byref(rec),
                                         None))
    data2 = prover.commit_record(pk, rec.value)
    assert data2.main_commit == data.main_commit
    assert prover.open(pk, data2, ch) == pf
    _lib.lib().bfz_record_free(rec)
    # a challenger that has not observed the key gives a proof the verifier rejects
    bad = prover.open(pk, data, prover.new_challenger())
    with pytest.raises(_lib.BfzError):
        client.verify(sdk.BfProofWithPublicValues(proof=bad, stdin=bytes([17])), vk)
    # main data committed for another key is refused; a key-less commit (the trait's commit
    # takes no key) opens under any key
    pk2, _ = client.setup(guests.HELLO)
    with pytest.raises(_lib.BfzError, match="another key"):
        prover.open(pk2, data, ch)
    mats, chips, ptrs, hs, ws, k = sdk._trace_args(traces)
    out = ctypes.c_void_p()
    root = (ctypes.c_uint32 * 8)()
    _lib.check(_lib.lib().bfz_main_commit(None, chips, ptrs, hs, ws, k, ctypes.byref(out), root))
    keyless = sdk.ShardMainData(out.value, root)
    assert keyless.main_commit == data.main_commit
    assert prover.open(pk, keyless, ch) == pf


def test_prove_batch_pipelined_matches_single(client):
    """bfz_prove_batch (execute + upload of job k+1 under prove(k)) returns, job for job, the
    bytes of single proofs and of the oracle, for every executor-thread count."""
    pk, vk = client.setup(guests.FIBO)
    stdins = [[5], [17], [30], [17], [1], [12], [9]]
    want = [O.prove(guests.FIBO, s) for s in stdins]
    for threads in (1, 2, 3):
        stats = {}
        got = client.prove_batch(pk, stdins, exec_threads=threads, stats=stats)
        assert [p.proof for p in got] == want, threads
        assert stats["exec_threads"] == threads and stats["wall_ms"] > 0
    client.verify(got[1], vk)
    assert got[1].public_values == client.execute(guests.FIBO, [17]).run()
    assert client.prove_batch(pk, []) == []


def test_prove_batch_error_does_not_hang(client):
    """An executor failure (missing input) in the middle of a batch is reported, the other
    threads stop, and the library stays usable."""
    pk, _ = client.setup(guests.FIBO)
    with pytest.raises(_lib.BfzError, match="input"):
        client.prove_batch(pk, [[5], [6], [], [7], [8]], exec_threads=2)
    assert client.prove_batch(pk, [[5]])[0].proof == O.prove(guests.FIBO, [5])


def test_setup_is_cached_per_program(client):
    """StarkMachine::setup (machine.rs:154-224) runs once per program: a second setup of the
    same ELF returns the same device-resident key at once."""
    import time
    elf = guests.FIBO + "\n"  # a program text no other test has set up
    t0 = time.perf_counter()
    pk1, vk1 = client.setup(elf)
    t1 = time.perf_counter()
    pk2, vk2 = client.setup(elf)
    t2 = time.perf_counter()
    assert vk1.commit == vk2.commit
    assert t2 - t1 < max(0.5 * (t1 - t0), 0.005)
    pf = client.prove(pk2, [5]).run()
    client.verify(pf, vk1)


def test_prove_traces_rejects_bad_shapes(client):
    pk, _ = client.setup(guests.HELLO)
    traces = sdk.generate_traces(guests.HELLO, [])
    c, name, t = traces[0]
    with pytest.raises(_lib.BfzError, match="width mismatch"):
        sdk.CoreProver().prove(pk, [(c, name, t[:, :-1])] + traces[1:])
    with pytest.raises(_lib.BfzError, match="power of two"):
        sdk.CoreProver().prove(pk, [(c, name, t[:-1])] + traces[1:])
    with pytest.raises(_lib.BfzError, match="repeated"):
        sdk.CoreProver().prove(pk, traces + traces[:1])
    bad = t.copy()
    bad[3, 0] = P  # a Montgomery word >= p
    with pytest.raises(_lib.BfzError, match="non-canonical"):
        sdk.CoreProver().prove(pk, [(c, name, bad)] + traces[1:])
    with pytest.raises(_lib.BfzError, match="power of two"):  # height 1
        sdk.CoreProver().prove(pk, [(c, name, t[:1])] + traces[1:])


def test_fibo17_end_to_end_sdk(client):
    """crates/sdk/src/lib.rs:186-196 test_e2e_core, through the SDK mirror."""
    pk, vk = client.setup(guests.FIBO)
    assert client.execute(guests.FIBO, [17]).run()[0] == 85
    proof = client.prove(pk, [17]).run()
    client.verify(proof, vk)


def test_random_programs_bytes_match_oracle(client):
    """Whole-proof parity beyond the reference programs: 16 seeded random halting programs
    (I/O, memory excursions, nested loops; some chips empty) give the oracle's bytes, and both
    verifiers accept them."""
    from bfgen import random_program
    rng = np.random.default_rng(11)
    for k in range(16):
        prog = random_program(rng, int(rng.integers(3, 120)), allow_negative=False)
        stdin = [int(x) for x in rng.integers(0, 256, size=prog.count(","))]
        pk, vk = client.setup(prog)
        pf = client.prove(pk, stdin).run()
        assert pf.proof == O.prove(prog, stdin), (k, prog)
        client.verify(pf, vk)
        assert O.verify(prog, pf.proof), (k, prog)


def test_pointer_below_zero_matches_reference_behaviour(client):
    """The reference executor wraps the memory pointer (u32, executor.rs:137-138) but its
    MemoryInstrs AIR range-checks it as a field word (air.rs:37-61): a program stepping below
    cell 0 executes and 'proves', and every verifier rejects the proof.  bfz reproduces that
    byte for byte (no early error the reference would not raise)."""
    prog, stdin = "<+.>,[->+<]>.", [7]
    pk, vk = client.setup(prog)
    pf = client.prove(pk, stdin).run()
    assert pf.proof == O.prove(prog, stdin)
    assert not O.verify(prog, pf.proof)
    with pytest.raises(_lib.BfzError, match="OOD evaluation mismatch on chip MemoryInstrs"):
        client.verify(pf, vk)


def test_fibo255_2pow20_parity(client):
    """fibonacci trace 2^20 rows (BASELINE config 3): full pipeline, bit-exact vs oracle."""
    pk, vk = client.setup(guests.FIBO)
    pf = client.prove(pk, [255]).run()
    client.verify(pf, vk)
    assert pf.proof == O.prove(guests.FIBO, [255])


@pytest.mark.slow
def test_fibo_x4_2pow22_bytes_match_oracle(client):
    """Headline workload (BASELINE.json metric: Cpu trace 2^22 rows, FIBO_X4 stdin [255],
    3,767,729 cycles): the GPU proof is byte-identical to the oracle's, both verifiers accept
    it, proving is deterministic, the bincode form round-trips, and tampering is rejected."""
    pk, vk = client.setup(guests.FIBO_X4)
    a = client.prove(pk, [255]).run()
    client.verify(a, vk)
    b = client.prove(pk, [255]).run()
    assert a.proof == b.proof
    ref = O.prove(guests.FIBO_X4, [255])
    assert a.proof == ref, "headline proof differs from the oracle"
    assert O.verify(guests.FIBO_X4, a.proof)
    bc = sdk.proof_to_bincode(a.proof)
    client.verify_bincode(bc, vk)
    assert sdk.proof_from_bincode(bc) == a.proof
    bad = bytearray(a.proof)
    bad[len(bad) // 3] ^= 4
    with pytest.raises(_lib.BfzError):
        client.verify(sdk.BfProofWithPublicValues(proof=bytes(bad), stdin=b"\xff"), vk)


def test_pcs_variant_parity(client):
    """Decision D1 switched off: GPU and oracle still agree bit for bit, and the
    proof differs from the default variant's."""
    prog = guests.FIBO
    pk, vk = client.setup(prog)
    try:
        sdk.set_pcs_variant(0)
        pf = client.prove(pk, [17]).run()
        client.verify(pf, vk)
        assert pf.proof == O.prove(prog, [17], observe_openings=False)
    finally:
        sdk.set_pcs_variant(-1)
    assert pf.proof != client.prove(pk, [17]).run().proof


def test_invalid_trace_rejected_by_verifiers(client):
    """An execution that violates the AIR (a memory pointer wrapping below zero breaks the
    KoalaBear word range check of MemoryInstrs) still yields a proof -- the quotient chunks
    are low-degree by construction, as in the reference -- but both verifiers reject it at
    the out-of-domain check (verifier.rs:194-208).  GPU and oracle agree bit for bit."""
    prog = "<+"
    pk, vk = client.setup(prog)
    pf = client.prove(pk, []).run()
    assert pf.proof == O.prove(prog, [])
    with pytest.raises(_lib.BfzError, match="OOD evaluation mismatch"):
        client.verify(pf, vk)
    assert not O.verify(prog, pf.proof)


def test_cpu_2pow23_proves_but_verifier_bounds_degree(client):
    """Largest provable size: 8 outer fibonacci loops (~7.5 M cycles) give a 2^23-row Cpu
    trace, whose LDE (2^24 rows) is KoalaBear's full two-adic subgroup.  The prover handles it;
    the verifier rejects Cpu log degree 23 > MAX_CPU_LOG_DEGREE = 22 exactly as
    crates/prover/src/verify.rs:20-28 (CpuLogDegreeTooLarge)."""
    prog = "++++++++[>" + guests.FIBO + "[-]<[-]<<-]"
    pk, vk = client.setup(prog)
    pf = client.prove(pk, [255]).run()
    with pytest.raises(_lib.BfzError, match="Cpu log degree too large"):
        client.verify(pf, vk)


def test_trace_beyond_two_adicity_is_an_error(client):
    """16 outer loops (~15 M cycles) need a 2^24-row Cpu trace and a 2^25-point LDE, beyond
    the 2^24-element two-adic subgroup of KoalaBear (p - 1 = 127 * 2^24): a clean error, no
    device fault, and the library keeps working afterwards."""
    prog = "++++++++++++++++[>" + guests.FIBO + "[-]<[-]<<-]"
    pk, vk = client.setup(prog)
    with pytest.raises(_lib.BfzError):
        client.prove(pk, [255]).run()
    pk2, vk2 = client.setup(guests.FIBO)
    client.verify(client.prove(pk2, [17]).run(), vk2)
