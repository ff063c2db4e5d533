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
    """16-lanes-per-state permutation (DPP cross-lane MDS, signed lazy form) == oracle, with the
    golden vector, the extreme states of the test above and 4096 random states."""
    rng = np.random.default_rng(3)
    st = rng.integers(0, P, size=(4096 + 16, 16), dtype=np.uint64).astype(np.uint32)
    st[0] = GOLDEN["poseidon2"][0]["in"]
    dev = mont(st).reshape(-1).copy()
    edge = [np.zeros(16), np.full(16, P - 1), np.ones(16), np.tile([P - 1, 0], 8),
            np.tile([0, P - 1], 8), np.full(16, (P - 1) // 2), np.full(16, (P + 1) // 2),
            np.arange(P - 16, P), np.tile([P - 1, 1], 8)]
    dev.reshape(-1, 16)[1:1 + len(edge)] = np.array(edge, dtype=np.uint64).astype(np.uint32)
    ref_in = unmont(dev).reshape(-1)
    _lib.check(_lib.lib().bfz_poseidon2_permute_small(dev.ctypes.data_as(P32), len(st)))
    got = unmont(dev).reshape(-1, 16)
    assert got[0].tolist() == GOLDEN["poseidon2"][0]["out"]
    assert np.array_equal(got, O.poseidon2(ref_in).reshape(-1, 16))


@pytest.mark.parametrize("logn,w", [(0, 3), (1, 2), (4, 31), (5, 1), (6, 64), (8, 3), (9, 2), (10, 45), (13, 7), (14, 5),
                                    (16, 4), (17, 9), (18, 3), (20, 2), (22, 1)])
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
    the split C ABI give the bytes of the one-call prove; open advances the challenger it is
    given (prove passes a clone, prover.rs:578) and the main data can be opened again."""
    pk, vk = client.setup(guests.FIBO)
    traces = sdk.generate_traces(guests.FIBO, [17])
    prover = sdk.CoreProver()
    data = prover.commit(pk, traces)
    ch0 = prover.new_challenger()
    prover.observe_into(pk, ch0)
    before = bytes(ch0)
    ch = _lib.Challenger.from_buffer_copy(before)  # prove opens on a clone (prover.rs:578)
    pf = prover.open(pk, data, ch)
    # open advances its &mut challenger through the whole transcript, the same
    # final state every time
    assert bytes(ch) != before
    after = bytes(ch)
    assert pf == client.prove(pk, [17]).run().proof
    assert pf == O.prove(guests.FIBO, [17])
    ch = _lib.Challenger.from_buffer_copy(before)
    assert prover.open(pk, data, ch) == pf and bytes(ch) == after
    ch = _lib.Challenger.from_buffer_copy(before)
    # the record path (device-generated traces) commits to the same root
    rec = ctypes.c_void_p()
    buf, n = _lib.u8buf(bytes([17]))
    _lib.check(_lib.lib().bfz_record_new(ctypes.c_void_p(pk.handle), buf, n, ctypes.byref(rec),
                                         None))
    data2 = prover.commit_record(pk, rec.value)
    assert data2.main_commit == data.main_commit
    assert prover.open(pk, data2, ch) == pf
    _lib.lib().bfz_record_free(rec)
    ch = _lib.Challenger.from_buffer_copy(before)
    # a challenger that has not observed the key gives a proof the verifier rejects
    bad = prover.open(pk, data, prover.new_challenger())
    with pytest.raises(_lib.BfzError):
        client.verify(sdk.BfProofWithPublicValues(proof=bad, stdin=bytes([17])), vk)
    # main data committed for another key is refused; a key-less commit (the trait's commit
    # takes no key) opens under any key
    pk2, _ = client.setup(guests.HELLO)
    with pytest.raises(_lib.BfzError, match="another key"):
        prover.open(pk2, data, ch)
    ch = _lib.Challenger.from_buffer_copy(before)
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


def test_record_prove_repeat_two_lanes_matches_oracle(client):
    """bfz_record_prove_repeat: proofs of one record back to back with one or
    two in flight, each on its own stream / pool / mailboxes; every proof is checked against the
    first inside the library and the first is the oracle's.  Then the default lane still proves."""
    from bfz import events
    prog, stdin = guests.FIBO, [255]
    pk, vk = client.setup(prog)
    rec = events.ExecutionRecordArrays.from_executor(prog, stdin)
    drec = events.record_from_events(pk, rec)
    want = O.prove(prog, stdin)
    L = _lib.lib()
    for inflight, count in ((1, 3), (2, 7), (4, 9)):
        ptr = ctypes.POINTER(ctypes.c_uint8)()
        n = ctypes.c_size_t()
        wall = ctypes.c_double()
        _lib.check(L.bfz_record_prove_repeat(ctypes.c_void_p(pk.handle), ctypes.c_void_p(drec.handle),
                                             count, inflight, ctypes.byref(ptr), ctypes.byref(n),
                                             ctypes.byref(wall)))
        assert _lib.take_bytes(ptr, n.value) == want, inflight
        assert wall.value > 0
    with pytest.raises(_lib.BfzError, match="inflight"):
        _lib.check(L.bfz_record_prove_repeat(ctypes.c_void_p(pk.handle), ctypes.c_void_p(drec.handle),
                                             2, 5, ctypes.byref(ptr), ctypes.byref(n), None))
    assert _prove_record(pk, drec) == want
    # every lane that proved holds a pool: at least the record's LDEs (2n rows of the main trace)
    held = []
    for lane in range(4):
        b = ctypes.c_uint64()
        _lib.check(L.bfz_device_pool_bytes(lane, ctypes.byref(b)))
        held.append(b.value)
    assert all(h > 0 for h in held), held
    with pytest.raises(_lib.BfzError, match="lane"):
        _lib.check(L.bfz_device_pool_bytes(4, ctypes.byref(b)))


def test_pool_reuse_across_shapes(client):
    """The lane pool (gpu.h DevicePool): a second proof of a shape the pool has already
    served allocates nothing, in either order of two shapes whose buffers differ by more than 2x
    (fibo17: Cpu 2^9 rows; fibo255: Cpu 2^20 rows), and the proving key, tables and the record's
    events are not in the lane's pool."""
    from bfz import events
    L = _lib.lib()

    def held():
        b = ctypes.c_uint64()
        _lib.check(L.bfz_device_pool_bytes(0, ctypes.byref(b)))
        return b.value

    pk, _ = client.setup(guests.FIBO)
    small = events.record_from_events(pk, events.ExecutionRecordArrays.from_executor(guests.FIBO, [17]))
    big = events.record_from_events(pk, events.ExecutionRecordArrays.from_executor(guests.FIBO, [255]))
    _prove_record(pk, small)
    _prove_record(pk, big)
    b0 = held()
    extra = events.record_from_events(pk, events.ExecutionRecordArrays.from_executor(guests.FIBO, [255]))
    assert held() == b0, "a record's device events went to the lane pool"
    del extra
    for rec in (small, big, small, big):
        _prove_record(pk, rec)
        assert held() == b0


def test_device_twiddle_table_matches_host():
    """The twiddle table is built on the device (runtime.hip k_twiddle_table, 2 x 2^24 words, once
    per process): identical to the host's running products (levels < 2^20 in full, a sample of
    every higher level)."""
    L = _lib.lib()
    assert L.bfz_selftest(b"twiddles") == 0, L.bfz_last_error()


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
    with pytest.raises(_lib.BfzError, match="power of two"):
        sdk.CoreProver().prove(pk, [(c, name, t[:6])] + traces[1:])


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
    # the Rust drop-in's path: the reference record's events through bfz_record_from_events
    from bfz import events
    rec = events.ExecutionRecordArrays.from_executor(guests.FIBO_X4, [255])
    assert len(rec.cpu) == 3767729
    assert _record_proof(pk, rec) == ref
    assert _record_proof(pk, rec, cycles=True) == ref  # the compact hand-over (16 B per cycle)
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


# ---------------------------------------------------------------- the Rust drop-in's flows
ONE_CYCLE = [("+", []), (".", []), (">", []), (",", [9]), ("-", [])]


@pytest.mark.parametrize("prog,stdin", ONE_CYCLE)
def test_one_cycle_programs_match_oracle(client, prog, stdin):
    """1-row Cpu traces (cpu/trace.rs:33, no minimum height): the GPU proof is the
    oracle's, both verifiers accept it; the host-trace path takes the 1-row trace too."""
    pk, vk = client.setup(prog)
    pf = client.prove(pk, stdin).run()
    assert pf.proof == O.prove(prog, stdin)
    client.verify(pf, vk)
    assert O.verify(prog, pf.proof)
    traces = sdk.generate_traces(prog, stdin)
    assert traces[0][2].shape[0] == 1
    assert sdk.CoreProver().prove(pk, traces) == pf.proof


@pytest.mark.parametrize("name,prog,stdin", guests.REFERENCE_PROGRAMS + [("fibo17", guests.FIBO, [17])])
def test_bfprover_host_key_flow_matches_oracle(name, prog, stdin):
    """BfProver<HipProverComponents> as the reference runs it (crates/prover/src/lib.rs:46-90):
    setup keeps only pk_to_host(pk) and drops the device key; every prove rebuilds it with
    pk_to_device (bfz_pk_from_host) and proves the executor's record through
    bfz_record_from_events (HipProver::prove).  Bytes = the oracle's."""
    bp = sdk.BfProver()
    pk, vk = bp.setup(prog)
    assert isinstance(pk.pk, sdk.StarkProvingKey) and pk.pk.commit == vk.commit
    assert [n for _, n, _ in pk.pk.traces] == ["Byte", "Program"]  # (Reverse(height), name)
    pf = bp.prove(pk, stdin)
    assert pf.proof == O.prove(prog, stdin), name
    bp.verify(pf, vk)
    assert pf.public_values == client_output(prog, stdin)


def client_output(prog, stdin):
    return sdk.ProverClient().execute(prog, stdin).run()


def test_pk_to_device_refuses_a_wrong_commit():
    """pk_to_device with a commit that is not the traces' (a key from another program, one word
    changed) is refused: the device key is never silently re-made."""
    bp = sdk.BfProver()
    pk, vk = bp.setup(guests.HELLO)
    other, _ = bp.setup(guests.FIBO)
    for commit in ([vk.commit[0] ^ 1] + vk.commit[1:], other.pk.commit):
        bad = sdk.StarkProvingKey(commit=commit, traces=pk.pk.traces,
                                  chip_ordering=pk.pk.chip_ordering, local_only=pk.pk.local_only)
        with pytest.raises(_lib.BfzError, match="commitment mismatch"):
            sdk.CoreProver.pk_to_device(bad)
    dpk = sdk.CoreProver.pk_to_device(pk.pk)  # the right one is a cache hit of setup's key
    assert dpk.commit == vk.commit


def _record_proof(pk, rec, cycles=False, pinned=False):
    from bfz import events
    drec = (events.record_from_cycles(pk, events.cycles_from_record(rec, pinned=pinned), rec.memory)
            if cycles else events.record_from_events(pk, rec))
    return _prove_record(pk, drec)


def _prove_record(pk, drec):
    ptr = ctypes.POINTER(ctypes.c_uint8)()
    n = ctypes.c_size_t()
    _lib.check(_lib.lib().bfz_record_prove(ctypes.c_void_p(pk.handle), ctypes.c_void_p(drec.handle),
                                           ctypes.byref(ptr), ctypes.byref(n), None))
    return _lib.take_bytes(ptr, n.value)


@pytest.mark.parametrize("name,prog,stdin", guests.REFERENCE_PROGRAMS + [("fibo255", guests.FIBO, [255])])
def test_record_from_events_matches_oracle(client, name, prog, stdin):
    """bfz_record_from_events: the reference record's event vectors (Executor::run) in HBM,
    traces generated there; the proof is the oracle's.  The memory events may come in any order
    (the reference drains a HashMap, executor.rs:74): they are put in address order."""
    from bfz import events
    pk, vk = client.setup(prog)
    rec = events.ExecutionRecordArrays.from_executor(prog, stdin)
    want = O.prove(prog, stdin)
    assert _record_proof(pk, rec) == want, name
    if len(rec.memory) > 1:
        rec.memory = np.ascontiguousarray(rec.memory[::-1])
        assert _record_proof(pk, rec) == want, name


def test_record_from_events_sub_events_and_bad_events(client):
    """Sub events in sub_events (chained after add_events, alu/mod.rs:72) give a valid proof of
    the same execution; out-of-range events are refused before any kernel reads them, and the
    library keeps working."""
    from bfz import events
    prog, stdin = guests.FIBO, [17]
    pk, vk = client.setup(prog)
    rec = events.ExecutionRecordArrays.from_executor(prog, stdin)
    subs = rec.add["opcode"] == events.SUB
    split = events.ExecutionRecordArrays(**{**rec.__dict__, "add": np.ascontiguousarray(rec.add[~subs]),
                                            "sub": np.ascontiguousarray(rec.add[subs])})
    pf = _record_proof(pk, split)
    client.verify(sdk.BfProofWithPublicValues(proof=pf, stdin=bytes(stdin)), vk)
    for field, idx, val, msg in (("cpu", 7, ("pc", 10 ** 6), "out of range"),
                                 ("cpu", 0, ("mv_access_kind", 3), "out of range"),
                                 ("jump", 0, ("opcode", 2), "out of range"),
                                 ("memory", 1, ("addr", None), "two memory events")):
        bad = events.ExecutionRecordArrays(**{k: (v.copy() if isinstance(v, np.ndarray) else v)
                                              for k, v in rec.__dict__.items()})
        arr = getattr(bad, field)
        arr[idx][val[0]] = arr[0][val[0]] if val[1] is None else val[1]
        with pytest.raises(_lib.BfzError, match=msg):
            _record_proof(pk, bad)
    empty = events.ExecutionRecordArrays(**{**rec.__dict__, "cpu": rec.cpu[:0]})
    with pytest.raises(_lib.BfzError, match="no cpu events"):
        _record_proof(pk, empty)
    assert _record_proof(pk, rec) == O.prove(prog, stdin)


@pytest.mark.parametrize("prog,stdin", [(guests.FIBO, [17]), (guests.HELLO, []), ("+", [])])
def test_logup_perm_trace_matches_oracle(prog, stdin):
    """a7 standalone: generate_permutation_trace (permutation.rs:75-148) on the
    device == the oracle's, every included chip: the flattened EF trace (batched fractions and
    running sum, flatten_to_base) and the cumulative sum, for seeded random LogUp challenges;
    plus uniformly random main traces (every row a different denominator)."""
    rng = np.random.default_rng(33)
    for trial in range(2):
        alpha = [int(x) for x in rng.integers(0, P, 4)]
        beta = [int(x) for x in rng.integers(0, P, 4)]
        for chip in range(8):
            main = O.trace(prog, stdin, chip)
            if main is None:
                continue
            if trial:
                main = rng.integers(0, P, size=main.shape, dtype=np.uint64).astype(np.uint32)
            prep = O.trace(prog, stdin, chip, prep=True) if chip in (1, 5) else None
            exp, exp_cs = O.perm_trace(chip, main, prep, alpha, beta)
            out = ctypes.POINTER(ctypes.c_uint32)()
            w = ctypes.c_size_t()
            cs = (ctypes.c_uint32 * 4)()
            m_dev = mont(main).copy()
            p_dev = mont(prep).copy() if prep is not None else None
            _lib.check(_lib.lib().bfz_perm_trace(
                chip, m_dev.ctypes.data_as(P32), p_dev.ctypes.data_as(P32) if p_dev is not None else None,
                main.shape[0], (ctypes.c_uint32 * 4)(*mont(alpha)), (ctypes.c_uint32 * 4)(*mont(beta)),
                ctypes.byref(out), ctypes.byref(w), cs))
            got = np.ctypeslib.as_array(out, shape=(main.shape[0] * w.value,)).copy()
            _lib.lib().bfz_free(out)
            assert np.array_equal(unmont(got).reshape(exp.shape), exp), (prog, chip, trial)
            assert unmont(list(cs)).tolist() == exp_cs, (prog, chip, trial)


def test_device_transcript_divergence_is_an_error(client, monkeypatch):
    """the LogUp alpha/beta, the quotient alpha, the FRI betas, the PoW check
    and the query indices are sampled on the device and replayed by the host.  A device sponge
    that is not the host's (fault injected into its uploaded state) must fail the proof with an
    error naming the divergence -- not return a proof the verifier rejects -- and the library
    must keep working afterwards."""
    prog, stdin = guests.FIBO, [17]
    pk, vk = client.setup(prog)
    _lib.check(_lib.lib().bfz_set_fault_injection(1))
    try:
        with pytest.raises(_lib.BfzError, match="device transcript diverged"):
            client.prove(pk, stdin).run()
    finally:
        _lib.check(_lib.lib().bfz_set_fault_injection(0))
    pf = client.prove(pk, stdin).run()
    assert pf.proof == O.prove(prog, stdin)


@pytest.mark.parametrize("name,prog,stdin", guests.REFERENCE_PROGRAMS + [("fibo255", guests.FIBO, [255])])
def test_record_from_cycles_matches_oracle(client, name, prog, stdin):
    """bfz_record_from_cycles: 16 B per cycle + the memory events; the device
    rebuilds every CpuEvent field and the add/jump/memory_instr/io events (executor.rs:108-239)
    and the proof is the oracle's -- also with the memory events in reverse order, and with the
    cycles in page-locked bfz_host_alloc memory (one DMA, no staging)."""
    from bfz import events
    pk, vk = client.setup(prog)
    rec = events.ExecutionRecordArrays.from_executor(prog, stdin)
    want = O.prove(prog, stdin)
    assert _record_proof(pk, rec, cycles=True) == want, name
    assert _record_proof(pk, rec, cycles=True, pinned=True) == want, name
    if len(rec.memory) > 1:
        rec.memory = np.ascontiguousarray(rec.memory[::-1])
        assert _record_proof(pk, rec, cycles=True) == want, name


@pytest.mark.parametrize("name,prog,stdin", guests.REFERENCE_PROGRAMS[:5] + [("fibo255", guests.FIBO, [255])])
def test_chunked_cycle_handover_matches_oracle(client, name, prog, stdin):
    """bfz_cycles_begin / push / finish: the cycles pushed in chunks (any
    order; chunk sizes 1 cycle, 7 cycles, a third of the run) give the oracle's proof, and so does
    the compiled stand-in of CycleArrays::new pushing chunks from its worker threads."""
    from bfz import events
    pk, vk = client.setup(prog)
    rec = events.ExecutionRecordArrays.from_executor(prog, stdin)
    cyc = events.cycles_from_record(rec, pinned=True)
    want = O.prove(prog, stdin)
    chunks = [7, max(1, len(cyc) // 3)] + ([1] if len(cyc) < 5000 else [])
    for ch in chunks:
        drec = events.record_from_cycle_chunks(pk, cyc, rec.memory, ch)
        assert _prove_record(pk, drec) == want, (name, ch)
    sa = events.CycleArraysStandin()
    out = events.pinned_empty(len(cyc), events.CYCLE)
    drec, _ = sa.handover(pk, events.rust_cpu_events(rec), rec.memory, out, 4, 1000)
    assert _prove_record(pk, drec) == want, name


def test_chunked_cycle_handover_refuses_gaps_and_overlaps(client):
    """A chunk outside the announced count, a missing cycle or one pushed twice is an error
    (the handle is consumed), and the library keeps working."""
    from bfz import events
    prog, stdin = guests.FIBO, [17]
    pk, vk = client.setup(prog)
    rec = events.ExecutionRecordArrays.from_executor(prog, stdin)
    cyc = events.cycles_from_record(rec)
    L = _lib.lib()
    n = len(cyc)
    base = cyc.ctypes.data
    for pushes, match in (([(0, n - 1)], "missing"), ([(0, n), (5, 3)], "twice"),
                          ([(0, 10), (20, n - 20)], "missing")):
        up = ctypes.c_void_p()
        _lib.check(L.bfz_cycles_begin(ctypes.c_void_p(pk.handle), n, ctypes.byref(up)))
        for a, k in pushes:
            _lib.check(L.bfz_cycles_push(up, a, base + 16 * a, k))
        out = ctypes.c_void_p()
        with pytest.raises(_lib.BfzError, match=match):
            _lib.check(L.bfz_cycles_finish(up, rec.memory.ctypes.data, len(rec.memory), ctypes.byref(out)))
    up = ctypes.c_void_p()
    _lib.check(L.bfz_cycles_begin(ctypes.c_void_p(pk.handle), n, ctypes.byref(up)))
    with pytest.raises(_lib.BfzError, match="outside"):
        _lib.check(L.bfz_cycles_push(up, n - 2, base, 3))
    L.bfz_cycles_abort(up)
    drec = events.record_from_cycle_chunks(pk, cyc, rec.memory, 100)
    assert _prove_record(pk, drec) == O.prove(prog, stdin)


def test_record_from_cycles_refuses_cycles_no_record_holds(client):
    """Cycles a reference record cannot hold are refused before any trace kernel runs (pc past
    the program, an access on a memory step, a previous timestamp at or after the cycle's own,
    a prev_value outside an Input, padding, a successor the executor would not step to), and the
    library keeps working."""
    from bfz import events
    prog, stdin = guests.FIBO, [17]
    pk, vk = client.setup(prog)
    rec = events.ExecutionRecordArrays.from_executor(prog, stdin)
    cyc = events.cycles_from_record(rec)
    ops = np.array([{"[": 0, "]": 1, "+": 2, "-": 3, ">": 4, "<": 5, ",": 6, ".": 7}[ch]
                    for ch in prog if ch in "[]+-><,."])
    op = ops[cyc["pc"]]
    mem_step = int(np.flatnonzero((op == 4) | (op == 5))[0])
    alu = int(np.flatnonzero((op == 2) | (op == 3))[3])
    for idx, field, val in ((5, "pc", len(ops)), (mem_step, "mv", 1), (mem_step, "prev_ts", 1),
                            (alu, "prev_ts", 2 * alu + 1), (alu, "prev_value", 9)):
        bad = cyc.copy()
        bad[idx][field] = val
        with pytest.raises(_lib.BfzError, match="out of range"):
            events.record_from_cycles(pk, bad, rec.memory)
    # a cycle's successor must be the executor's next step (executor.rs:107-176): pc + 1 after a
    # non-jump, op_a or pc + 1 after a loop as mv chooses, mp unchanged off a memory step, and
    # the last cycle must leave the program (a truncated record is refused)
    jmp = int(np.flatnonzero((op == 0) | (op == 1))[2])
    for idx, field, val in ((alu + 1, "pc", int(cyc[alu]["pc"])), (jmp, "mv", 1 - min(int(cyc[jmp]["mv"]), 1)),
                            (alu + 1, "mp", int(cyc[alu]["mp"]) + 1)):
        bad = cyc.copy()
        bad[idx][field] = val
        with pytest.raises(_lib.BfzError, match="out of range"):
            events.record_from_cycles(pk, bad, rec.memory)
    with pytest.raises(_lib.BfzError, match="out of range"):
        events.record_from_cycles(pk, cyc[:-1].copy(), rec.memory)
    raw = cyc.view(np.uint8).reshape(len(cyc), 16).copy()
    raw[3, 15] = 1
    with pytest.raises(_lib.BfzError, match="out of range"):
        events.record_from_cycles(pk, raw.view(events.CYCLE).reshape(-1), rec.memory)
    with pytest.raises(_lib.BfzError, match="no cycles"):
        events.record_from_cycles(pk, cyc[:0], rec.memory)
    assert _record_proof(pk, rec, cycles=True) == O.prove(prog, stdin)


def test_first_proof_of_a_fresh_process_costs_a_warm_proof():
    """a fresh process (init, setup, record, one prove -- what a
    ProverClient::prove().run() process does) proves the headline workload in about the time of
    a warm proof: no table is built between the first proof's launches (twiddles on the device in
    setup, coset-power and selector tables when the record is created).  scripts/cold_first_proof.py
    in a child process; bench.py reports the same figure as cold_first_proof_ms."""
    import subprocess
    import sys
    out = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "cold_first_proof.py"),
                          "--warm", "2"], capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    r = json.loads(out.stdout.strip().splitlines()[-1])
    assert r["cycles"] == 3767729
    assert r["first_prove_ms"] <= 1.5 * min(r["warm_prove_ms"]), r
