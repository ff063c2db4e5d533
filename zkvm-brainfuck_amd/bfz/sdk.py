"""Python mirror of the reference SDK (crates/sdk/src/lib.rs, action.rs, proof.rs) over the
bfz C ABI.  Same names, argument meaning and error behaviour:

    client = ProverClient()                      # ProverClient::new        lib.rs:31-33
    out = client.execute(elf, stdin).run()       # ProverClient::execute    lib.rs:57-59
    pk, vk = client.setup(elf)                   # ProverClient::setup      lib.rs:133-135
    proof = client.prove(pk, stdin).run()        # ProverClient::prove      lib.rs:92-94
    client.verify(proof, vk)                     # ProverClient::verify     lib.rs:110-116

and of the core MachineProver boundary (crates/stark/src/prover.rs:27-150):

    traces = generate_traces(elf, stdin)         # generate_traces          prover.rs:58-81
    prover = CoreProver()
    data = prover.commit(pk, traces)             # MachineProver::commit    prover.rs:209-236
    ch = prover.new_challenger()
    prover.observe_into(pk, ch)                  # pk.observe_into          prover.rs:595-601
    proof = prover.open(pk, data, ch)            # MachineProver::open      prover.rs:242-553
    proof = prover.prove(pk, traces)             # MachineProver::prove     prover.rs:560-582

Errors raise (the reference returns Err / panics in the same places).  Proving runs on the GPU
through libbfz; verification runs the host verifier compiled into the same library.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field
from typing import List, Optional

from . import _lib
from ._lib import BfzError, Challenger, check, init, lib, take_bytes, u8buf


@dataclass
class BfVerifyingKey:
    """StarkVerifyingKey: preprocessed commitment (Montgomery u32 x 8) + the program that
    determines chip_information (crates/prover/src/types.rs:17-20)."""
    commit: List[int]
    elf: str


@dataclass
class BfProvingKey:
    """BfProvingKey (crates/prover/src/types.rs:8-15): device-resident pk + elf + vk."""
    handle: int
    elf: str
    vk: BfVerifyingKey

    def __del__(self):
        try:
            if self.handle:
                lib().bfz_pk_free(ctypes.c_void_p(self.handle))
                self.handle = 0
        except Exception:
            pass


# KoalaBear word representation inside bincode (bfz_proof_to_bincode): the p3 MontyField31
# serde writes the Montgomery word [p3-recalled]; CANONICAL is the alternative.
FIELD_MONTGOMERY, FIELD_CANONICAL = 0, 1


def proof_to_bincode(proof: bytes, field_repr: int = FIELD_MONTGOMERY) -> bytes:
    """BFZ1 normal form -> bincode::serialize(&ShardProof<KoalaBearPoseidon2>) bytes
    (crates/stark/src/types.rs:66-73, crates/core/machine/src/utils/prove.rs:46)."""
    buf, n = u8buf(proof)
    ptr = ctypes.POINTER(ctypes.c_uint8)()
    olen = ctypes.c_size_t()
    check(lib().bfz_proof_to_bincode(buf, n, int(field_repr), ctypes.byref(ptr), ctypes.byref(olen)))
    return take_bytes(ptr, olen.value)


def proof_from_bincode(data: bytes, field_repr: int = FIELD_MONTGOMERY) -> bytes:
    """bincode ShardProof bytes -> BFZ1 normal form (chip_ordering applied)."""
    buf, n = u8buf(data)
    ptr = ctypes.POINTER(ctypes.c_uint8)()
    olen = ctypes.c_size_t()
    check(lib().bfz_proof_from_bincode(buf, n, int(field_repr), ctypes.byref(ptr),
                                       ctypes.byref(olen)))
    return take_bytes(ptr, olen.value)


@dataclass
class BfProofWithPublicValues:
    """crates/sdk/src/proof.rs:10-13 — the proof (BFZ1 normal-form bytes) and stdin.

    `to_bincode()` gives the reference's serialized form of this struct, bincode of
    { proof: ShardProof<CoreSC>, stdin: Vec<u8> }; `from_bincode()` reads it back."""
    proof: bytes
    stdin: bytes
    public_values: bytes = b""
    cycles: int = 0

    def to_bincode(self, field_repr: int = FIELD_MONTGOMERY) -> bytes:
        import struct
        return (proof_to_bincode(self.proof, field_repr) + struct.pack("<Q", len(self.stdin))
                + bytes(self.stdin))

    @staticmethod
    def from_bincode(data: bytes, field_repr: int = FIELD_MONTGOMERY) -> "BfProofWithPublicValues":
        import struct
        # the ShardProof is everything before the trailing Vec<u8> stdin; its length is found by
        # trying the stdin lengths the tail can hold (the u64 prefix sits right before stdin)
        for k in range(0, len(data) - 7):
            cut = len(data) - k - 8
            if cut < 0:
                break
            if struct.unpack_from("<Q", data, cut)[0] == k:
                try:
                    pf = proof_from_bincode(data[:cut], field_repr)
                except BfzError:
                    continue
                return BfProofWithPublicValues(proof=pf, stdin=bytes(data[cut + 8:]))
        raise BfzError("not a bincode BfProofWithPublicValues")


class Execute:
    """action::Execute (crates/sdk/src/action.rs:10-33)."""

    def __init__(self, elf: str, stdin: bytes):
        self.elf, self.stdin = elf, bytes(stdin)

    def run(self) -> bytes:
        buf, n = u8buf(self.stdin)
        cap = 1 << 20
        out = (ctypes.c_uint8 * cap)()
        olen = ctypes.c_size_t()
        cyc = ctypes.c_uint64()
        check(lib().bfz_execute(self.elf.encode(), buf, n, out, cap, ctypes.byref(olen),
                                ctypes.byref(cyc)))
        return bytes(out[: min(olen.value, cap)])


class Prove:
    """action::Prove (crates/sdk/src/action.rs:35-61)."""

    def __init__(self, pk: BfProvingKey, stdin: bytes):
        self.pk, self.stdin = pk, bytes(stdin)

    def run(self) -> BfProofWithPublicValues:
        init()
        buf, n = u8buf(self.stdin)
        ptr = ctypes.POINTER(ctypes.c_uint8)()
        plen = ctypes.c_size_t()
        check(lib().bfz_prove(ctypes.c_void_p(self.pk.handle), buf, n, ctypes.byref(ptr),
                              ctypes.byref(plen)))
        return BfProofWithPublicValues(proof=take_bytes(ptr, plen.value), stdin=self.stdin,
                                       public_values=Execute(self.pk.elf, self.stdin).run())


class ProverClient:
    """crates/sdk/src/lib.rs:20-136, backed by the MI355X prover."""

    def __init__(self, device: int = 0):
        self.device = device

    @staticmethod
    def new() -> "ProverClient":
        return ProverClient()

    def execute(self, elf: str, stdin) -> Execute:
        return Execute(elf, bytes(stdin))

    def setup(self, elf: str):
        init(self.device)
        h = ctypes.c_void_p()
        commit = (ctypes.c_uint32 * 8)()
        check(lib().bfz_setup(elf.encode(), ctypes.byref(h), commit))
        vk = BfVerifyingKey(commit=list(commit), elf=elf)
        return BfProvingKey(handle=h.value, elf=elf, vk=vk), vk

    def prove(self, pk: BfProvingKey, stdin) -> Prove:
        return Prove(pk, bytes(stdin))

    def prove_batch(self, pk: BfProvingKey, stdins, exec_threads: int = 0,
                    public_values: bool = True, stats: Optional[dict] = None):
        """Proofs of pk's program over many inputs, pipelined (bfz_prove_batch): executions run
        on host threads and uploads on a copy stream while the GPU proves the previous job.
        Each proof equals prove(pk, stdin).run()'s; stats (a dict) receives the batch timings."""
        init(self.device)
        ins = [bytes(x) for x in stdins]
        k = len(ins)
        bufs = [u8buf(x) for x in ins]
        arr = (ctypes.POINTER(ctypes.c_uint8) * max(k, 1))(
            *[ctypes.cast(b, ctypes.POINTER(ctypes.c_uint8)) for b, _ in bufs])
        lens = (ctypes.c_size_t * max(k, 1))(*[n for _, n in bufs])
        outs = (ctypes.POINTER(ctypes.c_uint8) * max(k, 1))()
        olens = (ctypes.c_size_t * max(k, 1))()
        st = _lib.BatchStats()
        check(lib().bfz_prove_batch(ctypes.c_void_p(pk.handle), arr, lens, k, int(exec_threads),
                                    outs, olens, ctypes.byref(st)))
        proofs = [take_bytes(outs[i], olens[i]) for i in range(k)]
        if stats is not None:
            stats.update({name: getattr(st, name) for name, _ in st._fields_})
        return [BfProofWithPublicValues(
            proof=pf, stdin=x,
            public_values=Execute(pk.elf, x).run() if public_values else b"")
            for pf, x in zip(proofs, ins)]

    def verify(self, proof: BfProofWithPublicValues, vk: BfVerifyingKey) -> None:
        buf, n = u8buf(proof.proof)
        commit = (ctypes.c_uint32 * 8)(*vk.commit)
        check(lib().bfz_verify(vk.elf.encode(), commit, buf, n))

    def verify_bincode(self, shard_proof: bytes, vk: BfVerifyingKey,
                       field_repr: int = FIELD_MONTGOMERY) -> None:
        """StarkMachine::verify on the reference's bincode ShardProof bytes."""
        buf, n = u8buf(shard_proof)
        commit = (ctypes.c_uint32 * 8)(*vk.commit)
        check(lib().bfz_verify_bincode(vk.elf.encode(), commit, buf, n, int(field_repr)))


# BfAir::chips() order (crates/core/machine/src/brainfuck/mod.rs:53-81) = chip index in the ABI
CHIPS = ("Cpu", "Program", "AddSub", "Jump", "Memory", "Byte", "MemoryInstrs", "IO")


def generate_traces(elf: str, stdin) -> list:
    """Execute + generate_dependencies + generate_traces: [(chip index, name, trace)] for the
    chips the record includes, each trace a (height, width) uint32 array in Montgomery form
    (the byte layout of the reference's RowMajorMatrix<KoalaBear>)."""
    import numpy as np
    buf, n = u8buf(bytes(stdin))
    out = []
    for c, name in enumerate(CHIPS):
        p = ctypes.POINTER(ctypes.c_uint32)()
        h, w = ctypes.c_size_t(), ctypes.c_size_t()
        rc = lib().bfz_trace(elf.encode(), buf, n, c, 0, ctypes.byref(p), ctypes.byref(h),
                             ctypes.byref(w))
        if rc == 1:
            continue
        check(rc)
        arr = np.ctypeslib.as_array(p, shape=(h.value * w.value,)).copy()
        lib().bfz_free(p)
        out.append((c, name, arr.reshape(h.value, w.value)))
    return out


def _trace_args(traces):
    import numpy as np
    mats = [np.ascontiguousarray(t, dtype=np.uint32) for _, _, t in traces]
    k = len(mats)
    chips = (ctypes.c_int * k)(*[c for c, _, _ in traces])
    ptrs = (ctypes.POINTER(ctypes.c_uint32) * k)(
        *[m.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)) for m in mats])
    hs = (ctypes.c_size_t * k)(*[m.shape[0] for m in mats])
    ws = (ctypes.c_size_t * k)(*[m.shape[1] for m in mats])
    return mats, chips, ptrs, hs, ws, k


class ShardMainData:
    """ShardMainData (crates/stark/src/types.rs:13-18) held in HBM by libbfz: the main traces'
    evaluations, LDEs and Merkle tree; main_commit is its root (8 Montgomery words)."""

    def __init__(self, handle: int, main_commit):
        self.handle = handle
        self.main_commit = list(main_commit)

    def __del__(self):
        if getattr(self, "handle", None):
            lib().bfz_main_data_free(ctypes.c_void_p(self.handle))
            self.handle = None


class CoreProver:
    """HIP implementation of the MachineProver trait (crates/stark/src/prover.rs:27-150) from
    host traces: `commit` (:209-236), `observe_into` (MachineProvingKey, :595-601), `open`
    (:242-553) and the default `prove` (:560-582) = commit + open on a clone of the
    challenger.  Every step runs on the device; the challenger is plain data (Challenger)."""

    def commit(self, pk: BfProvingKey, traces) -> ShardMainData:
        init()
        mats, chips, ptrs, hs, ws, k = _trace_args(traces)
        out = ctypes.c_void_p()
        root = (ctypes.c_uint32 * 8)()
        check(lib().bfz_main_commit(ctypes.c_void_p(pk.handle), chips, ptrs, hs, ws, k,
                                    ctypes.byref(out), root))
        return ShardMainData(out.value, root)

    def commit_record(self, pk: BfProvingKey, record_handle: int) -> ShardMainData:
        """commit from a device-resident record (bfz_record_new): traces generated on device."""
        init()
        out = ctypes.c_void_p()
        root = (ctypes.c_uint32 * 8)()
        check(lib().bfz_record_main_commit(ctypes.c_void_p(pk.handle),
                                           ctypes.c_void_p(record_handle), ctypes.byref(out), root))
        return ShardMainData(out.value, root)

    @staticmethod
    def new_challenger() -> Challenger:
        return Challenger()  # DuplexChallenger::new: all zero, empty buffers

    def observe_into(self, pk: BfProvingKey, ch: Challenger) -> None:
        check(lib().bfz_challenger_observe_pk(ctypes.c_void_p(pk.handle), ctypes.byref(ch)))

    def open(self, pk: BfProvingKey, data: ShardMainData, ch: Challenger) -> bytes:
        ptr = ctypes.POINTER(ctypes.c_uint8)()
        plen = ctypes.c_size_t()
        check(lib().bfz_open(ctypes.c_void_p(pk.handle), ctypes.c_void_p(data.handle),
                             ctypes.byref(ch), ctypes.byref(ptr), ctypes.byref(plen)))
        return take_bytes(ptr, plen.value)

    def prove(self, pk: BfProvingKey, traces) -> bytes:
        """One call (bfz_prove_traces): same bytes as commit + observe_into + open."""
        init()
        mats, chips, ptrs, hs, ws, k = _trace_args(traces)
        ptr = ctypes.POINTER(ctypes.c_uint8)()
        plen = ctypes.c_size_t()
        check(lib().bfz_prove_traces(ctypes.c_void_p(pk.handle), chips, ptrs, hs, ws, k,
                                     ctypes.byref(ptr), ctypes.byref(plen)))
        return take_bytes(ptr, plen.value)


@dataclass
class StarkProvingKey:
    """StarkProvingKey on the host (crates/stark/src/machine.rs:49-60) as pk_to_host returns it:
    the preprocessed commit and traces in the key's order (sorted (Reverse(height), name),
    machine.rs:182-183), chip_ordering and local_only.  traces: [(chip id, name, array)] with
    each array the row-major Montgomery matrix (RowMajorMatrix<KoalaBear>::values)."""
    commit: List[int]
    traces: list
    chip_ordering: dict
    local_only: list


class DeviceProvingKey:
    """MachineProver::DeviceProvingKey made by pk_to_device (a bfz_pk handle, freed on drop)."""

    def __init__(self, handle: int, commit):
        self.handle = handle
        self.commit = list(commit)

    def __del__(self):
        if getattr(self, "handle", None):
            lib().bfz_pk_free(ctypes.c_void_p(self.handle))
            self.handle = None


# local_only per chip (Chip::local_only; the preprocessed chips Program and Byte are not)
_LOCAL_ONLY = {"Cpu": False, "Program": False, "AddSub": True, "Jump": True, "Memory": False,
               "Byte": False, "MemoryInstrs": False, "IO": True}


def _pk_to_host(pk) -> StarkProvingKey:
    import numpy as np
    commit = (ctypes.c_uint32 * 8)()
    check(lib().bfz_pk_commit(ctypes.c_void_p(pk.handle), commit))
    named = []
    for c, name in enumerate(CHIPS):
        p = ctypes.POINTER(ctypes.c_uint32)()
        h, w = ctypes.c_size_t(), ctypes.c_size_t()
        buf, n = u8buf(b"")
        rc = lib().bfz_trace(pk.elf.encode(), buf, n, c, 1, ctypes.byref(p), ctypes.byref(h),
                             ctypes.byref(w))
        if rc == 1:
            continue
        check(rc)
        arr = np.ctypeslib.as_array(p, shape=(h.value * w.value,)).copy().reshape(h.value, w.value)
        lib().bfz_free(p)
        named.append((c, name, arr))
    named.sort(key=lambda t: (-t[2].shape[0], t[1]))  # machine.rs:182-183
    return StarkProvingKey(commit=list(commit), traces=named,
                           chip_ordering={name: i for i, (_, name, _) in enumerate(named)},
                           local_only=[_LOCAL_ONLY[name] for _, name, _ in named])


def _pk_to_device(hpk: StarkProvingKey) -> DeviceProvingKey:
    mats, chips, ptrs, hs, ws, k = _trace_args(hpk.traces)
    commit = (ctypes.c_uint32 * 8)(*hpk.commit)
    out = ctypes.c_void_p()
    check(lib().bfz_pk_from_host(chips, ptrs, hs, ws, k, commit, ctypes.byref(out)))
    return DeviceProvingKey(out.value, hpk.commit)


CoreProver.pk_to_host = staticmethod(_pk_to_host)
CoreProver.pk_to_host.__doc__ = "MachineProver::pk_to_host (prover.rs:55,205-207)."
CoreProver.pk_to_device = staticmethod(_pk_to_device)
CoreProver.pk_to_device.__doc__ = ("MachineProver::pk_to_device (prover.rs:52,201-203) -> "
                                   "bfz_pk_from_host: refuses traces or a commit that do not match.")


@dataclass
class HostBfProvingKey:
    """BfProvingKey (crates/prover/src/types.rs:8-15) exactly as BfProver::setup builds it:
    the HOST key pk_to_host(pk), the elf and the vk (crates/prover/src/lib.rs:46-56)."""
    pk: StarkProvingKey
    elf: str
    vk: BfVerifyingKey


class BfProver:
    """BfProver<HipProverComponents> (crates/prover/src/lib.rs:28-90) -- the reference's own
    flow around the HIP core prover:
      setup: MachineProver::setup, keep pk_to_host(pk)                       (lib.rs:46-56)
      prove: pk_to_device(pk.pk) every time, Executor::run, then the HipProver::prove override:
             observe_into, bfz_record_from_events (the record's events to HBM, traces and
             byte-lookup multiplicities generated there), commit, open on a clone (lib.rs:70-90,
             utils/prove.rs:23-66, prover.rs:560-582)."""

    def __init__(self):
        self.core = CoreProver()

    def setup(self, elf: str):
        init()
        h = ctypes.c_void_p()
        commit = (ctypes.c_uint32 * 8)()
        check(lib().bfz_setup(elf.encode(), ctypes.byref(h), commit))
        vk = BfVerifyingKey(commit=list(commit), elf=elf)
        dpk = BfProvingKey(handle=h.value, elf=elf, vk=vk)
        pk = HostBfProvingKey(pk=self.core.pk_to_host(dpk), elf=elf, vk=vk)
        del dpk  # the device key is dropped, as the reference keeps only the host key
        return pk, vk

    def prove(self, pk: HostBfProvingKey, stdin) -> BfProofWithPublicValues:
        from .events import ExecutionRecordArrays, record_from_events
        dpk = self.core.pk_to_device(pk.pk)                         # lib.rs:76
        rec = ExecutionRecordArrays.from_executor(pk.elf, stdin)    # Executor::run
        ch = self.core.new_challenger()                             # config().challenger()
        self.core.observe_into(dpk, ch)                             # prover.rs:572
        drec = record_from_events(dpk, rec)
        data = self.core.commit_record(dpk, drec.handle)
        opened = Challenger.from_buffer_copy(bytes(ch))             # challenger.clone()
        proof = self.core.open(dpk, data, opened)                   # prover.rs:578
        return BfProofWithPublicValues(proof=proof, stdin=bytes(stdin), public_values=rec.output,
                                       cycles=rec.global_clk)

    def verify(self, proof: BfProofWithPublicValues, vk: BfVerifyingKey) -> None:
        ProverClient().verify(proof, vk)


def set_num_queries(q: int) -> None:
    """FRI_QUERIES override (crates/stark/src/kb31_poseidon2.rs:59-62); 0 = environment/84."""
    check(lib().bfz_set_num_queries(int(q)))


def set_pcs_variant(observe_openings: int) -> None:
    """Decision D1: 1 = opened values observed before FRI alpha (default),
    0 = alpha sampled first, -1 = environment BFZ_OBSERVE_OPENINGS."""
    check(lib().bfz_set_pcs_variant(int(observe_openings)))
