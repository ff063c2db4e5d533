"""The reference's ExecutionRecord events (crates/core/executor/src/record.rs:15-34,
events/*.rs) as numpy structured arrays laid out exactly like the bfz_*_event structs of
include/bfz.h, and their hand-over to the device (bfz_record_from_events).

    rec = ExecutionRecordArrays.from_executor(elf, stdin)   # Executor::run's events
    handle = record_from_events(pk, rec)                     # -> bfz_record (HBM)

`from_executor` parses the field-by-field event stream of bfz_execute_events (the executor a
Rust caller would have run: `Executor::run`, executor.rs:71-79); a Rust HipProver fills the
same structs from `record.cpu_events`, `record.add_events`, ... directly.
"""
from __future__ import annotations

import ctypes
import struct
from dataclasses import dataclass

import numpy as np

from . import _lib
from ._lib import check, lib, u8buf


def _dt(fields, itemsize):
    names, formats, offsets = zip(*fields)
    return np.dtype({"names": list(names), "formats": list(formats), "offsets": list(offsets),
                     "itemsize": itemsize})


# bfz.h layouts (explicit padding; tests/test_abi.py checks them against the header)
ACCESS = [("kind", "u1", 0), ("value", "u1", 1), ("prev_value", "u1", 2), ("timestamp", "<u4", 4),
          ("prev_timestamp", "<u4", 8)]
CPU = _dt([("clk", "<u4", 0), ("pc", "<u4", 4), ("next_pc", "<u4", 8), ("mp", "<u4", 12),
           ("next_mp", "<u4", 16), ("mv", "u1", 20), ("next_mv", "u1", 21)]
          + [("mv_access_" + n, f, 24 + o) for n, f, o in ACCESS]
          + [("next_mv_access_" + n, f, 36 + o) for n, f, o in ACCESS], 48)
ALU = _dt([("pc", "<u4", 0), ("opcode", "u1", 4), ("next_mv", "u1", 5), ("mv", "u1", 6)], 8)
JUMP = _dt([("pc", "<u4", 0), ("next_pc", "<u4", 4), ("opcode", "u1", 8), ("dst", "<u4", 12),
            ("mv", "u1", 16)], 20)
MEM_INSTR = _dt([("clk", "<u4", 0), ("pc", "<u4", 4), ("opcode", "u1", 8), ("mp", "<u4", 12),
                 ("next_mp", "<u4", 16)], 20)
IO = _dt([("pc", "<u4", 0), ("opcode", "u1", 4), ("mp", "<u4", 8), ("mv", "u1", 12)], 16)
MEMORY = _dt([("addr", "<u4", 0), ("initial_timestamp", "<u4", 4), ("final_timestamp", "<u4", 8),
              ("initial_value", "u1", 12), ("final_value", "u1", 13)], 16)

# bfz_cycle: the compact hand-over of bfz_record_from_cycles (16 B per cycle)
CYCLE = _dt([("pc", "<u4", 0), ("mp", "<u4", 4), ("prev_ts", "<u4", 8), ("mv", "u1", 12),
             ("prev_value", "u1", 13)], 16)

# bfz_execute_events stream: the same fields packed (no padding), in declaration order
_P_ACCESS = [("kind", "u1"), ("value", "u1"), ("prev_value", "u1"), ("timestamp", "<u4"),
             ("prev_timestamp", "<u4")]
_PACKED = {
    "cpu": np.dtype([("clk", "<u4"), ("pc", "<u4"), ("next_pc", "<u4"), ("mp", "<u4"),
                     ("next_mp", "<u4"), ("mv", "u1"), ("next_mv", "u1")]
                    + [("mv_access_" + n, f) for n, f in _P_ACCESS]
                    + [("next_mv_access_" + n, f) for n, f in _P_ACCESS]),
    "alu": np.dtype([("pc", "<u4"), ("opcode", "u1"), ("next_mv", "u1"), ("mv", "u1")]),
    "jump": np.dtype([("pc", "<u4"), ("next_pc", "<u4"), ("opcode", "u1"), ("dst", "<u4"),
                      ("mv", "u1")]),
    "memory_instr": np.dtype([("clk", "<u4"), ("pc", "<u4"), ("opcode", "u1"), ("mp", "<u4"),
                              ("next_mp", "<u4")]),
    "io": np.dtype([("pc", "<u4"), ("opcode", "u1"), ("mp", "<u4"), ("mv", "u1")]),
    "memory": np.dtype([("addr", "<u4"), ("initial_timestamp", "<u4"), ("final_timestamp", "<u4"),
                        ("initial_value", "u1"), ("final_value", "u1")]),
}
_ALIGNED = {"cpu": CPU, "alu": ALU, "jump": JUMP, "memory_instr": MEM_INSTR, "io": IO,
            "memory": MEMORY}
# Opcode discriminants (crates/core/executor/src/opcode.rs:13-30)
ADD, SUB = 2, 3


def _aligned(packed: np.ndarray, dt: np.dtype) -> np.ndarray:
    out = np.zeros(len(packed), dtype=dt)
    for name in packed.dtype.names:
        out[name] = packed[name]
    return out


@dataclass
class ExecutionRecordArrays:
    """ExecutionRecord's event vectors (record.rs:15-34) in the bfz_events layout."""
    cpu: np.ndarray
    add: np.ndarray
    sub: np.ndarray
    jump: np.ndarray
    io: np.ndarray
    memory_instr: np.ndarray
    memory: np.ndarray  # cpu_memory_access, any order
    global_clk: int = 0
    output: bytes = b""

    @staticmethod
    def from_executor(elf: str, stdin, executor: int = 0) -> "ExecutionRecordArrays":
        """Executor::run (executor.rs:71-79) on (elf, stdin): every ALU event is an add_event
        (the reference executor pushes Add and Sub alike to add_events, executor.rs:219-226)."""
        buf, n = u8buf(bytes(stdin))
        p = ctypes.POINTER(ctypes.c_uint8)()
        ln = ctypes.c_size_t()
        check(lib().bfz_execute_events(elf.encode(), buf, n, int(executor), ctypes.byref(p),
                                       ctypes.byref(ln)))
        blob = _lib.take_bytes(p, ln.value)
        off = 0
        arrs = {}
        for key in ("cpu", "alu", "jump", "memory_instr", "io", "memory"):
            cnt = struct.unpack_from("<Q", blob, off)[0]
            off += 8
            dt = _PACKED[key]
            packed = np.frombuffer(blob, dtype=dt, count=cnt, offset=off)
            off += cnt * dt.itemsize
            arrs[key] = _aligned(packed, _ALIGNED[key])
        gclk = struct.unpack_from("<Q", blob, off)[0]
        off += 8 + 8  # global_clk, pc, mp
        nout = struct.unpack_from("<Q", blob, off)[0]
        out = bytes(blob[off + 8: off + 8 + nout])
        return ExecutionRecordArrays(cpu=arrs["cpu"], add=arrs["alu"],
                                     sub=np.zeros(0, dtype=ALU), jump=arrs["jump"], io=arrs["io"],
                                     memory_instr=arrs["memory_instr"], memory=arrs["memory"],
                                     global_clk=gclk, output=out)

    def as_c(self) -> "_lib.Events":
        ev = _lib.Events()
        for name in ("cpu", "add", "sub", "jump", "io", "memory_instr", "memory"):
            a = getattr(self, name)
            assert a.dtype == {"add": ALU, "sub": ALU}.get(name, _ALIGNED.get(name)), name
            assert a.flags["C_CONTIGUOUS"], name
            setattr(ev, name, a.ctypes.data if len(a) else None)
            setattr(ev, "n_" + name, len(a))
        return ev


INPUT = 6  # Opcode::Input (the only cycle whose mv_access is a write)


class _PinnedBuffer:
    """bfz_host_alloc memory (page-locked), freed with bfz_host_free when the last array view of
    it goes away."""

    def __init__(self, nbytes: int):
        _lib.init()
        p = ctypes.c_void_p()
        check(lib().bfz_host_alloc(max(int(nbytes), 1), ctypes.byref(p)))
        self.ptr = p.value

    def __del__(self):
        if getattr(self, "ptr", None):
            lib().bfz_host_free(ctypes.c_void_p(self.ptr))
            self.ptr = None


class PinnedArray(np.ndarray):
    """A numpy array over bfz_host_alloc memory (keeps the allocation alive, views included)."""

    def __array_finalize__(self, obj):
        self._owner = getattr(obj, "_owner", None)


def pinned_empty(n: int, dtype) -> PinnedArray:
    """An uninitialised array of n elements in page-locked host memory: bfz_record_from_cycles
    DMAs straight from it (what the Rust CycleArrays does through bfz_host_alloc)."""
    dtype = np.dtype(dtype)
    buf = _PinnedBuffer(n * dtype.itemsize)
    raw = (ctypes.c_uint8 * max(n * dtype.itemsize, 1)).from_address(buf.ptr)
    arr = np.frombuffer(raw, dtype=dtype, count=n).view(PinnedArray)
    arr._owner = buf
    return arr


def cycles_from_record(rec: "ExecutionRecordArrays", pinned: bool = False) -> np.ndarray:
    """The compact hand-over of bfz_record_from_cycles built from the record's cpu_events -- what
    the Rust HipProver's CycleArrays::new does over record.cpu_events: pc, mp, mv, the
    mv_access's prev_timestamp (0 when it is None) and, for a write (Input), its prev_value.
    Everything else in the record is rebuilt on the device.  pinned: build it in bfz_host_alloc
    memory (the upload is then one DMA, no staging copy)."""
    cpu = rec.cpu
    out = pinned_empty(len(cpu), CYCLE) if pinned else np.empty(len(cpu), dtype=CYCLE)
    out["pc"] = cpu["pc"]
    out["mp"] = cpu["mp"]
    out["prev_ts"] = cpu["mv_access_prev_timestamp"]
    out["mv"] = cpu["mv"]
    write = cpu["mv_access_kind"] == 2
    out["prev_value"] = np.where(write, cpu["mv_access_prev_value"], 0)
    out.view(np.uint8).reshape(-1, 16)[:, 14:16] = 0  # padding
    return out


class DeviceRecord:
    """bfz_record: the events resident in HBM (freed on drop)."""

    def __init__(self, handle: int):
        self.handle = handle

    def __del__(self):
        if getattr(self, "handle", None):
            lib().bfz_record_free(ctypes.c_void_p(self.handle))
            self.handle = None


def record_from_events(pk, rec: ExecutionRecordArrays) -> DeviceRecord:
    """bfz_record_from_events: the record utils::prove hands to MachineProver::prove, on the
    device (memory events put in address order; events validated)."""
    _lib.init()
    c = rec.as_c()
    out = ctypes.c_void_p()
    check(lib().bfz_record_from_events(ctypes.c_void_p(pk.handle), ctypes.byref(c),
                                       ctypes.byref(out)))
    return DeviceRecord(out.value)


def record_from_cycles(pk, cycles: np.ndarray, memory: np.ndarray) -> DeviceRecord:
    """bfz_record_from_cycles: the compact per-cycle hand-over (16 B per cycle) + the memory
    events; the device rebuilds the CpuEvents and every chip's events, then validates them."""
    _lib.init()
    assert cycles.dtype == CYCLE and cycles.flags["C_CONTIGUOUS"]
    assert memory.dtype == MEMORY and memory.flags["C_CONTIGUOUS"]
    out = ctypes.c_void_p()
    check(lib().bfz_record_from_cycles(ctypes.c_void_p(pk.handle),
                                       cycles.ctypes.data if len(cycles) else None, len(cycles),
                                       memory.ctypes.data if len(memory) else None, len(memory),
                                       ctypes.byref(out)))
    return DeviceRecord(out.value)


def record_from_cycle_chunks(pk, cycles: np.ndarray, memory: np.ndarray, chunk: int) -> DeviceRecord:
    """The chunked hand-over (bfz_cycles_begin / push / finish) of the same cycles, `chunk`
    cycles per push: the record (and proof) must equal bfz_record_from_cycles'."""
    _lib.init()
    assert cycles.dtype == CYCLE and cycles.flags["C_CONTIGUOUS"]
    assert memory.dtype == MEMORY and memory.flags["C_CONTIGUOUS"]
    L = lib()
    up = ctypes.c_void_p()
    check(L.bfz_cycles_begin(ctypes.c_void_p(pk.handle), len(cycles), ctypes.byref(up)))
    try:
        # pushed last chunk first: the library accepts any order
        starts = list(range(0, len(cycles), chunk))[::-1]
        for a in starts:
            n = min(chunk, len(cycles) - a)
            check(L.bfz_cycles_push(up, a, cycles.ctypes.data + a * CYCLE.itemsize, n))
    except BaseException:
        L.bfz_cycles_abort(up)
        raise
    out = ctypes.c_void_p()
    check(L.bfz_cycles_finish(up, memory.ctypes.data if len(memory) else None, len(memory),
                              ctypes.byref(out)))
    return DeviceRecord(out.value)


# Vec<CpuEvent> as rustc lays it out (repr(Rust): the u32 fields, the two 12-byte
# Option<MemoryRecordEnum> -- tag 0 Read, 1 Write, 2 None in the niche -- then mv, next_mv):
# the input of the compiled stand-in of CycleArrays::new (crates/bf-hip-prover/standin).
_RS_ACCESS = [("tag", "u1", 0), ("value", "u1", 1), ("prev_value", "u1", 2),
              ("timestamp", "<u4", 4), ("prev_timestamp", "<u4", 8)]
RUST_CPU = _dt([("clk", "<u4", 0), ("pc", "<u4", 4), ("next_pc", "<u4", 8), ("mp", "<u4", 12),
                ("next_mp", "<u4", 16)]
               + [("mv_access_" + n, f, 20 + o) for n, f, o in _RS_ACCESS]
               + [("next_mv_access_" + n, f, 32 + o) for n, f, o in _RS_ACCESS]
               + [("mv", "u1", 44), ("next_mv", "u1", 45)], 48)


def rust_cpu_events(rec: "ExecutionRecordArrays") -> np.ndarray:
    """record.cpu_events in the Rust layout above (what HipProver::prove iterates)."""
    cpu = rec.cpu
    out = np.zeros(len(cpu), dtype=RUST_CPU)
    for k in ("clk", "pc", "next_pc", "mp", "next_mp", "mv", "next_mv"):
        out[k] = cpu[k]
    tag = np.array([2, 0, 1], dtype=np.uint8)  # bfz kind None/Read/Write -> Rust tag
    for a in ("mv_access_", "next_mv_access_"):
        out[a + "tag"] = tag[cpu[a + "kind"]]
        for k in ("value", "prev_value", "timestamp", "prev_timestamp"):
            out[a + k] = cpu[a + k]
    return out


class CycleArraysStandin:
    """ctypes view of crates/bf-hip-prover/standin/libcycle_arrays.so: the compiled stand-in of
    the Rust CycleArrays::new (one parallel pass over cpu_events into page-locked memory) and its
    pipelined form over bfz_cycles_* (conversion of chunk k+1 overlaps the DMA of chunk k)."""

    def __init__(self):
        import os
        lib()  # libbfz first (the stand-in links it by its directory); no device needed to convert
        root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        path = os.path.join(root, "crates", "bf-hip-prover", "standin", "libcycle_arrays.so")
        self.so = ctypes.CDLL(path)
        self.so.ca_convert.restype = ctypes.c_int
        self.so.ca_convert.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int]
        self.so.ca_handover.restype = ctypes.c_int
        self.so.ca_handover.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                        ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                        ctypes.c_int, ctypes.c_size_t, ctypes.POINTER(ctypes.c_void_p),
                                        ctypes.POINTER(ctypes.c_double)]

    def convert(self, rust_cpu: np.ndarray, out: np.ndarray, threads: int) -> None:
        assert rust_cpu.dtype == RUST_CPU and out.dtype == CYCLE and len(out) == len(rust_cpu)
        if self.so.ca_convert(rust_cpu.ctypes.data, len(rust_cpu), out.ctypes.data, threads):
            raise RuntimeError("ca_convert failed")

    def handover(self, pk, rust_cpu: np.ndarray, memory: np.ndarray, out: np.ndarray,
                 threads: int, chunk: int):
        """(DeviceRecord, ms until the last chunk was pushed)."""
        assert rust_cpu.dtype == RUST_CPU and out.dtype == CYCLE and len(out) == len(rust_cpu)
        assert memory.dtype == MEMORY
        rec = ctypes.c_void_p()
        conv = ctypes.c_double()
        check(self.so.ca_handover(ctypes.c_void_p(pk.handle), rust_cpu.ctypes.data, len(rust_cpu),
                                  memory.ctypes.data if len(memory) else None, len(memory),
                                  out.ctypes.data, threads, chunk, ctypes.byref(rec),
                                  ctypes.byref(conv)))
        return DeviceRecord(rec.value), conv.value
