"""One core proof sharded over the ranks of a torch.distributed group.

Every rank holds the same record and proving key; bfz_record_prove_sharded hashes this
rank's subtree of every large Merkle tree and calls back here for the two exchanges: an
all-gather of subtree roots and a sum all-reduce of the owner-masked query openings.  The
callbacks receive device pointers: with the nccl backend (RCCL on ROCm) the collectives run on
zero-copy tensor views of them, over xGMI; with gloo (the tests, several ranks on one GPU) they
go through host tensors.
"""
from __future__ import annotations

import ctypes
import traceback

import numpy as np

from . import _lib


class _DeviceSpan:
    """A raw device pointer seen by torch.as_tensor through __cuda_array_interface__ (no copy)."""

    def __init__(self, ptr: int, nbytes: int, typestr: str = "|u1"):
        item = int(typestr[-1])
        self.__cuda_array_interface__ = {"shape": (nbytes // item,), "typestr": typestr,
                                         "data": (int(ptr), False), "version": 2, "strides": None}


class Collectives:
    """ctypes callbacks over a torch.distributed process group.

    libbfz passes DEVICE pointers on the rank's GPU (the send data complete; at the two quotient
    all-gathers later GPU work is still queued, which _sync's device-wide wait covers).  With the
    nccl backend (RCCL) the collective runs on views of those buffers, device to device over
    xGMI; with gloo (several test ranks sharing one GPU) the data goes through host tensors."""

    def __init__(self, dist, group=None, device=None, pointers="device"):
        """pointers="host" reads the callback buffers as host memory: only for testing the
        exchange logic on a machine without a GPU (libbfz always passes device pointers)."""
        import torch
        self.dist, self.group, self.torch = dist, group, torch
        self.world = dist.get_world_size(group)
        backend = str(dist.get_backend(group)).lower()
        self.cuda = torch.device("cuda", device if device is not None else 0)
        self.host_ptrs = pointers == "host"
        self.nccl = "nccl" in backend and not self.host_ptrs
        self.dev = self.cuda if self.nccl else torch.device("cpu")
        self.allgather = _lib.ALLGATHER_FN(self._allgather)
        self.allreduce = _lib.ALLREDUCE_FN(self._allreduce)
        self.alltoall = _lib.ALLTOALL_FN(self._alltoall)
        self.exchange = None  # (send, recv) device tensors of the pending all-to-all

    def _view(self, ptr, nbytes, typestr="|u1"):
        if self.host_ptrs:
            dt = {"|u1": np.uint8, "<i4": np.int32}[typestr]
            buf = (ctypes.c_uint8 * nbytes).from_address(ptr)
            return self.torch.from_numpy(np.frombuffer(buf, dtype=dt))
        return self.torch.as_tensor(_DeviceSpan(ptr, nbytes, typestr), device=self.cuda)

    def _sync(self):
        if not self.host_ptrs:
            self.torch.cuda.synchronize(self.cuda)

    def _allgather(self, _ctx, send, nbytes, recv):
        try:
            torch = self.torch
            src = self._view(send, nbytes)
            dst = self._view(recv, nbytes * self.world)
            if self.nccl:
                self.dist.all_gather_into_tensor(dst, src, group=self.group)
            else:
                parts = [torch.empty(nbytes, dtype=torch.uint8) for _ in range(self.world)]
                self.dist.all_gather(parts, src.cpu(), group=self.group)
                dst.copy_(torch.cat(parts))
            self._sync()
            return 0
        except Exception:  # noqa: BLE001 - reported to the C side as a failed collective
            traceback.print_exc()
            return 1

    def _allreduce(self, _ctx, data, n):
        try:
            torch = self.torch
            # exactly one rank contributes each word (< 2^31): an int32 sum is exact
            t = self._view(ctypes.cast(data, ctypes.c_void_p).value, 4 * n, "<i4")
            if self.nccl:
                self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM, group=self.group)
            else:
                h = t.cpu()
                self.dist.all_reduce(h, op=self.dist.ReduceOp.SUM, group=self.group)
                t.copy_(h)
            self._sync()
            return 0
        except Exception:  # noqa: BLE001
            traceback.print_exc()
            return 1

    def _alltoall(self, _ctx):
        """Equal-block all-to-all of the registered device tensors (RCCL with nccl; through
        host memory with gloo)."""
        try:
            send, recv = self.exchange
            if self.nccl:
                self.dist.all_to_all_single(recv, send, group=self.group)
                self.torch.cuda.synchronize(recv.device)
            else:
                r = self.torch.empty(send.shape, dtype=send.dtype)
                self.dist.all_to_all_single(r, send.cpu(), group=self.group)
                recv.copy_(r)
                self.torch.cuda.synchronize(recv.device)
            return 0
        except Exception:  # noqa: BLE001
            traceback.print_exc()
            return 1


def commit_fri_sharded(cols, log_n: int, coll: "Collectives | None", rank: int = 0, send=None,
                       recv=None):
    """bfz_commit_fri_sharded on this rank's columns.

    cols: int32 CUDA tensor of shape (w_local, 2^log_n): column-major, bit-reversed rows,
    Montgomery form, columns [rank w_local, (rank+1) w_local) of the trace.  send/recv:
    optional preallocated int32 CUDA exchange buffers of 2^(log_n+1) * w_local words.  Returns
    (root, fri_roots, final) as uint32 numpy arrays (identical on every rank)."""
    import torch
    L = _lib.lib()
    w_local = cols.shape[0]
    world = coll.world if coll else 1
    n2 = 2 << log_n
    if world > 1:
        if send is None or recv is None:
            send = torch.empty((w_local * n2,), dtype=torch.int32, device=cols.device)
            recv = torch.empty_like(send)
        coll.exchange = (send, recv)
    else:
        send = recv = None
    torch.cuda.synchronize(cols.device)  # cols may still be in flight on torch's stream
    cap = 8 + 8 * (log_n + 1) + 4
    out = (ctypes.c_uint32 * cap)()
    nw = ctypes.c_size_t()
    empty_a2a = _lib.ALLTOALL_FN(0)
    empty_ag = _lib.ALLGATHER_FN(0)
    try:
        _lib.check(L.bfz_commit_fri_sharded(
            ctypes.c_void_p(cols.data_ptr()), log_n, w_local, rank, world,
            ctypes.c_void_p(send.data_ptr() if send is not None else 0),
            ctypes.c_void_p(recv.data_ptr() if recv is not None else 0),
            coll.alltoall if coll else empty_a2a, coll.allgather if coll else empty_ag, None,
            out, cap, ctypes.byref(nw)))
    finally:
        if coll:
            coll.exchange = None
    words = np.frombuffer(bytes(out), dtype=np.uint32)[: nw.value]
    nfri = (nw.value - 12) // 8
    return words[:8].copy(), words[8:8 + 8 * nfri].reshape(nfri, 8).copy(), words[-4:].copy()


def prove_record_sharded(pk_handle, rec, coll: Collectives, rank: int, timings=None) -> bytes:
    """bfz_record_prove_sharded for this rank; returns the (rank-independent) proof bytes."""
    L = _lib.lib()
    ptr = ctypes.POINTER(ctypes.c_uint8)()
    plen = ctypes.c_size_t()
    _lib.check(L.bfz_record_prove_sharded(
        ctypes.c_void_p(pk_handle), rec, rank, coll.world, coll.allgather, coll.allreduce, None,
        ctypes.byref(ptr), ctypes.byref(plen), ctypes.byref(timings) if timings else None))
    return _lib.take_bytes(ptr, plen.value)


def new_record(pk_handle, stdin: bytes):
    """bfz_record_new: execute + upload the events (the proof's inputs) to this rank's GPU."""
    L = _lib.lib()
    rec = ctypes.c_void_p()
    cycles = ctypes.c_uint64()
    buf, n = _lib.u8buf(bytes(stdin))
    _lib.check(L.bfz_record_new(ctypes.c_void_p(pk_handle), buf, n, ctypes.byref(rec),
                                ctypes.byref(cycles)))
    return rec, cycles.value
