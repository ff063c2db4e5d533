"""N>1 path of bench.py on CPU: two gloo ranks run the same timed_steps() the GPU bench uses
(barriers + max over ranks); every rank proves its own replica, so no data-path collective."""
import os
import socket
import sys

import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, q):
    import time

    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    import bench
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    calls = []
    # rank 1 is the slow replica: 40 ms per step vs 5 ms
    ms = bench.timed_steps(lambda: (calls.append(1), time.sleep(0.04 if rank else 0.005)), 3,
                           dist)
    q.put((rank, ms, len(calls)))
    dist.destroy_process_group()


def test_timed_steps_two_gloo_ranks_take_max():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, ms0, n0), (_, ms1, n1) = res
    assert n0 == n1 == 3            # exactly K steps on every rank
    assert ms0 == ms1               # every rank reports the same (max) value
    assert ms0 >= 40.0              # ... which is the slow rank's pace


def _coll_rank(rank, world, port, q):
    """The host side of the sharded prover's two exchanges (bfz/shard.py Collectives), driven
    through the same ctypes callback objects libbfz calls, on a gloo group.  With no GPU here the
    buffers are host memory (pointers="host"); the GPU tests run the device-pointer form."""
    import ctypes

    import numpy as np
    import torch.distributed as dist
    sys.path.insert(0, os.path.join(ROOT, "zkvm-brainfuck_amd"))
    from bfz import shard
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    coll = shard.Collectives(dist, pointers="host")
    # all-gather of 32-byte subtree roots: rank r sends its own digest
    send = np.arange(1, 9, dtype=np.uint32) + 1000 * rank
    recv = np.zeros(8 * world, dtype=np.uint32)
    rc_ag = coll.allgather(None, send.ctypes.data, send.nbytes, recv.ctypes.data)
    # owner-masked all-reduce: word i is owned by rank i % world (others contribute 0)
    n = 37
    words = np.array([(0x7F000000 - i) if i % world == rank else 0 for i in range(n)],
                     dtype=np.uint32)
    rc_ar = coll.allreduce(None, words.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), n)
    q.put((rank, rc_ag, recv.tolist(), rc_ar, words.tolist()))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_shard_collectives_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_coll_rank, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    gathered = [v + 1000 * r for r in range(world) for v in range(1, 9)]
    reduced = [0x7F000000 - i for i in range(37)]  # exact: one owner per word, values < 2^31
    for rank, rc_ag, recv, rc_ar, words in res:
        assert rc_ag == 0 and rc_ar == 0
        assert recv == gathered, f"rank {rank}: all-gather out of rank order"
        assert words == reduced, f"rank {rank}: owner-masked all-reduce"


def test_run_with_limit_abandons_a_hung_extra():
    """bench.py runs the N>1 RCCL sharded-proof extra under a wall-clock limit: a result comes
    back as is, an exception as an error entry, and a call still blocked at the limit as None
    (the bench then reports it and exits without the teardown that would wait for it)."""
    import threading
    sys.path.insert(0, ROOT)
    import bench
    assert bench.run_with_limit(lambda: {"ms": 1.0}, 5) == {"ms": 1.0}
    err = bench.run_with_limit(lambda: 1 // 0, 5)
    assert "ZeroDivisionError" in err["error"]
    gate = threading.Event()
    assert bench.run_with_limit(gate.wait, 0.2) is None
    gate.set()
