"""One proof sharded over several ranks (bfz_record_prove_sharded).

Each test runs `world` processes with a gloo group on the one GPU of the box (RCCL needs
distinct devices; the exchanged data are the same).  Every rank must return the proof that
the unsharded prover returns, byte for byte, and rank 0 checks it against the oracle.
"""
import hashlib
import os
import socket
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, cases, q, fri_min=None):
    try:
        if fri_min is not None:  # shard the FRI rounds of these small proofs too
            os.environ["BFZ_FRI_SHARD_MIN"] = str(fri_min)
        sys.path.insert(0, os.path.join(ROOT, "zkvm-brainfuck_amd"))
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        import ctypes

        import torch.distributed as dist

        from bfz import _lib, sdk, shard
        dist.init_process_group("gloo", rank=rank, world_size=world)
        _lib.init(0)
        coll = shard.Collectives(dist)
        client = sdk.ProverClient()
        out = []
        for prog, stdin in cases:
            pk, vk = client.setup(prog)
            rec, _ = shard.new_record(pk.handle, bytes(stdin))
            sharded = shard.prove_record_sharded(pk.handle, rec, coll, rank)
            ptr = ctypes.POINTER(ctypes.c_uint8)()
            plen = ctypes.c_size_t()
            _lib.check(_lib.lib().bfz_record_prove(ctypes.c_void_p(pk.handle), rec,
                                                   ctypes.byref(ptr), ctypes.byref(plen), None))
            single = _lib.take_bytes(ptr, plen.value)
            _lib.lib().bfz_record_free(rec)
            ok_verify = True
            if rank == 0:
                client.verify(sdk.BfProofWithPublicValues(proof=sharded, stdin=bytes(stdin)), vk)
            out.append((hashlib.sha256(sharded).hexdigest(), hashlib.sha256(single).hexdigest(),
                        ok_verify, sharded if rank == 0 else b""))
        dist.destroy_process_group()
        q.put((rank, out, None))
    except Exception as e:  # noqa: BLE001 - reported to the parent
        import traceback
        q.put((rank, None, traceback.format_exc()))


def _run(world, cases, fri_min=None):
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, cases, q, fri_min))
          for r in range(world)]
    for p in ps:
        p.start()
    res = {}
    for _ in ps:
        rank, out, err = q.get(timeout=900)
        assert err is None, f"rank {rank}:\n{err}"
        res[rank] = out
    for p in ps:
        p.join(timeout=120)
        assert p.exitcode == 0
    return res


@pytest.mark.parametrize("world,fri_min", [(2, None), (4, None), (8, None), (2, 1024), (4, 1024)])
def test_sharded_proof_is_bit_exact(world, fri_min):
    """fri_min=1024 keeps every FRI round with >= world * 1024 leaves row-sharded (the default
    replicates the rounds below 2^18 leaves, i.e. all of these small proofs' rounds)."""
    from bfz import guests
    import oracle_lib as O
    cases = [(guests.FIBO, [17]), (guests.FIBO, [255])]
    res = _run(world, cases, fri_min)
    for i, (prog, stdin) in enumerate(cases):
        digests = {res[r][i][0] for r in range(world)}
        assert len(digests) == 1, "ranks disagree"
        assert res[0][i][0] == res[0][i][1], "sharded proof differs from the unsharded one"
        if stdin == [17]:
            assert res[0][i][3] == O.prove(prog, stdin)


@pytest.mark.slow
@pytest.mark.parametrize("world", [2, 4, 8])
def test_sharded_headline_is_bit_exact(world):
    """The headline workload (FIBO_X4 stdin [255], Cpu 2^22 rows) sharded over 2, 4 and 8 ranks
    -- the SCALE shapes; at 4 and 8 ranks every quotient point's next row lies in another
    residue class, so the next-residue LDE shards run at 2^22 -- every rank returns the
    unsharded proof byte for byte (which test_gpu.py checks against the oracle)."""
    from bfz import guests
    res = _run(world, [(guests.FIBO_X4, [255])])
    assert len({res[r][0][0] for r in range(world)}) == 1, "ranks disagree"
    assert res[0][0][0] == res[0][0][1], "sharded proof differs from the unsharded one"
