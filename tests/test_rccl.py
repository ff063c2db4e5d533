"""The RCCL branches of bfz/shard.py's Collectives on a real GPU.

The multi-rank sharded tests (test_sharded.py, test_pcs_sharded.py) run several ranks on the
box's one GPU, so they use gloo: RCCL refuses two ranks on one device.  This test runs the
nccl-backend branches (all_gather_into_tensor, all_reduce, all_to_all_single on zero-copy
__cuda_array_interface__ views of raw device pointers, as libbfz hands them to the callbacks)
in a one-rank RCCL group, where each collective is the identity: it checks the views, dtypes,
sizes and stream synchronisation that the 8-GPU run relies on.
"""
import os
import socket
import subprocess
import sys
import textwrap

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = textwrap.dedent("""
    import ctypes, os, sys
    sys.path.insert(0, os.path.join(sys.argv[1], "zkvm-brainfuck_amd"))
    import torch
    import torch.distributed as dist
    from bfz import shard
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=sys.argv[2])
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    coll = shard.Collectives(dist, device=0)
    assert coll.nccl, "expected the RCCL branch"
    g = torch.Generator().manual_seed(7)
    # all-gather of 32-byte subtree roots (libbfz: prover.hip subtree roots)
    src = torch.randint(0, 256, (32,), dtype=torch.uint8, generator=g).cuda()
    dst = torch.zeros(32, dtype=torch.uint8, device="cuda")
    assert coll._allgather(None, src.data_ptr(), 32, dst.data_ptr()) == 0
    assert torch.equal(src, dst)
    # sum all-reduce of owner-masked query words (int32, in place)
    words = torch.randint(0, 2**31 - 1, (4099,), dtype=torch.int32, generator=g).cuda()
    ref = words.clone()
    assert coll._allreduce(None, ctypes.c_void_p(words.data_ptr()), words.numel()) == 0
    assert torch.equal(words, ref)
    # equal-block all-to-all of registered exchange buffers (pcs_sharded.hip)
    send = torch.randint(0, 2**31 - 1, (1 << 16,), dtype=torch.int32, generator=g).cuda()
    recv = torch.zeros_like(send)
    coll.exchange = (send, recv)
    assert coll._alltoall(None) == 0
    assert torch.equal(send, recv)
    dist.destroy_process_group()
    print("rccl ok")
""")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_rccl_collective_branches_one_rank():
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, "-c", SCRIPT, ROOT, str(_free_port())], env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and "rccl ok" in r.stdout, r.stdout[-2000:] + r.stderr[-4000:]
