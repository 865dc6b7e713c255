"""The multi-GPU exchanges of shard.py over real RCCL (backend "nccl") with libfa.so as the local reduction.

The GPU box has one GPU, so the process group has world size 1: the reduce-scatter of a single partial
is a copy and the chain has no hand-off, so every layout must equal the single-GPU ordered chain
bit-for-bit.  What this pins beyond the gloo tests (tests/test_shard_gloo.py, world 2 and 3 on CPU):
the RCCL work handles and stream ordering around libfa's launches on a side stream (the reduce of
chunk c+1 is enqueued while the reduce-scatter of chunk c is in flight, buffers are reused after
wait()), raw device addresses as clients, and pieces that take the phased and the one-shot kernels.
"""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture(scope="module")
def rccl(fa, torch_gpu):
    import torch.distributed as dist
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % _free_port(), rank=0, world_size=1,
                            device_id=torch_gpu.device("cuda", 0))
    yield dist
    dist.destroy_process_group()


@pytest.mark.parametrize("n,D", [(64 * 20_011, 5), (64 * 400_000, 3)])  # 1.3 M (one-shot) and 25.6 M (phased)
def test_layouts_over_rccl_bitexact(fa, O, torch_gpu, rccl, n, D):
    import importlib
    torch = torch_gpu
    shard = importlib.import_module("mhfsl_amd.shard")
    seed = 0x5EED
    w = O.weights(D)
    clients = []
    for k in range(D):
        t = torch.empty(n, dtype=torch.float32, device="cuda")
        fa.fill_uniform(t, n, fa.F32, seed, k)
        clients.append(t)
    addrs = [t.data_ptr() for t in clients]
    ref = O.fedavg([O.gen(seed, k, n) for k in range(D)], w).view(np.uint32)
    stream = torch.cuda.Stream()
    red = shard.fa_reducer(fa, fa.F32, stream)
    dev = torch.device("cuda", 0)
    got = {}
    with torch.cuda.stream(stream):
        for ch in (1, 4, 16):
            got["rs_cyclic%d" % ch] = shard.reduce_rs_cyclic(red, rccl, addrs, w, n, dev, chunks=ch, itemsize=4)
        got["rs3"] = shard.reduce_rs(red, rccl, clients, w, n, dev, chunks=3)
        got["chain5"] = shard.reduce_chain(red, rccl, addrs, w, n, dev, chunks=5, itemsize=4)
        got["range"] = shard.reduce_range(red, clients, w, 0, n)
    torch.cuda.synchronize()
    assert shard.cyclic_bounds(n, 1, 0, 16)[0][0] == 0
    for name, t in got.items():
        a = t.cpu().numpy()
        assert a.size == n, name
        bad = np.flatnonzero(a.view(np.uint32) != ref)
        assert bad.size == 0, (name, bad[:8])
