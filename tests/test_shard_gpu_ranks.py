"""Two ranks on the GPU box's one GPU (gloo; RCCL needs one GPU per rank), each reducing its clients
with libfa.so on device buffers: the chain hand-off, both reduce-scatters and the range layout
against the oracle.  Beyond tests/test_shard_gloo.py (CPU tensors, oracle reducer) and
tests/test_shard_rccl.py (world 1), this runs the multi-rank exchange logic around real kernel
launches in separate processes: the chain continues rank 0's fp32 accumulator on rank 1 (d_init, in
place) and must stay bit-exact; device tensors cross gloo through host copies (shard._staged).
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, n, D, seed, w, q):
    import importlib
    import torch
    import torch.distributed as dist
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from conftest import load_pkg
    torch.cuda.set_device(0)
    fa = load_pkg()
    fa.lib()
    shard = importlib.import_module("mhfsl_amd.shard")
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    try:
        dev = torch.device("cuda", 0)
        stream = torch.cuda.Stream()
        red = shard.fa_reducer(fa, fa.F32, stream)
        res = {}
        with torch.cuda.stream(stream):
            lo, hi = shard.range_bounds(n, world, rank)
            sl = []
            for k in range(D):
                t = torch.empty(hi - lo, dtype=torch.float32, device=dev)
                fa.fill_uniform(t, hi - lo, fa.F32, seed, k, idx0=lo)
                sl.append(t)
            res["range"] = shard.reduce_range(red, sl, w, lo, hi)
            c0, c1 = shard.client_bounds(D, world, rank)
            mine = []
            for k in range(c0, c1):
                t = torch.empty(n, dtype=torch.float32, device=dev)
                fa.fill_uniform(t, n, fa.F32, seed, k)
                mine.append(t)
            res["chain"] = shard.reduce_chain(red, dist, [t.data_ptr() for t in mine], w[c0:c1], n, dev, chunks=5)
            res["rs"] = shard.reduce_rs(red, dist, mine, w[c0:c1], n, dev, chunks=3)
            res["rs_cyclic"] = shard.reduce_rs_cyclic(red, dist, mine, w[c0:c1], n, dev, chunks=4)
        torch.cuda.synchronize()
        q.put((rank, {k: v.cpu().numpy() for k, v in res.items()}))
    finally:
        dist.destroy_process_group()


def test_two_gpu_ranks_match_oracle(O, torch_gpu):
    import importlib
    shard = importlib.import_module("mhfsl_amd.shard")
    world, D, seed = 2, 5, 31
    n = 2 * shard.UNIT * 10_007  # a multiple of world * UNIT, as the reduce-scatters need
    w = [float(x) for x in O.weights(D)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, D, seed, w, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        out = dict(q.get(timeout=150) for _ in range(world))
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    assert all(p.exitcode == 0 for p in procs)
    wf = np.asarray(w, np.float32)
    xs = [O.gen(seed, k, n) for k in range(D)]
    ref = O.fedavg(xs, wf)
    for layout in ("range", "chain"):  # bit-exact with the single-GPU ordered chain
        got = np.concatenate([out[r][layout] for r in range(world)])
        assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), layout
    absw = sum(abs(np.float64(wk)) * np.abs(x.astype(np.float64)) for wk, x in zip(wf, xs))
    ok, worst = shard.tolerance_ok(np.concatenate([out[r]["rs"] for r in range(world)]), ref, absw)
    assert ok, ("rs", worst)
    got = np.empty(n, np.float32)
    for r in range(world):
        off = 0
        for a, b in shard.cyclic_bounds(n, world, r, 4):
            got[a:b] = out[r]["rs_cyclic"][off:off + b - a]
            off += b - a
    ok, worst = shard.tolerance_ok(got, ref, absw)
    assert ok, ("rs_cyclic", worst)
