"""Multi-rank layouts of shard.py on CPU with the gloo backend (world_size 2 and 3).

The exchange logic (range ownership, reduce-scatter of partials, the rank-to-rank
chain hand-off and final scatter) is the product code; only the local reduction
is the oracle here (on the GPU box it is libfa.so via shard.fa_reducer).
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import ROOT, load_pkg


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def worker(rank, world, port, n, D, seed, q):
    import torch
    import torch.distributed as dist
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle as O
    from conftest import load_pkg as lp
    shard = lp()
    import importlib
    shard = importlib.import_module("mhfsl_amd.shard")
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        w = O.weights(D)
        dev = torch.device("cpu")

        def reducer(clients, weights, m, init=None, out=None):
            xs = [c.numpy() for c in clients]
            r = torch.from_numpy(O.fedavg(xs, np.asarray(weights, np.float32),
                                          init=None if init is None else init.numpy()))
            if out is None:
                return r
            out.copy_(r)
            return out
        res = {}
        # range: this rank's slice of every client bucket
        lo, hi = shard.range_bounds(n, world, rank)
        sl = [torch.from_numpy(O.gen(seed, k, hi - lo, idx0=lo)) for k in range(D)]
        res["range"] = shard.reduce_range(reducer, sl, w, lo, hi).numpy() if hi > lo else np.zeros(0, np.float32)
        # client-sharded: whole buckets of this rank's clients
        c0, c1 = shard.client_bounds(D, world, rank)
        mine = [torch.from_numpy(O.gen(seed, k, n)) for k in range(c0, c1)]
        res["chain"] = shard.reduce_chain(reducer, dist, mine, w[c0:c1], n, dev, chunks=5).numpy()
        npad = -(-n // (world * shard.UNIT)) * world * shard.UNIT
        mine_p = [torch.nn.functional.pad(x, (0, npad - n)) for x in mine]
        res["rs"] = shard.reduce_rs(reducer, dist, mine_p, w[c0:c1], npad, dev).numpy()
        res["rs_chunked"] = shard.reduce_rs(reducer, dist, mine_p, w[c0:c1], npad, dev, chunks=3).numpy()
        for ch in (1, 4):
            res["rs_cyclic%d" % ch] = shard.reduce_rs_cyclic(reducer, dist, mine_p, w[c0:c1], npad, dev,
                                                              chunks=ch).numpy()
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


def run(world, n, D, seed=17):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=worker, args=(r, world, port, n, D, seed, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return out


@pytest.mark.parametrize("world,n,D", [(2, 10_000, 5), (3, 7_777, 7), (2, 4_099, 1), (3, 1_000, 2)])
def test_layouts_match_single_gpu_chain(O, record_property, world, n, D):
    fa = load_pkg()
    import importlib
    shard = importlib.import_module("mhfsl_amd.shard")
    del fa
    seed = 17
    out = run(world, n, D, seed)
    w = O.weights(D)
    xs = [O.gen(seed, k, n) for k in range(D)]
    ref = O.fedavg(xs, w)
    # range and chain are bit-exact with the single-GPU ordered chain
    for layout in ("range", "chain"):
        got = np.concatenate([out[r][layout] for r in range(world)])
        assert got.size == n
        assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), layout
    # rs changes the summation order: within 1e-6 of sum_k |w_k x_k|
    absw = sum(abs(np.float64(wk)) * np.abs(x.astype(np.float64)) for wk, x in zip(w, xs))
    for layout in ("rs", "rs_chunked"):  # chunked: reduce of chunk c+1 overlaps the reduce-scatter of chunk c
        got = np.concatenate([out[r][layout] for r in range(world)])[:n]
        ok, worst = shard.tolerance_ok(got, ref, absw)
        record_property("max_err_fraction_of_bound_%s" % layout, worst)
        print("%s world=%d n=%d D=%d: max |err| = %.3g of the bound 1e-6 sum|w x|" % (layout, world, n, D, worst))
        assert ok, (layout, worst)
    # block-cyclic rs: each rank's shard is its cyclic_bounds segments, concatenated
    npad = -(-n // (world * shard.UNIT)) * world * shard.UNIT
    for ch in (1, 4):
        got = np.full(npad, np.nan, np.float32)
        for r in range(world):
            segs = shard.cyclic_bounds(npad, world, r, ch)
            mine = out[r]["rs_cyclic%d" % ch]
            assert mine.size == sum(b - a for a, b in segs) == npad // world
            off = 0
            for a, b in segs:
                got[a:b] = mine[off:off + b - a]
                off += b - a
        assert not np.isnan(got).any()  # the segments of all ranks cover the bucket
        ok, worst = shard.tolerance_ok(got[:n], ref, absw)
        record_property("max_err_fraction_of_bound_rs_cyclic%d" % ch, worst)
        print("rs_cyclic%d world=%d n=%d D=%d: max |err| = %.3g of the bound 1e-6 sum|w x|" % (ch, world, n, D, worst))
        assert ok, ("rs_cyclic", ch, worst)
        assert np.all(got[n:] == 0)  # padding stays zero


def test_bounds_cover_and_align():
    load_pkg()
    import importlib
    shard = importlib.import_module("mhfsl_amd.shard")
    for n in [0, 1, 63, 64, 65, 1000, 123_457]:
        for world in [1, 2, 3, 8]:
            b = [shard.range_bounds(n, world, r) for r in range(world)]
            assert b[0][0] == 0 and b[-1][1] == n
            assert all(b[i][1] == b[i + 1][0] for i in range(world - 1))
            assert all(lo % shard.UNIT == 0 or lo == n for lo, _ in b)
    for D in [1, 2, 5, 32, 128]:
        for world in [1, 2, 3, 8]:
            c = [shard.client_bounds(D, world, r) for r in range(world)]
            assert c[0][0] == 0 and c[-1][1] == D and all(c[i][1] == c[i + 1][0] for i in range(world - 1))
