"""CPU: bench.py's parity objects (verdict r03 #1) -- the check every timed leg runs on its own result.

Every bench leg (the main line at any N, the N > 1 weak-range / rs / chain secondaries, the in-process
--ctx-multi children, the single-GPU secondaries and rounds) reads its result back after its timed region
and checks >= 1024 sampled elements per rank / GPU against the oracle's ordered chain (aggregator.cpp:59-93,
:112-150 with FedAvg semantics): bit-exact for range and chain, |err| <= 1e-6 * sum_k |w_k x_k| for the
RCCL reduce-scatter.  Here the checker itself is tested on results the oracle computes (and corrupts), and
the client-sharded legs' parity runs over a gloo world of 2 with the exchange code of shard.py, so the
fields the driver's first multi-GPU run will carry are known to be populated and to catch a wrong result.
"""
import os
import socket
import sys
import types

import numpy as np
import torch.multiprocessing as mp

from conftest import ROOT

sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_sample_positions_cover_every_segment():
    segs = [(100, 164), (1000, 1001), (5000, 9000)]
    pos, idx = bench.sample_positions(segs, k=1024)
    total = sum(b - a for a, b in segs)
    assert pos.min() >= 0 and pos.max() < total and np.all(np.diff(pos) > 0)
    # the ends of every segment are always among the samples
    for a, b in segs:
        assert a in idx and b - 1 in idx
        assert np.count_nonzero((idx >= a) & (idx < b)) >= 1
    assert np.all([any(a <= i < b for a, b in segs) for i in idx])
    # position p of the concatenated result holds global element idx[p]
    cat = np.concatenate([np.arange(a, b) for a, b in segs])
    assert np.array_equal(cat[pos], idx.astype(np.int64))
    assert bench.sample_positions([(0, 50)], k=1024)[0].size == 50  # small results: every element
    assert bench.sample_positions([], k=10)[0].size == 0


def _full(O, seed, D, n, idx0=0, clients=None):
    w = O.weights(D)
    xs = [O.gen(seed, k if clients is None else clients[k], n, idx0=idx0) for k in range(D)]
    return w, xs, O.fedavg(xs, w)


def test_parity_exact_passes_and_catches_one_flipped_bit(O):
    w, _, out = _full(O, 0x5EED, 5, 20_000, idx0=7_000)
    pos, idx = bench.sample_positions([(7_000, 27_000)])
    p = bench.parity_check(out, pos, idx, 0x5EED, w)
    assert p["ok"] and p["mismatches"] == 0 and p["samples"] >= 1024 and p["max_abs_err"] == 0.0
    bad = out.copy()
    bad.view(np.uint32)[pos[3]] ^= 1  # one ulp on one sampled element
    q = bench.parity_check(bad, pos, idx, 0x5EED, w)
    assert not q["ok"] and q["mismatches"] == 1 and 0 < q["max_abs_err"] < 1e-6


def test_parity_bf16_result_and_mapped_clients(O):
    D, n = 6, 3_000
    clients = [k % 2 for k in range(D)]  # --ctx-multi --h2d: client k submits host buffer k % 8
    w = O.weights(D)
    xs = [O.gen(0x5EED, c, n, dtype="bf16") for c in clients]
    out = O.fedavg(xs, w, out_dtype="bf16")
    pos, idx = bench.sample_positions([(0, n)])
    assert bench.parity_check(out, pos, idx, 0x5EED, w, clients=clients, bf16_in=True)["ok"]
    assert not bench.parity_check(out, pos, idx, 0x5EED, w, bf16_in=True)["ok"]  # wrong client map


def test_parity_tolerance_bound(O):
    w, xs, out = _full(O, 0x5EED, 8, 10_000)
    pos, idx = bench.sample_positions([(0, 10_000)])
    sabs = np.sum([np.abs(np.float64(w[k]) * xs[k].astype(np.float64)) for k in range(8)], axis=0)
    near = (out.astype(np.float64) + 0.5e-6 * sabs).astype(np.float32)
    p = bench.parity_check(near, pos, idx, 0x5EED, w, exact=False)
    assert p["ok"] and 0.3 < p["max_err_over_bound"] < 0.8  # 0.5 of the bound plus the fp32 rounding
    far = out.copy()
    far[pos[10]] += np.float32(3e-6 * sabs[idx[10]] + 1e-6)
    q = bench.parity_check(far, pos, idx, 0x5EED, w, exact=False)
    assert not q["ok"] and q["mismatches"] == 1 and q["max_err_over_bound"] > 1.0


def test_parity_literal(O):
    n = 4_000
    x = O.gen(0x5EED, 0, n)
    out = O.literal(x)
    pos, idx = bench.sample_positions([(0, n)])
    p = bench.parity_check(out, pos, idx, 0x5EED, np.ones(1, np.float32), literal=True)
    assert p["ok"] and "fl(fl(x+x)/1000)" in p["check"]


def test_parity_merge_and_guard():
    a = {"check": "c", "samples": 10, "mismatches": 0, "max_abs_err": 0.0, "ok": True}
    b = {"check": "c", "samples": 12, "mismatches": 2, "max_abs_err": 1e-3, "max_err_over_bound": 4.0, "ok": False}
    m = bench.parity_merge([a, b])
    assert m["samples"] == 22 and m["mismatches"] == 2 and not m["ok"] and m["max_err_over_bound"] == 4.0
    g = bench.parity_guarded(lambda: 1 / 0)
    assert g["ok"] is False and "ZeroDivisionError" in g["error"]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, n, D, q, corrupt):
    import importlib
    import torch
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import bench as B
    import oracle as O
    from conftest import load_pkg
    load_pkg()
    shard = importlib.import_module("mhfsl_amd.shard")
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    try:
        w = O.weights(D)

        def reducer(clients, weights, m, init=None, out=None):
            r = torch.from_numpy(O.fedavg([c.numpy() for c in clients], np.asarray(weights, np.float32),
                                          init=None if init is None else init.numpy()))
            if out is None:
                return r
            out.copy_(r)
            return out
        c0, c1 = shard.client_bounds(D, world, rank)
        mine = [torch.from_numpy(O.gen(0x5EED, k, n)) for k in range(c0, c1)]
        setup = types.SimpleNamespace(seed=0x5EED, in_dt=0, fa=types.SimpleNamespace(BF16=1))
        out = {}
        for layout in ("rs", "chain"):
            fn = shard.reduce_rs_cyclic if layout == "rs" else shard.reduce_chain
            res = fn(reducer, dist, mine, w[c0:c1], n, torch.device("cpu"), chunks=4)
            if corrupt and rank == 1:
                res[0] += 1.0  # the first element of every segment is always sampled
            p = B.client_sharded_parity(shard, setup, layout, res, n, world, rank, 4, D)
            out[layout] = B.parity_over_ranks(torch, dist, world, "gloo", p)
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def _run(world, n, D, corrupt=False):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, D, q, corrupt)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return out


def test_client_sharded_parity_over_gloo_ranks():
    """The N > 1 rs / chain legs' parity objects over a world of 2: populated on every rank (summed samples,
    ranks = 2), passing for the real exchange, failing when one rank's result is off."""
    n, D = 2 * 64 * 40, 7
    out = _run(2, n, D)
    for layout, exact in (("rs", False), ("chain", True)):
        for r in range(2):
            p = out[r][layout]
            assert p["ok"] and p["ranks"] == 2 and p["mismatches"] == 0, (layout, p)
            assert p["samples"] >= 2 * 1024 and ("max_err_over_bound" in p) == (not exact)
            assert p["check"].startswith("bit-exact") == exact
        if not exact:
            assert out[0][layout]["max_err_over_bound"] < 1.0
    bad = _run(2, n, D, corrupt=True)
    for layout in ("rs", "chain"):
        assert not bad[0][layout]["ok"] and bad[0][layout]["mismatches"] >= 1


def test_committed_round4_bench_line_has_every_field():
    """profiles/r04_bench.json (the full N = 1 bench of the round-4 tree, r04s07): the main line and every
    secondary that reduces carry a passing parity object; the CPU baseline is the whole north-star workload,
    and the other configs carry the reference's CPU path beside their device figure (verdict r03 #1, #3)."""
    import json
    with open(os.path.join(ROOT, "profiles", "r04_bench.json")) as f:
        line = json.load(f)
    assert line["parity"]["ok"] and line["parity"]["samples"] >= 1024
    cpu = line["cpu_baseline"]
    assert cpu["kind"] == "reference" and cpu["sample"].startswith("the whole workload") and cpu["cores"] >= 1
    sec = line["secondary"]
    for key, v in sec.items():
        if key.startswith("sync_") and "parity" not in v:  # r04s07 predates the sync legs' check
            continue
        assert v["parity"]["ok"] and v["parity"]["samples"] >= 1024, key
    for key in ("c2", "c3", "c4", "c5", "round_c2", "round_c4"):
        assert sec[key]["cpu_gib_s"] > 0 and sec[key]["cpu_cores"] >= 1 and sec[key]["host_cpu"], key


def test_parity_nan_is_a_mismatch_and_json_stays_standard(O):
    """A NaN where the oracle has a number fails both checks, and the parity object serializes as standard
    JSON (no NaN / Infinity literals the driver's parser would refuse)."""
    import json
    w, _, out = _full(O, 0x5EED, 4, 5_000)
    pos, idx = bench.sample_positions([(0, 5_000)])
    bad = out.copy()
    bad[pos[7]] = np.nan
    for exact in (True, False):
        p = bench.parity_check(bad, pos, idx, 0x5EED, w, exact=exact)
        assert not p["ok"] and p["mismatches"] == 1, p
        json.loads(json.dumps(p, allow_nan=False))
    m = bench.parity_merge([bench.parity_check(out, pos, idx, 0x5EED, w, exact=False),
                            bench.parity_check(bad, pos, idx, 0x5EED, w, exact=False)])
    assert not m["ok"] and m["max_err_over_bound"] is None


def test_ctx_children_the_n1_run_starts(monkeypatch):
    """Which --ctx-multi children the N = 1 bench starts: on the driver's 8-GPU node the real multi-GPU legs
    (C4's reduce-scatter on 4 and 8 GPUs, C5 host-inclusive on 8), on a one-GPU box the 8-GPU legs rehearsed
    as 8 shards of the one GPU; every child's JSON (with its parity object) lands under its key."""
    import json
    import subprocess
    calls = []

    class R:
        returncode = 0
        stderr = ""

        def __init__(self, cmd):
            self.stdout = json.dumps({"cmd": cmd, "parity": {"ok": True}}) + "\n"

    def fake_run(cmd, **kw):
        calls.append(cmd)
        return R(cmd)
    monkeypatch.setattr(subprocess, "run", fake_run)
    import time
    res = bench.ctx_multi_secondaries(8, time.monotonic() + 1000)
    sweep = {"ctx_rs_c4_4gpu_rschunks%d" % c for c in bench.RS_CHUNK_SWEEP}
    assert {"ns_h2d", "ctx_range_northstar_8gpu", "ctx_rs_northstar_8gpu", "ctx_rs_c4_4gpu", "ctx_rs_c4_8gpu",
            "ctx_range_c5_h2d_8gpu"} | sweep == set(res)
    # the north star host-inclusive on one GPU comes first, on every node
    assert calls[0][calls[0].index("--ctx-gpus") + 1] == "1" and "--h2d" in calls[0] and "northstar" in calls[0]
    assert all(r["parity"]["ok"] for r in res.values())
    c4 = [c for c in calls if "c4" in c and c[c.index("--ctx-gpus") + 1] == "4"]
    assert c4 and c4[0][c4[0].index("--ctx-multi") + 1] == "rs" and "--rs-chunks" not in c4[0]
    # the rs overlap-depth sweep of C4 at 4 GPUs comes last (the budget drops it first), one child per depth
    assert [c[c.index("--rs-chunks") + 1] for c in calls if "--rs-chunks" in c] == \
        [str(c) for c in bench.RS_CHUNK_SWEEP]
    assert all("--rs-chunks" not in c for c in calls[:-len(bench.RS_CHUNK_SWEEP)])
    calls.clear()
    res = bench.ctx_multi_secondaries(1, time.monotonic() + 1000)
    assert set(res) == {"ns_h2d", "ctx_rs_c4_8shard_rehearsal_on_one_gpu",
                        "ctx_range_c5r_h2d_8shard_rehearsal_on_one_gpu"}
    assert all("--ctx-shared" in c and c[c.index("--ctx-shared") + 1] == "8" for c in calls[1:])
    # no time left: skipped, never started
    calls.clear()
    res = bench.ctx_multi_secondaries(8, time.monotonic() + 10)
    assert not calls and all("skipped" in r for r in res.values())
