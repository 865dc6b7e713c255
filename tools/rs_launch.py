#!/usr/bin/env python3
"""Local-reduction launch pattern of the client-sharded layouts at W ranks, on one GPU, no collective.

  python tools/rs_launch.py [W=8] [chunks=16] [steps=10]

One rank of the bench's rs / chain layouts holds 32 whole 256 MiB clients and reduces them in
pieces before each RCCL exchange.  This times those local launches alone (wall clock, K steps,
synchronised at both ends) for
  * one     -- the whole bucket in one launch (no exchange at all: the lower bound);
  * rs_rng  -- shard.reduce_rs: chunks * W launches per step (one per rank range and chunk);
  * rs_cyc  -- shard.reduce_rs_cyclic: chunks launches per step (one contiguous piece per chunk);
  * chain   -- shard.reduce_chain on a middle rank: chunks launches with d_init.
so the gap between rs_rng and rs_cyc is the launch cost the cyclic layout removes.  One JSON line.
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    W = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    chunks = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    import bench
    import torch
    fa = bench.load_pkg()
    shard = bench.load_shard()
    fa.lib()
    D, n = 32, 64 << 20
    setup = bench.Setup(fa, torch, D, n, "f32", "f32", 0, 0)
    cl = setup.clients()
    stream = torch.cuda.Stream()
    red = shard.fa_reducer(fa, fa.F32, stream)
    per = n // W
    buf = torch.empty(n, dtype=torch.float32, device="cuda")
    acc = torch.empty(n, dtype=torch.float32, device="cuda")
    edges = sorted({min(per, (per * c // chunks) // shard.UNIT * shard.UNIT) for c in range(chunks)} | {per})
    pieces = shard.cyclic_pieces(n, W, chunks)
    cedges = sorted({min(n, (n * c // chunks) // shard.UNIT * shard.UNIT) for c in range(chunks)} | {n})

    def p(x, a, b):
        return x + a * 4

    def one():
        red(cl, setup.w, n, out=buf)

    def rs_rng():
        for a, b in zip(edges, edges[1:]):
            q = b - a
            for r in range(W):
                o0 = r * per + a
                red([p(x, o0, o0 + q) for x in cl], setup.w, q, out=buf[r * q:(r + 1) * q])

    def rs_cyc():
        for a, b in pieces:
            red([p(x, a, b) for x in cl], setup.w, b - a, out=buf[:b - a])

    def chain():
        for a, b in zip(cedges, cedges[1:]):
            red([p(x, a, b) for x in cl], setup.w, b - a, init=acc[a:b], out=buf[a:b])

    res = {"W": W, "chunks": chunks, "steps": steps, "D": D, "elems_per_client": n}
    with torch.cuda.stream(stream):
        for name, fn in (("one", one), ("rs_rng", rs_rng), ("rs_cyc", rs_cyc), ("chain", chain)):
            for _ in range(2):
                fn()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(steps):
                fn()
            t_enq = time.perf_counter() - t0
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            res[name] = {"ms_per_step": round(dt / steps * 1e3, 4), "enqueue_ms_per_step": round(t_enq / steps * 1e3, 4)}
    setup.close()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
