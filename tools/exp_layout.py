#!/usr/bin/env python3
"""Experiment (GPU box): does the placement of the D client buckets in HBM matter?

All buckets allocated separately sit at the same offset modulo their (2 MiB
aligned) size, so lane l of a wave reads the same low address bits from all U
clients it loads at once.  This places the D buckets (and optionally the
output) in one pool with a skew of `pad` elements between consecutive buckets
and times the north-star reduce, interleaved in rounds in one process.

  python tools/exp_layout.py [pads...]     (pads in fp32 elements; default set below)
"""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    import torch
    fa = bench.load_pkg()
    fa.lib()
    D, n = 32, 64 << 20
    w = bench.Setup._weights(D)
    pads = [int(x) for x in sys.argv[1:]] or [0, 16, 32, 64, 128, 256, 512, 1024]
    stream = torch.cuda.Stream()
    sep_out = torch.empty(n, dtype=torch.float32, device="cuda")
    pools = {}
    for pad in pads:
        # D client slots then the output slot, all `n + pad` apart
        pool = torch.empty((D + 1) * (n + pad), dtype=torch.float32, device="cuda")
        clients = [pool[k * (n + pad): k * (n + pad) + n] for k in range(D)]
        for k, c in enumerate(clients):
            fa.fill_uniform(c, n, fa.F32, 0x5EED, k)
        pools[pad] = (pool, clients, pool[D * (n + pad): D * (n + pad) + n])
    torch.cuda.synchronize()
    variants = [(pad, where, blk) for pad in pads for where in ("pool", "separate") for blk in (128, 256)]
    results = {v: [] for v in variants}
    for rnd in range(4):
        for v in variants:
            pad, where, blk = v
            fa.set_tuning(block=blk, max_blocks=-1, unroll=8, nontemporal=1)
            out = pools[pad][2] if where == "pool" else sep_out
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(5)]
            for a, b in ev:
                a.record(stream)
                fa.reduce_device(pools[pad][1], w, n, fa.F32, out, fa.F32, stream=stream)
                b.record(stream)
            torch.cuda.synchronize()
            results[v] += [a.elapsed_time(b) for a, b in ev[1:]]
    algo = (D + 1) * n * 4
    rows = []
    for v, t in results.items():
        med = statistics.median(t)
        rows.append({"pad_elems": v[0], "out": v[1], "block": v[2], "ms_median": round(med, 4),
                     "ms_min": round(min(t), 4), "GBs": round(algo / med / 1e6, 1)})
    rows.sort(key=lambda r: r["ms_median"])
    for r in rows:
        print(json.dumps(r))


if __name__ == "__main__":
    main()
