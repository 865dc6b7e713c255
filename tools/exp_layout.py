#!/usr/bin/env python3
"""Experiment (GPU box): does the placement of the D client buckets in HBM matter?

All buckets allocated separately sit at the same offset modulo their (2 MiB
aligned) size, so lane l of a wave reads the same low address bits from all U
clients it loads at once.  This places the D buckets in one pool with a skew of
`pad` elements between them and times the north-star reduce for several skews
and cache policies, interleaved in rounds in one process.
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
    pads = [0, 64, 1024, 4096 + 64, 65536 + 1024, 262144 + 4096, 524288 + 32768]
    pools = {}
    stream = torch.cuda.Stream()
    out = torch.empty(n, dtype=torch.float32, device="cuda")
    variants = []
    for pad in pads:
        pool = torch.empty(D * (n + pad), dtype=torch.float32, device="cuda")
        clients = [pool[k * (n + pad): k * (n + pad) + n] for k in range(D)]
        for k, c in enumerate(clients):
            fa.fill_uniform(c, n, fa.F32, 0x5EED, k)
        torch.cuda.synchronize()
        pools[pad] = (pool, clients)
        for nt in (1, 2):
            for unroll in (8, 16):
                variants.append((pad, nt, unroll))
        # keep memory bounded: time this pool now, then free it
    results = {v: [] for v in variants}
    for rnd in range(4):
        for v in variants:
            pad, nt, unroll = v
            fa.set_tuning(block=256, max_blocks=-1, unroll=unroll, nontemporal=nt)
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
        rows.append({"pad_elems": v[0], "nt": v[1], "unroll": v[2], "ms_median": round(med, 4),
                     "ms_min": round(min(t), 4), "GBs": round(algo / med / 1e6, 1)})
    rows.sort(key=lambda r: r["ms_median"])
    for r in rows:
        print(json.dumps(r))


if __name__ == "__main__":
    main()
