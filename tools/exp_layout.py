#!/usr/bin/env python3
"""Experiment (GPU box): is the FedAvg kernel's speed a property of the per-client
skew or of where an allocation happens to land physically?

For each skew (`pad` fp32 elements between consecutive client buckets inside
one pool) this allocates REPS independent pools, interleaving allocation order,
and times the reduce on every pool in interleaved rounds in one process.  A skew
effect shows as a shift of all REPS pools; a placement effect as spread within
one skew.

  python tools/exp_layout.py [n_log2] [reps] [pads...]
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
    n = 1 << int(sys.argv[1]) if len(sys.argv) > 1 else 32 << 20
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    pads = [int(x) for x in sys.argv[3:]] or [0, 64, 128, 1024]
    D = 32
    w = bench.Setup._weights(D)
    fa.set_tuning(block=128, max_blocks=-1, unroll=8, load_policy=2, store_policy=2)
    stream = torch.cuda.Stream()
    pools = {}
    for r in range(reps):
        for pad in pads:
            pool = torch.empty((D + 1) * (n + pad), dtype=torch.float32, device="cuda")
            clients = [pool[k * (n + pad): k * (n + pad) + n] for k in range(D)]
            for k, c in enumerate(clients):
                fa.fill_uniform(c, n, fa.F32, 0x5EED, k)
            pools[(pad, r)] = (pool, clients, pool[D * (n + pad): D * (n + pad) + n])
    torch.cuda.synchronize()
    results = {key: [] for key in pools}
    for rnd in range(4):
        for key, (pool, clients, out) in pools.items():
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(4)]
            for a, b in ev:
                a.record(stream)
                fa.reduce_device(clients, w, n, fa.F32, out, fa.F32, stream=stream)
                b.record(stream)
            torch.cuda.synchronize()
            results[key] += [a.elapsed_time(b) for a, b in ev[1:]]
    algo = (D + 1) * n * 4
    for pad in pads:
        meds = [statistics.median(results[(pad, r)]) for r in range(reps)]
        print(json.dumps({"pad_elems": pad, "pool_ms_medians": [round(m, 4) for m in meds],
                          "GBs": [round(algo / m / 1e6) for m in meds],
                          "base_mod_2MiB": [pools[(pad, r)][0].data_ptr() % (2 << 20) for r in range(reps)],
                          "base_GiB": [round(pools[(pad, r)][0].data_ptr() / 2**30, 2) for r in range(reps)]}))


if __name__ == "__main__":
    main()
