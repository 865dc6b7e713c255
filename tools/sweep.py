#!/usr/bin/env python3
"""Tuning sweep of the FedAvg kernel on a bench workload (GPU box tool).

  python tools/sweep.py [workload]   SWEEP_BLOCKS / SWEEP_MAXBLOCKS / SWEEP_UNROLLS / SWEEP_STORES / SWEEP_WALKS / SWEEP_POOLS:
                                     comma lists

Interleaves every configuration in rounds inside one process (rule: A/B deltas
come from one process), prints one JSON line per configuration with the median
and min kernel time over all rounds.
"""
import itertools
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
    workload = sys.argv[1] if len(sys.argv) > 1 else "northstar"
    D, n, i, o, _ = bench.WORKLOADS[workload]
    pools = int(os.environ.get("SWEEP_POOLS", "3"))
    setups = [bench.Setup(fa, torch, D, n, i, o, 0, 0) for _ in range(pools)]  # placement varies per pool
    setup = setups[0]
    stream = torch.cuda.Stream()
    def env_list(name, default):
        v = os.environ.get(name)
        return [int(x) for x in v.split(",")] if v else default
    grid = list(itertools.product(env_list("SWEEP_BLOCKS", [128, 256]), env_list("SWEEP_MAXBLOCKS", [0]), env_list("SWEEP_UNROLLS", [8, 16]), [2],
                                  env_list("SWEEP_STORES", [1, 2, 3, 4]), env_list("SWEEP_WALKS", [1])))
    times = {(g, p): [] for g in grid for p in range(pools)}
    for rnd in range(3):
        for g in grid:
            fa.set_tuning(block=g[0], max_blocks=g[1] if g[1] else -1, unroll=g[2], load_policy=g[3],
                          store_policy=g[4], walk=g[5])
            for p, st in enumerate(setups):
                ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(4)]
                for a, b in ev:
                    a.record(stream)
                    st.launch(0, stream)
                    b.record(stream)
                torch.cuda.synchronize()
                times[(g, p)] += [a.elapsed_time(b) for a, b in ev[1:]]
    rows = []
    for g in grid:
        meds = [statistics.median(times[(g, p)]) for p in range(pools)]
        med = statistics.mean(meds)
        rows.append({"block": g[0], "max_blocks": g[1], "unroll": g[2], "load_policy": g[3], "store_policy": g[4],
                     "walk": g[5],
                     "ms_mean_of_pool_medians": round(med, 4), "pool_ms": [round(m, 4) for m in meds],
                     "GBs": round(setup.algo_bytes() / med / 1e6, 1)})
    rows.sort(key=lambda r: r["ms_mean_of_pool_medians"])
    for r in rows:
        print(json.dumps(r))


if __name__ == "__main__":
    main()
