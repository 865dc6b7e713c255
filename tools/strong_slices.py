#!/usr/bin/env python3
"""One rank's share of the strong-scaled north star, on one GPU: 32 clients x (64 Mi / W) fp32 elements.

  python tools/strong_slices.py [steps=20] [W list, default 1,2,4,8]

bench.py --gpus W (strong scaling) gives rank r the elements [r*n/W, (r+1)*n/W) of every client bucket
(aggregator.cpp:59-93 sharded per SURVEY.md 8e).  This times that per-rank launch alone for each W, so
the kernel that each slice size takes can be tuned on the one-GPU box.  One JSON line per W.
"""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    ws = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [1, 2, 4, 8]
    import bench
    import torch
    fa = bench.load_pkg()
    if os.environ.get("FA_BENCH_WALK"):  # A/B of fa_tuning.walk (process default, before any context)
        fa.set_tuning(walk=int(os.environ["FA_BENCH_WALK"]))
    fa.lib()
    stream = torch.cuda.Stream()
    D, n = 32, 64 << 20
    for W in ws:
        s = bench.Setup(fa, torch, D, n // W, "f32", "f32", 0, 0)
        torch.cuda.synchronize()
        wall, ka, km = bench.timed_loop(torch, s, steps, 5, stream, None, lambda: None)
        print(json.dumps({"W": W, "elems": n // W, "sets": s.nsets, "kernel_ms_avg": round(ka, 4),
                          "kernel_ms_min_per_launch_events": round(min(km), 4), "wall_ms": round(wall / steps * 1e3, 4),
                          "frac": round(s.algo_bytes() / (ka * 1e-3) / 1e9 / bench.HBM_PEAK_GBS, 4)}), flush=True)
        s.close()


if __name__ == "__main__":
    main()
