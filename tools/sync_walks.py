#!/usr/bin/env python3
"""Compute-node state sync (fa_sync_part) under different grid walks, interleaved in one process
(GPU box tool).  Default shape: 8 client copies of VGG-19's FC part (119.6 M fp32 parameters).

  python tools/sync_walks.py [D] [n] [walks=2,5] [rounds=3]
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
    D = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 119_586_826
    walks = [int(x) for x in (sys.argv[3] if len(sys.argv) > 3 else "2,5").split(",")]
    rounds = int(sys.argv[4]) if len(sys.argv) > 4 else 3
    s = bench.SyncSetup(fa, torch, D, n, "f32", "f32", 0, 0)
    stream = torch.cuda.Stream()
    times = {w: [] for w in walks}
    for _ in range(rounds):
        for w in walks:
            fa.set_tuning(walk=w)
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(5)]
            for a, b in ev:
                a.record(stream)
                s.launch(0, stream)
                b.record(stream)
            torch.cuda.synchronize()
            times[w] += [a.elapsed_time(b) for a, b in ev[1:]]
    for w in walks:
        med = statistics.median(times[w])
        print(json.dumps({"walk": w, "D": D, "n": n, "median_ms": round(med, 4),
                          "GBs_2Ds": round(s.algo_bytes() / med / 1e6, 1)}))
    s.close()


if __name__ == "__main__":
    main()
