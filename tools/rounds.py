#!/usr/bin/env python3
"""Device time of one aggregator round on the buckets it forms (bench.ROUNDS), batched and per part.

  python tools/rounds.py [steps=20] [names, default round_c2,round_c3]

Under `rocprofv3 --kernel-trace --stats` this gives the per-kernel split of a round (profiles/).
One JSON line per (round, batched).
"""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    names = sys.argv[2].split(",") if len(sys.argv) > 2 else ["round_c2", "round_c3"]
    import bench
    import torch
    fa = bench.load_pkg()
    fa.lib()
    stream = torch.cuda.Stream()
    for name in names:
        for batched in (True, False):
            s = bench.RoundSetup(fa, torch, name, 0, batched=batched)
            torch.cuda.synchronize()
            wall, ka, km = bench.timed_loop(torch, s, steps, 5, stream, None, lambda: None)
            print(json.dumps({"round": name, "batched": batched, "sizes": s.sizes, "D": s.D,
                              "round_ms_avg": round(ka, 4), "round_ms_min_per_launch_events": round(min(km), 4),
                              "wall_ms": round(wall / steps * 1e3, 4),
                              "frac": round(s.algo_bytes() / (ka * 1e-3) / 1e9 / bench.HBM_PEAK_GBS, 4)}), flush=True)
            s.close()


if __name__ == "__main__":
    main()
