#!/usr/bin/env python3
"""Would range sub-shards inside one GPU pay? (GPU box diagnostic; DESIGN.md 4, round 3 "the address span")

  python tools/subshard_probe.py [launches=8] [configs=c4:5,c5:8]

For a config D x n (C4: 64 x 139.6 M, C5: 128 x 268 M fp32) and S sub-shards this times, with HIP events on
one stream (median over `launches`):
  * whole -- the product's launch over one pool (every client's bucket one contiguous slot);
  * split -- the same bytes as S pools of D slots of n/S elements each (what a range-major layout inside one
             GPU would hold), reduced by S launches back to back: each launch's clients span D * n/S * 4 bytes
             instead of D * n * 4.
Same elements reduced, same algorithmic bytes (one output per element).  Prints one JSON line per config.
"""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SHAPES = {"c4": (64, 139_611_210), "c5": (128, 1 << 28)}


def timed(torch, stream, fn, launches):
    evs = []
    for k in range(launches + 3):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        fn(k)
        b.record(stream)
        evs.append((a, b))
    torch.cuda.synchronize()
    return statistics.median([a.elapsed_time(b) for a, b in evs[3:]])


def main():
    launches = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    configs = [c.split(":") for c in (sys.argv[2] if len(sys.argv) > 2 else "c4:5,c5:8").split(",")]
    import torch
    import bench
    fa = bench.load_pkg()
    fa.lib()
    stream = torch.cuda.Stream()
    for name, S in configs:
        S = int(S)
        D, n = SHAPES[name]
        algo = (D + 1) * n * 4
        s = bench.Setup(fa, torch, D, n, "f32", "f32", 0, 0)
        torch.cuda.synchronize()
        whole = timed(torch, stream, lambda k: s.launch(k, stream), launches)
        s.close()
        per = (-(-n // S) + 63) // 64 * 64  # sub-shards of a multiple of 64 elements
        subs = []
        for i in range(S):
            lo, hi = min(n, i * per), min(n, (i + 1) * per)
            subs.append(bench.Setup(fa, torch, D, hi - lo, "f32", "f32", lo, 0, min_rotate_bytes=0))
        torch.cuda.synchronize()

        def split(k):
            for sub in subs:
                sub.launch(0, stream)
        sp = timed(torch, stream, split, launches)
        for sub in subs:
            sub.close()
        print(json.dumps({"config": name, "clients": D, "elems": n, "subshards": S,
                          "whole_ms": round(whole, 4), "whole_frac": round(algo / (whole * 1e-3) / 8e12, 4),
                          "split_ms": round(sp, 4), "split_frac": round(algo / (sp * 1e-3) / 8e12, 4)}), flush=True)


if __name__ == "__main__":
    main()
