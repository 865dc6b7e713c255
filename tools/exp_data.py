#!/usr/bin/env python3
"""Experiment (GPU box): does the reduction's time depend on the VALUES in the client buckets?

The placement probe of fa_bucket_define times uninitialized pools (1.28 ms for the north star) while
the bench, over uniform[-1,1) data in the same pool, measures 1.32-1.34 ms.  This times one pool
(north-star shape) with different contents, interleaved in rounds in one process:
  random  fill_uniform (the bench's data)      zeros   all bits 0
  ones    every element 1.0f (0x3f800000)      alt     0x55555555 / 0xAAAAAAAA alternating per client
A value dependence with identical addresses and instructions points at power (HBM I/O toggling),
not at the access pattern.

  python tools/exp_data.py [rounds] [launches]
"""
import ctypes
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    launches = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    import torch
    fa = bench.load_pkg()
    fa.lib()
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemsetD32.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t]
    D, n, i, o, _ = bench.WORKLOADS["northstar"]
    s = bench.Setup(fa, torch, D, n, i, o, 0, 0)
    stream = torch.cuda.Stream()

    def fill(pattern):
        for k in range(D):
            ptr, cnt, _ = s.agg.slot(0, 0, k)
            if pattern == "random":
                fa.fill_uniform(ptr, cnt, fa.F32, 0x5EED, k)
            else:
                val = {"zeros": 0, "ones": 0x3F800000, "alt": 0x55555555 if k % 2 == 0 else 0xAAAAAAAA - (1 << 32)}[pattern]
                assert hip.hipMemsetD32(ctypes.c_void_p(ptr), val, cnt) == 0
        torch.cuda.synchronize()

    patterns = ["random", "zeros", "ones", "alt"]
    times = {p: [] for p in patterns}
    for _ in range(rounds):
        for p in patterns:
            fill(p)
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(launches)]
            for a, b in ev:
                a.record(stream)
                s.launch(0, stream)
                b.record(stream)
            torch.cuda.synchronize()
            times[p] += [a.elapsed_time(b) for a, b in ev[1:]]
    for p in patterns:
        med = statistics.median(times[p])
        print(json.dumps({"pattern": p, "median_ms": round(med, 4), "min_ms": round(min(times[p]), 4),
                          "GBs": round(s.algo_bytes() / med / 1e6, 1), "placement": s.placement}))
    s.close()


if __name__ == "__main__":
    main()
