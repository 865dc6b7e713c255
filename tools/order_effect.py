#!/usr/bin/env python3
"""Does a leg run slower right after a large allocation was freed in the same process? (experiment)

  python tools/order_effect.py [gib=129] [fa|torch|idle|ctx|ctx-small|fa-keep|torch-hi|torch-lo|alloc-only]

Keeps the c4 workload (bench.WORKLOADS["c4"], 36 GB) resident, times it, then allocates and frees `gib` GiB
(C5's 129 GiB by default, as bench.py's secondaries do before the round legs) and times c4 again at
intervals after the free.  A slowdown that fades with time is the driver clearing the freed memory in the
background.  One JSON line per measurement.
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    gib = float(sys.argv[1]) if len(sys.argv) > 1 else 129
    import bench
    import torch
    fa = bench.load_pkg()
    fa.lib()
    if len(sys.argv) > 2 and sys.argv[2] == "alloc-only":  # allocate, fill and free `gib` GiB, then exit
        big = bench.Setup(fa, torch, max(1, int(gib)), 1 << 28, "f32", "f32", 0, 0)
        torch.cuda.synchronize()
        big.close()
        return
    stream = torch.cuda.Stream()
    D, n, i, o, _ = bench.WORKLOADS["c4"]
    s = bench.Setup(fa, torch, D, n, i, o, 0, 0)

    def measure(tag, t0=None):
        torch.cuda.synchronize()
        t = time.perf_counter()
        _, ka, _ = bench.timed_loop(torch, s, 10, 2, stream, None, lambda: None, per_launch=1)
        print(json.dumps({"when": tag, "t_after_free_s": None if t0 is None else round(t - t0, 3),
                          "ms_avg": round(ka, 4),
                          "frac": round(s.algo_bytes() / (ka * 1e-3) / 1e9 / bench.HBM_PEAK_GBS, 4)}), flush=True)

    time.sleep(5)
    measure("before")
    measure("before")
    mode = sys.argv[2] if len(sys.argv) > 2 else "fa"
    if mode == "fa":  # gib GiB in 1 GiB client slots of one bucket (range pieces of <= 16 GiB), filled, freed
        big = bench.Setup(fa, torch, max(1, int(gib)), 1 << 28, "f32", "f32", 0, 0)
        torch.cuda.synchronize()
        big.close()
    elif mode == "torch":  # the same bytes through torch's allocator, released to the driver
        big = [torch.ones(1 << 28, device="cuda") for _ in range(max(1, int(gib)))]
        torch.cuda.synchronize()
        del big
        torch.cuda.empty_cache()
    elif mode == "ctx":  # a libfa context created and destroyed, nothing defined
        a = fa.Aggregator(devices=[0])
        a.close()
    elif mode == "ctx-small":  # a libfa context with one small part (1 MiB slots), filled, destroyed
        big = bench.Setup(fa, torch, 4, 1 << 18, "f32", "f32", 0, 0)
        torch.cuda.synchronize()
        big.close()
    elif mode == "fa-keep":  # the libfa allocation, filled, then kept (no free) for the waits
        keep = bench.Setup(fa, torch, max(1, int(gib)), 1 << 28, "f32", "f32", 0, 0)
        torch.cuda.synchronize()
    elif mode == "torch-hi":  # a high-priority torch stream (its pool) created and used once
        hs = torch.cuda.Stream(priority=-1)
        with torch.cuda.stream(hs):
            torch.ones(16, device="cuda").sum()
        torch.cuda.synchronize()
    elif mode == "torch-lo":  # normal-priority streams beside it: one more used once
        ls = torch.cuda.Stream()
        with torch.cuda.stream(ls):
            torch.ones(16, device="cuda").sum()
        torch.cuda.synchronize()
    # mode "idle": nothing allocated, the same waits (a control)
    t0 = time.perf_counter()
    for wait in (0, 0.5, 1, 2, 3, 4, 6, 8, 12, 20):
        while time.perf_counter() - t0 < wait:
            time.sleep(0.01)
        measure("after_free", t0)
    s.close()


if __name__ == "__main__":
    main()
