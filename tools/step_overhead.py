#!/usr/bin/env python3
"""Wall time per bench step with and without per-step HIP events (GPU box tool).

  python tools/step_overhead.py [workloads=northstar,ns_w8,ns_w4,c2] [steps=20] [reps=5]

bench.py's timed loop records an event pair around every launch (the roofline's kernel time); this
measures what those events add to the wall-clock step time that `value` is computed from: for each
workload, alternately, `steps` launches back to back with an event pair around each, and the same
launches with no events, each bracketed by synchronize, median over `reps` repetitions.
"""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    names = sys.argv[1].split(",") if len(sys.argv) > 1 else ["northstar", "ns_w8", "ns_w4", "c2"]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    import bench
    import torch
    fa = bench.load_pkg()
    fa.lib()
    stream = torch.cuda.Stream()
    for name in names:
        D, n, i, o, _ = bench.WORKLOADS[name]
        s = bench.Setup(fa, torch, D, n, i, o, 0, 0)
        for k in range(5):
            s.launch(k, stream)
        torch.cuda.synchronize()
        res = {"events": [], "plain": [], "kernel_ms": []}
        for _ in range(reps):
            for mode in ("events", "plain"):
                evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                       for _ in range(steps)] if mode == "events" else None
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for k in range(steps):
                    if evs:
                        evs[k][0].record(stream)
                    s.launch(k, stream)
                    if evs:
                        evs[k][1].record(stream)
                torch.cuda.synchronize()
                res[mode].append((time.perf_counter() - t0) / steps * 1e3)
                if evs:
                    res["kernel_ms"].append(statistics.mean(a.elapsed_time(b) for a, b in evs))
        out = {"workload": name, "steps": steps, "reps": reps}
        for k, v in res.items():
            out[k + "_ms_per_step_median"] = round(statistics.median(v), 4)
        out["events_cost_us_per_step"] = round((out["events_ms_per_step_median"] - out["plain_ms_per_step_median"]) * 1e3, 2)
        out["plain_minus_kernel_us"] = round((out["plain_ms_per_step_median"] - out["kernel_ms_ms_per_step_median"]) * 1e3, 2)
        print(json.dumps(out), flush=True)
        s.close()


if __name__ == "__main__":
    main()
