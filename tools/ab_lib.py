#!/usr/bin/env python3
"""A/B of two builds of the package on one bench workload (GPU box tool).

  python tools/ab_lib.py PKG_DIR [workload=northstar] [launches=30]      (workload "sync:<w>": state sync; round_c2/c3/c4: one round)
  AB_TUNE="slot_skew=4096,..." sets the process tuning defaults (fa_set_tuning) before the context exists.

PKG_DIR holds an ``__init__.py`` and ``lib/libfa.so`` (e.g. a build of an earlier commit); the
workload's buckets are set up through that build's own context and timed with HIP events on
one stream.  Run the builds alternately in separate processes on the same box.
"""
import importlib.util
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    pkg_dir = os.path.abspath(sys.argv[1])
    workload = sys.argv[2] if len(sys.argv) > 2 else "northstar"
    launches = int(sys.argv[3]) if len(sys.argv) > 3 else 30
    import torch
    spec = importlib.util.spec_from_file_location("mhfsl_amd", os.path.join(pkg_dir, "__init__.py"),
                                                  submodule_search_locations=[pkg_dir])
    fa = importlib.util.module_from_spec(spec)
    sys.modules["mhfsl_amd"] = fa
    spec.loader.exec_module(fa)
    fa.lib()
    tune = os.environ.get("AB_TUNE", "")  # e.g. "slot_skew=4096,rs_chunks=4": process tuning defaults
    if tune:
        fa.set_tuning(**{k: int(v) for k, v in (kv.split("=") for kv in tune.split(","))})
    import bench  # noqa: E402  (finds the package above in sys.modules)
    sync = workload.startswith("sync:")  # compute-node state sync (fa_sync_part) on a workload's shape
    if workload in bench.ROUNDS:  # one aggregator round on its own buckets (bench.RoundSetup)
        s = bench.RoundSetup(fa, torch, workload, 0)
    else:
        D, n, i, o, _ = bench.WORKLOADS[workload[5:] if sync else workload]
        s = (bench.SyncSetup if sync else bench.Setup)(fa, torch, D, n, i, o, 0, 0)
    stream = torch.cuda.Stream()
    evs = []
    for k in range(launches):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        s.launch(k, stream)
        b.record(stream)
        evs.append((a, b))
    torch.cuda.synchronize()
    ms = [a.elapsed_time(b) for a, b in evs[5:]]
    print(json.dumps({"pkg": pkg_dir, "workload": workload, "median_ms": round(statistics.median(ms), 4),
                      "min_ms": round(min(ms), 4)}))
    s.close()


if __name__ == "__main__":
    main()
