#!/usr/bin/env python3
"""Compute-node state sync (fa_sync_part) under the context tuning space, on one GPU.

  python tools/sync_sweep.py [workload=c2] [steps=20]

For the sync leg of bench.py (SyncSetup: D client copies of a bucket synced in place) this times every
store policy x grid cap x block of fa_tuning, and beside them the independent in-place read+write ceiling
on the same slots (bench.rw_plain_peak).  One JSON line per form; GB/s counts reads and writes.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "c2"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    import bench
    import torch
    fa = bench.load_pkg()
    fa.lib()
    stream = torch.cuda.Stream()
    D, n, si, so, _ = bench.WORKLOADS[wl]
    s = bench.SyncSetup(fa, torch, D, n, si, so, 0, 0)
    cp = bench.rw_plain_peak(fa, torch, s, stream)
    print(json.dumps({"workload": wl, "D": D, "n": n, "sets": s.nsets, "copy_ceiling_GBs": cp["GBs"],
                      "form": cp["form"]}), flush=True)
    for block in (128, 256):
        for mb in (-1, 2048, 4096, 8192, 16384):
            for sp in (1, 2, 3, 4):
                s.agg.set_tuning(block=block, max_blocks=mb, store_policy=sp)
                torch.cuda.synchronize()
                _, ka, km = bench.timed_loop(torch, s, steps, 3, stream, None, lambda: None)
                gbs = s.algo_bytes() / (ka * 1e-3) / 1e9
                print(json.dumps({"block": block, "max_blocks": mb, "store_policy": sp, "ms": round(ka, 4),
                                  "GBs": round(gbs, 1), "frac_of_copy": round(gbs / cp["GBs"], 4)}), flush=True)
    s.agg.set_tuning(block=128, max_blocks=-1, store_policy=3)
    print(json.dumps({"parity": s.parity(0)["ok"]}), flush=True)
    s.close()


if __name__ == "__main__":
    main()
