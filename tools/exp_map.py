#!/usr/bin/env python3
"""Experiment (GPU box): FedAvg reduce speed vs absolute position inside one large
allocation.  A WINDOW = 32 clients + output of 128 MiB each (4.1 GiB) placed at
consecutive offsets of a `GiB`-sized hipMalloc arena; every window is timed in
interleaved rounds.

  python tools/exp_map.py [arena_GiB]
"""
import ctypes
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
    hip = ctypes.CDLL("libamdhip64.so.7")
    hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
    gib = int(sys.argv[1]) if len(sys.argv) > 1 else 96
    n, D = 32 << 20, 32
    cb = n * 4
    wbytes = (D + 1) * cb
    p = ctypes.c_void_p()
    rc = hip.hipMalloc(ctypes.byref(p), gib << 30)
    if rc:
        sys.exit("alloc failed %d" % rc)
    base = p.value
    nwin = (gib << 30) // wbytes
    fa.fill_uniform(base, (gib << 30) // 4, fa.F32, 3, 0)
    w = bench.Setup._weights(D)
    fa.set_tuning(block=128, max_blocks=-1, unroll=16, load_policy=2, store_policy=2)
    stream = torch.cuda.Stream()
    torch.cuda.synchronize()
    res = {i: [] for i in range(nwin)}
    for rnd in range(3):
        for i in range(nwin):
            o = base + i * wbytes
            clients = [o + k * cb for k in range(D)]
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(3)]
            for x, y in ev:
                x.record(stream)
                fa.reduce_device(clients, w, n, fa.F32, o + D * cb, fa.F32, stream=stream)
                y.record(stream)
            torch.cuda.synchronize()
            res[i] += [x.elapsed_time(y) for x, y in ev[1:]]
    meds = [round(statistics.median(res[i]), 4) for i in range(nwin)]
    print(json.dumps({"window_GiB": round(wbytes / 2**30, 3), "arena_GiB": gib, "ms": meds,
                      "TBs": [round(wbytes / m / 1e9, 2) for m in meds]}))


if __name__ == "__main__":
    main()
