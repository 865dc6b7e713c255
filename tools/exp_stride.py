#!/usr/bin/env python3
"""Experiment (GPU box): FedAvg reduce speed vs the relative placement of the 33
streams (32 clients + output) inside ONE allocation.

Arenas: a physically contiguous one (hipExtMallocWithFlags(hipDeviceMallocContiguous))
and a plain hipMalloc one.  Layouts place client k at k * stride (+ optional
per-client jitter) and the output after the last client.  All layouts share the
arena (timing only; the values are garbage after the first launch).

  python tools/exp_stride.py [n_log2]
"""
import ctypes
import json
import os
import random
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

MiB = 1 << 20


def main():
    import torch
    fa = bench.load_pkg()
    fa.lib()
    hip = ctypes.CDLL("libamdhip64.so.7")
    hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
    hip.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
    n = 1 << int(sys.argv[1]) if len(sys.argv) > 1 else 32 << 20
    D = 32
    cb = n * 4
    w = bench.Setup._weights(D)
    fa.set_tuning(block=128, max_blocks=-1, unroll=16, load_policy=2, store_policy=2)
    rng = random.Random(7)
    layouts = {
        "pow2": [k * cb for k in range(D + 1)],
        "+256B": [k * (cb + 256) for k in range(D + 1)],
        "+512B": [k * (cb + 512) for k in range(D + 1)],
        "+4KiB": [k * (cb + 4096) for k in range(D + 1)],
        "+64KiB": [k * (cb + 65536) for k in range(D + 1)],
        "+2MiB": [k * (cb + 2 * MiB) for k in range(D + 1)],
        "+2MiB+256B": [k * (cb + 2 * MiB + 256) for k in range(D + 1)],
        "+6MiB": [k * (cb + 6 * MiB) for k in range(D + 1)],
        "+6MiB+512B": [k * (cb + 6 * MiB + 512) for k in range(D + 1)],
        "jitter": [k * (cb + 8 * MiB) + rng.randrange(0, 4 * MiB, 256) for k in range(D + 1)],
    }
    span = max(max(v) for v in layouts.values()) + cb
    stream = torch.cuda.Stream()
    arenas = {}
    for name, flag in (("contiguous", 0x4), ("hipMalloc", None)):
        p = ctypes.c_void_p()
        rc = hip.hipMalloc(ctypes.byref(p), span) if flag is None else hip.hipExtMallocWithFlags(
            ctypes.byref(p), span, flag)
        if rc:
            print(json.dumps({"arena": name, "alloc_error": rc}))
            continue
        fa.fill_uniform(p.value, span // 4, fa.F32, 1, 0)
        arenas[name] = p.value
    torch.cuda.synchronize()
    res = {(a, l): [] for a in arenas for l in layouts}
    for rnd in range(4):
        for (a, l) in res:
            base = arenas[a]
            offs = layouts[l]
            clients = [base + o for o in offs[:D]]
            out = base + offs[D]
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(4)]
            for x, y in ev:
                x.record(stream)
                fa.reduce_device(clients, w, n, fa.F32, out, fa.F32, stream=stream)
                y.record(stream)
            torch.cuda.synchronize()
            res[(a, l)] += [x.elapsed_time(y) for x, y in ev[1:]]
    algo = (D + 1) * cb
    for a in arenas:
        row = {"arena": a}
        for l in layouts:
            m = statistics.median(res[(a, l)])
            row[l] = [round(m, 4), round(algo / m / 1e6)]
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
