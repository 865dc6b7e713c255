#!/usr/bin/env python3
"""Experiment (GPU box): with the 32 input buckets fixed, does the OUTPUT buffer's
placement decide the reduce time?  Times the same inputs into K separately
allocated output buffers (hipMalloc) and into K outputs carved from one arena.

  python tools/exp_out.py [n_log2] [K]
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
    n = 1 << int(sys.argv[1]) if len(sys.argv) > 1 else 32 << 20
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    D = 32
    w = bench.Setup._weights(D)
    fa.set_tuning(block=128, max_blocks=-1, unroll=8, load_policy=2, store_policy=2)
    agg = fa.Aggregator(1)
    agg.define(0, n, fa.F32, fa.F32, D, fa.FEDAVG)
    clients = []
    for k in range(D):
        p, cnt, _ = agg.slot(0, 0, k)
        fa.fill_uniform(p, cnt, fa.F32, 1, k)
        clients.append(p)
    outs = {}
    for i in range(K):
        p = ctypes.c_void_p()
        assert hip.hipMalloc(ctypes.byref(p), n * 4) == 0
        outs["sep%d" % i] = p.value
    arena = ctypes.c_void_p()
    assert hip.hipMalloc(ctypes.byref(arena), K * n * 4) == 0
    for i in range(K):
        outs["arena%d" % i] = arena.value + i * n * 4
    outs["ctx_out"] = agg.output(0)
    stream = torch.cuda.Stream()
    torch.cuda.synchronize()
    res = {k: [] for k in outs}
    for rnd in range(4):
        for name, o in outs.items():
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(4)]
            for a, b in ev:
                a.record(stream)
                fa.reduce_device(clients, w, n, fa.F32, o, fa.F32, stream=stream)
                b.record(stream)
            torch.cuda.synchronize()
            res[name] += [a.elapsed_time(b) for a, b in ev[1:]]
    print(json.dumps({name: round(statistics.median(t), 4) for name, t in res.items()}))
    print(json.dumps({name: "%x" % (o % (1 << 32)) for name, o in outs.items()}))


if __name__ == "__main__":
    main()
