#!/usr/bin/env python3
"""Experiment (GPU box): FedAvg reduce speed vs how the client pool is allocated.

Methods: torch caching allocator, plain hipMalloc, hipExtMallocWithFlags with
hipDeviceMallocContiguous.  REPS pools per method, timed in interleaved rounds.

  python tools/exp_alloc.py [n_log2] [reps]
"""
import ctypes
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

HIP_CONTIGUOUS = 0x4


def main():
    import torch
    fa = bench.load_pkg()
    fa.lib()
    hip = ctypes.CDLL("libamdhip64.so.7")
    hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
    hip.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
    n = 1 << int(sys.argv[1]) if len(sys.argv) > 1 else 32 << 20
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    D = 32
    w = bench.Setup._weights(D)
    fa.set_tuning(block=128, max_blocks=-1, unroll=8, load_policy=2, store_policy=2)
    stream = torch.cuda.Stream()
    nbytes = (D + 1) * n * 4
    pools = {}
    keep = []
    for r in range(reps):
        for method in ("torch", "hipMalloc", "contiguous"):
            if method == "torch":
                t = torch.empty((D + 1) * n, dtype=torch.float32, device="cuda")
                keep.append(t)
                base = t.data_ptr()
            else:
                p = ctypes.c_void_p()
                rc = (hip.hipMalloc(ctypes.byref(p), nbytes) if method == "hipMalloc"
                      else hip.hipExtMallocWithFlags(ctypes.byref(p), nbytes, HIP_CONTIGUOUS))
                if rc != 0:
                    print(json.dumps({"method": method, "rep": r, "alloc_error": rc}), flush=True)
                    continue
                base = p.value
            clients = [base + k * n * 4 for k in range(D)]
            for k, c in enumerate(clients):
                fa.fill_uniform(c, n, fa.F32, 0x5EED, k)
            pools[(method, r)] = (clients, base + D * n * 4)
    torch.cuda.synchronize()
    results = {key: [] for key in pools}
    for rnd in range(4):
        for key, (clients, out) in pools.items():
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(4)]
            for a, b in ev:
                a.record(stream)
                fa.reduce_device(clients, w, n, fa.F32, out, fa.F32, stream=stream)
                b.record(stream)
            torch.cuda.synchronize()
            results[key] += [a.elapsed_time(b) for a, b in ev[1:]]
    algo = (D + 1) * n * 4
    for method in ("torch", "hipMalloc", "contiguous"):
        meds = [statistics.median(results[(method, r)]) for r in range(reps) if (method, r) in results]
        print(json.dumps({"method": method, "pool_ms_medians": [round(m, 4) for m in meds],
                          "GBs": [round(algo / m / 1e6) for m in meds]}), flush=True)


if __name__ == "__main__":
    main()
