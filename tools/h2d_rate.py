#!/usr/bin/env python3
"""Host-inclusive aggregation rate (GPU box tool): client buckets start in host
memory (as they arrive from network_layer.cpp's receiver) and the reduced
bucket ends in host memory (as it leaves through new_message()).

One round = D x fa_submit (or fa_submit_pinned) + fa_finalize (reduce + D2H).
Reports GiB/s of client input per round, for pageable and pinned host buffers,
and the device-resident rate of the same round for comparison.

  python tools/h2d_rate.py [D] [n_log2] [rounds] [shards]

shards > 1 runs a range-sharded context of that many shards; on a one-GPU box they share GPU 0
(FA_TEST_SHARED_DEVICE), so the PCIe link is the same and an unchanged rate shows that the shards'
copies overlap (the host side issues every shard's H2D / D2H before it waits for any).
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    import numpy as np
    import torch
    fa = bench.load_pkg()
    fa.lib()
    D = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    n = 1 << int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 26
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    shards = int(sys.argv[4]) if len(sys.argv) > 4 else 1
    w = bench.Setup._weights(D)
    rng = np.random.default_rng(0)
    # at most 8 distinct host buffers, client k uses buffer k % 8 (timing does not depend on values; keeps
    # C5's share, 128 x 128 MiB, at 1 GiB of pageable + 1 GiB of pinned host memory)
    pageable = [rng.uniform(-1, 1, n).astype(np.float32) for _ in range(min(D, 8))]
    pinned = []
    for x in pageable:
        t = torch.empty(n, dtype=torch.float32, pin_memory=True)
        t.numpy()[:] = x
        pinned.append(t)
    out = np.empty(n, np.float32)
    # modes: pageable (fa_submit / fa_finalize of numpy arrays), pinned (fa_submit_pinned, pageable result),
    # pinned_io (pinned receipts and the result DMA'd straight into pinned memory: fa_finalize_gather with
    # FA_HOST_PINNED, the drop-in aggregator's own path, host/aggregator_main.cpp)
    modes = os.environ.get("H2D_MODES", "pageable,pinned").split(",")
    out_pinned = fa.PinnedBuffer(n * 4) if "pinned_io" in modes else None
    res = {"D": D, "n": n, "bytes_per_client": n * 4, "distinct_host_buffers": len(pageable), "shards": shards}
    if shards == 1:
        ctx = fa.Aggregator(1)
    elif fa.device_count() >= shards:
        ctx = fa.Aggregator(shards)
    else:
        ctx = fa.Aggregator(devices=[0] * shards, shared_device=True)
        res["shared_device"] = True
    with ctx as agg:
        agg.define(1, n, fa.F32, fa.F32, D, fa.FEDAVG)
        for mode in modes:
            times = []
            for r in range(rounds + 1):
                t0 = time.perf_counter()
                for k in range(D):
                    if mode in ("pinned", "pinned_io"):
                        agg.submit(1, k, pinned[k % len(pinned)].numpy(), w[k], pinned=True)
                    else:
                        agg.submit(1, k, pageable[k % len(pageable)], w[k])
                if mode == "pinned_io":
                    agg.finalize_gather(1, [out_pinned.view(np.float32, count=n)], pinned=True)
                else:
                    agg.finalize(1, out)
                times.append(time.perf_counter() - t0)
            t = min(times[1:])
            res[mode] = {"round_s": round(t, 4), "GiB_s_input": round(D * n * 4 / t / 2**30, 2),
                         "GB_s_pcie_bytes": round((D + 1) * n * 4 / t / 1e9, 2)}
        if shards > 1:
            print(json.dumps(res))
            return
        # device-resident round on the same slots
        stream = torch.cuda.Stream()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(5)]
        for a, b in ev:
            a.record(stream)
            agg.reduce(1, w, stream=stream)
            b.record(stream)
        torch.cuda.synchronize()
        ms = min(a.elapsed_time(b) for a, b in ev[1:])
        res["device_resident"] = {"round_ms": round(ms, 4), "GiB_s_input": round(D * n * 4 / ms / 1e-3 / 2**30, 1)}
        agg.sync()
    # Drain before exit: the context is destroyed (fa_destroy synchronizes its streams), then the whole device,
    # and the profiler gets a moment to deliver its last copy records (a marker trace of this tool lost its
    # DEVICE_TO_HOST rows to "completion callbacks were not delivered" at exit, gpurun_out r03s46).
    torch.cuda.synchronize()
    if out_pinned is not None:
        out_pinned.close()
    time.sleep(float(os.environ.get("H2D_EXIT_DRAIN_S", "2")))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
