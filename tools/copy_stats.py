#!/usr/bin/env python3
"""Both directions of a host-inclusive round's copies from one rocprofv3 run (round 4).

`rocprofv3 --marker-trace --kernel-trace --memory-copy-trace` of tools/h2d_rate.py records every
HOST_TO_DEVICE copy as a memory-copy record (SDMA), but no DEVICE_TO_HOST one: on this ROCm stack the HIP
runtime performs device-to-host copies with its blit kernel `__amd_rocclr_copyBuffer` (the GPU writes the
host memory over PCIe), which the kernel trace records -- and for which rocprofiler-sdk's async-copy
tracer waits in vain at exit ("N completion callbacks were not delivered", one per D2H copy;
tools/copy_trace_probe.py shows the same for torch's own x.cpu() and pinned copy_, gpurun_out r04s04).
So the D2H half is read from the kernel trace here.

  python tools/copy_stats.py <rocprofv3 output dir> <out.csv> [pinned_round_json]

Writes one CSV (HOST_TO_DEVICE from the memory-copy trace, DEVICE_TO_HOST from the copyBuffer dispatches,
with bytes and GB/s where the marker trace names the sizes) and prints a JSON breakdown of the run: host
ranges per entry (fa_submit*, fa_finalize*, fa_copy_output, fa_reduce*), device time per kind.
"""
import collections
import csv
import glob
import json
import os
import sys


def rows(d, suffix):
    f = glob.glob(os.path.join(d, "**", "*" + suffix), recursive=True)
    return list(csv.DictReader(open(f[0]))) if f else []


def dur(r):
    return int(r["End_Timestamp"]) - int(r["Start_Timestamp"])


def main():
    d, out = sys.argv[1], sys.argv[2]
    copies = rows(d, "memory_copy_trace.csv")
    kernels = rows(d, "kernel_trace.csv")
    markers = rows(d, "marker_api_trace.csv")
    per = collections.defaultdict(list)
    for r in copies:
        per[r["Direction"].replace("MEMORY_COPY_", "")].append(dur(r))
    blits = [r for r in kernels if "__amd_rocclr_copyBuffer" in r["Kernel_Name"]]
    for r in blits:
        per["DEVICE_TO_HOST"].append(dur(r))
    reductions = [dur(r) for r in kernels if "fedavg" in r["Kernel_Name"]]
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs", "Source"])
        for name, src in (("HOST_TO_DEVICE", "memory-copy trace (SDMA)"),
                          ("DEVICE_TO_HOST", "kernel trace: __amd_rocclr_copyBuffer (HIP's blit kernel)")):
            v = per.get(name, [])
            if v:
                w.writerow(["MEMORY_COPY_" + name, len(v), sum(v), round(sum(v) / len(v), 1), min(v), max(v), src])
        if reductions:
            w.writerow(["KERNEL_fedavg_reduce", len(reductions), sum(reductions),
                        round(sum(reductions) / len(reductions), 1), min(reductions), max(reductions), "kernel trace"])
    host = collections.defaultdict(list)
    for r in markers:
        name = r.get("Function") or r.get("Name") or ""
        key = name.split(" part")[0].split(" slot")[0].split(" n ")[0].split(" D ")[0]
        if "Start_Timestamp" in r and "End_Timestamp" in r:
            host[key].append(dur(r))
    res = {"device_ns": {k: {"calls": len(v), "total": sum(v), "avg": round(sum(v) / len(v), 1)} for k, v in per.items()},
           "reduce_kernel_ns": {"calls": len(reductions), "total": sum(reductions)},
           "host_range_ns": {k: {"calls": len(v), "total": sum(v)} for k, v in sorted(host.items())}}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
