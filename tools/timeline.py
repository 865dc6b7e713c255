#!/usr/bin/env python3
"""Per-workgroup timeline of the phased kernel (GPU box diagnostic; run with FA_TIMELINE=1).

  FA_TIMELINE=1 python tools/timeline.py [workloads, default northstar,ns_w2,ns_w4,ns_w8] [launches=8]

The kernel's thread 0 of every workgroup stamps the 100 MHz wall clock at its start, at its arrival at /
departure from the first and the last meeting (the last phase has none), and once its stores have completed (fedavg_phased_kernel,
FA_TIMELINE); fa_diag_phased_timeline copies them out after each launch.  Per workload this prints the
median over launches of: the start spread (dispatch ramp), the read time to the first meeting (min /
median / max over workgroups and per XCD = blockIdx % 8), the meeting wait, the last meeting's arrival
spread, the write time after it, and the whole span -- where a launch loses time against its bytes.
"""
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

TICK_US = 0.01  # 100 MHz


def summarize(tl, G):
    rows = [tl[b * 8:(b + 1) * 8] for b in range(G)]
    start = [r[0] for r in rows]
    t0 = min(start)
    us = lambda x: round(x * TICK_US, 2)  # noqa: E731
    whole = [r[5] - r[0] for r in rows]  # start to stores completed, per workgroup
    base = {
        "meetings": int(rows[0][6]),
        "span_us": us(max(r[5] for r in rows) - t0),
        "start_spread_us": us(max(start) - t0),
        "workgroup_us": {"min": us(min(whole)), "median": us(statistics.median(whole)), "max": us(max(whole))},
        "end_spread_us": us(max(r[5] for r in rows) - min(r[5] for r in rows)),
        "workgroup_median_per_xcd_us": {x: us(statistics.median(whole[x::8])) for x in range(8)},
    }
    if base["meetings"] == 0:  # a launch without meetings (one sized phase): the meeting stamps stay 0
        return base
    read0 = [r[1] - r[0] for r in rows]
    lds0 = [r[7] - r[0] for r in rows]  # phase 0's LDS part; the register part follows until r[1]
    wait0 = [r[2] - r[1] for r in rows]
    write = [r[5] - r[4] for r in rows]
    arrive_last = [r[3] for r in rows]
    per_xcd, lds_xcd = {}, {}
    for x in range(8):
        per_xcd[x] = us(statistics.median([read0[b] for b in range(x, G, 8)]))
        lds_xcd[x] = us(statistics.median([lds0[b] for b in range(x, G, 8)]))
    return dict(base, **{
        "read0_us": {"min": us(min(read0)), "median": us(statistics.median(read0)), "max": us(max(read0))},
        "read0_median_per_xcd_us": per_xcd,
        "lds0_median_per_xcd_us": lds_xcd,
        "wait0_us": {"median": us(statistics.median(wait0)), "max": us(max(wait0))},
        "last_arrival_spread_us": us(max(arrive_last) - min(arrive_last)),
        "write_after_last_meeting_us": {"min": us(min(write)), "median": us(statistics.median(write)),
                                         "max": us(max(write))},
    })


def main():
    if os.environ.get("FA_TIMELINE") != "1":
        sys.exit("run with FA_TIMELINE=1")
    names = sys.argv[1].split(",") if len(sys.argv) > 1 else ["northstar", "ns_w2", "ns_w4", "ns_w8"]
    launches = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    import bench
    import torch
    fa = bench.load_pkg()
    if os.environ.get("FA_BENCH_WALK"):  # A/B of fa_tuning.walk (process default, before any context)
        fa.set_tuning(walk=int(os.environ["FA_BENCH_WALK"]))
    lib = fa.lib()
    lib.fa_diag_phased_timeline.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    G = torch.cuda.get_device_properties(0).multi_processor_count
    buf = (ctypes.c_ulonglong * (8 * G))()
    stream = torch.cuda.Stream()
    for name in names:
        D, n, in_dt, out_dt, _ = bench.WORKLOADS[name]
        s = bench.Setup(fa, torch, D, n, in_dt, out_dt, 0, 0)
        torch.cuda.synchronize()
        recs, ms, raws = [], [], []
        for i in range(launches + 2):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            s.launch(i, stream)
            b.record(stream)
            torch.cuda.synchronize()
            got = lib.fa_diag_phased_timeline(0, buf, 8 * G)
            if got != 8 * G:
                sys.exit("no timeline (%d): is the phased kernel taking this workload?" % got)
            if i >= 2:
                recs.append(summarize(list(buf), G))
                ms.append(a.elapsed_time(b))
                if os.environ.get("TL_DUMP") == "1":  # raw per-workgroup times (us), launch by launch
                    raws.append([round((buf[g * 8 + 5] - buf[g * 8]) * TICK_US, 1) for g in range(G)])

        def med(path):
            vals = []
            for r in recs:
                v = r
                for k in path:
                    v = v[k]
                vals.append(v)
            return round(statistics.median(vals), 2)
        out = {"workload": name, "launches": launches, "event_ms_median": round(statistics.median(ms), 4),
               "algorithmic_bytes": s.algo_bytes(), "meetings": recs[0]["meetings"]}
        for key in ("span_us", "start_spread_us", "last_arrival_spread_us", "end_spread_us"):
            if key in recs[0]:
                out[key] = med([key])
        for key in ("workgroup_us", "read0_us", "wait0_us", "write_after_last_meeting_us"):
            if key in recs[0]:
                out[key] = {k: med([key, k]) for k in recs[0][key]}
        out["workgroup_median_per_xcd_us"] = {x: med(["workgroup_median_per_xcd_us", x]) for x in range(8)}
        if out["meetings"]:
            out["read0_median_per_xcd_us"] = {x: med(["read0_median_per_xcd_us", x]) for x in range(8)}
            out["lds0_median_per_xcd_us"] = {x: med(["lds0_median_per_xcd_us", x]) for x in range(8)}
        if raws:
            out["workgroup_us_per_launch"] = raws
        print(json.dumps(out), flush=True)
        s.close()


if __name__ == "__main__":
    main()
