#!/usr/bin/env python3
"""Summarise a gpu_session.sh output directory into profiles/.

  python tools/pmc_traffic.py gpurun_out/<tag> <round> [workload]

* kernel-trace stats (rocprofv3 --kernel-trace --stats) of the bench run ->
  profiles/<round>_kernel_stats.csv (copied) + per-(kernel, grid) averages.
* PMC passes (separate FETCH_SIZE and WRITE_SIZE runs, as the MI355X guide
  prescribes) -> HBM bytes per launch of the dominant kernel:
      traffic = (2 * FETCH_SIZE + WRITE_SIZE) * 1024
  (FETCH_SIZE/WRITE_SIZE are KiB; gfx950 FETCH_SIZE counts half the bytes of a
  wide coalesced streaming read, so it is doubled).  Written to
  profiles/pmc_traffic.json[workload], which bench.py reads for roofline.traffic.
"""
import collections
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PER_LAUNCH_STEPS = 10  # bench.timed_loop(per_launch=10): steps timed one by one after the region


def per_kernel(path, value_col=None, counter=None):
    rows = list(csv.DictReader(open(path)))
    g = collections.defaultdict(list)
    for r in rows:
        if counter and r.get("Counter_Name") != counter:
            continue
        grid = r.get("Grid_Size") or r.get("Grid_Size_X")
        key = (r["Kernel_Name"], int(grid))
        if value_col:
            g[key].append(float(r[value_col]))
        else:
            g[key].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    if not value_col:  # launch order, durations only
        g = {k: [d for _, d in sorted(v)] for k, v in g.items()}
    return g


def dominant(g):
    return max(g.items(), key=lambda kv: sum(kv[1]))


def main():
    src, rnd = sys.argv[1], sys.argv[2]
    workload = sys.argv[3] if len(sys.argv) > 3 else "northstar"
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    sp = os.path.join(prof, rnd + "_summary.json")
    summary = json.load(open(sp)) if os.path.exists(sp) else {}  # keep the round's other records
    summary.update({"round": rnd, "workload": workload, "source_dir": os.path.basename(os.path.normpath(src))})

    kt = os.path.join(src, "prof", "run_kernel_trace.csv")
    if os.path.exists(kt):
        shutil.copy(os.path.join(src, "prof", "run_kernel_stats.csv"), os.path.join(prof, rnd + "_kernel_stats.csv"))
        g = per_kernel(kt)
        bj = os.path.join(src, "prof_bench.json")
        steps = warmup = 0
        if os.path.exists(bj) and os.path.getsize(bj):
            line = json.loads(open(bj).read().strip().splitlines()[-1])
            summary["bench_under_profiler"] = line["roofline"]
            steps, warmup = int(line["steps"]), int(line["warmup"])
        # the dominant kernel's launches in bench order: warm-ups, the timed region's `steps`, then the
        # separate per-launch-event loop (bench.timed_loop)
        summary["kernels"] = []
        for k, v in sorted(g.items(), key=lambda kv: -sum(kv[1])):
            rec = {"kernel": k[0], "grid": k[1], "calls": len(v), "avg_ns": round(sum(v) / len(v), 1), "min_ns": min(v)}
            if steps and len(v) >= warmup + steps and not summary["kernels"]:
                rec["timed_launches"] = steps
                rec["timed_avg_ns"] = round(sum(v[warmup:warmup + steps]) / steps, 1)
            summary["kernels"].append(rec)

    fetch = os.path.join(src, "pmc_FETCH_SIZE", "run_counter_collection.csv")
    write = os.path.join(src, "pmc_WRITE_SIZE", "run_counter_collection.csv")
    if workload != "northstar" or not os.path.exists(fetch):  # tools/pmc_workloads.sh layout
        fetch = os.path.join(src, "pmc_%s_FETCH_SIZE" % workload, "run_counter_collection.csv")
        write = os.path.join(src, "pmc_%s_WRITE_SIZE" % workload, "run_counter_collection.csv")
    if os.path.exists(fetch) and os.path.exists(write):
        fk, fv = dominant(per_kernel(fetch, "Counter_Value", "FETCH_SIZE"))
        wg = per_kernel(write, "Counter_Value", "WRITE_SIZE")
        wv = wg[fk]
        f_kib, w_kib = sum(fv) / len(fv), sum(wv) / len(wv)
        traffic = (2 * f_kib + w_kib) * 1024
        # launches of the dominant kernel per bench step (C5's range pieces: one launch per piece): the pass ran
        # warmup + steps timed steps + bench.timed_loop's per-launch loop (PER_LAUNCH_STEPS)
        per_step = 1
        bj = os.path.join(os.path.dirname(fetch), os.pardir, "pmc_%s_FETCH_SIZE.json" % workload)
        if os.path.exists(bj) and os.path.getsize(bj):
            line = json.loads(open(bj).read().strip().splitlines()[-1])
            n_steps = int(line["warmup"]) + int(line["steps"]) + PER_LAUNCH_STEPS
            per_step = max(1, round(len(fv) / n_steps))
        rec = {"kernel": fk[0], "grid": fk[1], "launches": len(fv), "FETCH_SIZE_KiB": f_kib,
               "WRITE_SIZE_KiB": w_kib, "hbm_bytes_per_launch": round(traffic), "launches_per_step": per_step,
               "hbm_bytes_per_step": round(traffic * per_step),
               "formula": "(2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE half-count correction)"}
        if workload == "northstar":
            summary["pmc"] = rec
        else:
            summary.setdefault("pmc_workloads", {})[workload] = rec
        tp = os.path.join(prof, "pmc_traffic.json")
        d = json.load(open(tp)) if os.path.exists(tp) else {}
        d[workload] = {"hbm_bytes_per_launch": round(traffic), "launches_per_step": per_step,
                       "hbm_bytes_per_step": round(traffic * per_step), "kernel": fk[0], "grid": fk[1],
                       "FETCH_SIZE_KiB": f_kib, "WRITE_SIZE_KiB": w_kib, "round": rnd,
                       "source": "profiles/%s_summary.json (gpurun_out/%s)" % (rnd, os.path.basename(os.path.normpath(src)))}
        json.dump(d, open(tp, "w"), indent=1)
    for extra in ("hbm_probe.json",):
        p = os.path.join(src, extra)
        if os.path.exists(p) and os.path.getsize(p):
            summary["hbm_probe"] = json.load(open(p))
    for sw in ("sweep_northstar.jsonl", "sweep_c2.jsonl"):
        p = os.path.join(src, sw)
        if os.path.exists(p):
            summary[sw.split(".")[0]] = [json.loads(l) for l in open(p) if l.strip()][:8]
    json.dump(summary, open(sp, "w"), indent=1)
    print(json.dumps({k: v for k, v in summary.items() if k in ("pmc", "bench_under_profiler")}, indent=1))


if __name__ == "__main__":
    main()
