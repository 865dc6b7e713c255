#!/usr/bin/env python3
"""BASELINE C2 end to end: the reference's own aggregator process against the drop-in, same blobs (GPU box).

  python tools/e2e_c2_ref.py [ref_rounds=3] [rounds=10]

C2 is ResNet-18 split "3,8" with 8 data owners (buckets 83 584 / 9 442 304 / 5 130 fp32).  The receipt
templates are made here by oracle/_ref/ref_harness (the reference's own model builders and torch::save), so
the reference process can torch::load them into its modules.  Then, over loopback with the fake data owners
(tests/tools, every reply checked against the oracle):
  * oracle/_ref/ref_cpu_aggregator 8 1 -- the reference's systemAPI / network_layer process on CPU libtorch,
    aggregator.cpp:55-167 restated (literal mode: the owners send in turn, as its result depends on order);
  * bin/fa_aggregator -d 8 in literal mode (the same exchange) and in FedAvg mode (owners at once).
The owners send the routing table in the refactor message (--routing-table): the reference cannot reach an
owner id above 3 without it.  One JSON line per leg.
"""
import json
import os
import signal
import statistics
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

HARNESS = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
SPEC = ["1", "1", "9", "3", "10"]  # resnet, resnet18, start 9, end 3 (split "3,8"), 10 classes
D = 8


def owners(blobs, mode, port_base, rounds, cwd, extra=()):
    return subprocess.run([bench.FAKE_OWNERS, "--blobs", blobs, "--parts", "1,2,3", "-d", str(D), "-c", "1",
                           "--rounds", str(rounds), "--port-base", str(port_base), "--model-name", "1",
                           "--model-type", "1", "--start", "9", "--end", "3", "--mode", mode,
                           "--reply-timeout", "120", "--routing-table"] + list(extra),
                          capture_output=True, text=True, timeout=900, cwd=cwd)


def leg(name, agg_cmd, mode, port_base, rounds, blobs, startup_s):
    with tempfile.TemporaryDirectory(prefix="fa_c2_") as tmp:
        agg = subprocess.Popen(agg_cmd, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, cwd=tmp,
                               start_new_session=True)
        try:
            time.sleep(startup_s)
            if agg.poll() is not None:
                raise RuntimeError("%s exited early (rc %s)" % (name, agg.returncode))
            r = owners(blobs, mode, port_base, rounds, tmp)
        finally:
            if agg.poll() is None:
                try:
                    agg.wait(timeout=10)
                except subprocess.TimeoutExpired:
                    os.killpg(agg.pid, signal.SIGKILL)  # the reference's loop never returns
                    agg.wait()
    res = json.loads(r.stdout.strip().splitlines()[-1])
    ms = res["round_ms"][1:]
    return {"leg": name, "mode": mode, "ok": res["ok"], "rounds_timed": len(ms),
            "round_ms_median": round(statistics.median(ms), 3), "round_ms_min": min(ms),
            "round0_ms": res["round_ms"][0], "checked_elems": res["checked_elems"]}


def main():
    ref_rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    with tempfile.TemporaryDirectory(prefix="fa_c2_blobs_") as blobs:
        for mp in ("-1", "2"):  # the small buckets' templates, then the 9.4 M one
            subprocess.run([HARNESS, "golden"] + SPEC + [str(D), "24301", "7", blobs, mp], check=True,
                           capture_output=True, timeout=600)
        if bench.ports_free(bench.REF_PORTS):
            print(json.dumps(dict(leg("reference_process_cpu", [bench.REF_CPU_AGGREGATOR, str(D), "1"], "literal",
                                      8079, ref_rounds + 1, blobs, 2.5),
                                  path="oracle/_ref/ref_cpu_aggregator: the reference's systemAPI / network_layer / "
                                       "torch::load / torch::save, aggregator.cpp:55-167 restated on CPU libtorch")),
                  flush=True)
        for mode in ("literal", "fedavg"):
            base = bench.free_port_base()
            print(json.dumps(leg("fa_aggregator", [bench.FA_AGGREGATOR, "-i", "-1", "-d", str(D), "-c", "1", "--mode",
                                                   mode, "--rounds", str(rounds + 1), "--port-base", str(base)],
                                 mode, base, rounds + 1, blobs, 0.5)), flush=True)


if __name__ == "__main__":
    main()
