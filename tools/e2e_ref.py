#!/usr/bin/env python3
"""A BASELINE config end to end: the reference's own aggregator process against the drop-in, same receipts.

  python tools/e2e_ref.py [c2|c3|c4] [ref_rounds=3] [rounds=10]     (GPU box)

C2 is ResNet-18 split "3,8" with 8 data owners (buckets 83 584 / 9 442 304 / 5 130), C3 ResNet-101 split
"10,19" with 32 (2 594 688 / 29 511 680 / 5 130), both fp32 here: the reference has no bf16 path.  The
receipt templates are made here by oracle/_ref/ref_harness (the reference's own model builders and
torch::save), so the reference process can torch::load them into its modules.  Then, over loopback with the fake data owners
(tests/tools, every reply checked against the oracle):
  * oracle/_ref/ref_cpu_aggregator 8 1 -- the reference's systemAPI / network_layer process on CPU libtorch,
    aggregator.cpp:55-167 restated (literal mode: the owners send in turn, as its result depends on order);
  * bin/fa_aggregator -d 8 in literal mode (the same exchange) and in FedAvg mode (owners at once).
  * oracle/_ref/ref_aggregator -- the same process with the INTEGRATION.md 2 binding on libfa (FedAvg).
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
# name -> (ref_harness spec: model_name, model_type, start, end, classes; D; template model parts to write)
CONFIGS = {
    "c2": (["1", "1", "9", "3", "10"], 8, ["-1", "2"]),         # ResNet-18 split "3,8"
    "c3": (["1", "4", "20", "10", "10"], 32, ["-1", "1", "2"]),  # ResNet-101 split "10,19"
    "c4": (["0", "6", "20", "3", "10"], 64, ["-1", "2", "3"]),    # VGG-19 split "3,19"
}
# The reference process holds ~3x a phase's receipts (C2: 0.94 GB peak RSS for 302 MB) and queues its
# replies: its address space is capped so that C4 (30.6 GB of FC receipts per phase) fails by itself
# rather than crowd the host.
REF_AS_LIMIT = 160 << 30


def owners(spec, D, blobs, mode, port_base, rounds, cwd, extra=()):
    return subprocess.run([bench.FAKE_OWNERS, "--blobs", blobs, "--parts", "1,2,3", "-d", str(D), "-c", "1",
                           "--rounds", str(rounds), "--port-base", str(port_base), "--model-name", spec[0],
                           "--model-type", spec[1], "--start", spec[2], "--end", spec[3], "--mode", mode,
                           "--reply-timeout", "300", "--routing-table"] + list(extra),
                          capture_output=True, text=True, timeout=1500, cwd=cwd)


def cap_address_space():
    import resource
    resource.setrlimit(resource.RLIMIT_AS, (REF_AS_LIMIT, REF_AS_LIMIT))


def leg(name, spec, D, agg_cmd, mode, port_base, rounds, blobs, startup_s, extra=(), cap=False):
    with tempfile.TemporaryDirectory(prefix="fa_e2e_") as tmp:
        agg_out = open(os.path.join(tmp, "agg.out"), "w+")
        agg = subprocess.Popen(agg_cmd, stdout=agg_out, stderr=subprocess.DEVNULL, cwd=tmp, start_new_session=True,
                               preexec_fn=cap_address_space if cap else None)
        try:
            time.sleep(startup_s)
            if agg.poll() is not None:
                raise RuntimeError("%s exited early (rc %s)" % (name, agg.returncode))
            r = owners(spec, D, blobs, mode, port_base, rounds, tmp, extra)
        finally:
            if agg.poll() is None:
                try:
                    agg.wait(timeout=10)
                except subprocess.TimeoutExpired:
                    os.killpg(agg.pid, signal.SIGKILL)  # the reference's loop never returns
                    agg.wait()
        agg_out.seek(0)
        lines = [json.loads(l) for l in agg_out.read().splitlines() if l.startswith("{")]  # fa_aggregator's
        agg_out.close()
    res = json.loads(r.stdout.strip().splitlines()[-1])
    ms = res["round_ms"][1:]
    view = None
    if len(lines) > 1:  # medians over rounds 1.. of the aggregator's own phase times
        med = lambda f: round(statistics.median(f(p) for p in lines[1:]) * 1e3, 3)  # noqa: E731
        view = {k: med(lambda p, k=k: p[k.split(".")[0]][k.split(".")[1]])
                for k in ("phase1.receive_s", "phase1.absorb_s", "phase1.reduce_s", "phase2.receive_s",
                          "phase2.absorb_s", "phase2.reduce_s", "phase2.finalize_s", "phase2.frame_s",
                          "phase2.send_s")}
    if lines:  # streaming ingest (fa_aggregator, round 6): receipts committed from their streams, cumulative
        view = dict(view or {}, streamed=lines[-1].get("streamed"), stream_fallbacks=lines[-1].get("stream_fallbacks"))
    return {"leg": name, "mode": mode, "ok": res["ok"], "rounds_timed": len(ms), "aggregator_view_ms": view,
            "round_ms_median": round(statistics.median(ms), 3), "round_ms_min": min(ms),
            "round0_ms": res["round_ms"][0], "checked_elems": res["checked_elems"]}


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
    ref_rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    spec, D, mps = CONFIGS[cfg]
    with tempfile.TemporaryDirectory(prefix="fa_%s_blobs_" % cfg) as blobs:
        for mp in mps:  # the small buckets' templates (-1), then the large ones one by one; client 0's archive
            # is the template whatever D is (the owners write their own values into it), so D = 1 here
            subprocess.run([HARNESS, "golden"] + spec + ["1", "24301", "7", blobs, mp], check=True,
                           capture_output=True, timeout=1200)
        only_fa = os.environ.get("E2E_ONLY_FA") == "1"  # the drop-in's legs alone
        if not only_fa and bench.ports_free(bench.REF_PORTS):
            print(json.dumps(dict(leg("reference_process_cpu", spec, D, [bench.REF_CPU_AGGREGATOR, str(D), "1"],
                                      "literal", 8079, ref_rounds + 1, blobs, 2.5, cap=True), config=cfg,
                                  path="oracle/_ref/ref_cpu_aggregator: the reference's systemAPI / network_layer / "
                                       "torch::load / torch::save, aggregator.cpp:55-167 restated on CPU libtorch")),
                  flush=True)
        binding = os.environ.get("E2E_NO_BINDING") != "1"
        if not only_fa and binding and os.access(bench.REF_BINDING_AGGREGATOR, os.X_OK) and \
                bench.ports_free(bench.REF_PORTS):
            print(json.dumps(dict(leg("reference_process_with_binding", spec, D,
                                      [bench.REF_BINDING_AGGREGATOR, str(D), "1"], "fedavg", 8079, ref_rounds + 1,
                                      blobs, 2.5, ["--sequential"], cap=True), config=cfg,
                                  path="oracle/_ref/ref_aggregator: the reference's process with aggregator.cpp:55-167 "
                                       "replaced by the INTEGRATION.md 2 binding on libfa (torch::load / torch::save "
                                       "stay)")), flush=True)
        for mode in ("literal", "fedavg"):
            base = bench.free_port_base()
            print(json.dumps(dict(leg("fa_aggregator", spec, D, [bench.FA_AGGREGATOR, "-i", "-1", "-d", str(D), "-c",
                                                                 "1", "--mode", mode, "--rounds", str(rounds + 1),
                                                                 "--port-base", str(base)] +
                                      os.environ.get("E2E_AGG_ARGS", "").split(),
                                      mode, base, rounds + 1, blobs, 0.5), config=cfg,
                                  agg_args=os.environ.get("E2E_AGG_ARGS", ""))), flush=True)


if __name__ == "__main__":
    main()
