"""CPU: the bench's stdout line stays small enough for the driver to parse.

BENCH_r05's line was 20.3 KB and the driver's parse returned null.  bench.compact_line keeps the required
keys, roofline, cpu_baseline (with its spread), parity and one small object per secondary leg, and the full
object goes to a side file.  Here the compaction runs on the round-5 final-tree line (profiles/r05s53_bench.json)
and on the shapes of the lines a multi-GPU node produces (the N = 1 run with 8 in-process multi-GPU children,
and the N = 8 main line with its layout secondaries).
"""
import copy
import json
import os
import sys

from conftest import ROOT

sys.path.insert(0, ROOT)

REQUIRED = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline", "parity")
ROOFLINE = ("bound", "achieved", "peak", "unit", "frac", "traffic")
CPU = ("value", "unit", "cores", "kind", "sample")


def _r05():
    with open(os.path.join(ROOT, "profiles", "r05s53_bench.json")) as f:
        return json.load(f)


def _check(line, bench):
    s = json.dumps(bench.compact_line(line, "gpurun_out/bench_full.json"))
    assert len(s.encode()) <= bench.LINE_MAX_BYTES, len(s)
    got = json.loads(s)
    for k in REQUIRED:
        assert k in got, k
    for k in ROOFLINE:
        assert k in got["roofline"], k
    if line.get("cpu_baseline"):
        for k in CPU:
            assert k in got["cpu_baseline"], k
    assert got["value"] == line["value"] and got["roofline"]["frac"] == line["roofline"]["frac"]
    assert "\n" not in s
    return got


def test_round5_line_compacts_under_the_bound():
    import bench
    line = _r05()
    assert len(json.dumps(line)) > 20000  # the line the driver could not parse
    got = _check(line, bench)
    sec = got["secondary"]
    assert set(sec) == set(line["secondary"])
    assert sec["c4"]["frac"] == line["secondary"]["c4"]["frac"] and sec["c4"]["parity_ok"] is True
    assert sec["c4"]["cpu_gib_s"] == line["secondary"]["c4"]["cpu_gib_s"]
    assert sec["round_c2"]["ms"] == line["secondary"]["round_c2"]["round_ms_avg"]
    assert sec["round_c1"]["e2e_literal_ms"] == line["secondary"]["round_c1"]["e2e_loopback_literal"]["round_ms_median"]
    assert sec["round_c1"]["cpu_e2e_ms"] == line["secondary"]["round_c1"]["cpu_e2e_loopback"]["round_ms_median"]
    assert sec["round_c1"]["e2e_parity_ok"] is True
    rs = sec["ctx_rs_c4_8shard_rehearsal_on_one_gpu"]
    assert rs["rehearsal"] and rs["err_over_bound"] == round(
        line["secondary"]["ctx_rs_c4_8shard_rehearsal_on_one_gpu"]["parity"]["max_err_over_bound"], 3)
    assert got["full_record"] == "gpurun_out/bench_full.json"


def test_eight_gpu_node_n1_line_compacts():
    """The N = 1 run on an 8-GPU node: every single-GPU leg plus eight in-process multi-GPU children, some of
    them failed with long error text, and a host-inclusive leg with its split."""
    import bench
    line = _r05()
    sec = line["secondary"]
    child = sec.pop("ctx_rs_c4_8shard_rehearsal_on_one_gpu")
    sec.pop("ctx_range_c5r_h2d_8shard_rehearsal_on_one_gpu")
    for key in ("ctx_range_northstar_8gpu", "ctx_rs_northstar_8gpu", "ctx_rs_c4_4gpu", "ctx_rs_c4_8gpu",
                "ctx_range_c5_h2d_8gpu", "ctx_rs_c4_4gpu_rschunks2", "ctx_rs_c4_4gpu_rschunks4"):
        sec[key] = dict(copy.deepcopy(child), shared_device_rehearsal=False)
    sec["ctx_rs_c4_4gpu_rschunks16"] = {"error": "rc 1: " + "x" * 300}
    sec["ns_h2d"] = {"gib_s": 50.1, "ms_per_round": 166.0, "h2d_ms": 160.1, "reduce_ms": 1.3, "d2h_ms": 4.6,
                     "pcie_GBs": 55.0, "parity": {"ok": True, "samples": 1026}, "description": "y" * 300}
    e2e = {"aggregator_view": {"phase1_reduce_ms": 0.4, "phase2_reduce_ms": 1.3, "streamed": 63, "note": "z" * 200},
           "rounds_timed": 7, "round_ms_median": 25.1, "parity": {"ok": True, "samples": 10}}
    sec["round_c2"]["e2e_loopback_fedavg"] = e2e
    sec["round_c2"]["e2e_loopback_fedavg_no_streaming"] = dict(e2e, round_ms_median=27.0,
                                                                aggregator_view=dict(e2e["aggregator_view"],
                                                                                     phase2_reduce_ms=7.2))
    got = _check(line, bench)
    c2 = got["secondary"]["round_c2"]
    assert c2["e2e_fedavg_ms"] == 25.1 and c2["e2e_fedavg_tail_ms"] == 1.3
    assert c2["e2e_fedavg_nostream_ms"] == 27.0 and c2["e2e_fedavg_nostream_tail_ms"] == 7.2 and c2["e2e_parity_ok"]
    err = got["secondary"]["ctx_rs_c4_4gpu_rschunks16"]["error"]
    assert err.startswith("rc 1: x") and len(err) <= 80
    assert got["secondary"]["ns_h2d"]["h2d_ms"] == 160.1
    assert "secondary_truncated" not in got


def test_eight_gpu_main_line_compacts():
    """The --gpus 8 main line: range over 8 ranks and the weak-range / rs / chain secondaries."""
    import bench
    line = _r05()
    line["n_gpus"] = 8
    line["roofline"]["kernel_ms_avg_max_over_ranks"] = 0.17
    line["parity"] = dict(line["parity"], ranks=8)
    line["cpu_baseline"] = None  # rank 0 at N = 1 only
    desc = "client-sharded: each rank reduces its 4 whole clients into fp32 partials " * 3
    line["secondary"] = {L: {"description": desc, "clients": 32, "steps": 20, "ms_per_step": 0.2, "gib_s": 40000.0,
                             "phased_meeting_timeouts": 0,
                             "parity": {"check": "c", "samples": 8000, "mismatches": 0, "max_abs_err": 1e-7,
                                        "max_err_over_bound": 0.2, "ok": True, "ranks": 8}}
                         for L in ("weak_range", "rs", "chain")}
    line["secondary_error"] = "secondary layouts did not finish within 90 s"
    got = _check(line, bench)
    assert got["secondary"]["rs"] == {"gib_s": 40000.0, "ms": 0.2, "parity_ok": True, "err_over_bound": 0.2}
    assert got["parity"]["ranks"] == 8


def test_line_printer_writes_compact_line_and_full_record(tmp_path):
    import io
    import bench
    out = io.StringIO()
    full = tmp_path / "full.json"
    p = bench.LinePrinter(0, out, full_path=str(full))
    line = _r05()
    p.emit(line)
    p.emit(line)  # once only
    printed = out.getvalue().splitlines()
    assert len(printed) == 1 and len(printed[0]) <= bench.LINE_MAX_BYTES
    assert json.loads(full.read_text()) == line
    assert json.loads(printed[0])["value"] == line["value"]


def test_cpu_baseline_cores_spread_over_ccds(monkeypatch):
    """The CPU legs run pinned on one CPU per physical core of one NUMA node, dealt over
    its L3 domains: a 64-core, 8-CCD, SMT-2 mask gives 16 cores as 2 per CCD and never an SMT sibling."""
    import bench
    cpus = list(range(128))  # cpu c and c + 64 are SMT siblings; CCD = (c % 64) // 8
    monkeypatch.setattr(bench.os, "sched_getaffinity", lambda pid: set(cpus))

    def topo(c, what):
        core = c % 64
        if what.startswith("topology"):
            return "%d,%d" % (core, core + 64)
        return "ccd%d" % (core // 8)
    monkeypatch.setattr(bench, "_cpu_topology", topo)
    monkeypatch.setattr(bench, "_numa_node", lambda c: 0)
    got = bench.pick_cores(16)
    assert len(set(got)) == 16 and all(c < 64 for c in got)
    assert sorted((c // 8) for c in got) == sorted(list(range(8)) * 2)
    assert bench.pick_cores(1) == [0]
    assert len(bench.pick_cores(100)) == 100  # SMT siblings once every core is taken
    # two sockets (node = core // 32): 16 cores fit one node, so they all come from node 0's 4 CCDs
    monkeypatch.setattr(bench, "_numa_node", lambda c: (c % 64) // 32)
    got = bench.pick_cores(16)
    assert all((c % 64) < 32 for c in got) and sorted(c // 8 for c in got) == sorted(list(range(4)) * 4)
    assert len(set(bench.pick_cores(40))) == 40  # more than a node holds: the rest from the other
    assert bench.compact_cpus([0, 1, 2, 3, 8, 16, 17]) == "0-3,8,16-17"
    s = bench.spread([0.5, 0.25, 1.0], 2**30)
    assert s == {"min": 1.0, "median": 2.0, "max": 4.0, "reps": 3}


def test_round6_full_record_compacts_to_its_printed_line():
    """The round's final-tree run (r06s25): the line the bench printed is compact_line of the full record it
    wrote beside it, within the bound, with the sync legs' copy-ceiling fraction and the C2 end-to-end keys."""
    import bench
    with open(os.path.join(ROOT, "profiles", "r06s25_bench_full.json")) as f:
        full = json.load(f)
    with open(os.path.join(ROOT, "profiles", "r06s25_bench_line.json")) as f:
        printed = json.load(f)
    got = _check(full, bench)
    assert json.loads(json.dumps(bench.compact_line(full, printed["full_record"]))) == printed
    assert "frac_copy_ind" in got["secondary"]["sync_c2"] and "e2e_fedavg_tail_ms" in got["secondary"]["round_c2"]


def test_timed_loop_refuses_a_non_stream():
    """timed_loop records HIP events on the stream it is given; anything else (a bool once reached it and
    crashed inside the HIP runtime, r06s11-s20) is a TypeError before any launch."""
    import pytest
    import bench

    class NoLaunch:
        def launch(self, step, stream):
            raise AssertionError("launched")

    for bad in (True, False, None, 0):
        with pytest.raises(TypeError):
            bench.timed_loop(None, NoLaunch(), 1, 0, bad, None, lambda: None)
