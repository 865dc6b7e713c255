"""CPU: bench.py's live roofline.traffic (two rocprofv3 PMC child passes before the GPU is touched).

A stand-in `rocprofv3` on PATH writes the counter CSV the real one writes (one row per dispatch and
counter); the test checks the pass layout (one counter per run, the bench child after `--`), the choice of
the reduction kernel over the fill / probe kernels, and the gfx950 formula (2 FETCH_SIZE + WRITE_SIZE) KiB.
"""
import json
import os
import stat
import sys

from conftest import ROOT

sys.path.insert(0, ROOT)
import bench  # noqa: E402

FAKE = r'''#!/usr/bin/env python3
import json, os, sys
a = sys.argv[1:]
log = os.environ["FAKE_ROCPROF_LOG"]
with open(log, "a") as f:
    f.write(json.dumps(a + ["WORLD_SIZE=%s" % os.environ.get("WORLD_SIZE")]) + "\n")
counter = a[a.index("--pmc") + 1]
out = a[a.index("-d") + 1]
assert a[a.index("--") + 2].endswith("bench.py") and "--no-cpu-baseline" in a
os.makedirs(out, exist_ok=True)
vals = {"FETCH_SIZE": {"fill": 10.0, "red": 4194304.0, "probe": 9999999.0},
        "WRITE_SIZE": {"fill": 262144.0, "red": 262144.0, "probe": 0.0}}[counter]
names = {"fill": "void fa::fill_kernel<float>(void*, long)", "red": "void fa::fedavg_phased_kernel<float>(x)",
         "probe": "fa::read_probe_kernel(x)"}
with open(os.path.join(out, "run_counter_collection.csv"), "w") as f:
    f.write('"Kernel_Name","Grid_Size","Counter_Name","Counter_Value"\n')
    for k, n in (("fill", 8), ("red", 5), ("probe", 9)):
        for i in range(n):
            f.write('"%s",65536,"%s",%s\n' % (names[k], counter, vals[k] + (i % 2)))
'''


def test_live_traffic_two_passes_reduction_kernel(tmp_path, monkeypatch):
    fake = tmp_path / "rocprofv3"
    fake.write_text(FAKE)
    fake.chmod(fake.stat().st_mode | stat.S_IEXEC)
    log = tmp_path / "calls.jsonl"
    monkeypatch.setenv("PATH", str(tmp_path) + os.pathsep + os.environ["PATH"])
    monkeypatch.setenv("FAKE_ROCPROF_LOG", str(log))
    monkeypatch.setenv("WORLD_SIZE", "4")  # a launcher's variables must not reach the child
    traffic, src = bench.live_traffic("ns_w4", timeout=60)
    calls = [json.loads(l) for l in log.read_text().splitlines()]
    assert [c[c.index("--pmc") + 1] for c in calls] == ["FETCH_SIZE", "WRITE_SIZE"]
    assert all("--workload" in c and c[c.index("--workload") + 1] == "ns_w4" for c in calls)
    assert all(c[-1] == "WORLD_SIZE=None" for c in calls)
    f, w = 4194304.4, 262144.4  # means over 5 launches alternating +0 / +1
    assert traffic == round((2 * f + w) * 1024)
    assert "fedavg_phased_kernel" in src and "5 launches" in src


def test_live_traffic_reports_a_missing_profiler(monkeypatch, tmp_path):
    monkeypatch.setenv("PATH", str(tmp_path))
    assert bench.live_traffic("northstar") == (None, "rocprofv3 not on PATH")


def test_bench_skips_live_pmc_under_a_profiler(monkeypatch):
    monkeypatch.setenv("ROCPROF_COUNTERS", "FETCH_SIZE")
    assert bench.under_profiler()


HANG = r'''#!/usr/bin/env python3
import os, subprocess, sys, time
# a profiler whose child hangs: both must die when the pass times out
child = subprocess.Popen([sys.executable, "-c", "import time; time.sleep(600)"])
open(os.environ["FAKE_ROCPROF_PIDS"], "w").write("%d %d" % (os.getpid(), child.pid))
time.sleep(600)
'''


def test_live_traffic_timeout_kills_the_whole_pass(tmp_path, monkeypatch):
    fake = tmp_path / "rocprofv3"
    fake.write_text(HANG)
    fake.chmod(fake.stat().st_mode | stat.S_IEXEC)
    pids = tmp_path / "pids"
    monkeypatch.setenv("PATH", str(tmp_path) + os.pathsep + os.environ["PATH"])
    monkeypatch.setenv("FAKE_ROCPROF_PIDS", str(pids))
    traffic, reason = bench.live_traffic("northstar", timeout=3)
    assert traffic is None and "timed out" in reason
    import time
    for pid in map(int, pids.read_text().split()):
        for _ in range(50):  # reaped by now, or about to be
            try:
                os.kill(pid, 0)
            except ProcessLookupError:
                break
            time.sleep(0.1)
        else:
            raise AssertionError("process %d of the timed-out pass survived" % pid)
