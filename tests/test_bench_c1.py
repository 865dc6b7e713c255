"""CPU: bench.py's BASELINE C1 legs (secondary.round_c1) that need no GPU.

`cpu_c1` times the reference's CPU path for C1 (LeNet-5, two data owners): its receive loop alone
(oracle/_ref/ref_harness bench-round, aggregator.cpp:59-93 / :108-150 with torch::load) and its own
aggregator process over loopback (oracle/_ref/ref_cpu_aggregator against the fake owners, every reply
checked against the oracle).  The same function runs on the GPU box before the GPU is touched; here it runs
in the CPU suite so the fields the bench line carries are known to be filled and their parity object true.
"""
import os
import sys

import pytest

from conftest import ROOT

sys.path.insert(0, ROOT)
import bench  # noqa: E402

pytestmark = pytest.mark.skipif(
    not (os.access(bench.REF_CPU_AGGREGATOR, os.X_OK) and os.access(os.path.join(ROOT, "oracle", "_ref",
                                                                                 "ref_harness"), os.X_OK)),
    reason="oracle/_ref not built (make -f oracle/Makefile.ref)")


def test_cpu_c1_fields():
    import subprocess
    subprocess.run(["make", "-C", os.path.join(ROOT, "tests", "tools")], check=True, capture_output=True)
    if not bench.ports_free(bench.REF_PORTS):
        pytest.skip("the reference's fixed ports 8080-8083 are in use")
    r = bench.cpu_c1(2, "test")
    assert "cpu_error" not in r, r
    assert r["cpu_kind"] == "reference" and r["cpu_round_ms"] > 0 and r["cpu_round_ms_1_core"] > 0
    e2e = r["cpu_e2e_loopback"]
    assert e2e["parity"]["ok"] and e2e["parity"]["samples"] == bench.C1_E2E_ROUNDS * 2 * (50_536 + 10_164 + 850)
    assert e2e["rounds_timed"] == bench.C1_E2E_ROUNDS - 1 and 0 < e2e["round_ms_min"] <= e2e["round_ms_median"]
    assert e2e["aggregator_view"] is None  # the reference process prints no round lines
