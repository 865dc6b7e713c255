"""The phased kernel's dynamic row pool (FA_PHASED_DYN) on the GPU against the one-shot walk (whole buckets, bit
for bit) and the oracle (sampled elements), at one row per workgroup, the measured size, every LDS row of a
phase in the pool and more rows than a phase holds.  Shapes: multi-phase f32 buckets, LDS-only and near-empty
remainders, 1 to 64 clients, a sized phase, a d_init continuation, and bf16 buckets of the 512-thread form
(tests/phased_child.py); and 52 launches at once on as many streams, beyond the 48 stream-owned counter slots.
Each setting runs in its own child process (the knobs are read once per process),
one after another."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_child(env_extra):
    env = dict(os.environ, **env_extra)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "phased_child.py")], env=env, cwd=ROOT,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    for c in res["cases"]:
        assert c["same_bits"], c
        assert c["oracle_sampled_ok"] in (None, True), c
    assert res["streams"]["mismatched_outputs"] == 0, res["streams"]
    return res


@pytest.mark.parametrize("dyn", [1, 8, 38, 200])
def test_dyn_pool_same_bits(dyn):
    res = run_child({"FA_PHASED_DYN": str(dyn)})
    for c in res["cases"]:
        if not c["bf16"]:  # the f32 form has a dynamic instantiation: it must be what ran
            assert c["dyn_launches"] >= 1, c
    # concurrent launches on 52 streams: the streams that got a counter slot of their own took the dynamic form
    assert res["streams"]["dyn_launches"] >= 1, res["streams"]
