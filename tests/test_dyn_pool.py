"""The phased kernel's dynamic row pool (FA_PHASED_DYN, fa_kernels.hip) on the GPU: every pool size -- one
row per workgroup, the product's default, every LDS row of a phase in the pool, more rows than a phase holds
-- gives the bits of the one-shot walk and of the oracle, over multi-phase buckets, LDS-only and near-empty
last phases, 1 to 64 clients and a d_init continuation; and the dynamic form is what ran.  Each pool size
runs in its own child process (the knob is read once per process), one after another."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("dyn", [1, 8, 38, 200])
def test_dyn_pool_same_bits(dyn):
    env = dict(os.environ, FA_PHASED_DYN=str(dyn))
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "dyn_child.py")], env=env, cwd=ROOT,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    for c in res["cases"]:
        assert c["same_bits"], c
        assert c["oracle_sampled_ok"] in (None, True), c
        assert c["dyn_launches"] >= 1, c  # the phased launch of the case took the dynamic form
