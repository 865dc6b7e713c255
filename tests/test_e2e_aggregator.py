"""End-to-end (GPU): the drop-in aggregator process against fake data owners over loopback TCP.

BASELINE.json config C1: LeNet-5 model parts, data owners speaking the
reference's wire protocol (Message.h frames carrying torch::save archives made
by the reference's own builders).  The fake owners (tests/tools/fake_owners.cpp)
check every reply bit-for-bit against the oracle: FedAvg (uniform weights) and
the reference-literal last/500 mode, several rounds.
"""
import json
import os
import random
import socket
import subprocess
import time

import pytest

from conftest import GOLDEN, PKG_DIR, ROOT

pytestmark = pytest.mark.gpu

AGG = os.path.join(PKG_DIR, "bin", "fa_aggregator")
OWNERS = os.path.join(ROOT, "tests", "tools", "bin", "fa_fake_owners")


def ports_free(base, span=40):
    for p in range(base, base + span):
        with socket.socket() as s:
            try:
                s.bind(("127.0.0.1", p))
            except OSError:
                return False
    return True


def pick_base():
    for _ in range(50):
        b = random.randrange(20000, 60000, 100)
        if ports_free(b):
            return b
    pytest.skip("no free port range")


@pytest.fixture(scope="module", autouse=True)
def built():
    subprocess.run(["make", "-C", os.path.join(ROOT, "tests", "tools")], check=True, capture_output=True)
    assert os.access(AGG, os.X_OK), "build the package first (make -C %s)" % PKG_DIR


@pytest.mark.parametrize("mode,D,rounds", [("fedavg", 2, 3), ("literal", 2, 2), ("fedavg", 5, 2)])
def test_lenet_rounds_over_tcp(torch_gpu, mode, D, rounds):
    base = pick_base()
    agg = subprocess.Popen([AGG, "-i", "-1", "-d", str(D), "-c", "1", "--mode", mode, "--rounds", str(rounds),
                            "--port-base", str(base)], stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    try:
        time.sleep(0.5)
        r = subprocess.run([OWNERS, "--blobs", os.path.join(GOLDEN, "lenet5_c1"), "--parts", "1,2,3", "-d", str(D),
                            "-c", "1", "--rounds", str(rounds), "--mode", mode, "--port-base", str(base),
                            "--model-name", "2", "--start", "6", "--end", "1"],
                           capture_output=True, text=True, timeout=240)
        assert r.returncode == 0, r.stderr[-2000:]
        res = json.loads(r.stdout.strip().splitlines()[-1])
        assert res["ok"] and res["rounds"] == rounds
        assert res["checked_elems"] == rounds * D * (50_536 + 10_164 + 850)
        out, err = agg.communicate(timeout=60)
        assert agg.returncode == 0, err[-2000:]
        stats = [json.loads(l) for l in out.splitlines() if l.startswith("{")]
        assert len(stats) == rounds and stats[0]["phase2"]["layers"] == 2
    finally:
        if agg.poll() is None:
            agg.kill()
