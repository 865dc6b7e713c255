"""CPU: BASELINE config C1 through the reference's own aggregator process on CPU libtorch.

oracle/_ref/ref_cpu_aggregator (oracle/Makefile.ref) is the reference's systemAPI + network_layer + model
builders compiled from /root/reference as they lie, with aggregator.cpp:55-167 restated on CPU libtorch
(oracle/ref_cpu_aggregator.cpp; aggregator.cpp itself needs the absent third_party/argparse).  The fake data
owners (tests/tools/fake_owners.cpp, speaking the reference's frame) drive it over loopback and check every
reply against the oracle's literal result fl(fl(x_last + x_last) / 1000): the reference's CPU path runs and is
pinned here, with no GPU.  bench.py times the same pairing as `secondary.round_c1.cpu_e2e_loopback`.

The second test shows what the drop-in's receipt ledger exists for (host/receipts.h,
tests/test_e2e_aggregator.py::test_late_duplicates_of_earlier_rounds_are_dropped): the wire carries no round
number, so the reference takes a late copy of an earlier round's part 1 as a receipt -- phase 1 ends on the
stale parameters, and the current part 1, arriving in phase 2, indexes parts[1].layers[model_part - 2] =
layers[-1] (aggregator.cpp:118): the process dies.
"""
import json
import os
import socket
import subprocess
import tempfile
import time

import pytest

from conftest import GOLDEN, ROOT

REF_CPU_AGG = os.path.join(ROOT, "oracle", "_ref", "ref_cpu_aggregator")
OWNERS = os.path.join(ROOT, "tests", "tools", "bin", "fa_fake_owners")
PORTS = (8080, 8081, 8082, 8083)  # the reference's fixed routing table (network_layer.h:80-86)


def ports_free():
    for p in PORTS:
        with socket.socket() as s:
            s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)  # as the reference binds (network_layer.cpp:99)
            try:
                s.bind(("0.0.0.0", p))
            except OSError:
                return False
    return True


pytestmark = [
    pytest.mark.skipif(not os.access(REF_CPU_AGG, os.X_OK),
                       reason="oracle/_ref/ref_cpu_aggregator not built (make -f oracle/Makefile.ref)"),
]


@pytest.fixture(scope="module", autouse=True)
def built():
    subprocess.run(["make", "-C", os.path.join(ROOT, "tests", "tools")], check=True, capture_output=True)


def run_pair(owner_flags, rounds, reply_timeout=30):
    if not ports_free():
        pytest.skip("the reference's fixed ports 8080-8083 are in use")
    with tempfile.TemporaryDirectory() as tmp:  # the reference process writes its logs in cwd
        agg = subprocess.Popen([REF_CPU_AGG, "2", "1"], stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, cwd=tmp,
                               start_new_session=True)
        try:
            time.sleep(2.5)  # the reference's receiver binds its port a second after it is released
            assert agg.poll() is None, agg.stderr.read()
            r = subprocess.run([OWNERS, "--blobs", os.path.join(GOLDEN, "lenet5_c1"), "--parts", "1,2,3", "-d", "2",
                                "-c", "1", "--rounds", str(rounds), "--port-base", "8079", "--model-name", "2",
                                "--start", "6", "--end", "1", "--mode", "literal",
                                "--reply-timeout", str(reply_timeout)] + owner_flags,
                               capture_output=True, text=True, timeout=120, cwd=tmp)
            time.sleep(0.5)
            status = agg.poll()
        finally:
            if agg.poll() is None:
                os.killpg(agg.pid, 9)  # the reference's loop never returns (aggregator.cpp:55)
            agg.wait(timeout=30)
    return r, status


def test_reference_cpu_process_serves_c1_bit_exact():
    r, status = run_pair([], rounds=5)
    assert r.returncode == 0, r.stderr[-2000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["ok"] and res["rounds"] == 5
    assert res["checked_elems"] == 5 * 2 * (50_536 + 10_164 + 850)
    assert status is None  # still serving


def test_reference_cpu_process_serves_c2_eight_owners(tmp_path):
    """BASELINE C2 (ResNet-18 split "3,8", 8 owners) through the reference's process: receipt templates from
    the reference's own builders (ref_harness golden), the owners' addresses in the refactor message
    (fake_owners --routing-table; without it the reference cannot reach owner ids above 3), one round,
    every reply bit-exact.  tools/e2e_ref.py c2 times the same pairing against fa_aggregator."""
    harness = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
    for mp in ("-1", "2"):
        subprocess.run([harness, "golden", "1", "1", "9", "3", "10", "1", "24301", "7", str(tmp_path), mp],
                       check=True, capture_output=True, timeout=600)
    if not ports_free():
        pytest.skip("the reference's fixed ports 8080-8083 are in use")
    with tempfile.TemporaryDirectory() as cwd:
        agg = subprocess.Popen([REF_CPU_AGG, "8", "1"], stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, cwd=cwd,
                               start_new_session=True)
        try:
            time.sleep(2.5)
            assert agg.poll() is None, agg.stderr.read()
            r = subprocess.run([OWNERS, "--blobs", str(tmp_path), "--parts", "1,2,3", "-d", "8", "-c", "1",
                                "--rounds", "1", "--port-base", "8079", "--model-name", "1", "--model-type", "1",
                                "--start", "9", "--end", "3", "--mode", "literal", "--reply-timeout", "120",
                                "--routing-table"], capture_output=True, text=True, timeout=300, cwd=cwd)
        finally:
            if agg.poll() is None:
                os.killpg(agg.pid, 9)
            agg.wait(timeout=30)
    assert r.returncode == 0, r.stderr[-2000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["ok"] and res["checked_elems"] == 8 * (83_584 + 9_442_304 + 5_130)


def test_reference_cpu_process_takes_a_late_copy():
    r, status = run_pair(["--retransmit-late", "1"], rounds=2, reply_timeout=5)
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert not res["ok"]  # round 1 never completes correctly
    assert status not in (None, 0), status  # the process died (SIGSEGV: layers[-1])
