"""GPU: the reference-side binding of INTEGRATION.md section 2 run for real, inside the reference's own
process structure (VERDICT r02 "next" #3).

oracle/_ref/ref_aggregator (oracle/Makefile.ref, built in the build container from /root/reference's
sources as they lie) is the reference's systemAPI + network_layer + model builders + libtorch, with
aggregator.cpp:55-167 replaced by the INTEGRATION.md block `aggregate_rounds` (extracted verbatim) calling
libfa.so.  Only aggregator.cpp's argparse and multicast discovery are left out (oracle/ref_aggregator_main.cpp).
One LeNet-5 round (BASELINE config C1: 2 data owners) goes through it: the fake owners (tests/tools,
speaking the reference's frame) send the refactor message and the receipts, and check every reply --
serialized by the reference's own new_message / torch::save -- bit-for-bit against the oracle's FedAvg.

The reference's routing table is fixed (network_layer.h:80-86): the aggregator listens on 8080 and replies
to owners 0 and 2 on 8081 and 8083, so the test needs those ports free (the GPU box).
"""
import json
import os
import socket
import subprocess
import time

import pytest

from conftest import GOLDEN, ROOT

pytestmark = pytest.mark.gpu

REF_AGG = os.path.join(ROOT, "oracle", "_ref", "ref_aggregator")
OWNERS = os.path.join(ROOT, "tests", "tools", "bin", "fa_fake_owners")


def ports_free(ports):
    for p in ports:
        with socket.socket() as s:
            try:
                s.bind(("0.0.0.0", p))
            except OSError:
                return False
    return True


@pytest.mark.skipif(not os.access(REF_AGG, os.X_OK), reason="oracle/_ref/ref_aggregator not built (needs the "
                    "reference tree in the build container: make -f oracle/Makefile.ref)")
def test_reference_process_with_the_binding_runs_a_lenet_round(torch_gpu, tmp_path):
    if not ports_free([8080, 8081, 8082, 8083]):
        pytest.skip("the reference's fixed ports 8080-8083 are in use")
    D, C = 2, 1
    log_out, log_err = open(tmp_path / "ref_agg.out", "w"), open(tmp_path / "ref_agg.err", "w")
    agg = subprocess.Popen([REF_AGG, str(D), str(C)], stdout=log_out, stderr=log_err, start_new_session=True)
    err = lambda: open(tmp_path / "ref_agg.err").read()[-3000:]  # noqa: E731
    try:
        time.sleep(2.5)  # the reference's receiver binds 8080 one second after it is released
        assert agg.poll() is None, err()
        # owners in id order (--sequential): the binding's chain order is the owners' ids, the oracle's too
        r = subprocess.run([OWNERS, "--blobs", os.path.join(GOLDEN, "lenet5_c1"), "--parts", "1,2,3", "-d", str(D),
                            "-c", str(C), "--rounds", "1", "--port-base", "8079", "--model-name", "2", "--start",
                            "6", "--end", "1", "--sequential", "--reply-timeout", "90"],
                           capture_output=True, text=True, timeout=240)
        assert r.returncode == 0, (r.stdout[-1000:], r.stderr[-2000:])
        res = json.loads(r.stdout.strip().splitlines()[-1])
        # parts 1, 2, 3 of LeNet-5 (C1), every element of every reply bit-exact
        assert res["ok"] and res["rounds"] == 1 and res["checked_elems"] > 0, res
    finally:
        if agg.poll() is None:
            os.killpg(agg.pid, 9)  # the reference's loop never returns (aggregator.cpp:55)
        agg.wait(timeout=30)
        log_out.close()
        log_err.close()
    assert "refactor done" in err(), err()


REF_CN = os.path.join(ROOT, "oracle", "_ref", "ref_compute_node")


@pytest.mark.skipif(not os.access(REF_CN, os.X_OK), reason="oracle/_ref/ref_compute_node not built (needs the "
                    "reference tree in the build container: make -f oracle/Makefile.ref)")
@pytest.mark.parametrize("D,spec", [(8, ("1", "1", "4", "8")),    # C2: ResNet-18 split 3,8 -> layers 4..8
                                    (3, ("2", "0", "2", "5"))])   # LeNet-5's middle layers
def test_compute_node_binding_on_the_reference_states(torch_gpu, tmp_path, D, spec):
    """INTEGRATION.md section 5 run for real: the reference's own compute node state --
    systemAPI(false, id) + refactor() -> init_state_vector (systemAPI.cpp:3-15), one State per data owner
    with the layers the reference's builders make for the node's part -- aggregated through libfa.so by the
    binding block extracted verbatim (oracle/_ref/compute_node_fa.cpp).  Every client's every layer must equal
    the oracle's ordered FedAvg chain over the same values with the binding's weights (n_k differ), bit for
    bit.  The reference never aggregates a compute node's states (compute_node.cpp:16-84)."""
    if not ports_free([8080, 8081, 8082, 8083]):
        pytest.skip("the reference's fixed ports 8080-8083 are in use")
    r = subprocess.run([REF_CN, str(D)] + list(spec), capture_output=True, text=True, timeout=240, cwd=str(tmp_path))
    assert r.returncode == 0, (r.stdout[-1000:], r.stderr[-2000:])
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["ok"] and res["mismatches"] == 0 and res["clients"] == D and res["layers"] >= 1
    assert res["checked_elems"] >= D * res["layer0_elems"] > 0
