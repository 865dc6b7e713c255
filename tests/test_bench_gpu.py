"""GPU: bench.py's own legs on the one-GPU box, each ending with its parity object (verdict r03 #1).

* A workload held in range pieces (forced small with --piece-split-kib / --piece-span-kib, as C5's 128 x 1 GiB
  is on one GPU) prints its line: read_stream_peak walks the pieces instead of asking fa_bucket_slot for a
  contiguous slot, and the client-sharded layout builds contiguous slots.
* `--ctx-multi range|rs` (the in-process multi-GPU children the N = 1 run starts on a node with several
  GPUs) and `--gpus 2` (two ranks sharing the GPU over gloo: the driver's N > 1 launch, rehearsed) carry
  a passing parity object on the main line and on every secondary, so the first run on an 8-GPU node is
  also the first parity test of its reduce-scatter and range legs.
"""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu
BENCH = os.path.join(ROOT, "bench.py")


def run_bench(args, env=None, timeout=240, tmp=None):
    """The bench's own output: the full object (the side file its compact stdout line names) for a main line,
    the printed object for a --ctx-multi child."""
    import tempfile
    with tempfile.TemporaryDirectory(prefix="fa_bench_") as d:
        full = os.path.join(d, "full.json")
        r = subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True, timeout=timeout, cwd=ROOT,
                           env=dict(os.environ, FA_BENCH_FULL=full, **(env or {})))
        assert r.returncode == 0, r.stderr[-3000:]
        printed = r.stdout.strip().splitlines()
        line = json.loads(printed[-1])
        if "full_record" not in line:
            return line
        assert len(printed) == 1, printed[:-1]  # a main line: one line on stdout, nothing else
        assert len(printed[-1]) <= 6000
        with open(full) as f:
            return json.load(f)


def ok(p, samples=1024):
    assert p and p["ok"] and p["mismatches"] == 0 and p["samples"] >= samples, p


PIECES = ["--piece-split-kib", "-1", "--piece-span-kib", str(256 << 10)]  # ns_w8's 1 GiB of slots -> 4 pieces


@pytest.mark.parametrize("layout", ["range", "rs"])
def test_pieced_workload_prints_its_line(fa, torch_gpu, layout):
    line = run_bench(["--workload", "ns_w8", "--layout", layout, "--steps", "3", "--warmup", "1", "--no-cpu-baseline",
                      "--no-secondary", "--no-live-pmc"] + PIECES)
    ok(line["parity"])
    assert line["value"] > 0 and line["roofline"]["phased_meeting_timeouts"] == 0
    if layout == "range":
        assert line["roofline"]["read_stream_peak"] > 0
        assert line["parity"]["check"].startswith("bit-exact")


@pytest.mark.parametrize("workload", ["c3", "c2"])
def test_read_stream_peak_of_bf16_and_rotated_workloads(fa, torch_gpu, workload):
    """The read-only rate beside a config's kernel: a bf16 workload (C3) is read as the fp32 words its bytes
    make, and a workload whose input set fits the MALL (C2, 3 sets rotated) is read set by set."""
    line = run_bench(["--workload", workload, "--steps", "3", "--warmup", "1", "--no-cpu-baseline", "--no-secondary",
                      "--no-live-pmc"])
    ok(line["parity"])
    rf = line["roofline"]
    assert rf["read_stream_peak"] > 1000 and 0.5 < rf["frac_of_read_stream"] < 1.2, rf


@pytest.mark.parametrize("layout", ["range", "rs"])
def test_ctx_multi_child_carries_parity(fa, torch_gpu, layout):
    res = run_bench(["--ctx-multi", layout, "--workload", "ns_w8", "--steps", "3", "--warmup", "1"])
    ok(res["parity"])
    assert res["gpus"] >= 1 and len(res["parity"]["per_gpu_samples"]) == res["gpus"]
    assert all(s >= 1024 for s in res["parity"]["per_gpu_samples"])


def test_ctx_multi_host_inclusive_parity(fa, torch_gpu):
    """--h2d: every client submitted from pinned host memory (its own buffer: 32 x 32 MiB fit the 16 GiB
    bound) and the result finalized into a pinned host buffer; checked against the oracle's chain, with the
    round's H2D / reduce / D2H split reported."""
    res = run_bench(["--ctx-multi", "range", "--workload", "ns_w8", "--h2d", "--steps", "2", "--warmup", "1",
                     "--ctx-gpus", "1"])
    ok(res["parity"])
    assert res["host_inclusive"] and res["distinct_host_buffers"] == 32
    assert res["h2d_ms"] > 0 and res["reduce_ms"] > 0 and res["d2h_ms"] > 0 and res["pcie_GBs"] > 0


def test_two_rank_rehearsal_parity_everywhere(fa, torch_gpu):
    """The driver's N > 1 launch rehearsed on one GPU (bench.py spawns 2 ranks, gloo): the main range line
    and the weak-range, rs and chain secondaries each carry a parity object summed over both ranks."""
    line = run_bench(["--gpus", "2", "--workload", "ns_w8", "--steps", "3", "--warmup", "1", "--no-live-pmc"],
                     timeout=300)
    assert line["n_gpus"] == 2
    ok(line["parity"], 2 * 1024)
    assert line["parity"]["ranks"] == 2
    for leg in ("weak_range", "rs", "chain"):
        p = line["secondary"][leg]["parity"]
        ok(p, 2 * 1024)
        assert p["ranks"] == 2
    assert line["secondary"]["rs"]["parity"]["max_err_over_bound"] < 1.0


@pytest.mark.parametrize("args", [["--ctx-multi", "rs", "--workload", "c4"],
                                  ["--ctx-multi", "range", "--workload", "c5r", "--h2d"]])
def test_eight_gpu_children_rehearsed_on_one_gpu(fa, torch_gpu, args):
    """The N = 1 run's children on the driver's 8-GPU node (ctx_rs_c4_8gpu; ctx_range_c5_h2d_8gpu with C5's
    per-GPU share, so that 128 clients fit the box's host budget) rehearsed as 8 shards of GPU 0
    (FA_TEST_SHARED_DEVICE: the same dealing, pieces, shard offsets and copy-out; the exchange replaced by its
    definition in ring order): the parity object covers all 8 shards, >= 1024 samples each."""
    res = run_bench(args + ["--ctx-shared", "8", "--steps", "2", "--warmup", "1"], timeout=300)
    assert res["gpus"] == 8 and res["shared_device_rehearsal"]
    ok(res["parity"], 8 * 1024)
    assert len(res["parity"]["per_gpu_samples"]) == 8 and min(res["parity"]["per_gpu_samples"]) >= 1024
    if "rs" in args:
        assert res["parity"]["max_err_over_bound"] < 1.0


@pytest.mark.parametrize("chunks", [2, 16])
def test_rs_chunk_sweep_child_rehearsed_on_one_gpu(fa, torch_gpu, chunks):
    """The rs overlap-depth sweep the N = 1 run starts on a multi-GPU node (ctx_rs_c4_4gpu_rschunks<K>),
    rehearsed as 4 shards of GPU 0 on a smaller bucket: the context takes the piece count it was given, and
    every GPU's block-cyclic segments still pass the 1e-6 bound."""
    res = run_bench(["--ctx-multi", "rs", "--workload", "ns_w8", "--ctx-shared", "4", "--rs-chunks", str(chunks),
                     "--steps", "2", "--warmup", "1"])
    assert res["tuning"]["rs_chunks"] == chunks and res["gpus"] == 4
    ok(res["parity"], 4 * 1024)
    assert res["parity"]["max_err_over_bound"] < 1.0
