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
        b = random.randrange(10000, 32000, 100)  # below the ephemeral port range
        if ports_free(b):
            return b
    pytest.skip("no free port range")


@pytest.fixture(scope="module", autouse=True)
def built():
    subprocess.run(["make", "-C", os.path.join(ROOT, "tests", "tools")], check=True, capture_output=True)
    assert os.access(AGG, os.X_OK), "build the package first (make -C %s)" % PKG_DIR


@pytest.mark.parametrize("mode,D,rounds,table", [("fedavg", 2, 3, False), ("literal", 2, 2, False),
                                                  ("fedavg", 5, 2, False), ("fedavg", 21, 2, True)])
def test_lenet_rounds_over_tcp(torch_gpu, mode, D, rounds, table):
    """table: the refactor message carries the owners' addresses (read_table 1, owner ids 4..21: both of the
    reference's port ranges, network_layer.cpp:510-534), as the reference's init node sends it."""
    base = pick_base()
    agg = subprocess.Popen([AGG, "-i", "-1", "-d", str(D), "-c", "1", "--mode", mode, "--rounds", str(rounds),
                            "--port-base", str(base)], stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    try:
        time.sleep(0.5)
        r = subprocess.run([OWNERS, "--blobs", os.path.join(GOLDEN, "lenet5_c1"), "--parts", "1,2,3", "-d", str(D),
                            "-c", "1", "--rounds", str(rounds), "--mode", mode, "--port-base", str(base),
                            "--model-name", "2", "--start", "6", "--end", "1"] + (["--routing-table"] if table else []),
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


def _large_parts(d, bf16=False):
    """Model-part archives of a few MB (torch.jit.save: the same zip/pickle layout as torch::save), big
    enough that the aggregator receives them into its pooled pinned buffers and replies from them;
    bf16 parameters (BFloat16Storage records) with bf16=True."""
    import torch
    import torch.nn as nn
    torch.manual_seed(1)
    parts = {1: nn.Sequential(nn.Conv2d(3, 64, 3), nn.ReLU(), nn.Conv2d(64, 64, 3)),
             2: nn.Sequential(nn.Linear(1024, 2304), nn.ReLU()),  # 9.4 MB: above the receive gate's 8 MiB
             3: nn.Sequential(nn.Linear(2304, 1000), nn.ReLU(), nn.Linear(1000, 10))}
    for mp, m in parts.items():
        if bf16:
            m = m.to(torch.bfloat16)
        torch.jit.save(torch.jit.script(m), os.path.join(d, "mp%d_client0.pt" % mp))
    return {mp: sum(p.numel() for p in m.parameters()) for mp, m in parts.items()}


@pytest.mark.parametrize("pinned,sequential,extra", [
    (True, False, []), (False, False, []), (True, True, []),
    (True, True, ["--eager"]),                          # chains advance as the in-order receipts land
    (True, False, ["--eager"]),
    (True, False, ["--layout", "rs", "--rs-chunks", "3"]),  # RCCL reduce-scatter layout (one GPU: a copy)
    (True, False, ["--rx-concurrency", "2"]),           # 6 owners at once, 2 large receipts received at a time
    (False, False, ["--rx-concurrency", "0"]),          # no receive gate
    (True, False, ["--crc", "host"]),                   # reply CRC-32s from the host (default: the GPU's)
])
def test_multi_mb_parts_concurrent_owners(torch_gpu, tmp_path, pinned, sequential, extra):
    """D=6 owners sending at once (or one after another) multi-MB parts: pinned zero-copy ingest
    (fa_submit_gather_pinned from the received frame) and D2H into the reply frame
    (fa_finalize_gather), or the pageable staging path with --no-pinned; phase 2's two buckets reduced
    by one batched launch (fa_reduce_parts), or accumulated on arrival (--eager), or through the rs
    layout; bit-exact FedAvg every round."""
    sizes = _large_parts(str(tmp_path))
    D, rounds = 6, 2
    base = pick_base()
    cmd = [AGG, "-i", "-1", "-d", str(D), "-c", "1", "--rounds", str(rounds), "--port-base", str(base)] + extra
    agg = subprocess.Popen(cmd + ([] if pinned else ["--no-pinned"]), stdout=subprocess.PIPE,
                           stderr=subprocess.PIPE, text=True)
    try:
        time.sleep(0.5)
        r = subprocess.run([OWNERS, "--blobs", str(tmp_path), "--parts", "1,2,3", "-d", str(D), "-c", "1",
                            "--rounds", str(rounds), "--port-base", str(base), "--model-name", "1", "--start", "9",
                            "--end", "3"] + (["--sequential"] if sequential else []),
                           capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        res = json.loads(r.stdout.strip().splitlines()[-1])
        assert res["ok"] and res["checked_elems"] == rounds * D * sum(sizes.values())
        out, err = agg.communicate(timeout=60)
        assert agg.returncode == 0, err[-2000:]
        stats = [json.loads(l) for l in out.splitlines() if l.startswith("{")]
        assert len(stats) == rounds
    finally:
        if agg.poll() is None:
            agg.kill()


@pytest.mark.parametrize("extra,tol", [
    (["--gpus", "2"], 0),                                            # range shards: bit-exact
    (["--gpus", "3", "--eager"], 0),                                 # range shards, accumulate on arrival
    (["--gpus", "3", "--layout", "rs", "--rs-chunks", "3"], 1e-6),   # client shards + the exchange: tolerance
    (["--gpus", "4", "--layout", "rs"], 1e-6),                       # a GPU holds 1-2 of the 6 clients
])
def test_multi_gpu_layouts_through_the_process(torch_gpu, tmp_path, extra, tol):
    """fa_aggregator --gpus G, the drop-in process's multi-GPU layouts end to end, rehearsed as G shards of
    the box's one GPU (--test-shared-device: FA_TEST_SHARED_DEVICE; the rs exchange replaced by its
    definition in ring order): receipts split over the shards from the frames they arrived in, the replies
    gathered back from every shard into one frame.  Range shards must be bit-exact; the client-sharded rs
    layout is held to 1e-6 * sum_k |w_k x_k| element by element (fake_owners --rel-tol)."""
    sizes = _large_parts(str(tmp_path))
    D, rounds = 6, 2
    base = pick_base()
    agg = subprocess.Popen([AGG, "-i", "-1", "-d", str(D), "-c", "1", "--rounds", str(rounds), "--port-base",
                            str(base), "--test-shared-device"] + extra,
                           stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    try:
        time.sleep(0.5)
        r = subprocess.run([OWNERS, "--blobs", str(tmp_path), "--parts", "1,2,3", "-d", str(D), "-c", "1",
                            "--rounds", str(rounds), "--port-base", str(base), "--model-name", "1", "--start", "9",
                            "--end", "3"] + (["--rel-tol", str(tol)] if tol else []),
                           capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        res = json.loads(r.stdout.strip().splitlines()[-1])
        assert res["ok"] and res["checked_elems"] == rounds * D * sum(sizes.values())
        if tol:
            assert 0 <= res["max_err_over_bound"] < 1.0
        out, err = agg.communicate(timeout=60)
        assert agg.returncode == 0, err[-2000:]
        assert len([l for l in out.splitlines() if l.startswith("{")]) == rounds
    finally:
        if agg.poll() is None:
            agg.kill()


@pytest.mark.parametrize("drop_phase", [1, 2])
def test_missing_owner_is_reported_and_times_out(torch_gpu, drop_phase):
    """Failure detection: one data owner never sends its phase-1 (or phase-2) receipts.  The
    reference's aggregator blocks forever (its receive loop, network_layer.cpp:654-665); fa_aggregator names
    the missing owner after --stall-report seconds of silence and exits with code 3 after --receipt-timeout."""
    D, base = 3, pick_base()  # owner ids 0, 2, 3 (aggregator.cpp:103-105 with C = 1); owner k = 1 is id 2
    agg = subprocess.Popen([AGG, "-i", "-1", "-d", str(D), "-c", "1", "--rounds", "1", "--port-base", str(base),
                            "--stall-report", "1", "--receipt-timeout", "3"],
                           stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    try:
        time.sleep(0.5)
        r = subprocess.run([OWNERS, "--blobs", os.path.join(GOLDEN, "lenet5_c1"), "--parts", "1,2,3", "-d", str(D),
                            "-c", "1", "--port-base", str(base), "--model-name", "2", "--start", "6", "--end", "1",
                            "--drop-owner", "1", "--drop-phase", str(drop_phase), "--reply-timeout", "8"],
                           capture_output=True, text=True, timeout=120)
        assert r.returncode == 1  # the owners never get their replies
        out, err = agg.communicate(timeout=60)
        assert agg.returncode == 3, err[-2000:]
        stalls = [l for l in err.splitlines() if "no receipt for" in l]
        assert len(stalls) >= 2 and "giving up" in stalls[-1]
        if drop_phase == 1:
            assert "phase 1" in stalls[0] and "part 1: 1 owner(s) [2]" in stalls[0]
        else:
            assert "phase 2" in stalls[0] and "part 2: 1 owner(s) [2]; part 3: 1 owner(s) [2]" in stalls[0]
            assert sum(l.startswith("{") for l in out.splitlines()) == 0  # no round completed
    finally:
        if agg.poll() is None:
            agg.kill()


@pytest.mark.parametrize("extra", [[], ["--eager"]])
def test_retransmitted_receipts_count_once(torch_gpu, extra):
    """One data owner sends every receipt twice.  The reference counts raw receipts (aggregator.cpp:59-92,
    :112-149), so its phase would end one owner short; fa_aggregator counts distinct (owner, bucket) pairs:
    the duplicate replaces the slot, the round waits for every owner and every reply is bit-exact."""
    D, rounds, base = 4, 2, pick_base()
    agg = subprocess.Popen([AGG, "-i", "-1", "-d", str(D), "-c", "1", "--rounds", str(rounds), "--port-base",
                            str(base), "--stall-report", "5", "--receipt-timeout", "30"] + extra,
                           stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    try:
        time.sleep(0.5)
        r = subprocess.run([OWNERS, "--blobs", os.path.join(GOLDEN, "lenet5_c1"), "--parts", "1,2,3", "-d", str(D),
                            "-c", "1", "--rounds", str(rounds), "--port-base", str(base), "--model-name", "2",
                            "--start", "6", "--end", "1", "--retransmit", "2", "--reply-timeout", "60"],
                           capture_output=True, text=True, timeout=180)
        assert r.returncode == 0, r.stderr[-2000:]
        res = json.loads(r.stdout.strip().splitlines()[-1])
        assert res["ok"] and res["rounds"] == rounds
        out, err = agg.communicate(timeout=60)
        assert agg.returncode == 0, err[-2000:]
        assert sum(l.startswith("{") for l in out.splitlines()) == rounds
        assert "sent it again" in err or "ignored" in err  # the duplicates were seen, and not counted
    finally:
        if agg.poll() is None:
            agg.kill()


def _run_late_copies(extra, owner_flags, rounds=3, D=4):
    """fa_aggregator against fake owners with the given failure injection; returns the round lines."""
    base = pick_base()
    agg = subprocess.Popen([AGG, "-i", "-1", "-d", str(D), "-c", "1", "--rounds", str(rounds), "--port-base",
                            str(base), "--stall-report", "5", "--receipt-timeout", "30"] + extra,
                           stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    try:
        time.sleep(0.5)
        r = subprocess.run([OWNERS, "--blobs", os.path.join(GOLDEN, "lenet5_c1"), "--parts", "1,2,3", "-d", str(D),
                            "-c", "1", "--rounds", str(rounds), "--port-base", str(base), "--model-name", "2",
                            "--start", "6", "--end", "1", "--reply-timeout", "60"] + owner_flags
                           + (["--mode", "literal"] if "literal" in extra else []),
                           capture_output=True, text=True, timeout=180)
        assert r.returncode == 0, r.stderr[-2000:]
        res = json.loads(r.stdout.strip().splitlines()[-1])
        assert res["ok"] and res["rounds"] == rounds
        out, err = agg.communicate(timeout=60)
        assert agg.returncode == 0, err[-2000:]
        lines = [json.loads(l) for l in out.splitlines() if l.startswith("{")]
        assert len(lines) == rounds
        return lines, err
    finally:
        if agg.poll() is None:
            agg.kill()


def _assert_late_copies_counted(lines, parts=3):
    """Owner K sends its previous round's receipt of every bucket twice per round (once before and once after
    the current one).  Both copies of every bucket are dropped, none absorbed: the counts are exact.  K sends
    in order and the aggregator takes receipts in accept order, so by the end of round r every copy of
    rounds < r and all of round r's but (at most) the after-copy of its last bucket have been seen; that one
    lands in the next round's phase 1 (an other-phase byte copy, also counted) or after the last round."""
    assert lines[0]["stale_dropped"] == 0  # round 0 has no earlier round to be late from
    for r, l in enumerate(lines[1:], start=1):
        assert 2 * parts * r - 1 <= l["stale_dropped"] <= 2 * parts * r, (r, l)
        assert l["replaced"] == 0 and l["ignored"] == 0, l  # no copy replaced a slot or was taken for a resend


@pytest.mark.parametrize("extra", [[], ["--eager"], ["--mode", "literal"]])
def test_late_duplicates_of_earlier_rounds_are_dropped(torch_gpu, extra):
    """Owner 2 re-sends its previous round's receipts during the next round, once before and once after the
    current ones (fake_owners --retransmit-late).  The wire has no round number; a late copy is a byte copy
    of a frame already reduced, t_start included (stamped when the owner sent it, network_layer.cpp:761), so
    fa_aggregator drops it by its (t_start, length, content) key: it neither counts as the owner's receipt nor
    replaces the newer one, every reply of every round stays bit-exact against the oracle over THIS round's
    values, and the counts are exact (aggregator.cpp:59-92 would reduce the stale parameters without a word)."""
    lines, err = _run_late_copies(extra, ["--retransmit-late", "2"])
    assert "stale part" in err, err[-2000:]
    _assert_late_copies_counted(lines)
    assert all(l["clock_back"] == 0 for l in lines)


@pytest.mark.parametrize("extra", [[], ["--eager"], ["--mode", "literal"]])
def test_owner_clock_going_back_does_not_stall(torch_gpu, extra):
    """Owner 1's clock steps back 10 minutes every round (fake_owners --clock-skew 1,600000: an NTP step, a VM
    resume), so each round its genuine receipts are stamped before its receipts of the previous round.  The
    ledger drops only byte copies of reduced receipts, so they are accepted (the log names the clock), the
    rounds complete and every reply is bit-exact.  The same owner also re-sends its previous round's receipts
    late (--retransmit-late 1): those copies now carry stamps NEWER than the current receipts, and are still
    dropped, every one."""
    lines, err = _run_late_copies(extra, ["--clock-skew", "1,600000", "--retransmit-late", "1"])
    assert "clock went back" in err, err[-2000:]
    for r, l in enumerate(lines):
        assert l["clock_back"] == r, (r, l)  # its part 1 of every later round (phase 2 follows its own part 1)
    _assert_late_copies_counted(lines)


@pytest.mark.parametrize("extra", [[], ["--eager"], ["--mode", "literal"], ["--layout", "rs", "--rs-chunks", "3"]])
def test_bf16_parts_over_tcp(torch_gpu, tmp_path, extra):
    """BASELINE config C3's dtype through the drop-in process: owners send bf16 model parts
    (BFloat16Storage records); the aggregator reduces them in bf16 buckets (fp32 chain, one rounding)
    and replies in bf16, bit-exact against the oracle's bf16 FedAvg (or the literal last/500 in bf16);
    the rs layout too (one GPU: the reduce-scatter is a copy, then the one rounding to bf16)."""
    sizes = _large_parts(str(tmp_path), bf16=True)
    D, rounds = 5, 2
    base = pick_base()
    literal = "literal" in extra
    agg = subprocess.Popen([AGG, "-i", "-1", "-d", str(D), "-c", "1", "--rounds", str(rounds), "--port-base",
                            str(base)] + extra, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    try:
        time.sleep(0.5)
        r = subprocess.run([OWNERS, "--blobs", str(tmp_path), "--parts", "1,2,3", "-d", str(D), "-c", "1",
                            "--rounds", str(rounds), "--port-base", str(base), "--model-name", "1", "--start", "9",
                            "--end", "3"] + (["--mode", "literal"] if literal else []),
                           capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        res = json.loads(r.stdout.strip().splitlines()[-1])
        assert res["ok"] and res["checked_elems"] == rounds * D * sum(sizes.values())
        out, err = agg.communicate(timeout=60)
        assert agg.returncode == 0, err[-2000:]
    finally:
        if agg.poll() is None:
            agg.kill()


def _stream_run(blobs, parts_spec, D, rounds, agg_extra, owner_extra, timeout=300):
    """fa_aggregator with streaming ingest against fake owners whose frames go out in random pieces
    (fake_owners --chunked); returns (owners' result, the aggregator's round lines, its stderr)."""
    base = pick_base()
    agg = subprocess.Popen([AGG, "-i", "-1", "-d", str(D), "-c", "1", "--rounds", str(rounds), "--port-base",
                            str(base), "--stall-report", "20", "--receipt-timeout", "120"] + agg_extra,
                           stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    try:
        time.sleep(0.5)
        r = subprocess.run([OWNERS, "--blobs", blobs, "--parts", "1,2,3", "-d", str(D), "-c", "1", "--rounds",
                            str(rounds), "--port-base", str(base), "--reply-timeout", "120"] + parts_spec + owner_extra,
                           capture_output=True, text=True, timeout=timeout)
        assert r.returncode == 0, r.stderr[-2000:]
        res = json.loads(r.stdout.strip().splitlines()[-1])
        out, err = agg.communicate(timeout=60)
        assert agg.returncode == 0, err[-2000:]
        lines = [json.loads(l) for l in out.splitlines() if l.startswith("{")]
        assert len(lines) == rounds
        return res, lines, err
    finally:
        if agg.poll() is None:
            agg.kill()


LENET = ["--model-name", "2", "--start", "6", "--end", "1"]
LARGE = ["--model-name", "1", "--start", "9", "--end", "3"]


@pytest.mark.parametrize("chunks,extra", [
    ("1,64,7", []),                               # 1..64-byte pieces: every record boundary splits somewhere
    ("1,65536,8", []),                            # 1 B .. 64 KiB
    ("1,65536,9", ["--eager"]),                   # the chain advances on commits
    ("1,65536,10", ["--mode", "literal"]),        # literal: owners in turn, the last committed receipt
    ("1,4096,11", ["--gpus", "2", "--test-shared-device"]),  # range shards: each piece split over the GPUs
])
def test_streaming_ingest_lenet_random_pieces(torch_gpu, chunks, extra):
    """Streaming ingest: every frame (--stream-min-bytes 1) is DMA'd to its slot record by
    record while it arrives, the owners writing their frames in random pieces of 1 byte to 64 KiB with random
    pauses, all owners at once, so the frames land interleaved in random order.  Once a bucket's first receipt
    has given its layout, receipts are committed from their streams; every reply bit-exact."""
    D, rounds = 3, 3
    owner = ["--chunked", chunks] + (["--mode", "literal"] if "literal" in extra else [])
    res, lines, err = _stream_run(os.path.join(GOLDEN, "lenet5_c1"), LENET, D, rounds,
                                  ["--stream-min-bytes", "1"] + extra, owner)
    assert res["ok"] and res["checked_elems"] == rounds * D * (50_536 + 10_164 + 850)
    # the layout of a bucket comes from its first receipt: later frames of the same round stream already
    assert lines[0]["streamed"] <= D * 3 - 3
    # most later receipts (a tiny frame can land whole before the main thread has claimed it: the plain path)
    assert lines[-1]["streamed"] >= (rounds - 1) * D * 3 // 2, lines[-1]
    assert lines[-1]["stream_fallbacks"] == 0 and lines[-1]["streamed_bytes"] > 0


@pytest.mark.parametrize("extra", [[], ["--eager"], ["--layout", "rs", "--rs-chunks", "3"],
                                   ["--gpus", "3", "--test-shared-device"]])
def test_streaming_ingest_multi_mb_parts(torch_gpu, tmp_path, extra):
    """Multi-MB parts at the default threshold (frames of >= 1 MiB stream) in random 4..64 KiB pieces: parts
    2 and 3 are streamed from round 1 on, part 1 (150 KB) is not; every reply bit-exact (rs: the bound)."""
    sizes = _large_parts(str(tmp_path))
    D, rounds = 6, 3
    tol = ["--rel-tol", "1e-6"] if "rs" in extra else []
    res, lines, err = _stream_run(str(tmp_path), LARGE, D, rounds, extra, ["--chunked", "4096,65536,3"] + tol)
    assert res["ok"] and res["checked_elems"] == rounds * D * sum(sizes.values())
    assert lines[-1]["streamed"] >= (rounds - 1) * D * 2 - 4, lines[-1]
    assert lines[-1]["stream_fallbacks"] == 0


@pytest.mark.parametrize("extra", [[], ["--eager"]])
def test_streaming_with_late_copies_and_retransmissions(torch_gpu, extra):
    """Streamed frames that must NOT end up in a slot: owner 2 re-sends its previous round's receipts before
    and after the current ones (late byte copies, stale), all of it in random pieces, streamed.  A stale copy may stream into the empty slot but is never committed, and a
    receipt that lands whole stops any other frame streaming into its slot: every reply bit-exact and the
    stale counts exact, as without streaming."""
    D, rounds = 4, 3
    res, lines, err = _stream_run(os.path.join(GOLDEN, "lenet5_c1"), LENET, D, rounds,
                                  ["--stream-min-bytes", "1"] + extra,
                                  ["--chunked", "1,65536,5", "--retransmit-late", "2"])
    assert res["ok"] and res["rounds"] == rounds
    for r, l in enumerate(lines[1:], start=1):
        assert 2 * 3 * r - 1 <= l["stale_dropped"] <= 2 * 3 * r, (r, l)
    assert lines[-1]["streamed"] > 0
