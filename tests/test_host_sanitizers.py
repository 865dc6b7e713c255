"""CPU: sanitizer builds of the host code that network bytes flow through (SURVEY.md 5 "Race detection").

The reference has no sanitizer runs and known races (network_layer.cpp:395-401: check_new_task drops and
re-takes its lock by hand; the receiver thread is a second consumer at startup).  Here:

* ASan + UBSan: tests/tools/fuzz_host.cpp mutates the committed receipts (torch::save archives built by
  the reference's own model builders, and wire frames encoded by its Message.h) -- truncations, bit
  flips, extreme 16/32/64-bit fields at the zip headers, the data.pkl record and the frame header -- and
  runs every parser stage the aggregator applies to a receipt.  The round-1 parser failed this within
  the first thousand mutations (heap-buffer-overflow in the zip central directory walk).
* TSan: tests/tools/net_selftest.cpp (concurrent senders into one receiver with per-connection reader
  threads and a reorder buffer, pooled pinned frames, 8 sender threads fanning out) under
  ThreadSanitizer.  It found a race between NetLayer::stop() closing the listening socket and the
  receiver thread still polling it.
"""
import glob
import json
import os
import subprocess

import pytest

from conftest import GOLDEN, ROOT

BIN = os.path.join(ROOT, "tests", "tools", "bin")


@pytest.fixture(scope="module", autouse=True)
def sanitizer_builds():
    r = subprocess.run(["make", "-C", os.path.join(ROOT, "tests", "tools"), "sanitizers"], capture_output=True,
                       text=True, timeout=600)
    if r.returncode != 0:
        pytest.fail("sanitizer build failed:\n" + r.stderr[-3000:])


def seeds():
    files = sorted(glob.glob(os.path.join(GOLDEN, "*", "mp*_client0.pt")))
    files += sorted(glob.glob(os.path.join(GOLDEN, "frames", "*.bin")))
    assert len(files) >= 8
    return files


@pytest.mark.parametrize("seed", [1, 2])
def test_parsers_under_asan_ubsan_mutation_fuzz(seed):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([os.path.join(BIN, "fuzz_host_asan"), "1500", str(seed)] + seeds(), capture_output=True,
                       text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-4000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["ok"] and res["runs"] == 1500 * len(seeds())
    assert res["archives_ok"] > 0 and res["frames_ok"] > 0  # the mutations reach past the first checks


def test_network_layer_under_tsan():
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1")
    for _ in range(2):  # interleavings differ run to run
        r = subprocess.run([os.path.join(BIN, "net_selftest_tsan"),
                            os.path.join(GOLDEN, "resnet18_c2", "mp1_client0.pt")],
                           capture_output=True, text=True, timeout=300, env=env)
        assert r.returncode == 0, r.stderr[-4000:]
        assert json.loads(r.stdout.strip().splitlines()[-1])["ok"]


def test_reply_crc32_matches_zlib():
    """The CRC-32 that seals every reply's zip records (host/archive.cpp: PCLMULQDQ folding where the CPU has
    it) equals zlib's and the table form on every length 0..2999 at five misalignments and on multi-MB buffers
    (tests/tools/crc_selftest.cpp); the reference's torch::load would reject a reply with a wrong one."""
    subprocess.run(["make", "-C", os.path.join(ROOT, "tests", "tools")], capture_output=True, timeout=600, check=True)
    r = subprocess.run([os.path.join(BIN, "crc_selftest")], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr[-2000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["bad"] == 0 and res["checks"] > 15_000


def test_archive_layout_cache():
    """Every receipt of a bucket is the same module saved again, so the archive parse caches its tensor views
    by structure + pickle + code records (host/archive.cpp): on every committed receipt archive a second copy
    with other parameter values, elsewhere in memory, hits the cache and its views equal the walk's, rebased;
    a changed pickle byte misses it (tests/tools/archive_cache_selftest.cpp)."""
    import glob
    subprocess.run(["make", "-C", os.path.join(ROOT, "tests", "tools")], capture_output=True, timeout=600, check=True)
    blobs = sorted(glob.glob(os.path.join(GOLDEN, "*", "mp*_client0.pt")))
    assert len(blobs) >= 5
    r = subprocess.run([os.path.join(BIN, "archive_cache_selftest")] + blobs, capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr[-2000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["failed"] == 0 and res["checks"] == 6 * len(blobs) and res["hits"] == 2 * len(blobs)


def test_receipt_ledger_under_asan_ubsan():
    """fa_aggregator's receipt ledger (host/receipts.h): late byte copies of earlier rounds, before and after
    the current receipt, in both phases, dropped; an owner clock stepped back, a frozen part resent under a new
    stamp and a retransmission of the current receipt kept (tests/tools/receipts_selftest.cpp)."""
    for exe in ("receipts_selftest", "receipts_selftest_asan"):
        if exe == "receipts_selftest":
            subprocess.run(["make", "-C", os.path.join(ROOT, "tests", "tools")], capture_output=True, timeout=600,
                           check=True)
        r = subprocess.run([os.path.join(BIN, exe)], capture_output=True, text=True, timeout=60,
                           env=dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1"))
        assert r.returncode == 0, r.stderr[-2000:]
        res = json.loads(r.stdout.strip().splitlines()[-1])
        assert res["failed"] == 0 and res["checks"] >= 50
