"""CPU tests of the C ABI boundary: libfa.so loads and exports every symbol that
include/fedavg/fa.h declares; argument checking and error reporting work
without touching a GPU (no compute calls here)."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "fedavg", "fa.h")


def declared_symbols():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(fa_[a-z_]+)\s*\(", src)))


def test_header_declares_the_abi():
    syms = declared_symbols()
    for s in ["fa_create", "fa_bucket_define", "fa_submit", "fa_finalize", "fa_reduce_device", "fa_last_error",
              "fa_destroy"]:
        assert s in syms


def test_library_exports_every_declared_symbol(fa):
    out = subprocess.run(["nm", "-D", "--defined-only", fa.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r" T (fa_\w+)", out))
    missing = [s for s in declared_symbols() if s not in exported]
    assert not missing, missing
    L = fa.lib()
    for s in declared_symbols():
        assert getattr(L, s) is not None


def test_library_is_gfx950_code(fa, tmp_path):
    """The kernels are CDNA4 code objects (gfx950 only, no other targets)."""
    fb = str(tmp_path / "fatbin.bin")
    subprocess.run(["objcopy", "--dump-section", ".hip_fatbin=" + fb, fa.LIB_PATH, str(tmp_path / "scratch.so")],
                   check=True)  # explicit output: objcopy would rewrite the mapped library in place
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/clang-offload-bundler", "--list", "--type=o", "--input=" + fb],
                         capture_output=True, text=True)
    if out.returncode != 0:
        pytest.skip("offload bundler listing unavailable")
    targets = [t for t in out.stdout.split() if "amdgcn" in t]
    assert targets and all("gfx950" in t for t in targets), out.stdout


def test_version_and_errors_without_gpu(fa):
    L = fa.lib()
    assert L.fa_version() == 7
    # argument errors are reported before any device work
    rc = L.fa_reduce_device(None, 0, None, None, 0, 16, 0, None, 0, 0, None, None)
    assert rc == fa.ERR_ARG and "null" in fa.last_error()
    assert L.fa_fill_uniform(None, 4, 7, 0, 0, 0, None) == fa.ERR_ARG
    t = fa._Tuning(96, 0, 0, 0, 0, 0, 0, 0, 0, 0)
    assert L.fa_set_tuning(ctypes.byref(t)) == fa.ERR_ARG
    assert L.fa_bucket_define(None, 1, 10, 0, 0, 1, 0) == fa.ERR_ARG
    assert fa.last_error() == "ctx is null"
    assert L.fa_finalize_gather(None, 1, 0, None, None, 0) == fa.ERR_ARG
    assert L.fa_finalize_gather(None, 1, 0, None, None, 4) == fa.ERR_ARG and "flags" in fa.last_error()
    assert L.fa_submit_gather_pinned(None, 1, 0, 0, None, None, ctypes.c_float(1.0)) == fa.ERR_ARG
    out = ctypes.c_void_p(1)
    assert L.fa_host_alloc(ctypes.c_size_t(0), ctypes.byref(out)) == 0 and out.value is None
    assert L.fa_host_free(None) == 0


def test_tuning_roundtrip(fa):
    before = fa.get_tuning()
    fa.set_tuning(block=128, unroll=16, load_policy=1, store_policy=4, rs_chunks=5)
    assert fa.get_tuning() == {"block": 128, "max_blocks": before["max_blocks"], "unroll": 16, "load_policy": 1,
                               "store_policy": 4, "slot_skew": before["slot_skew"], "walk": before["walk"],
                               "rs_chunks": 5, "piece_span_kib": 16 << 20, "piece_split_kib": 48 << 20}
    with pytest.raises(fa.FaError):
        fa.set_tuning(store_policy=5)
    assert fa.get_tuning()["store_policy"] == 4  # a rejected call changes nothing
    assert before["slot_skew"] == -2  # default: by slot size
    fa.set_tuning(slot_skew=-1)
    assert fa.get_tuning()["slot_skew"] == 0
    fa.set_tuning(slot_skew=-2)
    assert fa.get_tuning()["slot_skew"] == -2
    # range pieces (the former FA_PIECE_SPAN / FA_PIECE_SPLIT environment knobs): -1 = never / always cut
    fa.set_tuning(piece_span_kib=-1, piece_split_kib=-1)
    assert fa.get_tuning()["piece_span_kib"] == -1 and fa.get_tuning()["piece_split_kib"] == -1
    fa.set_tuning(piece_span_kib=16 << 20, piece_split_kib=48 << 20)
    for bad in (dict(slot_skew=100), dict(slot_skew=-3), dict(walk=7), dict(rs_chunks=2000), dict(block=96),
                dict(piece_span_kib=-2), dict(piece_split_kib=-5)):
        with pytest.raises(fa.FaError):
            fa.set_tuning(**bad)
    fa.set_tuning(**{k: (v or -1) if k in ("max_blocks", "slot_skew") else v for k, v in before.items()})
    assert fa.get_tuning() == before


def test_ctx_tuning_needs_a_ctx(fa):
    L = fa.lib()
    t = fa._Tuning()
    assert L.fa_ctx_set_tuning(None, ctypes.byref(t)) == fa.ERR_ARG
    assert L.fa_ctx_get_tuning(None, ctypes.byref(t)) == fa.ERR_ARG
    assert L.fa_reduce_parts(None, 0, None, None, None) == fa.ERR_ARG
    assert L.fa_bucket_progress(None, 1, None, None) == fa.ERR_ARG
    k = ctypes.c_int(7)
    assert L.fa_bucket_host_read(None, 1, ctypes.byref(k)) == fa.ERR_ARG


def test_no_experiment_knobs_in_the_product():
    """The library and the drop-in process read only two environment variables:
    FA_TIMELINE (a diagnostic) and FA_HOST_READ (fa.h); the closed experiments' knobs are gone."""
    from conftest import PKG_DIR
    names = set()
    for sub in ("csrc", "host"):
        d = os.path.join(PKG_DIR, sub)
        for f in os.listdir(d):
            if f.endswith((".hip", ".cpp", ".h")):
                src = open(os.path.join(d, f)).read()
                assert "getenv(name)" not in src and "getenv(k)" not in src, f  # no indirect lookups
                names |= set(re.findall(r'getenv\("([A-Z_0-9]+)"\)', src))
    assert names == {"FA_TIMELINE", "FA_HOST_READ"}, names


@pytest.mark.parametrize("n,world,chunks", [(64, 1, 1), (1000, 2, 1), (10_000, 2, 4), (7_777, 3, 5),
                                            (123_457, 8, 16), (256 * 8, 8, 3), (1 << 20, 4, 8)])
def test_rs_segments_match_shard_cyclic_bounds(fa, n, world, chunks):
    """The C ABI's rs ownership (fa_rs_segments, used by FA_SHARD_CLIENT_RS to copy each GPU's shard out)
    equals shard.cyclic_bounds, whose exchange the gloo tests check against the oracle; together the GPUs'
    segments tile the padded bucket exactly once."""
    import importlib
    shard = importlib.import_module("mhfsl_amd.shard")
    unit = world * shard.UNIT
    npad = -(-n // unit) * unit
    seen = np.zeros(npad, np.int32)
    for g in range(world):
        segs = fa.rs_segments(n, world, chunks, g)
        assert segs == shard.cyclic_bounds(npad, world, g, chunks)
        assert sum(b - a for a, b in segs) == npad // world
        for a, b in segs:
            seen[a:b] += 1
    assert np.all(seen == 1)
    with pytest.raises(fa.FaError):
        fa.rs_segments(n, world, chunks, world)


def test_no_device_fails_loudly(fa):
    """No CPU fallback: without a GPU the context cannot be created."""
    import torch  # noqa: F401  (same import order as the product users)
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    with pytest.raises(fa.FaError) as e:
        fa.Aggregator(1)
    assert e.value.code in (fa.ERR_NODEV, fa.ERR_ARG)


def test_native_bench_built_and_checks_arguments():
    """bin/fa_bench (the C++-only round timer) is built with the library; bad arguments exit with 2
    before any device work (so this runs without a GPU)."""
    import os
    import subprocess
    from conftest import PKG_DIR
    exe = os.path.join(PKG_DIR, "bin", "fa_bench")
    assert os.access(exe, os.X_OK)
    for bad in (["--workload", "nope"], ["--steps", "0"], ["--layout", "ring"], ["--frobnicate"]):
        r = subprocess.run([exe] + bad, capture_output=True, text=True, timeout=60)
        assert r.returncode == 2, (bad, r.stderr)
