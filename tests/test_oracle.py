"""CPU tests: the oracle against the reference-generated golden vectors.

tests/golden/<cfg>/ was produced by tools/gen_golden.py running
oracle/_ref/ref_harness: the reference's own model builders + libtorch running
the aggregator op sequence (aggregator.cpp:63-88) through torch::save/load
blobs, and libtorch's acc.add_(x_k, w_k) FedAvg chain.  These tests pin the
C restatement (oracle/fa_oracle.c) to those outputs bit-for-bit.
"""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN

CONFIGS = ["lenet5_c1", "resnet18_c2", "resnet101_c3", "vgg19_c4"]
KINDS = {"fedavg.f32": np.float32, "literal.f32": np.float32, "fedavg_bf16.bf16": np.uint16,
         "fedavg_bf16.f32": np.float32}


def manifest(cfg):
    with open(os.path.join(GOLDEN, cfg, "manifest.json")) as f:
        return json.load(f)


def check_output(cfg, rec, got):
    """Compare with a committed file, or with SHA-256 + sampled bit patterns."""
    if "file" in rec:
        ref = np.fromfile(os.path.join(GOLDEN, cfg, rec["file"]), dtype=got.dtype)
        assert ref.size == got.size
        ut = np.uint32 if got.dtype == np.float32 else np.uint16
        bad = np.flatnonzero(ref.view(ut) != got.view(ut))
        assert bad.size == 0, "%d mismatches, first at %s" % (bad.size, bad[:5])
    else:
        idx = np.asarray(rec["sample_idx"])
        bits = got.view(np.uint32 if got.dtype == np.float32 else np.uint16)[idx]
        assert np.array_equal(bits, np.asarray(rec["sample_bits"], bits.dtype))
        assert hashlib.sha256(got.tobytes()).hexdigest() == rec["sha256"]


def oracle_outputs(O, m, b, kinds):
    n, s = b["numel"], b["bucket_seed"]
    w = O.weights(m["D"])
    xs = [O.gen(s, k, n) for k in range(m["D"])]
    out = {}
    if "fedavg.f32" in kinds:
        out["fedavg.f32"] = O.fedavg(xs, w, threads=4)
    if "literal.f32" in kinds:
        out["literal.f32"] = O.literal(xs[-1])
    xb = [O.f32_to_bf16(x) for x in xs]
    if "fedavg_bf16.bf16" in kinds:
        out["fedavg_bf16.bf16"] = O.fedavg(xb, w, out_dtype="bf16", threads=4)
    if "fedavg_bf16.f32" in kinds:
        out["fedavg_bf16.f32"] = O.fedavg(xb, w, out_dtype="f32", threads=4)
    return out


@pytest.mark.parametrize("cfg", CONFIGS)
def test_weights_match_golden(O, cfg):
    m = manifest(cfg)
    w = O.weights(m["D"])
    assert np.array_equal(w, np.asarray(m["weights"], np.float32))
    assert abs(float(w.astype(np.float64).sum()) - 1.0) < 1e-6


@pytest.mark.parametrize("cfg", CONFIGS)
def test_oracle_matches_reference_golden(O, cfg):
    m = manifest(cfg)
    for b in m["buckets"]:
        if b["numel"] > 20_000_000:  # VGG FC part: covered by the GPU golden test at full size
            continue
        got = oracle_outputs(O, m, b, KINDS)
        for kind, arr in got.items():
            check_output(cfg, b["outputs"][kind], arr)


def test_literal_is_last_over_500(O):
    """aggregator.cpp:63-88 with parts/parts_ aliased: the round result is fl(2x_last)/1000."""
    m = manifest("resnet18_c2")
    b = m["buckets"][0]
    x_last = O.gen(b["bucket_seed"], m["D"] - 1, b["numel"])
    lit = np.fromfile(os.path.join(GOLDEN, "resnet18_c2", b["outputs"]["literal.f32"]["file"]), np.float32)
    assert np.array_equal(lit, (x_last + x_last) / np.float32(1000.0))
    # ... and it is not the mean the north star asks for
    fed = O.fedavg([O.gen(b["bucket_seed"], k, b["numel"]) for k in range(m["D"])], O.weights(m["D"]))
    assert not np.allclose(lit, fed)


def test_generator_is_exact_and_bounded(O):
    x = O.gen(0x5EED, 3, 100_000)
    assert x.min() >= -1.0 and x.max() < 1.0
    # u24 * 2^-23 - 1 is exact: every value is a multiple of 2^-23
    assert np.all(np.floor(x.astype(np.float64) * 2**23) == x.astype(np.float64) * 2**23)
    assert np.array_equal(O.gen(0x5EED, 3, 10, idx0=500), x[500:510])
    assert np.array_equal(O.gen_at(0x5EED, 3, [0, 7, 99_999]), x[[0, 7, 99_999]])


def test_fedavg_chain_properties(O):
    """Init continuation == one long chain; threads do not change bits; bf16 rounding is RNE."""
    w = O.weights(9)
    xs = [O.gen(11, k, 50_001) for k in range(9)]
    full = O.fedavg(xs, w)
    part = O.fedavg(xs[:4], w[:4])
    assert np.array_equal(O.fedavg(xs[4:], w[4:], init=part), full)
    assert np.array_equal(O.fedavg(xs, w, threads=7), full)
    assert np.array_equal(O.fedavg_at(11, w, [0, 17, 50_000]), full[[0, 17, 50_000]])
    v = np.array([1.0, 1.00390625, 1.01171875, -3.5, 0.0], np.float32)  # ties round to even
    assert O.bf16_to_f32(O.f32_to_bf16(v)).tolist() == [1.0, 1.0, 1.015625, -3.5, 0.0]


@pytest.mark.parametrize("cfg", CONFIGS)
def test_layout_fixture_consistent(cfg):
    """Bucket numel = sum of its named_parameters (models/*: what aggregator.cpp:72 iterates)."""
    with open(os.path.join(GOLDEN, "layouts", cfg + ".json")) as f:
        lay = json.load(f)
    m = manifest(cfg)
    assert [b["model_part"] for b in lay["buckets"]] == [b["model_part"] for b in m["buckets"]]
    for lb, mb in zip(lay["buckets"], m["buckets"]):
        assert lb["numel"] == sum(p["numel"] for p in lb["params"]) == mb["numel"]
        for p in lb["params"]:
            assert p["numel"] == int(np.prod(p["shape"]))


def test_reference_sizes_match_survey():
    """ResNet-18 split 3,8 / ResNet-101 10,19 / VGG-19 3,19 bucket sizes."""
    def sizes(cfg):
        with open(os.path.join(GOLDEN, "layouts", cfg + ".json")) as f:
            return [b["numel"] for b in json.load(f)["buckets"]]
    assert sizes("resnet18_c2") == [83_584, 9_442_304, 5_130]
    assert sizes("resnet101_c3") == [2_594_688, 29_511_680, 5_130]
    assert sizes("vgg19_c4") == [38_720, 2_359_808, 119_586_826]
