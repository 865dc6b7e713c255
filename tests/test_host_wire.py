"""CPU tests of the C++ host side: the torch::save archive view and the Message.h frame.

The archives under tests/golden/<cfg>/mp*_client0.pt were written by the
reference's own model builders through libtorch's torch::save (oracle/_ref), so
they are real wire payloads of the reference (network_layer.cpp:305-313).
"""
import io
import json
import os
import subprocess
import zipfile

import numpy as np
import pytest

from conftest import GOLDEN, PKG_DIR, ROOT

TOOL = os.path.join(PKG_DIR, "bin", "fa_archive_tool")
BLOBS = [(cfg, mp) for cfg in ("lenet5_c1", "resnet18_c2") for mp in (1, 2, 3)
         if os.path.exists(os.path.join(GOLDEN, cfg, "mp%d_client0.pt" % mp))]


def tool(*args):
    return subprocess.run([TOOL, *map(str, args)], capture_output=True, text=True, check=True).stdout


def layout(cfg, mp):
    with open(os.path.join(GOLDEN, "layouts", cfg + ".json")) as f:
        return [b for b in json.load(f)["buckets"] if b["model_part"] == mp][0]


def manifest_bucket(cfg, mp):
    with open(os.path.join(GOLDEN, cfg, "manifest.json")) as f:
        return [b for b in json.load(f)["buckets"] if b["model_part"] == mp][0]


def test_fixture_blobs_present():
    assert len(BLOBS) >= 5


@pytest.mark.parametrize("cfg,mp", BLOBS)
def test_archive_layout_matches_reference_builders(cfg, mp):
    """Parameter names/shapes in named_parameters() order, buffers in named_buffers() order."""
    d = json.loads(tool("dump", os.path.join(GOLDEN, cfg, "mp%d_client0.pt" % mp)))
    ref = layout(cfg, mp)
    assert [(p["name"], p["shape"]) for p in d["params"]] == [(p["name"], p["shape"]) for p in ref["params"]]
    assert [b["name"] for b in d["buffers"]] == [b["name"] for b in ref["buffers"]]
    assert d["param_numel"] == ref["numel"]
    assert all(p["storage"] == "FloatStorage" and p["contiguous"] for p in d["params"])


@pytest.mark.parametrize("cfg,mp", BLOBS)
def test_archive_values_are_the_senders(O, cfg, mp, tmp_path):
    """The mapped parameter records hold exactly what the data owner put in (client 0's generator values)."""
    out = tmp_path / "p.f32"
    tool("gather", os.path.join(GOLDEN, cfg, "mp%d_client0.pt" % mp), out)
    b = manifest_bucket(cfg, mp)
    got = np.fromfile(out, np.float32)
    assert np.array_equal(got.view(np.uint32), O.gen(b["bucket_seed"], 0, b["numel"]).view(np.uint32))


@pytest.mark.parametrize("cfg,mp", BLOBS)
def test_patched_archive_loads_in_libtorch(cfg, mp, tmp_path):
    """with_params(): CRCs valid for zipfile, and libtorch's loader sees the new parameters + old buffers."""
    import torch
    src = os.path.join(GOLDEN, cfg, "mp%d_client0.pt" % mp)
    n = json.loads(tool("dump", src))["param_numel"]
    vals = np.random.default_rng(mp).standard_normal(n).astype(np.float32)
    vals.tofile(tmp_path / "v.f32")
    tool("patch", src, tmp_path / "v.f32", tmp_path / "out.pt")
    data = (tmp_path / "out.pt").read_bytes()
    assert zipfile.ZipFile(io.BytesIO(data)).testzip() is None
    m = torch.jit.load(io.BytesIO(data))
    flat = torch.cat([p.detach().reshape(-1) for _, p in m.named_parameters()]) if n else torch.zeros(0)
    assert np.array_equal(flat.numpy().view(np.uint32), vals.view(np.uint32))
    orig = torch.jit.load(src)
    for (na, a), (nb, b) in zip(m.named_buffers(), orig.named_buffers()):
        assert na == nb and torch.equal(a, b)


def test_patched_multi_mb_archive_crcs(tmp_path):
    """The reply seal on a multi-MB archive (seal_params: every record's CRC-32 in 1 MiB chunks over threads,
    joined with crc32_combine): records of 0.5-9.4 MB and one empty one, checked by zipfile against zlib."""
    import torch
    import torch.nn as nn
    torch.manual_seed(3)
    m = nn.Sequential(nn.Linear(1024, 2304), nn.Linear(2304, 1000), nn.Linear(1000, 123), nn.Linear(7, 0))
    src = str(tmp_path / "big.pt")
    torch.jit.save(torch.jit.script(m), src)
    n = json.loads(tool("dump", src))["param_numel"]
    vals = np.random.default_rng(5).standard_normal(n).astype(np.float32)
    vals.tofile(tmp_path / "v.f32")
    tool("patch", src, tmp_path / "v.f32", tmp_path / "out.pt")
    data = (tmp_path / "out.pt").read_bytes()
    assert len(data) > 4 << 20
    assert zipfile.ZipFile(io.BytesIO(data)).testzip() is None
    got = torch.jit.load(io.BytesIO(data))
    flat = torch.cat([p.detach().reshape(-1) for _, p in got.named_parameters()])
    assert np.array_equal(flat.numpy().view(np.uint32), vals.view(np.uint32))


def test_frame_round_trip_and_grammar(tmp_path):
    """[int32 len] + Message.h text; `values` is the archive, binary-safe, followed by ',\\n}'."""
    src = os.path.join(GOLDEN, "lenet5_c1", "mp2_client0.pt")
    tool("frame", src, tmp_path / "f.bin")
    f = (tmp_path / "f.bin").read_bytes()
    blob = open(src, "rb").read()
    n = int.from_bytes(f[:4], "little")
    assert n == len(f) - 4
    head = (b"{,\nsave_connection : 0,\ntype : 0,\nclient_id : 7,\nprev_node : -1,\nsize_ : 0,\ntype_op : 5,\n"
            b"model_part : 2,\nt_start : 1700000000000,\nbatch0 : -1,\nvalues : ")
    assert f[4:4 + len(head)] == head
    assert f[4 + len(head):] == blob + b",\n}"
    meta = json.loads(tool("unframe", tmp_path / "f.bin", tmp_path / "back.pt"))
    assert meta == {"client_id": 7, "model_part": 2, "type_op": 5, "bytes": len(blob)}
    assert (tmp_path / "back.pt").read_bytes() == blob


def test_archive_rejects_garbage(tmp_path):
    p = tmp_path / "bad.pt"
    p.write_bytes(b"PK\x03\x04" + b"\x00" * 100)
    r = subprocess.run([TOOL, "dump", str(p)], capture_output=True, text=True)
    assert r.returncode != 0 and "zip" in r.stderr


@pytest.mark.parametrize("cfg", ["lenet5_c1", "resnet18_c2"])
def test_net_layer_and_buffer_pool_selftest(cfg):
    """CPU: concurrent per-connection receive in accept order, pooled frame buffers recycled after
    round 1, serialize-once fan-out in order per destination, and the split reply-archive copy
    (layout_into + seal_params == with_params_into) on a reference-built archive."""
    subprocess.run(["make", "-C", os.path.join(ROOT, "tests", "tools")], check=True, capture_output=True)
    exe = os.path.join(ROOT, "tests", "tools", "bin", "net_selftest")
    r = subprocess.run([exe, os.path.join(GOLDEN, cfg, "mp1_client0.pt")], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["ok"] and res["archive_bytes"] > 0


FRAMES = os.path.join(GOLDEN, "frames")


def _frame_cases():
    with open(os.path.join(FRAMES, "manifest.json")) as f:
        return json.load(f)["cases"]


@pytest.mark.parametrize("case", _frame_cases(), ids=lambda c: c["name"])
def test_wire_matches_reference_encoder_and_parser(case, tmp_path):
    """host/wire.cpp against the reference's own Message.h (tests/golden/frames, tools/gen_wire_golden.py):
    the same arguments give the reference's bytes, and our parser reads the reference's bytes into the
    fields the reference's parser found."""
    tool = os.path.join(PKG_DIR, "bin", "fa_archive_tool")
    args = [a.replace("GOLDEN", GOLDEN).replace("FRAMES", FRAMES) for a in case["args"]]
    ours = str(tmp_path / "ours.bin")
    subprocess.run([tool, "encode", "out=" + ours] + args, check=True)
    ref_path = os.path.join(FRAMES, case["name"] + ".bin")
    with open(ours, "rb") as a, open(ref_path, "rb") as b:
        mine, ref = a.read(), b.read()
    assert len(mine) == case["bytes"] and mine == ref
    got = json.loads(subprocess.run([tool, "decode", ref_path], check=True, capture_output=True, text=True).stdout)
    assert got == case["fields"]
