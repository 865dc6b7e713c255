#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ (runs in the build container only).

Drives oracle/_ref/ref_harness -- the reference's own model builders
(/root/reference/models/*.cpp, compiled by oracle/Makefile.ref) linked with
libtorch -- to emit, per configuration of BASELINE.json:

* ``layouts/<cfg>.json``: the bucket layout (named_parameters order, shapes,
  buffers) of every model part the aggregator reduces (aggregator.cpp:64,118),
  built exactly as systemAPI.cpp:17-38 builds it.
* ``<cfg>/manifest.json`` + small binaries: for D synthetic clients, the
  reference-literal result of the aggregator loop (aggregator.cpp:63-88 run on
  torch::save/torch::load blobs), and the libtorch FedAvg restatements
  (``acc.add_(x_k, w_k)`` in fp32, and over bf16-rounded inputs).  Buckets
  larger than SMALL elements are stored as SHA-256 + sampled elements.

The GPU box never runs this script and never reads /root/reference.
"""
import hashlib
import json
import os
import shutil
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HARNESS = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
GOLD = os.path.join(ROOT, "tests", "golden")
SMALL = 131072
N_SAMPLES = 1024
SEED = 0x5EED
WSEED = 7

# name, (model_name, model_type, start, end, num_classes), D, blob model_part
# model_name: vgg=0, resnet=1, letnet=2 (models.h:10-14); resnet18=1, resnet101=4
# (resnet.h:7-11); vgg19 = v19 = 6 (vgg_help.h:12-20).  start/end follow the
# refactor message of data_owner.cpp:99-100: end = cut[0], start = cut[-1] + 1.
CONFIGS = [
    ("lenet5_c1", (2, 0, 6, 1, 10), 2, -1),       # C1: LeNet-5, 2 data owners
    ("resnet18_c2", (1, 1, 9, 3, 10), 8, -1),     # C2: ResNet-18 split "3,8", 8 owners
    ("resnet101_c3", (1, 4, 20, 10, 10), 32, 0),  # C3: ResNet-101 split "10,19", 32 data owners
    ("vgg19_c4", (0, 6, 20, 3, 10), 64, 0),       # C4: VGG-19 split "3,19", 64 data owners
]


def run(args, timeout=3600):
    out = subprocess.run([HARNESS] + [str(a) for a in args], check=True, capture_output=True,
                         timeout=timeout, text=True).stdout
    return json.loads(out.strip().splitlines()[-1])


def sha(path):
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for chunk in iter(lambda: f.read(1 << 24), b""):
            h.update(chunk)
    return h.hexdigest()


def samples(path, dtype, numel):
    a = np.fromfile(path, dtype=dtype)
    assert a.size == numel, (path, a.size, numel)
    rng = np.random.default_rng(1234)
    idx = np.unique(np.concatenate([np.arange(min(16, numel)), np.arange(max(0, numel - 16), numel),
                                    rng.integers(0, numel, N_SAMPLES)]))
    return idx.tolist(), a[idx].view(np.uint32 if dtype == np.float32 else np.uint16).tolist()


def main():
    if not os.path.exists(HARNESS):
        sys.exit("build oracle/_ref first: make -f oracle/Makefile.ref")
    os.makedirs(os.path.join(GOLD, "layouts"), exist_ok=True)
    only = set(sys.argv[1:])  # optional: regenerate only the named configs
    for name, spec, D, blob_mp in CONFIGS:
        if only and name not in only:
            continue
        layout = run(["layout", *spec])
        layout["spec"] = dict(zip(["model_name", "model_type", "start", "end", "num_classes"], spec))
        with open(os.path.join(GOLD, "layouts", name + ".json"), "w") as f:
            json.dump(layout, f, indent=1)
        outdir = os.path.join(GOLD, name)
        shutil.rmtree(outdir, ignore_errors=True)
        os.makedirs(outdir)
        res = run(["golden", *spec, D, SEED, WSEED, outdir, blob_mp])
        manifest = {"config": name, "spec": layout["spec"], "D": D, "seed": SEED, "wseed": WSEED,
                    "weights": res["weights"], "buckets": []}
        for b in res["buckets"]:
            mp, numel = b["model_part"], b["numel"]
            entry = {"model_part": mp, "numel": numel, "bucket_seed": b["seed"], "outputs": {}}
            for kind, dt in (("literal.f32", np.float32), ("fedavg.f32", np.float32),
                             ("fedavg_bf16.bf16", np.uint16), ("fedavg_bf16.f32", np.float32),
                             ("buffers.f32", np.float32)):
                p = os.path.join(outdir, "mp%d_%s" % (mp, kind))
                if not os.path.exists(p):
                    continue
                n = os.path.getsize(p) // np.dtype(dt).itemsize
                rec = {"sha256": sha(p), "numel": n}
                if n > SMALL:
                    idx, vals = samples(p, np.float32 if dt == np.float32 else np.uint16, n)
                    rec["sample_idx"], rec["sample_bits"] = idx, vals
                    os.remove(p)
                else:
                    rec["file"] = os.path.basename(p)
                entry["outputs"][kind] = rec
            blob = os.path.join(outdir, "mp%d_client0.pt" % mp)
            if os.path.exists(blob):
                entry["client0_blob"] = {"file": os.path.basename(blob), "sha256": sha(blob)}
            manifest["buckets"].append(entry)
        with open(os.path.join(outdir, "manifest.json"), "w") as f:
            json.dump(manifest, f, indent=1)
        print(name, [(b["model_part"], b["numel"]) for b in manifest["buckets"]], flush=True)


if __name__ == "__main__":
    main()
