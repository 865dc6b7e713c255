#!/usr/bin/env python3
"""End-to-end rounds of the drop-in aggregator process (GPU box tool).

Builds model-part archives shaped like BASELINE.json C4 (VGG-19 split "3,19":
part 1 = 38 720, last part = 2 359 808 + 119 586 826 fp32 parameters) with
torch.jit.save (the same zip/pickle format as the reference's C++ torch::save),
starts fa_aggregator and the fake data owners (tests/tools) on loopback TCP and
reports the data owners' round time and the aggregator's per-phase split.
Beside it, oracle/_ref/ref_harness times the reference-literal receive loop
(torch::load + (p+p)/1000 + copy_, aggregator.cpp:63-88) on the VGG FC part.

  python tools/e2e_bench.py [D] [rounds] [aggregator args...]   (e.g. --layout rs, --eager)

E2E_MODEL=c3 uses BASELINE C3's bucket sizes instead (ResNet-101 split "10,19": 2 594 688 / 29 511 680 /
5 130 parameters) in bf16, E2E_MODEL=c2 C2's (ResNet-18 split "3,8": 83 584 / 9 442 304 / 5 130) in fp32
-- Linear layers with exactly those parameter counts; the aggregator only sees flat parameter buckets,
so their shapes do not matter.
"""
import json
import os
import random
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
AGG = os.path.join(ROOT, "multihop-federeated-split-learning_amd", "bin", "fa_aggregator")
OWNERS = os.path.join(ROOT, "tests", "tools", "bin", "fa_fake_owners")
REF = os.path.join(ROOT, "oracle", "_ref", "ref_harness")


def vgg_c4_parts(d):
    import torch
    import torch.nn as nn
    torch.manual_seed(0)
    parts = {
        1: nn.Sequential(nn.Conv2d(3, 64, 3, padding=1), nn.ReLU(), nn.Conv2d(64, 64, 3, padding=1), nn.ReLU()),
        2: nn.Sequential(nn.Conv2d(512, 512, 3, padding=1), nn.ReLU(), nn.MaxPool2d(2)),
        3: nn.Sequential(nn.Linear(512 * 7 * 7, 4096), nn.ReLU(), nn.Dropout(), nn.Linear(4096, 4096), nn.ReLU(),
                         nn.Dropout(), nn.Linear(4096, 10)),
    }
    sizes = {}
    for mp, m in parts.items():
        torch.jit.save(torch.jit.script(m), os.path.join(d, "mp%d_client0.pt" % mp))
        sizes[mp] = sum(p.numel() for p in m.parameters())
    return sizes


def resnet_parts(d, c3):
    import torch
    import torch.nn as nn
    torch.manual_seed(0)
    if c3:
        parts = {1: nn.Sequential(nn.Linear(347, 7456)),    # 2 594 688 parameters
                 2: nn.Sequential(nn.Linear(4095, 7205)),   # 29 511 680
                 3: nn.Sequential(nn.Linear(512, 10))}      # 5 130 (the ResNet fc)
    else:
        parts = {1: nn.Sequential(nn.Linear(31, 2612)),     # 83 584
                 2: nn.Sequential(nn.Linear(9220, 1024)),   # 9 442 304
                 3: nn.Sequential(nn.Linear(512, 10))}      # 5 130
    sizes = {}
    for mp, m in parts.items():
        if c3:
            m = m.to(torch.bfloat16)
        torch.jit.save(torch.jit.script(m), os.path.join(d, "mp%d_client0.pt" % mp))
        sizes[mp] = sum(p.numel() for p in m.parameters())
    return sizes


def heartbeat(every=20):
    """A progress line on stderr every `every` s: large rounds (D = 64 VGG owners, 30 GB of receipts per
    round over loopback) run for minutes with nothing else to print."""
    import threading
    t0 = time.time()

    def beat():
        while True:
            time.sleep(every)
            print("e2e_bench: %.0f s" % (time.time() - t0), file=sys.stderr, flush=True)
    threading.Thread(target=beat, daemon=True).start()


def main():
    heartbeat()
    D = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    extra = sys.argv[3:]
    model = os.environ.get("E2E_MODEL", "c4")
    resnet = model in ("c2", "c3")
    out = {"workload": {"c2": "ResNet-18 C2 bucket sizes (split 3,8), fp32",
                        "c3": "ResNet-101 C3 bucket sizes (split 10,19), bf16"}.get(
                            model, "VGG-19 C4 model parts (split 3,19)") + ", %d data owners, loopback TCP" % D,
           "aggregator_args": extra}
    with tempfile.TemporaryDirectory() as d:
        sizes = resnet_parts(d, model == "c3") if resnet else vgg_c4_parts(d)
        out["params_per_part"] = sizes
        base = random.randrange(10000, 32000, 100)  # below the ephemeral port range
        agg = subprocess.Popen([AGG, "-i", "-1", "-d", str(D), "-c", "1", "--rounds", str(rounds), "--port-base",
                                str(base)] + extra, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
        time.sleep(0.5)
        t0 = time.perf_counter()
        r = subprocess.run([OWNERS, "--blobs", d, "--parts", "1,2,3", "-d", str(D), "-c", "1", "--rounds",
                            str(rounds), "--port-base", str(base)] +
                           (["--model-name", "1", "--start", "19", "--end", "10"] if resnet else
                            ["--model-name", "0", "--start", "20", "--end", "3"]),
                           capture_output=True, text=True, timeout=900)
        wall = time.perf_counter() - t0
        a_out, a_err = agg.communicate(timeout=120)
        if r.returncode != 0 or agg.returncode != 0:
            print(json.dumps({"error": (r.stderr + a_err)[-3000:]}))
            sys.exit(1)
        owners = json.loads(r.stdout.strip().splitlines()[-1])
        phases = [json.loads(l) for l in a_out.splitlines() if l.startswith("{")]
        in_bytes = sum(p["phase1"]["bytes_in"] + p["phase2"]["bytes_in"] for p in phases) / len(phases)
        out.update({"ok": owners["ok"], "round_ms_owner_view": owners["round_ms"], "aggregator_phases": phases,
                    "bytes_in_per_round": in_bytes, "wall_s": round(wall, 3),
                    "ingest_GBs_per_round": [round(in_bytes / (ms / 1e3) / 1e9, 2) for ms in owners["round_ms"]]})
    if os.access(REF, os.X_OK) and not os.environ.get("E2E_NO_REF"):
        threads = str(min(16, len(os.sched_getaffinity(0))))
        lit = subprocess.run([REF, "bench-literal", "0", "6", "20", "3", "10", str(D), threads, "3"],
                             capture_output=True, text=True, timeout=900)
        if lit.returncode == 0:
            out["reference_literal_receive_loop"] = json.loads(lit.stdout.strip().splitlines()[-1])
    print(json.dumps(out))


if __name__ == "__main__":
    main()
