"""Child process of tests/test_phased_forms.py (GPU): the phased kernel's dynamic row pool (FA_PHASED_DYN, read
once per process) against the one-shot walk on the same device inputs, whole buckets bit for bit, plus sampled
elements against the oracle (the bf16 shapes run the static 512-thread form, which has no dynamic one).
Prints one JSON line.

  FA_PHASED_DYN=8 python tests/phased_child.py
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

# (clients, vectors per lane, fraction of one lane-vector row cut from the end, continue a d_init chain, bf16)
# f32, a full phase of 38 LDS + 48 register vectors per lane (the plan takes the phased form from 88 per lane
# up): 3 phases and a partial one (58% of a phase); 2 phases whose last is LDS-only (35%); one phase and a
# last of a few vectors per lane; 64 clients, the same; a 64-client sized phase (one phase with a register
# stage); d_init.  bf16 -> bf16, the 512-thread form (a phase of 20 LDS + 12 register vectors per lane): one
# phase and 28% of one (C3's shape), and 2 phases and 3 vectors per lane.
CASES = [(4, 86 * 2 + 50, 0.3, False, False), (33, 86 + 30, 0.5, False, False), (1, 88 + 1, 0.0, False, False),
         (64, 88 + 1, 0.7, False, False), (64, 70, 0.5, False, False), (8, 86 * 2 + 50, 0.2, True, False),
         (32, 32 + 9, 0.4, False, True), (16, 64 + 3, 0.1, False, True)]


def main():
    import torch
    import __graft_entry__ as g
    import oracle as O
    fa = g._load_pkg()
    fa.lib()
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    before = fa.get_tuning()
    results = []
    for D, q, frac, with_init, bf in CASES:
        lanes, V = (cus * 512, 8) if bf else (cus * 256, 4)
        dt, tdt, idt = (fa.BF16, torch.int16, torch.int16) if bf else (fa.F32, torch.float32, torch.int32)
        n = q * lanes * V - int(frac * lanes * V) - 3
        seed = 4100 + q + D
        w = O.weights(D)
        clients = []
        for k in range(D):
            t = torch.empty(n, dtype=tdt, device="cuda")
            fa.fill_uniform(t, n, dt, seed, k)
            clients.append(t)
        init = None
        if with_init:
            init = torch.empty(n, dtype=torch.float32, device="cuda")
            fa.fill_uniform(init, n, fa.F32, seed + 1, 999)
        outs = {}
        d0 = fa.diag_dyn_launches()
        try:
            for walk in (2, 5):
                fa.set_tuning(walk=walk)
                out = torch.empty(n, dtype=tdt, device="cuda")
                fa.reduce_device(clients, w, n, dt, out, dt, fa.FEDAVG, init=init)
                torch.cuda.synchronize()
                outs[walk] = out
        finally:
            fa.set_tuning(walk=before["walk"])
        same = bool(torch.equal(outs[2].view(idt), outs[5].view(idt)))
        mism = 0 if same else int((outs[2].view(idt) != outs[5].view(idt)).sum().item())
        plan = fa.plan_chain(dt, dt, n, D, cus=cus)
        oracle_ok = None
        if not with_init and not bf:
            rng = np.random.default_rng(q + D)
            idx = np.unique(np.concatenate([[0, n - 1], rng.integers(0, n, 512)]))
            ref = O.fedavg_at(seed, w, idx)
            got = outs[5][torch.as_tensor(idx, device="cuda")].cpu().numpy()
            oracle_ok = bool(np.array_equal(got.view(np.uint32), ref.view(np.uint32)))
        results.append({"clients": D, "n": n, "bf16": bf, "init": with_init, "plan": list(plan),
                        "same_bits": same, "mismatches": mism,
                        "oracle_sampled_ok": oracle_ok, "dyn_launches": fa.diag_dyn_launches() - d0})
        del clients, outs, init
        torch.cuda.empty_cache()
    # many streams at once: 52 launches of one two-phase bucket, each on a stream of its own, enqueued without a
    # sync in between -- the first 48 streams own their counter slots (the dynamic form), the rest share hashed
    # slots (the static form); grids that cannot all be resident meet late (bounded waits), never wrongly
    n = 89 * cus * 256 * 4 - 5
    D = 3
    w = O.weights(D)
    clients = []
    for k in range(D):
        t = torch.empty(n, dtype=torch.float32, device="cuda")
        fa.fill_uniform(t, n, fa.F32, 77, k)
        clients.append(t)
    ref = torch.empty(n, dtype=torch.float32, device="cuda")
    fa.reduce_device(clients, w, n, fa.F32, ref, fa.F32, fa.FEDAVG)
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream() for _ in range(52)]
    outs = [torch.empty(n, dtype=torch.float32, device="cuda") for _ in streams]
    d0 = fa.diag_dyn_launches()
    for s, o in zip(streams, outs):
        fa.reduce_device(clients, w, n, fa.F32, o, fa.F32, fa.FEDAVG, stream=s)
    torch.cuda.synchronize()
    bad = sum(0 if torch.equal(o.view(torch.int32), ref.view(torch.int32)) else 1 for o in outs)
    print(json.dumps({"dyn": int(os.environ.get("FA_PHASED_DYN", "0")), "cases": results,
                      "streams": {"launches": len(streams), "mismatched_outputs": bad,
                                  "dyn_launches": fa.diag_dyn_launches() - d0}}))


if __name__ == "__main__":
    main()
