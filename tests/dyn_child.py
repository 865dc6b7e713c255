"""Child process of tests/test_dyn_pool.py (GPU): the phased kernel's dynamic form (FA_PHASED_DYN, read once
per process) against the one-shot walk on the same device inputs, whole buckets bit for bit, plus sampled
elements against the oracle.  Prints one JSON line.

  FA_PHASED_DYN=8 python tests/dyn_child.py
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

# (clients, vectors per lane, fraction of one lane-vector row cut from the end, continue a d_init chain)
# for a full f32 phase of 38 LDS + 48 register vectors per lane (the plan takes the phased form from 88 per
# lane up): 3 phases and a partial one; 2 phases whose last is LDS-only; one phase and a last of a few
# vectors per lane; 64 clients, the same; a 64-client sized phase (one phase with a register stage); d_init
CASES = [(4, 86 * 2 + 50, 0.3, False), (33, 86 + 30, 0.5, False), (1, 88 + 1, 0.0, False),
         (64, 88 + 1, 0.7, False), (64, 70, 0.5, False), (8, 86 * 2 + 50, 0.2, True)]


def main():
    import torch
    import __graft_entry__ as g
    import oracle as O
    fa = g._load_pkg()
    fa.lib()
    lanes = torch.cuda.get_device_properties(0).multi_processor_count * 256
    before = fa.get_tuning()
    results = []
    for D, q, frac, with_init in CASES:
        n = q * lanes * 4 - int(frac * lanes * 4) - 3
        seed = 4100 + q + D
        w = O.weights(D)
        clients = []
        for k in range(D):
            t = torch.empty(n, dtype=torch.float32, device="cuda")
            fa.fill_uniform(t, n, fa.F32, seed, k)
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
                out = torch.empty(n, dtype=torch.float32, device="cuda")
                fa.reduce_device(clients, w, n, fa.F32, out, fa.F32, fa.FEDAVG, init=init)
                torch.cuda.synchronize()
                outs[walk] = out
        finally:
            fa.set_tuning(walk=before["walk"])
        same = bool(torch.equal(outs[2].view(torch.int32), outs[5].view(torch.int32)))
        mism = 0 if same else int((outs[2].view(torch.int32) != outs[5].view(torch.int32)).sum().item())
        oracle_ok = None
        if not with_init:
            rng = np.random.default_rng(q + D)
            idx = np.unique(np.concatenate([[0, n - 1], rng.integers(0, n, 512)]))
            ref = O.fedavg_at(seed, w, idx)
            got = outs[5][torch.as_tensor(idx, device="cuda")].cpu().numpy()
            oracle_ok = bool(np.array_equal(got.view(np.uint32), ref.view(np.uint32)))
        results.append({"clients": D, "n": n, "init": with_init, "same_bits": same, "mismatches": mism,
                        "oracle_sampled_ok": oracle_ok, "dyn_launches": fa.diag_dyn_launches() - d0})
        del clients, outs, init
        torch.cuda.empty_cache()
    print(json.dumps({"dyn": int(os.environ.get("FA_PHASED_DYN", "0")), "cases": results}))


if __name__ == "__main__":
    main()
