#!/usr/bin/env python3
"""Which device-to-host copies does rocprofv3 --memory-copy-trace record?  (GPU box tool, round 4.)

The host-inclusive marker trace (tools/h2d_rate.py under `gpu_session.sh markers`) records every
HOST_TO_DEVICE copy but no DEVICE_TO_HOST one, and rocprofiler-sdk reports "completion callbacks were
not delivered" at exit.  This probe issues D2H copies of several kinds, one kind per phase, separated
by roctx-free sleeps so their records can be told apart by time, and prints what it did:
  torch_pageable  -- x.cpu()                                 (torch, pageable destination)
  torch_pinned    -- pinned.copy_(x, non_blocking=True)       (torch, pinned destination)
  fa_pageable     -- fa_finalize into a numpy array           (libfa: staged through pinned chunks)
  fa_pinned       -- fa_finalize_gather(FA_HOST_PINNED)       (libfa: straight into pinned memory)
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    import numpy as np
    import torch
    fa = bench.load_pkg()
    fa.lib()
    n = 1 << 22
    reps = 3
    x = torch.ones(n, dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    log = []

    def phase(name, fn):
        t0 = time.time_ns()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        log.append({"kind": name, "reps": reps, "t0_ns": t0, "t1_ns": time.time_ns()})
        time.sleep(0.2)

    phase("torch_pageable", lambda: x.cpu())
    pin = torch.empty(n, dtype=torch.float32, pin_memory=True)
    phase("torch_pinned", lambda: pin.copy_(x, non_blocking=True))
    with fa.Aggregator(1) as agg:
        agg.define(1, n, fa.F32, fa.F32, 2, fa.FEDAVG)
        host = np.ones(n, np.float32)
        out = np.empty(n, np.float32)
        pbuf = fa.PinnedBuffer(n * 4)

        def fa_pageable():
            for k in range(2):
                agg.submit(1, k, host, 0.5)
            agg.finalize(1, out)

        def fa_pinned():
            for k in range(2):
                agg.submit(1, k, host, 0.5)
            agg.finalize_gather(1, [pbuf.view(np.float32, count=n)], pinned=True)
        phase("fa_pageable", fa_pageable)
        phase("fa_pinned", fa_pinned)
        agg.sync()
        pbuf.close()
    torch.cuda.synchronize()
    time.sleep(2)
    print(json.dumps({"n": n, "phases": log}))


if __name__ == "__main__":
    main()
