#!/usr/bin/env python3
"""Why many clients read slower (GPU box diagnostic; DESIGN.md 9 item 5, VERDICT r02 "next" #2).

  python tools/many_clients.py [launches=12] [configs=ns,d16,d64,d128,c4,c5r] [groups=0,32]

For every config (D clients x n fp32 elements, same total input where the name is d<D>) this times, with
HIP events on one stream (median over `launches`):
  * group 0  -- the product's launch (fa_reduce_part on the context's slots: one ordered chain over D);
  * group -1 -- the read-only probe over the same slots (fa_diag_read_stream: the phased kernel with its
                output switched off from one phase up; FA_PHASED_MIN_VECS=0 extends that to smaller buckets);
  * group G  -- the same chain cut into launches of G clients (fa_reduce_device: the first into the fp32
                output, the rest continuing it in place through d_init) -- same bits, 2 N * 4 extra bytes
                per extra launch.
If the G = 32 split of a 64- or 128-client bucket runs faster than the single launch in spite of its extra
bytes, the number of concurrent client streams is what costs.  Prints one JSON line per (config, group).
"""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CONFIGS = {
    "ns": (32, 64 << 20),
    "d16": (16, 128 << 20),
    "d64": (64, 32 << 20),
    "d128": (128, 16 << 20),
    "c4": (64, 139_611_210),
    "c5r": (128, 1 << 25),
    "c4r": (64, 34_902_848),  # C4's rank-0 range share at 4 GPUs
    "c5": (128, 1 << 28),
    # C4's slots (64 x 533 MiB), but every launch reduces only their first 32 M elements -- d64's launch on
    # C4's addresses: slow like C4 -> the slots' placement costs; fast like d64 -> the launch's length does
    "c4sub": (64, 139_611_210, 32 << 20),
    "c5sub": (128, 1 << 28, 1 << 25),  # C5's slots, c5r's launch
    # c5r's launch inside C5's pool at c5r's own slot spacing (128 MiB + 512 B): the same relative addresses as
    # c5r, C5's allocation -- slow like c5sub -> the allocation costs, fast like c5r -> the spacing does
    "c5sub_s128": (128, 1 << 28, 1 << 25, (128 << 20) + 512),
    "c5sub_s1g": (128, 1 << 28, 1 << 25, (1 << 30) + 512 + 4096),  # 1 GiB spacing with a 4.5 KiB skew
}
for _mib in (256, 512, 768, 1022, 958, 1024):  # spacing sweep inside C5's pool (r03s13)
    CONFIGS["c5sub_m%d" % _mib] = (128, 1 << 28, 1 << 25, (_mib << 20) + 512)


def main():
    launches = int(sys.argv[1]) if len(sys.argv) > 1 else 12
    names = sys.argv[2].split(",") if len(sys.argv) > 2 else list(CONFIGS)
    groups = [int(g) for g in sys.argv[3].split(",")] if len(sys.argv) > 3 else [0, 32]
    import torch
    import bench
    fa = bench.load_pkg()
    fa.lib()
    tune = os.environ.get("MC_TUNE", "")  # e.g. "slot_skew=4608": process tuning defaults before any context
    if tune:
        fa.set_tuning(**{k: int(v) for k, v in (kv.split("=") for kv in tune.split(","))})
    stream = torch.cuda.Stream()
    for name in names:
        D, n, *sub = CONFIGS[name]
        s = bench.Setup(fa, torch, D, n, "f32", "f32", 0, 0)
        torch.cuda.synchronize()
        # raw slot addresses only for the probe / split / sub legs (a pieced part has none: FA_PIECE_SPAN=0
        # keeps C5's pool whole for them)
        cl = s.clients(0) if sub or any(g != 0 for g in groups) else None
        out = s.agg.output(0)
        if sub:  # only the first sub[0] elements of every slot, through fa_reduce_device
            n = sub[0]
            if len(sub) > 1:  # the clients at another spacing inside the same pool
                cl = [cl[0] + k * sub[1] for k in range(D)]
        for G in groups:
            if G and G >= D:
                continue
            if sub and G == 0:
                G = D  # one fa_reduce_device launch over all D clients

            def launch(k):
                if G < 0:  # read-only probe over the same slots (fa_diag_read_stream; FA_PHASED_MIN_VECS=0
                    fa.diag_read_stream(cl, n - n % 4, stream=stream)  # gives sub-phase buckets the phased form)
                    return
                if not G:
                    s.launch(k, stream)
                    return
                for k0 in range(0, D, G):
                    fa.reduce_device(cl[k0:k0 + G], s.w[k0:k0 + G], n, fa.F32, out, fa.F32, fa.FEDAVG,
                                     init=out if k0 else None, stream=stream)
            evs = []
            for k in range(launches + 3):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(stream)
                launch(k)
                b.record(stream)
                evs.append((a, b))
            torch.cuda.synchronize()
            ms = statistics.median([a.elapsed_time(b) for a, b in evs[3:]])
            algo = (D + 1) * n * 4
            moved = D * n * 4 if G < 0 else algo + (2 * n * 4 * (-(-D // G) - 1) if G else 0)
            print(json.dumps({"tune": os.environ.get("MC_TUNE", ""), "config": name, "clients": D, "elems": n, "group": G, "median_ms": round(ms, 4),
                              "algo_frac": round(algo / (ms * 1e-3) / 8e12, 4),
                              "moved_TBs": round(moved / (ms * 1e-3) / 1e12, 3),
                              "timeouts": fa.phased_timeouts(0)}), flush=True)
        s.close()


if __name__ == "__main__":
    main()
