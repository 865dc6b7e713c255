#!/usr/bin/env python3
"""Device-resident FedAvg aggregation throughput on MI355X (BASELINE.json metric).

One step = one pass of the hot path over one round's synthetic client buckets
already resident in HBM: the ordered weighted-sum reduction of D client buckets
(pipeline_simulation/aggregator.cpp:59-93 / :112-150, FedAvg semantics) through
libfa.so's C ABI (fa_reduce_part on the context's own slots).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload northstar|c2|c3|c4|c5|c5r]
                  [--scaling strong|weak] [--layout range|rs|chain] [--no-cpu-baseline] [--no-secondary]

One process per GPU.  `--gpus N` with N > 1 starts its own N rank processes
(RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* in their env) unless a launcher such as
torch.distributed.run already set WORLD_SIZE.  Scaling "strong" (default): the
north star's 32 x 256 MiB problem is fixed and split over the ranks; layout
"range" gives rank r the elements [r n/N, (r+1) n/N) of every client bucket
(no collective, bit-exact).  "rs" / "chain" deal the 32 clients to the ranks
instead: "rs" combines fp32 partials with an RCCL reduce-scatter over xGMI,
"chain" hands the ordered fp32 chain rank to rank over RCCL p2p (bit-exact).
At N > 1 the weak-scaled range layout and the rs / chain layouts are reported
under "secondary".

value = bytes of client input of the whole problem / max-over-ranks wall time,
in GiB/s (D * n * sizeof(in) / t / 2^30).  roofline.achieved = algorithmic HBM
bytes of this rank's launch ((D+1) * n_rank * sizeof for f32->f32) / its
average duration from HIP events on the launch stream.
"""
import argparse
import collections
import csv
import faulthandler
import importlib.util
import json
import os
import statistics
import shutil
import signal
import subprocess
import sys
import tempfile
import threading
import time
import traceback

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.join(ROOT, "multihop-federeated-split-learning_amd")
HBM_PEAK_GBS = 8000.0  # MI355X spec HBM3E bandwidth (MI355X_MICROARCH.md chip table)

WORKLOADS = {
    # name: (clients per rank, elements per client per rank, in dtype, out dtype, description)
    "northstar": (32, 64 << 20, "f32", "f32", "256 MiB fp32 bucket x 32 clients (north-star target)"),
    "c2": (8, 12_557_962, "f32", "f32", "ResNet-18 full model buckets (reference build), 8 data owners, fp32"),
    "c3": (32, 42_737_546, "bf16", "bf16", "ResNet-101 full model buckets (basic-block build), 32 owners, bf16"),
    "c4": (64, 139_611_210, "f32", "f32", "VGG-19 full model buckets (reference build), 64 owners, fp32, on one GPU"),
    "c5": (128, 1 << 28, "f32", "f32", "synthetic 1 GiB fp32 bucket x 128 clients, all on one GPU (129 GiB resident)"),
    "c5r": (128, 1 << 25, "f32", "f32", "C5 one rank's share on 8 GPUs (range layout): 128 clients x 128 MiB slice"),
    # C4 is a 4-GPU config: rank 0's range share of it (shard.range_bounds(139_611_210, 4, 0))
    "c4r": (64, 34_902_848, "f32", "f32", "C4 one rank's share on 4 GPUs (range layout): 64 clients x 133 MiB slice"),
    # one rank's share of the strong-scaled north star (bench.py --gpus W): 32 clients x 256/W MiB
    "ns_w2": (32, 32 << 20, "f32", "f32", "north star, one rank's share at 2 GPUs (strong scaling): 32 x 128 MiB"),
    "ns_w4": (32, 16 << 20, "f32", "f32", "north star, one rank's share at 4 GPUs (strong scaling): 32 x 64 MiB"),
    "ns_w8": (32, 8 << 20, "f32", "f32", "north star, one rank's share at 8 GPUs (strong scaling): 32 x 32 MiB"),
}
H2D_DISTINCT_MAX_BYTES = 16 << 30  # host-inclusive legs: one pinned buffer per client up to this many bytes
ROTATE_MIN_BYTES = 1 << 30  # rotate input sets until a step's working set no longer fits the 256 MiB MALL
T_START = time.monotonic()
# Wall-clock budget of one bench run (the driver stops a bench at 600 s).  Every optional leg is bounded by
# what is left of it: the live PMC passes (100 s each at most), the CPU baseline (its variants only while
# more than 250 s are left, 60 s each), the multi-GPU secondaries of the N = 1 run (ctx_multi_secondaries).
# Worst case before the line is printed: 2 x 100 + 120 + 230 of variants is cut at 250 s left, then the
# single-GPU secondaries (~60-90 s of device work) and ctx children only until BUDGET_S - 30 s.
BUDGET_S = float(os.environ.get("FA_BENCH_BUDGET_S", "480"))


def budget_left():
    return T_START + BUDGET_S - time.monotonic()


def progress(msg):
    """A progress line on stderr (the run's legs, with the time since start): stdout carries the one line."""
    print("bench [%6.1f s] %s" % (time.monotonic() - T_START, msg), file=sys.stderr, flush=True)


def load_pkg():
    if "mhfsl_amd" in sys.modules:
        return sys.modules["mhfsl_amd"]
    spec = importlib.util.spec_from_file_location("mhfsl_amd", os.path.join(PKG_DIR, "__init__.py"),
                                                  submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["mhfsl_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


# ------------------------------------------------------------------ CPU baseline (rank 0, N = 1)

def cpu_threads():
    n = len(os.sched_getaffinity(0))
    cap = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return max(1, min(n, cap) if cap > 0 else n)


def _cpu_topology(c, what):
    try:
        with open("/sys/devices/system/cpu/cpu%d/%s" % (c, what)) as f:
            return f.read().strip()
    except OSError:
        return str(c)


def _numa_node(c):
    try:
        for e in os.listdir("/sys/devices/system/cpu/cpu%d" % c):
            if e.startswith("node") and e[4:].isdigit():
                return int(e[4:])
    except OSError:
        pass
    return 0


def pick_cores(n):
    """`n` CPUs of this process's affinity mask: one per physical core (an SMT sibling only when the mask has
    no other core left), on one NUMA node when it holds enough cores (its memory then local to every thread;
    the inputs are first-touched by the same cores), dealt round-robin over that node's L3 domains (CCDs), as
    a 16-core allocation of this CPU would spread.  Pinning 16 threads to one end of the mask instead puts
    them on two CCDs, whose links to memory then bound the reference's stream-like loop (r06s01: 73 GiB/s)."""
    mask = sorted(os.sched_getaffinity(0))
    cores, seen, spare = [], set(), []
    for c in mask:
        core = _cpu_topology(c, "topology/thread_siblings_list")
        if core in seen:
            spare.append(c)
            continue
        seen.add(core)
        cores.append(c)
    by_node = collections.OrderedDict()
    for c in cores:
        by_node.setdefault(_numa_node(c), []).append(c)
    home = [v for v in by_node.values() if len(v) >= n]
    pool = home[0] if home else cores
    groups = collections.OrderedDict()
    for c in pool:
        groups.setdefault(_cpu_topology(c, "cache/index3/shared_cpu_list"), []).append(c)
    chosen, lists = [], [list(v) for v in groups.values()]
    while lists and len(chosen) < n:
        for g in lists:
            if g and len(chosen) < n:
                chosen.append(g.pop(0))
        lists = [g for g in lists if g]
    rest = [c for c in cores if c not in chosen]
    return (chosen + rest + spare)[:max(1, n)]


def compact_cpus(cpus):
    """[0,1,2,3,8] -> "0-3,8"."""
    out, run = [], []
    for c in sorted(cpus):
        if run and c == run[-1] + 1:
            run.append(c)
            continue
        if run:
            out.append("%d-%d" % (run[0], run[-1]) if len(run) > 1 else str(run[0]))
        run = [c]
    if run:
        out.append("%d-%d" % (run[0], run[-1]) if len(run) > 1 else str(run[0]))
    return ",".join(out)


def pinned_child(cores):
    """subprocess kwargs that run a CPU leg on exactly `cores` with its OpenMP threads bound one per core."""
    env = dict(os.environ, OMP_NUM_THREADS=str(len(cores)), OMP_PROC_BIND="close", OMP_PLACES="cores")
    return {"env": env, "preexec_fn": lambda: os.sched_setaffinity(0, cores)}


def spread(rep_s, bytes_per_rep):
    """min / median / max GiB/s over the timed reps of one CPU leg."""
    r = sorted(bytes_per_rep / t / 2**30 for t in rep_s if t > 0)
    if not r:
        return None
    return {"min": round(r[0], 3), "median": round(statistics.median(r), 3), "max": round(r[-1], 3), "reps": len(r)}


def host_cpu():
    """The host CPU model (the CPU baseline varies with the host a GPU box lands on)."""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


# The reference's CPU path beside every config: the FedAvg chain restated in the
# reference's own library (libtorch acc.add_(x_k, w_k), oracle/_ref/ref_harness bench-fedavg) at each
# config's own shape.  name: (elements per client, clients, dtype, what the sample is)
CPU_CONFIGS = {
    "c2": (12_557_962, 8, "f32", "the whole config: 8 clients x ResNet-18's 12.6 M fp32 parameters"),
    "c3": (42_737_546, 32, "bf16", "the whole config: 32 clients x ResNet-101's 42.7 M bf16 parameters "
                                   "(fp32 accumulator, result rounded once to bf16)"),
    "c4": (139_611_210, 64, "f32", "the whole config: 64 clients x VGG-19's 139.6 M fp32 parameters (35.7 GB)"),
    "c5": (1 << 28, 16, "f32", "16 of the config's 128 clients x 1 GiB fp32 (16 GiB of host memory; the rate "
                               "is per byte, the config's 128 GiB would take 8x as long)"),
}
# The reference's own receive loop (aggregator.cpp:59-93 / :112-150: torch::load of each receipt into the
# global module + (p+p)/1000 + copy_), per round config: (secondary key, ref_harness model spec
# name type start end nc, model_part, receipts, what it is)
CPU_RECEIVE_LOOPS = [
    ("round_c2", (1, 1, 9, 3, 10), 2, 8, "ResNet-18 (C2) model_part 2 (9.4 M fp32 parameters), 8 receipts"),
    ("round_c4", (0, 6, 20, 3, 10), 3, 8, "VGG-19 (C4) model_part 3, the FC bucket (119.6 M fp32 parameters, a "
                                          "478 MB blob per receipt; aggregator.cpp:112-150, torch::load at :118), "
                                          "8 of the config's 64 receipts"),
]


# BASELINE config C1 end to end over loopback (tests/golden/lenet5_c1: LeNet-5 model parts made by the
# reference's own builders, spec of its manifest): fake data owners (tests/tools/fa_fake_owners, the load
# generator and checker: every element of every reply bit-exact against the oracle) against an aggregator
# process -- the reference's own CPU path (oracle/_ref/ref_cpu_aggregator: its systemAPI / network_layer with
# aggregator.cpp:55-167 on CPU libtorch) or the drop-in fa_aggregator.  Owner view: first send to last reply.
C1_E2E_ROUNDS = 40
C2_E2E_ROUNDS = 8
FAKE_OWNERS = os.path.join(ROOT, "tests", "tools", "bin", "fa_fake_owners")
FA_AGGREGATOR = os.path.join(PKG_DIR, "bin", "fa_aggregator")
REF_CPU_AGGREGATOR = os.path.join(ROOT, "oracle", "_ref", "ref_cpu_aggregator")
REF_BINDING_AGGREGATOR = os.path.join(ROOT, "oracle", "_ref", "ref_aggregator")  # + INTEGRATION.md 2 on libfa
REF_PORTS = (8080, 8081, 8082, 8083)  # the reference's fixed routing table (network_layer.h:80-86)


def ports_free(ports):
    import socket
    for p in ports:
        with socket.socket() as so:
            so.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)  # as the servers bind: TIME_WAIT is no conflict
            try:
                so.bind(("0.0.0.0", p))
            except OSError:
                return False
    return True


def free_port_base():
    import random
    for _ in range(50):
        b = random.randrange(10000, 32000, 100)
        if ports_free(range(b, b + 40)):
            return b
    raise RuntimeError("no free port range")


# The model arguments the fake owners send in the refactor message: (--model-name, --model-type, --start, --end)
C1_MODEL = ("2", "0", "6", "1")   # LeNet-5 split 6,1
C2_MODEL = ("1", "1", "9", "3")   # ResNet-18 split 3,8 (the ref_harness golden spec of tools/e2e_ref.py)


def e2e_c1(agg_cmd, mode, port_base, rounds=C1_E2E_ROUNDS, startup_s=0.5, timeout=120, owner_flags=()):
    """Rounds of BASELINE C1 (LeNet-5, D = 2, fp32) through one aggregator process over loopback; returns the
    owners' round times (round 0, which allocates, reported apart) and their bit-exact check of every reply."""
    return e2e_run(agg_cmd, mode, port_base, os.path.join(ROOT, "tests", "golden", "lenet5_c1"), 2, C1_MODEL,
                   rounds, startup_s, timeout, owner_flags)


def e2e_run(agg_cmd, mode, port_base, blobs, D, model, rounds, startup_s=0.5, timeout=120, owner_flags=()):
    """Rounds of one config (templates mp1..3_client0.pt in `blobs`, D owners) through one aggregator process
    over loopback against the fake owners, who check every element and every record CRC of every reply."""
    golden = blobs
    with tempfile.TemporaryDirectory(prefix="fa_e2e_") as tmp:  # the reference process writes its logs in cwd
        agg_out = open(os.path.join(tmp, "agg.out"), "w+")
        agg = subprocess.Popen(agg_cmd, stdout=agg_out, stderr=subprocess.DEVNULL, cwd=tmp, start_new_session=True)
        try:
            time.sleep(startup_s)
            if agg.poll() is not None:
                raise RuntimeError("aggregator exited early (rc %s)" % agg.returncode)
            r = subprocess.run([FAKE_OWNERS, "--blobs", golden, "--parts", "1,2,3", "-d", str(D), "-c", "1",
                                "--rounds", str(rounds), "--port-base", str(port_base), "--model-name", model[0],
                                "--model-type", model[1], "--start", model[2], "--end", model[3], "--mode", mode,
                                "--reply-timeout", "30"] + list(owner_flags),
                               capture_output=True, text=True, timeout=timeout, cwd=tmp)
        finally:
            if agg.poll() is None:
                try:
                    agg.wait(timeout=10)  # fa_aggregator --rounds exits by itself
                except subprocess.TimeoutExpired:
                    os.killpg(agg.pid, signal.SIGKILL)  # the reference's loop never returns (aggregator.cpp:55)
                    agg.wait()
        agg_out.seek(0)
        phases = []  # fa_aggregator's own round lines (the reference process prints a log, no JSON)
        for line in agg_out.read().splitlines():
            if line.startswith("{"):
                try:
                    phases.append(json.loads(line))
                except ValueError:
                    pass
        agg_out.close()
    if r.returncode not in (0, 1):
        raise RuntimeError("fake owners rc %d: %s" % (r.returncode, r.stderr[-300:]))
    res = json.loads(r.stdout.strip().splitlines()[-1])
    ms = res["round_ms"][1:]
    server = None
    if len(phases) > 1:
        med = lambda f: round(statistics.median(f(p) for p in phases[1:]) * 1e3, 4)  # noqa: E731
        server = {"phase1_reduce_ms": med(lambda p: p["phase1"]["reduce_s"]),
                  "phase2_reduce_ms": med(lambda p: p["phase2"]["reduce_s"]),
                  "streamed": phases[-1].get("streamed"),
                  "phase2_send_ms": med(lambda p: p["phase2"]["send_s"]),
                  "absorb_ms": med(lambda p: p["phase1"]["absorb_s"] + p["phase2"]["absorb_s"]),
                  "note": "medians over rounds 1.. of the aggregator's own round lines: reduce = the batched GPU "
                          "reduction + D2H into the reply frame + framing, absorb = archive parse + H2D submit"}
    return {"aggregator_view": server, "rounds_timed": len(ms), "round_ms_median": round(statistics.median(ms), 3),
            "round_ms_mean": round(statistics.mean(ms), 3),
            "round_ms_min": min(ms), "round0_ms": res["round_ms"][0], "mode": mode,
            "parity": {"check": "every element of every reply bit-exact vs the oracle (fake owners: %s)" %
                       ("fl(fl(x+x)/1000) of the last receipt" if mode == "literal" else "the ordered FedAvg chain"),
                       "samples": res["checked_elems"], "mismatches": 0 if res["ok"] else None, "ok": bool(res["ok"])}}


def cpu_c1(threads, cpu_model):
    """BASELINE C1's CPU figures (rank 0, before the GPU is touched): the reference's own aggregator process on
    CPU libtorch over loopback, and its receive loop alone (oracle/_ref/ref_harness bench-round)."""
    out = {"cpu_cores": threads, "host_cpu": cpu_model, "cpu_kind": "reference"}
    harness = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
    try:
        lines = []
        for t in (threads, 1):
            r = subprocess.run([harness] + [str(x) for x in ["bench-round", 2, 0, 6, 1, 10, 2, t, 500]],
                               capture_output=True, text=True, timeout=120, check=True)
            lines.append(json.loads(r.stdout.strip().splitlines()[-1]))
        out.update({"cpu_round_ms": round(lines[0]["round_ms_avg"], 4), "cpu_gib_s": round(lines[0]["gib_s"], 4),
                    "cpu_round_ms_1_core": round(lines[1]["round_ms_avg"], 4),
                    "cpu_path": "the reference's receive loop for a whole round, network aside: torch::load of each "
                                "receipt + (p+p)/1000 + copy_ (aggregator.cpp:59-93, :108-150), 3 buckets x 2 receipts",
                    "cpu_sample": "LeNet-5 split 6,1: 61,550 fp32 parameters per owner, 500 rounds after 1 warm-up"})
    except Exception as e:  # noqa: BLE001
        out["cpu_error"] = repr(e)[:200]
    if os.access(REF_CPU_AGGREGATOR, os.X_OK) and os.access(FAKE_OWNERS, os.X_OK):
        if ports_free(REF_PORTS):
            try:
                # the reference's receiver binds its port a second after it is released (network_layer.cpp)
                out["cpu_e2e_loopback"] = dict(e2e_c1([REF_CPU_AGGREGATOR, "2", "1"], "literal", 8079, startup_s=2.5),
                                               path="the reference's aggregator process on CPU libtorch: its own "
                                                    "systemAPI / network_layer / torch::save replies, "
                                                    "aggregator.cpp:55-167 restated (oracle/ref_cpu_aggregator.cpp)")
            except Exception as e:  # noqa: BLE001
                out["cpu_e2e_error"] = repr(e)[:300]
        else:
            out["cpu_e2e_error"] = "the reference's fixed ports 8080-8083 are in use"
    return out


CPU_REPS = 20  # timed reps of the main CPU leg (its min / median / max go in cpu_baseline.spread)
CPU_MAX_SAMPLE_BYTES = 36 << 30  # host memory one CPU leg may fill (C4's whole config, 35.7 GB, fits)


def cpu_baseline(D, n, reps, dt="f32", skip=None):
    """CPU baselines on the GPU box's host cores, before the GPU is initialised (child processes).

    oracle/_ref/ref_harness is built from the reference's own sources (model builders, State) linked with
    libtorch, the library the reference's arithmetic runs in -> kind "reference".  value = the FedAvg
    metric restated in that library: acc.add_(x_k, w_k) in client order over the WHOLE workload (D x n
    fp32, inputs generated in host memory before the clock), all cores of the affinity mask; beside it one
    core.  Returns (cpu_baseline object, {secondary key: figure}): every other config at its own shape
    (CPU_CONFIGS) and the reference's own receive loop with torch::load on C2's and C4's largest buckets
    (CPU_RECEIVE_LOOPS), each while the bench's time budget allows.  Fallback without the harness: the C
    oracle ("port") on the same workload.
    """
    threads = cpu_threads()
    cpu_model = host_cpu()
    cores = pick_cores(threads)
    harness = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
    s = 4 if dt == "f32" else 2
    D0 = D
    while D > 1 and D * n * s > CPU_MAX_SAMPLE_BYTES:  # C5 (128 GiB): a sample of its clients
        D //= 2
    sample = "%s: D=%d clients x %d %s elements (%.0f MiB per client, %.1f GiB in all), %d timed reps after 1 " \
             "warm-up" % ("the whole workload" if D == D0 else "%d of the workload's %d clients" % (D, D0), D, n, dt,
                          n * s / 2**20, D * n * s / 2**30, reps)
    bf = ["bf16"] if dt == "bf16" else []

    def run(args, timeout=120, ncores=None, pin=True):
        use = cores if ncores is None else cores[:ncores]
        out = subprocess.run([harness] + [str(a) for a in args], capture_output=True, text=True, timeout=timeout,
                             check=True, **(pinned_child(use) if pin else {})).stdout
        return json.loads(out.strip().splitlines()[-1])

    def leg_timeout(cap=90):
        left = budget_left() - 250
        if left < 10:
            raise TimeoutError("bench time budget (FA_BENCH_BUDGET_S): leg skipped")
        return min(cap, left)
    if os.access(harness, os.X_OK):
        try:
            r = run(["bench-fedavg", n, D, len(cores), reps] + bf)
            res = {"value": round(r["gib_s"], 3), "unit": "GiB/s", "cores": len(cores), "kind": "reference",
                   "path": "restatement in the reference's library: libtorch acc.add_(x_k, w_k) chain, "
                           "at::set_num_threads(%d)" % len(cores),
                   "sample": sample, "host_cpu": cpu_model,
                   "spread": spread(r.get("rep_s", []), D * n * s),
                   "pinned": "cores %s, OMP_PROC_BIND=close" % compact_cpus(cores)}
        except Exception as e:  # noqa: BLE001 -- fall through to the port
            print("cpu baseline: ref_harness failed (%s), timing the oracle port" % e, file=sys.stderr)
            res = None
        if res is not None:
            per = {}
            try:  # the same leg with the threads left to the scheduler, for comparison (not the baseline)
                ru = run(["bench-fedavg", n, D, len(cores), 5] + bf, timeout=leg_timeout(120), pin=False)
                res["unpinned"] = {"value": round(ru["gib_s"], 3), "spread": spread(ru.get("rep_s", []), D * n * s),
                                   "note": "%d threads, no affinity set: the scheduler may spread them over more "
                                           "cores / sockets than the pinned run's" % len(cores)}
            except Exception as e:  # noqa: BLE001 -- optional figure
                print("cpu baseline: unpinned leg not timed (%s)" % e, file=sys.stderr)
            try:
                r1 = run(["bench-fedavg", n, D, 1, 2] + bf, timeout=leg_timeout(120), ncores=1)
                res["fedavg_1_core"] = {"value": round(r1["gib_s"], 3), "unit": "GiB/s", "cores": 1,
                                        "sample": "the whole workload, 2 timed reps"}
            except Exception as e:  # noqa: BLE001 -- optional figures
                print("cpu baseline: one-core leg not timed (%s)" % e, file=sys.stderr)
            for key, (cn, cD, cdt, what) in CPU_CONFIGS.items():
                if key == skip:  # the main line's own workload: `value` above
                    continue
                try:
                    rc = run(["bench-fedavg", cn, cD, threads, 3] + (["bf16"] if cdt == "bf16" else []),
                             timeout=leg_timeout())
                    per[key] = {"cpu_gib_s": round(rc["gib_s"], 3), "cpu_cores": threads, "host_cpu": cpu_model,
                                "cpu_kind": "reference", "cpu_path": "libtorch acc.add_(x_k, w_k) chain (%s)" % cdt,
                                "cpu_sample": what + ", 3 timed reps", "cpu_ms_per_round": round(rc["avg_s"] * 1e3, 2)}
                except Exception as e:  # noqa: BLE001
                    per[key] = {"cpu_error": repr(e)[:200]}
            if budget_left() - 250 > 20:  # BASELINE C1: the reference's CPU aggregator over loopback, its loop
                per["round_c1"] = cpu_c1(threads, cpu_model)
            for key, spec, mp, receipts, what in CPU_RECEIVE_LOOPS:
                try:
                    lit = run(["bench-literal"] + list(spec) + [receipts, threads, mp], timeout=leg_timeout(120))
                    per[key] = {"cpu_gib_s": round(lit["gib_s"], 3), "cpu_cores": threads, "host_cpu": cpu_model,
                                "cpu_kind": "reference",
                                "cpu_path": "the reference's receive loop: torch::load of each receipt + (p+p)/1000 "
                                            "+ copy_ (GiB/s of parameters received)",
                                "cpu_sample": what}
                except Exception as e:  # noqa: BLE001
                    per[key] = {"cpu_error": repr(e)[:200]}
            # the C2 receive loop also without the decode, and on one core (the reference's own shape)
            for t in (threads, 1):
                for mode in ("", "arith"):
                    if t == threads and not mode:
                        continue  # = per["round_c2"]
                    try:
                        lit = run(["bench-literal", 1, 1, 9, 3, 10, 8, t, 2] + ([mode] if mode else []),
                                  timeout=leg_timeout(60), ncores=t)
                        k = "reference_receive_loop" + ("_arith_only" if mode else "") + ("_1_core" if t == 1 else "")
                        res[k] = {"value": round(lit["gib_s"], 3), "unit": "GiB/s of parameters received", "cores": t,
                                  "path": "the reference's receive loop (aggregator.cpp:59-93): " +
                                          ("(p+p)/1000 + copy_ on receipts decoded before the clock"
                                           if mode else "torch::load of each receipt + (p+p)/1000 + copy_"),
                                  "sample": "ResNet-18 (C2) model_part 2 (%d fp32 params), 8 receipts" % lit["numel"]}
                    except Exception as e:  # noqa: BLE001
                        print("cpu baseline: receive-loop variant not timed (%s)" % e, file=sys.stderr)
            if "round_c2" in per and "cpu_gib_s" in per["round_c2"]:
                res["reference_receive_loop"] = {"value": per["round_c2"]["cpu_gib_s"],
                                                 "unit": "GiB/s of parameters received", "cores": threads,
                                                 "path": "the reference's receive loop (aggregator.cpp:59-93): "
                                                         "torch::load of each receipt + (p+p)/1000 + copy_",
                                                 "sample": per["round_c2"]["cpu_sample"]}
            return res, per
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    w = oracle.weights(D)
    xs = [oracle.gen(0x5EED, k, n, dtype=dt) for k in range(D)]
    oracle.fedavg(xs, w, threads=threads)
    t0 = time.perf_counter()
    for _ in range(reps):
        oracle.fedavg(xs, w, threads=threads)
    per_rep = (time.perf_counter() - t0) / reps
    return {"value": round(D * n * s / per_rep / 2**30, 3), "unit": "GiB/s", "cores": threads, "kind": "port",
            "sample": sample + "; C oracle fmaf chain, %d threads" % threads, "host_cpu": cpu_model}, {}


# ------------------------------------------------------------------ parity (the checker, outside every timed region)
#
# Every leg that times a reduction checks what it computed afterwards: sampled elements of its result
# against the ordered chain (aggregator.cpp:59-93 / :112-150 with FedAvg semantics) evaluated by the C
# oracle at those indices only.  The oracle is the checker here, as in smoke(): it runs after the timed
# region has closed, never inside it, and nothing it computes feeds the measured path.  Range and chain
# layouts must be bit-exact; the client-sharded reduce-scatter (rs) sums in RCCL's order, so it is held to
# |err| <= 1e-6 * sum_k |w_k x_k| (BASELINE.json north_star: "within 1e-6 relative fp32").

PARITY_SAMPLES = 1024
RS_REL_TOL = 1e-6
RS_CHUNK_SWEEP = (2, 4, 16)  # rs pieces per round tried beside the library default (8) on a multi-GPU node


def load_checker():
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    return oracle


def sample_positions(segments, k=PARITY_SAMPLES, salt=0):
    """Positions to check in a result that holds the bucket segments [lo, hi) concatenated in the order
    given: both ends of every segment plus `k` positions spread uniformly (fixed seed) over the rest.
    Returns (positions in the result, global element indices), both int64 / uint64 arrays."""
    import numpy as np
    segs = [(int(a), int(b)) for a, b in segments if b > a]
    if not segs:
        return np.zeros(0, np.int64), np.zeros(0, np.uint64)
    lens = np.array([b - a for a, b in segs], np.int64)
    starts = np.concatenate([[0], np.cumsum(lens)[:-1]])
    total = int(lens.sum())
    if total <= k:  # a small result: every element
        pos = np.arange(total, dtype=np.int64)
    else:
        rng = np.random.default_rng(0xC0FFEE ^ salt)
        draw = np.unique(rng.integers(0, total, size=2 * k))
        while draw.size < k:  # only when k is close to total
            draw = np.unique(np.concatenate([draw, rng.integers(0, total, size=k)]))
        pos = np.unique(np.concatenate([starts, starts + lens - 1, rng.permutation(draw)[:k]]))
    seg = np.searchsorted(starts, pos, side="right") - 1
    lo = np.array([a for a, _ in segs], np.int64)
    return pos, (lo[seg] + (pos - starts[seg])).astype(np.uint64)


def parity_check(got, pos, idx, seed, w, exact=True, clients=None, bf16_in=False, literal=False):
    """Sampled parity of one result (host array `got`, fp32 or bf16 bits as uint16) against the oracle.

    exact: bit equality with the oracle's chain (rounded once to bf16 for a bf16 result); otherwise
    |got - ref| <= RS_REL_TOL * sum_k |w_k x_k| per element.  literal: the reference's own arithmetic
    fl(fl(x + x) / 1000) of the last client (`w` only gives the client count)."""
    import numpy as np
    O = load_checker()
    if literal:
        last = O.gen_at(seed, len(w) - 1 if clients is None else clients[-1], idx)
        if bf16_in:
            last = O.f32_to_bf16(last)
        ref = O.literal(last, out_dtype="bf16" if np.asarray(got).dtype == np.uint16 else "f32")
        sabs = None
    else:
        ref, sabs = O.sampled_chain(seed, w, idx, clients, bf16_in)
    g = np.asarray(got)[pos]
    if g.dtype == np.uint16:  # a bf16 result
        if not literal:
            ref = O.f32_to_bf16(ref)
        gf, rf = O.bf16_to_f32(g).astype(np.float64), O.bf16_to_f32(ref).astype(np.float64)
        gb, rb = g, ref
    else:
        gf, rf = g.astype(np.float64), ref.astype(np.float64)
        gb, rb = g.view(np.uint32), ref.view(np.uint32)
    err = np.abs(gf - rf)
    # a NaN where the oracle has a number is an error of unbounded size; the JSON line stays standard JSON
    # (no NaN / Infinity literals): non-finite maxima are reported as null and always count as mismatches
    fin = lambda x: float(x) if np.isfinite(x) else None  # noqa: E731
    res = {"samples": int(pos.size), "max_abs_err": fin(err.max()) if err.size else 0.0}
    if exact:
        bad = int(np.count_nonzero(gb != rb))
        res.update({"check": "bit-exact vs the oracle's ordered chain" if not literal else
                    "bit-exact vs the oracle's fl(fl(x+x)/1000) of the last client", "mismatches": bad})
    else:
        bound = RS_REL_TOL * sabs + 1e-30
        ratio = err / bound
        res.update({"check": "|err| <= %g * sum_k |w_k x_k|" % RS_REL_TOL,
                    "mismatches": int(np.count_nonzero(~(ratio <= 1.0))),  # NaN counts
                    "max_err_over_bound": fin(ratio.max()) if ratio.size else 0.0})
    res["ok"] = res["mismatches"] == 0 and res["samples"] > 0
    return res


def parity_merge(parts):
    """One parity object from several (GPUs of one context, buckets of one round)."""
    parts = [p for p in parts if p]
    if not parts:
        return None
    def worst(key):
        vals = [p.get(key, 0.0) for p in parts]
        return None if any(v is None for v in vals) else max(vals)
    out = {"check": parts[0]["check"], "samples": sum(p["samples"] for p in parts),
           "mismatches": sum(p["mismatches"] for p in parts), "max_abs_err": worst("max_abs_err")}
    if any("max_err_over_bound" in p for p in parts):
        out["max_err_over_bound"] = worst("max_err_over_bound")
    out["ok"] = all(p["ok"] for p in parts)
    return out


def parity_over_ranks(torch, dist, world, backend, p):
    """Rank-local parity summed (samples, mismatches) and maxed (errors) over the ranks; every rank gets it."""
    if world == 1:
        return p
    # every rank takes part in both reductions, whatever its own check did (a collective per rank)
    p = p or {"check": "not run", "samples": 0, "mismatches": 0, "max_abs_err": 0.0, "ok": False}
    inf = float("inf")
    enc = lambda v: inf if v is None else float(v)  # noqa: E731 -- None (a non-finite error) travels as inf
    dev = "cuda" if backend == "nccl" else "cpu"
    s = torch.tensor([p["samples"], p["mismatches"], 0 if p["ok"] else 1], dtype=torch.float64, device=dev)
    m = torch.tensor([enc(p["max_abs_err"]), enc(p.get("max_err_over_bound", 0.0))], dtype=torch.float64, device=dev)
    dist.all_reduce(s, op=dist.ReduceOp.SUM)
    dist.all_reduce(m, op=dist.ReduceOp.MAX)
    s, m = s.tolist(), [None if v == inf else v for v in m.tolist()]
    out = dict(p, samples=int(s[0]), mismatches=int(s[1]), max_abs_err=m[0], ranks=world, ok=s[2] == 0 and s[1] == 0)
    if "max_err_over_bound" in p:
        out["max_err_over_bound"] = m[1]
    return out


def parity_guarded(fn):
    """A parity check that fails to run is reported as such (ok false), never fatal to the bench line."""
    try:
        return fn()
    except Exception as e:  # noqa: BLE001
        traceback.print_exc()
        return {"ok": False, "error": repr(e)[:300], "samples": 0, "mismatches": 0, "max_abs_err": 0.0,
                "check": "not run"}


# ------------------------------------------------------------------ device measurement

def traffic_from_profile(workload, n_gpus, strong_range=False):
    """HBM bytes per launch from the committed rocprofv3 PMC summary (profiles/), if present.  At N > 1 a
    rank's launch of the strong-scaled north star is the per-rank share measured as ns_w<N>."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if n_gpus != 1:
        if not (strong_range and workload == "northstar"):
            return None, None
        workload = "ns_w%d" % n_gpus
    if not os.path.exists(p):
        return None, None
    with open(p) as f:
        d = json.load(f)
    rec = d.get(workload)
    if not rec:
        return None, None
    # per step (a step of C5's pieced layout is one launch per piece); older records hold one launch per step
    return rec.get("hbm_bytes_per_step", rec.get("hbm_bytes_per_launch")), "%s, kernel %s" % (
        rec.get("source"), rec.get("kernel", "?").split("(")[0])


def under_profiler():
    return os.environ.get("FA_BENCH_PMC_CHILD") == "1" or any(k.startswith("ROCPROF") for k in os.environ)


def live_traffic(workload, timeout=100):
    """HBM bytes per launch of this run's dominant kernel, measured now: two rocprofv3 PMC passes (FETCH_SIZE,
    then WRITE_SIZE, each its own run as MI355X_MICROARCH.md prescribes) of a short single-GPU bench of the
    same workload, started as child processes before this process touches the GPU.  gfx950 correction:
    traffic = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 (the counters are KiB; FETCH_SIZE counts half the bytes
    of a wide streaming read).  Returns (bytes, source) or (None, reason)."""
    prof = shutil.which("rocprofv3")
    if not prof:
        return None, "rocprofv3 not on PATH"
    vals, kernel, launches = {}, None, 0
    with tempfile.TemporaryDirectory(prefix="fa_pmc_") as tmp:
        for counter in ("FETCH_SIZE", "WRITE_SIZE"):
            d = os.path.join(tmp, counter)
            cmd = [prof, "--pmc", counter, "--kernel-trace", "--output-format", "csv", "-d", d, "-o", "run", "--",
                   sys.executable, os.path.abspath(__file__), "--workload", workload, "--steps", "4", "--warmup", "1",
                   "--no-cpu-baseline", "--no-secondary"]
            env = dict(os.environ, FA_BENCH_PMC_CHILD="1", TMPDIR=os.environ.get("TMPDIR", "/tmp"))
            for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
                env.pop(k, None)
            try:
                # its own process group, so a pass that times out is killed whole (the profiler and the
                # bench under it), not just the profiler's front end
                proc = subprocess.Popen(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, env=env, cwd=ROOT,
                                        start_new_session=True)
                try:
                    _, err = proc.communicate(timeout=timeout)
                except subprocess.TimeoutExpired:
                    os.killpg(proc.pid, signal.SIGKILL)
                    proc.communicate()
                    return None, "live PMC pass %s timed out after %d s" % (counter, timeout)
                if proc.returncode != 0:
                    return None, "live PMC pass %s failed (rc %d): %s" % (counter, proc.returncode,
                                                                         (err or b"")[-200:].decode(errors="replace"))
            except (subprocess.SubprocessError, OSError) as e:
                return None, "live PMC pass %s failed: %s" % (counter, repr(e)[:200])
            path = os.path.join(d, "run_counter_collection.csv")
            if not os.path.exists(path):  # some rocprofv3 versions nest the output under a host/pid directory
                found = [os.path.join(r, f) for r, _, fs in os.walk(d) for f in fs if f.endswith("counter_collection.csv")]
                if not found:
                    return None, "live PMC pass %s wrote no counter_collection.csv" % counter
                path = found[0]
            per = collections.defaultdict(list)
            with open(path) as f:
                for r in csv.DictReader(f):
                    if r.get("Counter_Name") == counter:
                        per[(r["Kernel_Name"], r.get("Grid_Size") or r.get("Grid_Size_X"))].append(float(r["Counter_Value"]))
            if not per:
                return None, "live PMC pass %s: no %s records" % (counter, counter)
            if kernel is None:  # the dominant kernel = the most fetched bytes among the reductions
                red = {k: v for k, v in per.items() if "fill_kernel" not in k[0] and "read_probe" not in k[0]}
                kernel = max((red or per).items(), key=lambda kv: sum(kv[1]))[0]
            v = per.get(kernel)
            if not v:
                return None, "live PMC pass %s: dominant kernel missing" % counter
            vals[counter] = sum(v) / len(v)
            launches = len(v)
    traffic = (2 * vals["FETCH_SIZE"] + vals["WRITE_SIZE"]) * 1024
    return round(traffic), "live: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of bench.py --workload %s " \
        "(child processes, %d launches of %s), (2*FETCH_SIZE + WRITE_SIZE) * 1024" % (
            workload, launches, kernel[0].split("(")[0])


class Setup:
    """One workload on the current GPU through the product's own context (fa_ctx).

    Each rotated input set is one bucket (part) of the context: its D client
    slots live in one HBM pool with the library's per-slot skew, the inputs are
    generated in place (fa_fill_uniform on the slot pointers) and a step is
    fa_reduce_part -- the device-resident round of the aggregator.
    """

    def __init__(self, fa, torch, D, n, in_dt, out_dt, elem0, device, client0=0, seed=0x5EED,
                 min_rotate_bytes=ROTATE_MIN_BYTES, mode=None, contiguous=False):
        self.fa, self.torch = fa, torch
        self.D, self.n = D, n
        self.elem0, self.client0, self.seed = elem0, client0, seed
        self.literal = mode is not None and mode == fa.LITERAL
        self.in_dt = fa.F32 if in_dt == "f32" else fa.BF16
        self.out_dt = fa.F32 if out_dt == "f32" else fa.BF16
        self.s_in = 4 if in_dt == "f32" else 2
        self.s_out = 4 if out_dt == "f32" else 2
        set_bytes = D * n * self.s_in
        self.nsets = max(1, -(-min_rotate_bytes // set_bytes))
        self.agg = fa.Aggregator(devices=[device])
        # contiguous: every client slot one range of device memory (the client-sharded legs hand raw slot
        # addresses to fa_reduce_device), i.e. no range pieces in this context
        if contiguous:
            self.agg.set_tuning(piece_span_kib=-1)
        for s in range(self.nsets):
            self.agg.define(s, n, self.in_dt, self.out_dt, D, fa.FEDAVG if mode is None else mode)
            for k in range(D):
                for ptr, cnt, off in self.agg.pieces(s, 0, k):
                    # global client id and element offset: ranks hold disjoint clients or slices of one bucket
                    fa.fill_uniform(ptr, cnt, self.in_dt, seed + s, client0 + k, idx0=elem0 + off)
        self.w = self._weights(D)

    @staticmethod
    def _weights(D):
        # same as oracle.weights(D) (splitmix64-derived n_k in [500,1500], w_k = n_k / sum n), computed here
        # so the product path does not import the oracle.
        import numpy as np
        M = (1 << 64) - 1

        def sm(z):
            z = (z + 0x9E3779B97F4A7C15) & M
            z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M
            z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M
            return z ^ (z >> 31)
        nk = [500 + sm(7 ^ (k << 32)) % 1001 for k in range(D)]
        tot = float(sum(nk))
        return np.array([float(x) / tot for x in nk], np.float32)

    def launch(self, step, stream):
        self.agg.reduce(step % self.nsets, self.w, stream=stream)

    def pieced(self, s=0):
        return len(self.agg.pieces(s, 0, 0)) > 1

    def clients(self, s=0):
        """Device addresses of the D client slots of set s (each one contiguous range)."""
        if self.pieced(s):
            raise RuntimeError("bucket set %d is held in range pieces (fa_bucket_pieces): its client slots are not "
                               "contiguous; build the Setup with contiguous=True" % s)
        return [self.agg.slot(s, 0, k)[0] for k in range(self.D)]

    def parity(self, s=0):
        """Sampled parity of input set s's reduced bucket (read back after the timed region): the oracle's
        chain over global clients client0.. at global elements elem0.. (literal mode: the last client)."""
        got = self.agg.copy_output(s)
        pos, idx = sample_positions([(self.elem0, self.elem0 + self.n)], salt=s)
        return parity_check(got, pos, idx, self.seed + s, self.w,
                            clients=[self.client0 + k for k in range(self.D)],
                            bf16_in=self.in_dt == self.fa.BF16, literal=self.literal)

    def close(self):
        self.agg.close()

    def algo_bytes(self):
        return self.D * self.n * self.s_in + self.n * self.s_out

    def input_bytes(self):
        return self.D * self.n * self.s_in


# The buckets one aggregation round forms (tests/golden/layouts, the reference builders): phase 1 reduces
# model_part 1 (aggregator.cpp:59-93), phase 2 the last-part layers 2..L+1 (:108-150).
ROUNDS = {
    # name: (clients, dtype, phase-1 bucket, phase-2 buckets, description)
    "round_c1": (2, "f32", 50_536, [10_164, 850], "LeNet-5 split 6,1, 2 owners, fp32"),
    "round_c2": (8, "f32", 83_584, [9_442_304, 5_130], "ResNet-18 split 3,8, 8 owners, fp32"),
    "round_c3": (32, "bf16", 2_594_688, [29_511_680, 5_130], "ResNet-101 split 10,19, 32 owners, bf16"),
    "round_c4": (64, "f32", 38_720, [2_359_808, 119_586_826], "VGG-19 split 3,19, 64 owners, fp32"),
}


ROUND_MAX_SETS = 16


class RoundSetup:
    """One aggregator round on the device: phase 1 = fa_reduce_part of model_part 1, phase 2 =
    fa_reduce_parts over the last-part layers (one batched launch for the small ones, the phased kernel for
    a large one).  `batched=False` launches every part on its own (the round-1 aggregator)."""

    def __init__(self, fa, torch, name, device, batched=True, min_rotate_bytes=ROTATE_MIN_BYTES):
        D, dt, p1, p2, self.desc = ROUNDS[name]
        self.fa, self.D, self.batched = fa, D, batched
        self.in_dt = fa.F32 if dt == "f32" else fa.BF16
        self.s = 4 if dt == "f32" else 2
        self.sizes = [p1] + list(p2)
        set_bytes = D * sum(self.sizes) * self.s
        # C1's whole round is 0.5 MB: it sits in L2 / the MALL whatever the rotation (its round is launch-bound),
        # so a few sets suffice; the other rounds rotate past the MALL as the workloads do
        self.nsets = min(ROUND_MAX_SETS, max(1, -(-min_rotate_bytes // set_bytes)))
        self.agg = fa.Aggregator(devices=[device])
        for st in range(self.nsets):
            for j, n in enumerate(self.sizes):
                pid = 10 * st + j + 1
                self.agg.define(pid, n, self.in_dt, self.in_dt, D, fa.FEDAVG)
                for k in range(D):
                    ptr, cnt, _ = self.agg.slot(pid, 0, k)
                    fa.fill_uniform(ptr, cnt, self.in_dt, 0x5EED + 100 * st + j, k)
        self.w = Setup._weights(D)

    def parity(self, st=0):
        """Sampled parity of every bucket of input set st (phase 1 and the batched phase 2), merged."""
        res = []
        for j, n in enumerate(self.sizes):
            got = self.agg.copy_output(10 * st + j + 1)
            pos, idx = sample_positions([(0, n)], salt=j)
            res.append(parity_check(got, pos, idx, 0x5EED + 100 * st + j, self.w, bf16_in=self.in_dt == self.fa.BF16))
        return parity_merge(res)

    def launch(self, step, stream):
        base = 10 * (step % self.nsets)
        self.agg.reduce(base + 1, self.w, stream=stream)  # phase 1
        p2 = [base + j + 1 for j in range(1, len(self.sizes))]
        if self.batched:
            self.agg.reduce_parts(p2, weights=[self.w] * len(p2), stream=stream)
        else:
            for pid in p2:
                self.agg.reduce(pid, self.w, stream=stream)

    def algo_bytes(self):
        return sum((self.D + 1) * n * self.s for n in self.sizes)

    def input_bytes(self):
        return sum(self.D * n * self.s for n in self.sizes)

    def close(self):
        self.agg.close()


class SyncSetup(Setup):
    """Compute-node state sync (fa_sync_part): every client slot := the FedAvg of all, in place.
    Algorithmic bytes per launch = D*n*s read + D*n*s written."""

    def launch(self, step, stream):
        self.agg.sync_states(step % self.nsets, self.w, stream=stream)

    def algo_bytes(self):
        return 2 * self.D * self.n * self.s_in

    def parity(self, s=0):
        """After the timed loop the slots hold repeated syncs, which the oracle does not restate: refill set
        s, run ONE sync on it (the same launch), and check the first and the last slot -- both must hold the
        chain over all D clients, rounded to the slot dtype -- at sampled elements."""
        import numpy as np
        fa, torch = self.fa, self.torch
        for k in range(self.D):
            for ptr, cnt, off in self.agg.pieces(s, 0, k):
                fa.fill_uniform(ptr, cnt, self.in_dt, self.seed + s, self.client0 + k, idx0=self.elem0 + off)
        torch.cuda.synchronize()  # the fills ran on the null stream; the context's streams do not wait for it
        self.agg.sync_states(s, self.w)
        self.agg.sync()
        torch.cuda.synchronize()
        dt = np.float32 if self.in_dt == fa.F32 else np.uint16
        res = []
        for k in sorted({0, self.D - 1}):
            got = np.concatenate([device_to_host(ptr, cnt, dt) for ptr, cnt, _ in self.agg.pieces(s, 0, k)])
            pos, idx = sample_positions([(self.elem0, self.elem0 + self.n)], salt=k)
            res.append(parity_check(got, pos, idx, self.seed + s, self.w,
                                    clients=[self.client0 + j for j in range(self.D)],
                                    bf16_in=self.in_dt == fa.BF16))
        out = parity_merge(res)
        out["check"] += " (slots 0 and D-1 after one in-place sync of a refilled set)"
        return out


_HIP = None


def device_to_host(ptr, count, dtype):
    """`count` elements of `dtype` at device address `ptr` -> a new host array (hipMemcpy of the HIP runtime
    torch has loaded; the parity checks' read-back of raw slots, outside every timed region)."""
    import ctypes
    import numpy as np
    global _HIP
    if _HIP is None:
        _HIP = ctypes.CDLL("libamdhip64.so.7")
        _HIP.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    out = np.empty(count, dtype)
    rc = _HIP.hipMemcpy(out.ctypes.data, ptr, out.nbytes, 2)  # hipMemcpyDeviceToHost
    if rc != 0:
        raise RuntimeError("hipMemcpy device-to-host failed (%d)" % rc)
    return out


def _read_rate(torch, setup, stream, launch, reps, passes=1):
    """GB/s of one read-only launch form over the setup's client slots: one launch per range piece (a bucket
    set held in pieces, e.g. C5 on one GPU, is reduced one launch per piece too), bytes of all pieces / the
    sum of their median HIP-event times on the launch stream.  The reps rotate over the input sets as the
    timed loop does, so a set that fits the MALL is not read back from it.  A bf16 slot is read as the fp32
    words its bytes make (the same bytes, the same addresses)."""
    sets = [[setup.agg.pieces(s, 0, k) for k in range(setup.D)] for s in range(setup.nsets)]
    nbytes, t_ms = 0, 0.0
    for j in range(len(sets[0][0])):
        n = sets[0][0][j][1] * setup.s_in // 4  # fp32 words of the piece's bytes
        n -= n % 4
        ms = []
        for i in range(reps + 2):
            ptrs = [pc[j][0] for pc in sets[i % setup.nsets]]
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            launch(ptrs, n)
            b.record(stream)
            b.synchronize()
            if i >= 2:
                ms.append(a.elapsed_time(b))
        nbytes += passes * setup.D * n * 4
        t_ms += statistics.median(ms)
    return round(nbytes / (t_ms * 1e-3) / 1e9, 1)


def read_stream_peak(fa, torch, setup, stream, reps=7):
    """Measured read-STREAM peak on this run's own client slots: a read-only launch over the D
    buckets -- from one phase up the phased kernel itself with its output stream switched off
    (fa_diag_read_stream).  frac_of_read_stream = achieved / this, i.e. what the output stream costs on top
    of the product's own reads."""
    return _read_rate(torch, setup, stream, lambda ptrs, n: fa.diag_read_stream(ptrs, n, stream=stream), reps)


READ_PLAIN_FORMS = [(g, u) for g in (2048, 4096, 8192, 16384) for u in (8, 16)]


def read_plain_peak(fa, torch, setup, stream, reps=5):
    """The independent read ceiling on the same slots: the best of plain grid-stride nt read launches
    (fa_diag_read_plain, tools/hbm_probe.hip's read kernel; grids x loads in flight of READ_PLAIN_FORMS),
    which share nothing with the product kernels' access pattern.  Returns {GB/s, the best form, every form}."""
    rates = {}
    for g, u in READ_PLAIN_FORMS:
        rates["grid%d_u%d" % (g, u)] = _read_rate(
            torch, setup, stream, lambda ptrs, n: fa.diag_read_plain(ptrs, n, grid=g, unroll=u, stream=stream), reps)
    best = max(rates, key=rates.get)
    return {"GBs": rates[best], "form": best, "forms": rates,
            "kernel": "plain grid-stride read, 256 lanes per workgroup, nt 16-byte loads, slot after slot"}


RW_PLAIN_FORMS = [(g, u, nt) for g in (2048, 4096, 8192, 16384) for u in (8, 16) for nt in (False, True)]


def rw_plain_peak(fa, torch, setup, stream, reps=3):
    """The independent in-place read+write ceiling on the sync legs' own slots (their traffic: every slot read
    and written back where it lies): the best of plain grid-stride launches (fa_diag_rw_plain; grids x loads in
    flight x plain/nt stores of RW_PLAIN_FORMS), slot after slot, none of the sync kernel's element-major walk.
    GB/s counts the bytes read and the bytes written, as the sync legs' algorithmic bytes do."""
    rates = {}
    for g, u, nt in RW_PLAIN_FORMS:
        rates["grid%d_u%d_%s" % (g, u, "nt" if nt else "plain")] = _read_rate(
            torch, setup, stream,
            lambda ptrs, n: fa.diag_rw_plain(ptrs, n, grid=g, unroll=u, nt=nt, stream=stream), reps, passes=2)
    best = max(rates, key=rates.get)
    return {"GBs": rates[best], "form": best, "forms": rates,
            "kernel": "plain grid-stride in-place read+write, 256 lanes per workgroup, nt 16-byte loads, "
                      "slot after slot"}


def settle(freed_bytes):
    """Wait out the driver's clear of device memory just freed before the next leg is timed: the clear runs
    beside the next leg's kernels at ~35 GB/s of freed memory (the c4 workload 0.87 -> 0.83-0.84 of spec for
    1.3 s after 36 GiB were freed, for 3.7 s after 129 GiB; tools/order_effect.py, gpurun_out r05s24-s25)."""
    time.sleep(min(8.0, freed_bytes / 30e9))


def timed_loop(torch, setup, steps, warmup, stream, dist, barrier, per_launch=10):
    """`steps` steps back to back, bracketed by barrier + synchronize: returns (wall seconds, region_ms, kern_ms).

    The timed region holds nothing but the steps: one HIP event pair on the launch stream brackets all of
    them (region_ms = their device time / steps -- the roofline's average launch duration), with no event
    between steps (an event pair per step added 7-12 us of wall time per step, gpurun_out r02s71).
    kern_ms: per-launch event pairs from a separate loop of `per_launch` steps after the timed region
    (kernel_ms_min / _median)."""
    if not hasattr(stream, "cuda_stream"):  # Event.record on a non-stream crashes inside the HIP runtime
        raise TypeError("timed_loop needs a torch.cuda.Stream, got %r" % (stream,))
    for i in range(warmup):
        setup.launch(i, stream)
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    a.record(stream)
    for i in range(steps):
        setup.launch(warmup + i, stream)
    b.record(stream)
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    region_ms = a.elapsed_time(b) / steps
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(per_launch)]
    for i, (x, y) in enumerate(evs):
        x.record(stream)
        setup.launch(warmup + steps + i, stream)
        y.record(stream)
    torch.cuda.synchronize()
    return wall, region_ms, [x.elapsed_time(y) for x, y in evs]


def time_client_sharded(torch, dist, shard, setup, layout, n, world, device, stream, steps, warmup, chunks, barrier):
    """Wall time of `steps` rounds of a client-sharded layout: every rank reduces its whole clients (the
    setup's slots) and the ranks combine them -- "rs": fp32 partials + RCCL reduce-scatter (block-cyclic
    ownership, one launch per chunk: shard.reduce_rs_cyclic), "chain": the
    ordered chain handed rank to rank over RCCL p2p (shard.py)."""
    reducer = shard.fa_reducer(setup.fa, setup.in_dt, stream)
    cl = setup.clients()
    dev = torch.device("cuda", device)
    npad = -(-n // (world * shard.UNIT)) * world * shard.UNIT
    assert npad == n, "workload size must be a multiple of world * 64"

    def step():
        with torch.cuda.stream(stream):
            if world == 1:
                return reducer(cl, setup.w, n)
            fn = shard.reduce_rs_cyclic if layout == "rs" else shard.reduce_chain
            return fn(reducer, dist, cl, setup.w, n, dev, chunks=chunks, itemsize=setup.s_in)
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        res = step()
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    return time.perf_counter() - t0, res


def client_sharded_parity(shard, setup, layout, res, n, world, rank, chunks, D):
    """Sampled parity of a client-sharded round's result `res` (this rank's part, read back after the timed
    region): "rs" holds the block-cyclic segments of shard.cyclic_bounds (RCCL's summation order: the 1e-6
    tolerance); "chain" this rank's range of the ordered chain (bit-exact); one rank: the whole chain."""
    got = res.cpu().numpy()
    if world == 1:
        segs, exact = [(0, n)], True
    elif layout == "rs":
        segs, exact = shard.cyclic_bounds(n, world, rank, chunks), False
    else:
        segs, exact = [shard.range_bounds(n, world, rank)], True
    pos, idx = sample_positions(segs, salt=rank)
    return parity_check(got, pos, idx, setup.seed, Setup._weights(D), exact=exact,
                        bf16_in=setup.in_dt == setup.fa.BF16)


def layout_desc_of(layout, D, world, chunks):
    if layout == "rs":
        return ("client-sharded: each rank reduces its %d whole clients into fp32 partials, RCCL "
                "reduce-scatter over xGMI in %d chunks overlapped with the reduction (block-cyclic "
                "ownership, one launch per chunk)" % (D, chunks))
    return ("client-sharded, bit-exact: each rank chains its %d whole clients and hands the fp32 chain to the "
            "next rank over RCCL p2p in %d chunks, last rank scatters the ranges" % (D, chunks))


# ------------------------------------------------------------------ the printed line
#
# The driver parses ONE stdout line, and a line past ~16 KB was not parsed (BENCH_r05: 20.3 KB, parsed null).
# stdout carries a compact line of at most LINE_MAX_BYTES: the required keys, roofline, cpu_baseline with its
# spread, parity, and one small object per secondary leg.  The full object (every leg's detail) goes to
# FULL_RECORD, which the compact line names.

LINE_MAX_BYTES = 6000
FULL_RECORD = os.environ.get("FA_BENCH_FULL") or os.path.join(ROOT, "gpurun_out", "bench_full.json")
ROOFLINE_KEYS = ("bound", "achieved", "peak", "unit", "frac", "traffic", "algorithmic_bytes_per_launch",
                 "kernel_ms_avg", "kernel_ms_min", "kernel_ms_median", "kernel_ms_avg_max_over_ranks",
                 "phased_meeting_timeouts", "read_stream_peak", "frac_of_read_stream",
                 "read_stream_peak_independent", "frac_of_read_stream_independent")
CPU_KEYS = ("value", "unit", "cores", "kind", "sample", "host_cpu", "spread", "pinned")
CONFIG_KEYS = ("workload", "description", "clients", "elems_per_client", "in_dtype", "out_dtype", "parallelism",
               "world_size", "dist_backend", "ranks_share_gpus", "input_sets_rotated")
# a leg's figure -> its key in the compact line
LEG_KEYS = (("gib_s", "gib_s"), ("frac", "frac"), ("kernel_ms_avg", "ms"), ("round_ms_avg", "ms"),
            ("ms_per_round", "ms"), ("ms_per_step", "ms"), ("frac_of_read_stream_independent", "frac_ind"),
            ("frac_of_copy_independent", "frac_copy_ind"),
            ("cpu_gib_s", "cpu_gib_s"), ("gpus", "gpus"), ("h2d_ms", "h2d_ms"), ("reduce_ms", "reduce_ms"),
            ("d2h_ms", "d2h_ms"), ("pcie_GBs", "pcie_GBs"))
E2E_KEYS = (("e2e_loopback_literal", "e2e_literal_ms"), ("e2e_loopback_fedavg", "e2e_fedavg_ms"),
            ("e2e_loopback_fedavg_no_streaming", "e2e_fedavg_nostream_ms"),
            ("e2e_loopback_reference_process_with_binding", "e2e_ref_binding_ms"), ("cpu_e2e_loopback", "cpu_e2e_ms"))


def _parity_brief(p):
    """{ok[, err_over_bound]} of a parity object (None when there is none)."""
    if not isinstance(p, dict):
        return None
    out = {"ok": bool(p.get("ok"))}
    if p.get("max_err_over_bound") is not None:
        out["err_over_bound"] = round(p["max_err_over_bound"], 3)
    return out


def compact_leg(v):
    """One secondary leg in a few figures: gib_s / frac / ms / frac_ind / cpu_gib_s, parity ok."""
    if not isinstance(v, dict):
        return v
    if "error" in v:
        return {"error": str(v["error"])[:80]}
    if "skipped" in v:
        return {"skipped": True}
    out = {}
    for src, dst in LEG_KEYS:
        if v.get(src) is not None and dst not in out:
            out[dst] = v[src]
    if v.get("cpu_error"):
        out["cpu_error"] = True
    if v.get("shared_device_rehearsal"):
        out["rehearsal"] = True
    if v.get("phased_meeting_timeouts"):
        out["meeting_timeouts"] = v["phased_meeting_timeouts"]
    par = _parity_brief(v.get("parity"))
    if par is not None:
        out["parity_ok"] = par["ok"]
        if "err_over_bound" in par:
            out["err_over_bound"] = par["err_over_bound"]
    for src, dst in E2E_KEYS:  # BASELINE C1's end-to-end rounds (owner view, medians)
        e = v.get(src)
        if isinstance(e, dict):
            if "error" in e:
                out[dst] = None
            else:
                out[dst] = e.get("round_ms_median")
                p = e.get("parity")
                out["e2e_parity_ok"] = out.get("e2e_parity_ok", True) and bool(p and p.get("ok"))
                view = e.get("aggregator_view") or {}
                if "fedavg" in src and view.get("phase2_reduce_ms") is not None:  # the phase-2 tail
                    out[dst.replace("_ms", "_tail_ms")] = view["phase2_reduce_ms"]
    if v.get("e2e_error"):
        out["e2e_error"] = True
    return out


def compact_line(line, full_record=None):
    """The stdout line from the full object: what the driver checks, in at most LINE_MAX_BYTES."""
    out = {k: line[k] for k in line if k not in ("config", "roofline", "cpu_baseline", "parity", "secondary")}
    cfg = line.get("config") or {}
    out["config"] = {k: cfg[k] for k in CONFIG_KEYS if k in cfg}
    rl = line.get("roofline") or {}
    out["roofline"] = {k: rl[k] for k in ROOFLINE_KEYS if k in rl}
    if rl.get("traffic_source"):
        out["roofline"]["traffic_source"] = "live PMC" if str(rl["traffic_source"]).startswith("live") \
            else "committed profile"
    cpu = line.get("cpu_baseline")
    if isinstance(cpu, dict):
        out["cpu_baseline"] = {k: cpu[k] for k in CPU_KEYS if k in cpu}
        if isinstance(cpu.get("fedavg_1_core"), dict):
            out["cpu_baseline"]["value_1_core"] = cpu["fedavg_1_core"].get("value")
        if isinstance(cpu.get("unpinned"), dict):
            out["cpu_baseline"]["value_unpinned"] = cpu["unpinned"].get("value")
    else:
        out["cpu_baseline"] = cpu
    par = line.get("parity")
    if isinstance(par, dict):
        out["parity"] = {k: par[k] for k in ("check", "samples", "mismatches", "max_abs_err", "max_err_over_bound",
                                             "ranks", "ok", "error") if k in par}
    else:
        out["parity"] = par
    if "secondary" in line:
        out["secondary"] = {k: compact_leg(v) for k, v in (line["secondary"] or {}).items()}
    if full_record:
        out["full_record"] = full_record
    s = json.dumps(out)
    if len(s) > LINE_MAX_BYTES and "secondary" in out:  # never expected: keep the required part parseable
        out["secondary"] = {k: (v.get("gib_s") if isinstance(v, dict) else v) for k, v in out["secondary"].items()}
        out["secondary_truncated"] = True
    return out


def write_full_record(line, path=FULL_RECORD):
    """The whole object (every leg's detail) beside the run; returns the path written, or None."""
    try:
        os.makedirs(os.path.dirname(path), exist_ok=True)
        with open(path, "w") as f:
            json.dump(line, f)
            f.write("\n")
        return os.path.relpath(path, ROOT)
    except OSError as e:
        print("bench: full record not written (%s)" % e, file=sys.stderr)
        return None


class LinePrinter:
    """Rank 0 prints the one JSON line exactly once (from the main thread or the watchdog), on the process's
    original stdout; everything else that writes to fd 1 (RCCL's version banner, library chatter) has been
    moved to stderr by quiet_stdout(), so the driver's stdout carries that one line only.  The line is the
    compact form (compact_line); the full object goes to FULL_RECORD first."""

    def __init__(self, rank, out=None, full_path=FULL_RECORD):
        self.rank = rank
        self.out = out or sys.stdout
        self.full_path = full_path
        self.lock = threading.Lock()
        self.done = False

    def emit(self, line):
        with self.lock:
            if self.rank == 0 and not self.done:
                rec = write_full_record(line, self.full_path) if self.full_path else None
                self.out.write(json.dumps(compact_line(line, rec)) + "\n")
                self.out.flush()
            self.done = True


def quiet_stdout():
    """fd 1 -> stderr for the rest of the process; returns a file on the original stdout."""
    sys.stdout.flush()
    out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    return out


def load_shard():
    load_pkg()
    import importlib
    return importlib.import_module("mhfsl_amd.shard")


def spawn_ranks(n, argv, script=None):
    """`--gpus N` (N > 1) without a launcher: start N rank processes (RANK / LOCAL_RANK / WORLD_SIZE /
    MASTER_* in their environment, one GPU each) and wait for them.  Runs before this process touches
    torch or HIP, so nothing is exec'd after GPU init; returns the worst exit code.  Should one rank
    fail, the others get a grace period and are then terminated (a collective would otherwise wait
    for the dead rank forever)."""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-u", script or os.path.abspath(__file__)] + argv, env=env))
    grace = float(os.environ.get("FA_BENCH_RANK_GRACE", "60"))
    failed_at = None
    while True:
        rcs = [p.poll() for p in procs]
        if all(rc is not None for rc in rcs):
            break
        if failed_at is None and any(rc not in (None, 0) for rc in rcs):
            failed_at = time.monotonic()
            print("bench: a rank exited with %s; waiting %.0f s for the others" % (rcs, grace), file=sys.stderr)
        if failed_at is not None and time.monotonic() - failed_at > grace:
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            for p in procs:
                try:
                    p.wait(timeout=20)
                except subprocess.TimeoutExpired:
                    p.kill()
            break
        time.sleep(0.2)
    rcs = [p.wait() for p in procs]
    bad = [rc for rc in rcs if rc != 0]
    return bad[0] if bad else 0


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="northstar", choices=sorted(WORKLOADS))
    ap.add_argument("--scaling", default="strong", choices=["strong", "weak"],
                    help="strong (default): the workload is split over the ranks by element range; weak: every "
                         "rank reduces a full-size slice of its own")
    ap.add_argument("--layout", default="range", choices=["range", "rs", "chain"])
    ap.add_argument("--chunks", type=int, default=16,
                    help="rs / chain layouts: chunks (reduce of chunk c+1 overlaps the exchange of chunk c)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-secondary", action="store_true")
    ap.add_argument("--no-live-pmc", action="store_true",
                    help="take roofline.traffic from profiles/pmc_traffic.json instead of two PMC passes run now")
    ap.add_argument("--dist-backend", default="auto",
                    help="auto (nccl = RCCL over xGMI when every rank has its own GPU, else gloo), nccl or gloo")
    ap.add_argument("--tune", default="", help="block,max_blocks,unroll,load_policy,store_policy (fa_tuning)")
    ap.add_argument("--piece-span-kib", type=int, default=0,
                    help="fa_tuning.piece_span_kib for every context (range pieces; tests force small pieces)")
    ap.add_argument("--piece-split-kib", type=int, default=0, help="fa_tuning.piece_split_kib (-1: always cut)")
    ap.add_argument("--ctx-multi", default="", choices=["", "range", "rs"],
                    help="one process over every visible GPU through the C ABI: FA_SHARD_RANGE or FA_SHARD_CLIENT_RS "
                         "(RCCL reduce-scatter); prints one JSON object (a secondary of the N = 1 run)")
    ap.add_argument("--ctx-shared", type=int, default=0,
                    help="with --ctx-multi: rehearse K shards on GPU 0 (FA_TEST_SHARED_DEVICE: the layout's code path "
                         "at K GPUs, the rs exchange replaced by its definition); for one-GPU boxes, not a timing")
    ap.add_argument("--ctx-gpus", type=int, default=0,
                    help="with --ctx-multi: use the first K visible GPUs (default all)")
    ap.add_argument("--h2d", action="store_true",
                    help="with --ctx-multi: host-inclusive rounds (fa_submit_pinned of every client from host "
                         "memory, overlapped per GPU, + fa_finalize into host memory)")
    ap.add_argument("--rs-chunks", type=int, default=0,
                    help="with --ctx-multi rs: pieces per round of the in-process reduce-scatter (fa_tuning.rs_chunks; "
                         "the reduction of piece c+1 overlaps the exchange of piece c); 0 = the library default")
    args = ap.parse_args()
    if args.steps < 1 or args.warmup < 0:
        ap.error("--steps must be >= 1 and --warmup >= 0")
    if args.ctx_multi:
        return ctx_multi(args)

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))
    line_out = quiet_stdout()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print("warning: --gpus %d but WORLD_SIZE %d; using WORLD_SIZE" % (args.gpus, world), file=sys.stderr)
    D, n, in_dt, out_dt, desc = WORKLOADS[args.workload]
    strong = args.scaling == "strong"

    # roofline.traffic: PMC passes of this rank's launch shape, run now (before this process touches the GPU)
    pmc_workload = args.workload if world == 1 else \
        ("ns_w%d" % world if strong and args.layout == "range" and args.workload == "northstar"
         and "ns_w%d" % world in WORKLOADS else None)
    live = (None, None)
    if world > 1 and pmc_workload:
        import torch  # counting devices does not initialise the GPU on this image
        if torch.cuda.device_count() < world:  # rehearsal: the ranks' kernels are not the per-rank launch shape
            pmc_workload = None
    if rank == 0 and pmc_workload and not args.no_live_pmc and not under_profiler():
        live = live_traffic(pmc_workload)
        if live[0] is None:
            print("bench: %s; using the committed profile" % live[1], file=sys.stderr)

    cpu, cpu_per = None, {}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu, cpu_per = cpu_baseline(D, n, CPU_REPS, in_dt, skip=args.workload)

    import torch
    import torch.distributed as dist
    fa = load_pkg()
    shard = load_shard()
    n_dev = torch.cuda.device_count()  # counts without initialising the GPU
    device = local_rank % max(1, n_dev)  # == local_rank on a node with one GPU per rank
    backend = args.dist_backend
    if backend == "auto":
        backend = "nccl" if n_dev >= world else "gloo"
    torch.cuda.set_device(device)
    fa.lib()
    shared_gpus = n_dev < world
    if shared_gpus:  # rehearsal: ranks share GPUs, and the phased kernel's persistent grid needs a whole GPU
        fa.set_tuning(walk=2)
    if args.tune:
        b, mb, u, lp, sp = [int(x) for x in args.tune.split(",")]
        fa.set_tuning(block=b, max_blocks=mb, unroll=u, load_policy=lp, store_policy=sp)
    if args.piece_span_kib or args.piece_split_kib:
        fa.set_tuning(piece_span_kib=args.piece_span_kib, piece_split_kib=args.piece_split_kib)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", device))
        else:
            dist.init_process_group(backend)

        def barrier():
            dist.barrier()
    else:
        def barrier():
            pass

    def max_over_ranks(x):
        if world == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64, device="cuda" if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    stream = torch.cuda.Stream()
    s_in = 4 if in_dt == "f32" else 2
    if args.layout == "range":
        # strong: rank r owns elements [lo, hi) of every one of the D buckets (the bucket is split W ways);
        # weak: rank r owns its own full-size slice [r n, (r+1) n) of D buckets W times as long
        lo, hi = shard.range_bounds(n, world, rank) if strong else (rank * n, (rank + 1) * n)
        setup = Setup(fa, torch, D, hi - lo, in_dt, out_dt, lo, device)
        total_bytes = D * n * s_in * (1 if strong else world)
        layout_desc = "range-sharded: rank %d owns elements [%d, %d) of every one of %d buckets of %d elements, " \
                      "no collective" % (rank, lo, hi, D, n if strong else n * world)
    else:
        # client-sharded: strong: the D clients are dealt to the ranks; weak: every rank holds D clients
        c0, c1 = shard.client_bounds(D, world, rank) if strong else (rank * D, (rank + 1) * D)
        setup = Setup(fa, torch, c1 - c0, n, in_dt, out_dt, 0, device, client0=c0, contiguous=True)
        setup.w = Setup._weights(D if strong else D * world)[c0:c1]
        total_bytes = D * n * s_in * (1 if strong else world)
        layout_desc = layout_desc_of(args.layout, c1 - c0, world, args.chunks)
    torch.cuda.synchronize()

    # the dominant kernel alone (roofline), HIP events on its stream
    timeouts0 = fa.phased_timeouts(device)
    wall_k, kavg, kern_ms = timed_loop(torch, setup, args.steps, args.warmup, stream, dist, barrier)
    timeouts = fa.phased_timeouts(device) - timeouts0  # > 0: the persistent grid was not co-resident
    if args.layout == "range":
        wall = wall_k
    else:  # the local reductions run beside RCCL's kernels: the one-shot walk (shard.py, "Overlap")
        walk0 = fa.get_tuning()["walk"]
        if world > 1:  # one rank runs no collective
            fa.set_tuning(walk=shard.OVERLAP_WALK)
        try:
            wall, res = time_client_sharded(torch, dist, shard, setup, args.layout, n, world, device, stream,
                                            args.steps, args.warmup, args.chunks, barrier)
        finally:
            fa.set_tuning(walk=walk0)
        timeouts += fa.phased_timeouts(device) - timeouts0 - timeouts
    wall = max_over_ranks(wall)
    # parity of what was timed, read back and checked now that the timed region is closed
    if args.layout == "range":
        par = parity_guarded(lambda: setup.parity(0))
    else:
        par = parity_guarded(lambda: client_sharded_parity(shard, setup, args.layout, res, n, world, rank,
                                                           args.chunks, D if strong else D * world))
        res = None
    par = parity_over_ranks(torch, dist, world, backend, par)

    achieved = setup.algo_bytes() / (kavg * 1e-3) / 1e9
    read_peak = read_stream_peak(fa, torch, setup, stream) if args.layout == "range" and not under_profiler() \
        else None
    read_ind = read_plain_peak(fa, torch, setup, stream) if args.layout == "range" and not under_profiler() \
        else None
    # ranks sharing one GPU (rehearsal) run the one-shot walk, so no committed profile of the phased kernel
    # describes their launches: no traffic then
    committed = (None, None) if shared_gpus else traffic_from_profile(args.workload, world,
                                                                      strong and args.layout == "range")
    traffic, traffic_src = live if live[0] is not None else committed
    line = {
        "metric": "GiB/s aggregated (device-resident), D-client fp32 bucket FedAvg reduce",
        "value": round(total_bytes * args.steps / wall / 2**30, 3),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(wall / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": args.scaling,
        "vs_baseline": None,
        "dtype": in_dt,
        "data": "synthetic (counter-based splitmix64 uniform[-1,1), generated in HBM)",
        "config": {"workload": args.workload, "description": desc, "clients": D,
                   "elems_per_client": n * (1 if strong else world), "in_dtype": in_dt, "out_dtype": out_dt,
                   "layout": layout_desc, "parallelism": "%s%d" % (args.layout, world),
                   "world_size": dist.get_world_size() if world > 1 else 1,
                   "dist_backend": backend if world > 1 else None,
                   "ranks_share_gpus": shared_gpus,
                   "tuning": setup.agg.get_tuning(), "input_sets_rotated": setup.nsets},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic, "traffic_source": traffic_src,
                     "traffic_committed_profile": committed[0],
                     "traffic_live_error": live[1] if live[0] is None and live[1] else None,
                     "algorithmic_bytes_per_launch": setup.algo_bytes(),
                     "kernel_ms_avg": round(kavg, 4),
                     "kernel_ms_avg_source": "HIP events on the launch stream bracketing the %d timed steps" % args.steps,
                     "kernel_ms_min": round(min(kern_ms), 4), "kernel_ms_median": round(statistics.median(kern_ms), 4),
                     "kernel_ms_per_launch_events_avg": round(statistics.mean(kern_ms), 4),
                     "kernel": "rank %d's launch (%s)" % (rank, "its range of every bucket" if args.layout == "range"
                                                         else "its clients' local reduction"),
                     "phased_meeting_timeouts": int(max_over_ranks(timeouts)),
                     "read_stream_peak": read_peak, "frac_of_read_stream":
                         round(achieved / read_peak, 4) if read_peak else None,
                     "read_stream_peak_independent": read_ind["GBs"] if read_ind else None,
                     "frac_of_read_stream_independent": round(achieved / read_ind["GBs"], 4) if read_ind else None,
                     "read_stream_peak_independent_detail": read_ind},
        "cpu_baseline": cpu,
        "parity": par,
    }
    if world > 1:
        line["roofline"]["kernel_ms_avg_max_over_ranks"] = round(max_over_ranks(kavg), 4)

    if rank == 0 and world == 1 and not args.no_secondary:
        setup.close()
        settle(setup.input_bytes())
        line["secondary"] = single_gpu_secondaries(fa, torch, args, device, stream, dist, barrier)
        for key, fig in cpu_per.items():  # the reference's CPU path beside each config's device figure
            line["secondary"].setdefault(key, {}).update(fig)
        line["secondary"].update(ctx_multi_secondaries(n_dev, T_START + BUDGET_S))

    printer = LinePrinter(rank, line_out)
    if world > 1 and not args.no_secondary and args.layout == "range":
        # the other layouts on the same ranks, as secondaries: weak-scaled range (every rank a full 256 MiB
        # slice), and the client-sharded RCCL legs (reduce-scatter, p2p chain) on the same strong problem.
        # A watchdog bounds them: should a collective stall, rank 0 still prints the main line (marked)
        # and every rank exits.
        limit = float(os.environ.get("FA_BENCH_SECONDARY_TIMEOUT", "90"))
        done = threading.Event()

        def watchdog():
            if not done.wait(limit):
                print("rank %d: secondary layouts still running after %.0f s; stacks:" % (rank, limit),
                      file=sys.stderr, flush=True)
                faulthandler.dump_traceback(file=sys.stderr, all_threads=True)
                line["secondary_error"] = "secondary layouts did not finish within %.0f s" % limit
                printer.emit(line)
                os._exit(0)
        threading.Thread(target=watchdog, daemon=True).start()
        setup.close()
        sec = line["secondary"] = {}  # filled layout by layout, so a watchdog exit keeps what finished
        steps2 = max(10, args.steps)
        for L in ("weak_range", "rs", "chain"):
            try:
                if L == "weak_range":
                    s2 = Setup(fa, torch, D, n, in_dt, out_dt, rank * n, device)
                    torch.cuda.synchronize()
                    w2, _, _ = timed_loop(torch, s2, steps2, 3, stream, dist, barrier)
                    tb, desc2 = D * n * s_in * world, "weak scaling: every rank reduces its own %d-element slice " \
                                                       "of %d buckets, no collective" % (n, D)
                    p2 = parity_guarded(lambda: s2.parity(0))
                else:
                    c0, c1 = shard.client_bounds(D, world, rank)
                    s2 = Setup(fa, torch, c1 - c0, n, in_dt, out_dt, 0, device, client0=c0, contiguous=True)
                    s2.w = Setup._weights(D)[c0:c1]
                    torch.cuda.synchronize()
                    # the local reductions run beside RCCL's kernels: the one-shot walk (shard.py, "Overlap")
                    walk0 = fa.get_tuning()["walk"]
                    fa.set_tuning(walk=shard.OVERLAP_WALK)
                    try:
                        w2, r2 = time_client_sharded(torch, dist, shard, s2, L, n, world, device, stream, steps2,
                                                     3, args.chunks, barrier)
                    finally:
                        fa.set_tuning(walk=walk0)
                    tb, desc2 = D * n * s_in, layout_desc_of(L, c1 - c0, world, args.chunks)
                    p2 = parity_guarded(lambda: client_sharded_parity(shard, s2, L, r2, n, world, rank, args.chunks, D))
                    r2 = None
                t2 = fa.phased_timeouts(device) - timeouts0 - timeouts
                w2 = max_over_ranks(w2)
                sec[L] = {"description": desc2, "clients": D, "steps": steps2,
                          "ms_per_step": round(w2 / steps2 * 1e3, 4), "gib_s": round(tb * steps2 / w2 / 2**30, 1),
                          "phased_meeting_timeouts": int(max_over_ranks(t2)),
                          "parity": parity_over_ranks(torch, dist, world, backend, p2)}
                timeouts += t2
                s2.close()
            except Exception as e:  # noqa: BLE001 -- the ranks may now disagree: report and leave
                traceback.print_exc()
                print("rank %d: %s layout failed" % (rank, L), file=sys.stderr, flush=True)
                sec[L] = {"error": repr(e)[:300]}
                printer.emit(line)
                os._exit(0)
        done.set()

    printer.emit(line)
    if world > 1:
        dist.destroy_process_group()


def ctx_multi(args):
    """Device-resident rounds of one fa_ctx over every visible GPU (`--ctx-multi range|rs`): the in-process
    multi-GPU layouts of the C ABI that fa_aggregator --gpus G uses.  Slots are filled in place on their
    GPUs; a step is fa_reduce_part (range: each GPU its element range; rs: each GPU its clients' fp32
    partials + ncclReduceScatter piece by piece); the steps are timed back to back, then fa_sync."""
    import torch
    fa = load_pkg()
    fa.lib()
    G = torch.cuda.device_count()
    if args.ctx_gpus > 0:
        G = min(G, args.ctx_gpus)
    shared = args.ctx_shared > 0
    if shared:  # K shards of GPU 0: the K-GPU code path rehearsed on a one-GPU box
        G = args.ctx_shared
        # the shards' launches share the GPU's CUs, and the phased kernel's persistent grid needs all of them:
        # the one-shot walk, as for ranks sharing a GPU
        fa.set_tuning(walk=2)
    dev_of = (lambda g: 0) if shared else (lambda g: g)  # noqa: E731
    D, n, in_dt, _, desc = WORKLOADS[args.workload]
    idt = fa.F32 if in_dt == "f32" else fa.BF16
    s_in = 4 if in_dt == "f32" else 2
    rs = args.ctx_multi == "rs"
    if args.rs_chunks:
        fa.set_tuning(rs_chunks=args.rs_chunks)  # the process default the context starts from
    agg = fa.Aggregator(devices=[dev_of(g) for g in range(G)], rs=rs, shared_device=shared)
    agg.define(1, n, idt, fa.F32, D, fa.FEDAVG)
    for g in range(G):
        with torch.cuda.device(dev_of(g)):
            for k in range(D):
                try:
                    pcs = agg.pieces(1, g, k)
                except fa.FaError:  # rs: the client lives on another GPU
                    continue
                for ptr, cnt, off in pcs:
                    fa.fill_uniform(ptr, cnt, idt, 0x5EED, k, idx0=off)
    for g in range(G):
        torch.cuda.synchronize(dev_of(g))
    w = Setup._weights(D)
    import numpy as np
    clients = None  # chain position k holds generator client k
    if args.h2d:
        # client buckets in pinned host memory, submitted each round (fa_submit_pinned); the result lands in a
        # pinned host buffer (fa_finalize_gather, FA_HOST_PINNED).  One buffer per client while the round's
        # receipts fit 16 GiB of host memory (the north star: 32 x 256 MiB), else 8 distinct buffers that client
        # k takes k % 8 of (C5 stays at 8 GiB).  Buffer i holds generator client i (filled on the device, copied
        # once, outside the timed region), so the result can be checked.
        nbuf = D if D * n * s_in <= H2D_DISTINCT_MAX_BYTES else min(D, 8)
        hosts = [fa.PinnedBuffer(n * s_in) for _ in range(nbuf)]
        tmp = torch.empty(n * s_in // 4, dtype=torch.float32, device="cuda:0")
        for i, h in enumerate(hosts):
            fa.fill_uniform(tmp, n, idt, 0x5EED, i)
            torch.from_numpy(h.view(np.float32, count=n * s_in // 4)).copy_(tmp)
        del tmp
        torch.cuda.synchronize(0)
        clients = [k % len(hosts) for k in range(D)]
        res_buf = fa.PinnedBuffer(n * 4)
        res = res_buf.view(np.float32, count=n)

        def submit_all():
            for k in range(D):
                agg.submit(1, k, hosts[k % len(hosts)].view(np.uint8), w[k], pinned=True)

        def step():
            submit_all()
            agg.finalize_gather(1, [res], pinned=True)
    else:
        def step():
            agg.reduce(1, w)
    devs = sorted({dev_of(g) for g in range(G)})
    t_before = {d: fa.phased_timeouts(d) for d in devs}
    for _ in range(args.warmup):
        step()
    agg.sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    agg.sync()
    dt = (time.perf_counter() - t0) / args.steps
    split = None
    if args.h2d:
        # where a host-inclusive round goes, from one more round run phase by phase after the timed ones:
        # every receipt's H2D (submits + fa_sync), the reduction alone (fa_reduce_parts + fa_sync), the D2H of
        # the result into the pinned reply (fa_finalize_gather, which then only copies)
        ta = time.perf_counter()
        submit_all()
        agg.sync()
        tb = time.perf_counter()
        agg.reduce_parts([1])
        agg.sync()
        tc = time.perf_counter()
        agg.finalize_gather(1, [res], pinned=True)
        td = time.perf_counter()
        pcie = D * n * s_in + n * 4
        split = {"h2d_ms": round((tb - ta) * 1e3, 3), "reduce_ms": round((tc - tb) * 1e3, 3),
                 "d2h_ms": round((td - tc) * 1e3, 3), "pcie_bytes_per_round": pcie,
                 "pcie_GBs": round(pcie / dt / 1e9, 2), "distinct_host_buffers": len(hosts)}
    # > 0: a phased launch's grid was not co-resident on some GPU (the rs layout never takes that kernel)
    timeouts = sum(fa.phased_timeouts(d) - t_before[d] for d in devs)
    tuning = agg.get_tuning()
    # parity of the last round, read back now that the timed region is closed: >= 1024 sampled elements of
    # every GPU's share of the result (range: its element range, pieces included; rs: its block-cyclic
    # segments after the RCCL reduce-scatter, held to the 1e-6 tolerance)
    def check():
        got = res if args.h2d else agg.copy_output(1)
        per_gpu = []
        for g in range(G):
            if rs:
                segs = [(lo, min(hi, n)) for lo, hi in fa.rs_segments(n, G, tuning["rs_chunks"], g) if lo < n]
            else:
                segs = [(off, off + cnt) for _, cnt, off in agg.pieces(1, g, 0)]
            pos, idx = sample_positions(segs, salt=g)
            # the whole result is on the host: position = element index
            per_gpu.append(parity_check(got, idx.astype(np.int64), idx, 0x5EED, w, exact=not rs or G == 1,
                                        clients=clients, bf16_in=idt == fa.BF16))
        p = parity_merge(per_gpu)
        p["per_gpu_samples"] = [q["samples"] for q in per_gpu]
        return p
    parity = parity_guarded(check)
    out = {"layout": args.ctx_multi, "gpus": G, "shared_device_rehearsal": shared, "workload": args.workload,
           "description": desc, "clients": D,
           "elems_per_client": n, "host_inclusive": args.h2d, "ms_per_round": round(dt * 1e3, 4),
           "gib_s": round(D * n * s_in / dt / 2**30, 1), "steps": args.steps,
           "phased_meeting_timeouts": timeouts, "parity": parity, "tuning": tuning}
    if split:
        out.update(split)
    agg.close()
    print(json.dumps(out), flush=True)


def ctx_multi_secondaries(n_dev, deadline, timeout=120):
    """On a node with several visible GPUs, the N = 1 run also times the in-process multi-GPU layouts over
    all of them (child processes, time-limited: a stalled collective cannot take the main line with it).
    Every child gets min(timeout, what is left before `deadline` - a 30 s margin); once less than 20 s is left
    the rest are skipped (reported as such), so the line is printed before the driver's limit (600 s).
    On a one-GPU box the 8-GPU children are rehearsed instead as 8 shards of the one GPU (--ctx-shared 8:
    the layouts' code paths with the exchange replaced by its definition; a parity check, not a timing)."""
    # BASELINE C4 is quoted on 4 GPUs (RCCL reduce-scatter), C5 on 8 (128 x 1 GiB buckets arriving from host
    # memory, H2D overlapped over every GPU's link); the north star on all of them
    # the north star host-inclusive on one GPU (pinned host -> GPU -> pinned host, every receipt's H2D in the
    # round; network_layer.cpp:33-74 in, aggregator.cpp:96-106 out): reported as ns_h2d with its split
    legs = [("range", "northstar", True, 1, 0, 0)]
    if n_dev >= 2:
        legs += [("range", "northstar", False, n_dev, 0, 0), ("rs", "northstar", False, n_dev, 0, 0),
                ("rs", "c4", False, min(4, n_dev), 0, 0), ("rs", "c4", False, n_dev, 0, 0),
                ("range", "c5", True, min(8, n_dev), 0, 0)]
        # the rs overlap depth on real xGMI (untuned so far: one-GPU boxes have no exchange to overlap): C4's
        # 4-GPU reduce-scatter at other piece counts than the default, last, so the budget drops them first
        legs += [("rs", "c4", False, min(4, n_dev), 0, c) for c in RS_CHUNK_SWEEP]
    else:  # C5's per-GPU share (c5r) keeps the host-inclusive rehearsal at 16 GiB of input per round
        legs += [("rs", "c4", False, 8, 8, 0), ("range", "c5r", True, 8, 8, 0)]
    res = {}
    for layout, workload, h2d, gpus, shared, chunks in legs:
        key = "ctx_%s_%s%s_%d%s%s" % (layout, workload, "_h2d" if h2d else "", gpus,
                                     "shard_rehearsal_on_one_gpu" if shared else "gpu",
                                     "_rschunks%d" % chunks if chunks else "")
        if (layout, workload, h2d, gpus, shared) == ("range", "northstar", True, 1, 0):
            key = "ns_h2d"
        if key in res:
            continue
        left = deadline - time.monotonic() - 30  # deadline = T_START + BUDGET_S
        if left < 20:
            res[key] = {"skipped": "the bench's time budget is spent (FA_BENCH_BUDGET_S)"}
            continue
        cmd = [sys.executable, os.path.abspath(__file__), "--ctx-multi", layout, "--workload", workload]
        cmd += ["--ctx-shared", str(shared)] if shared else ["--ctx-gpus", str(gpus)]
        cmd += ["--rs-chunks", str(chunks)] if chunks else []
        cmd += ["--h2d", "--steps", "3", "--warmup", "1"] if h2d else ["--steps", "3" if shared else "10", "--warmup",
                                                                        "1" if shared else "2"]
        try:
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=min(timeout, left))
            res[key] = json.loads(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 else \
                {"error": "rc %d: %s" % (r.returncode, r.stderr[-300:])}
        except Exception as e:  # noqa: BLE001 -- reported, never fatal
            res[key] = {"error": repr(e)[:300]}
    return res


def single_gpu_secondaries(fa, torch, args, device, stream, dist, barrier):
    """The other BASELINE configs' single-GPU shapes, compute-node sync and literal mode (rank 0, N = 1)."""
    sec = {}
    skip = set(os.environ.get("FA_BENCH_SKIP", "").split(","))  # diagnostics: legs left out of this run
    for name in sorted(WORKLOADS):
        if name == args.workload or "workloads" in skip:
            continue
        sD, sn, si, so, sdesc = WORKLOADS[name]
        progress("workload " + name)
        s = Setup(fa, torch, sD, sn, si, so, 0, device)
        torch.cuda.synchronize()
        w2, ka, _ = timed_loop(torch, s, max(10, args.steps), 3, stream, dist, barrier)
        achieved = s.algo_bytes() / (ka * 1e-3) / 1e9
        # the same config's own read-only rate (its slots, its size): how far its kernel is from reading alone
        rp = None if under_profiler() else read_stream_peak(fa, torch, s, stream)
        ri = None if under_profiler() else read_plain_peak(fa, torch, s, stream, reps=3)
        sec[name] = {"description": sdesc, "gib_s": round(s.input_bytes() * max(10, args.steps) / w2 / 2**30, 1),
                     "kernel_ms_avg": round(ka, 4),
                     "achieved_GBs": round(achieved, 1),
                     "algorithmic_bytes_per_launch": s.algo_bytes(),
                     "traffic": traffic_from_profile(name, 1)[0],
                     "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "read_stream_peak": rp, "frac_of_read_stream": round(achieved / rp, 4) if rp else None,
                     "read_stream_peak_independent": ri["GBs"] if ri else None,
                     "read_stream_peak_independent_form": ri["form"] if ri else None,
                     "frac_of_read_stream_independent": round(achieved / ri["GBs"], 4) if ri else None,
                     "input_sets_rotated": s.nsets, "parity": parity_guarded(lambda: s.parity(0))}
        s.close()
        settle(s.nsets * s.input_bytes())

    # the buckets of one aggregator round as it forms them: per-round device time and roofline fraction,
    # phase 2 batched (fa_reduce_parts) and, for comparison, one launch per part
    for name in sorted(ROUNDS) if "rounds" not in skip else []:
        for batched in (True, False):
            progress("round %s%s" % (name, "" if batched else " unbatched"))
            s = RoundSetup(fa, torch, name, device, batched=batched)
            torch.cuda.synchronize()
            w2, ka, _ = timed_loop(torch, s, max(10, args.steps), 3, stream, dist, barrier)
            sec[name + ("" if batched else "_unbatched")] = {
                "description": "one aggregator round: " + s.desc + ", buckets " + "/".join(map(str, s.sizes)) +
                               (" (phase 2 batched: fa_reduce_parts)" if batched else " (one launch per part)"),
                "round_ms_avg": round(ka, 4), "algorithmic_bytes_per_round": s.algo_bytes(),
                "achieved_GBs": round(s.algo_bytes() / (ka * 1e-3) / 1e9, 1),
                "frac": round(s.algo_bytes() / (ka * 1e-3) / 1e9 / HBM_PEAK_GBS, 4), "input_sets_rotated": s.nsets,
                "parity": parity_guarded(lambda: s.parity())}
            s.close()
            settle(s.nsets * s.input_bytes())

    # BASELINE C1 end to end: the drop-in process fa_aggregator on this GPU against the fake owners over
    # loopback, FedAvg (owners at once) and the reference-literal mode (owners in turn, as the CPU reference
    # leg runs); both checked reply by reply against the oracle
    if os.access(FA_AGGREGATOR, os.X_OK) and os.access(FAKE_OWNERS, os.X_OK) and "c1e2e" not in skip:
        c1 = sec.setdefault("round_c1", {})
        progress("C1 end to end")
        for mode in ("fedavg", "literal"):
            try:
                base = free_port_base()
                c1["e2e_loopback_" + mode] = e2e_c1(
                    [FA_AGGREGATOR, "-i", "-1", "-d", "2", "-c", "1", "--mode", mode, "--rounds", str(C1_E2E_ROUNDS),
                     "--port-base", str(base)], mode, base)
            except Exception as e:  # noqa: BLE001
                c1["e2e_loopback_" + mode] = {"error": repr(e)[:300]}
        # the maintainer's other option: the reference's own process with its reduction
        # replaced by the libfa binding -- its network layer, torch::load per receipt, torch::save per reply
        if os.access(REF_BINDING_AGGREGATOR, os.X_OK) and ports_free(REF_PORTS):
            try:
                c1["e2e_loopback_reference_process_with_binding"] = dict(
                    e2e_c1([REF_BINDING_AGGREGATOR, "2", "1"], "fedavg", 8079, startup_s=2.5,
                           owner_flags=["--sequential"]),
                    path="the reference's aggregator process (systemAPI / network_layer / torch::load / "
                         "torch::save) with aggregator.cpp:55-167 replaced by the INTEGRATION.md 2 binding on "
                         "libfa.so (oracle/_ref/ref_aggregator)")
            except Exception as e:  # noqa: BLE001
                c1["e2e_loopback_reference_process_with_binding"] = {"error": repr(e)[:300]}

    # BASELINE C2 end to end through the drop-in (FedAvg, 8 owners at once, ResNet-18 receipts made by the
    # reference's builders): the owner-view round and the phase-2 tail (last receipt -> replies framed), with
    # streaming ingest (the default) and without it (--stream-min-bytes 0)
    harness = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
    if os.access(FA_AGGREGATOR, os.X_OK) and os.access(FAKE_OWNERS, os.X_OK) and os.access(harness, os.X_OK) \
            and budget_left() > 90 and "c2e2e" not in skip:
        c2 = sec.setdefault("round_c2", {})
        progress("C2 end to end")
        try:
            with tempfile.TemporaryDirectory(prefix="fa_c2_blobs_") as blobs:
                for mp in ("-1", "2"):  # the reference's ResNet-18 parts saved by torch::save (client 0's)
                    subprocess.run([harness, "golden", "1", "1", "9", "3", "10", "1", "24301", "7", blobs, mp],
                                   check=True, capture_output=True, timeout=120)
                for streamed in (True, False):
                    base = free_port_base()
                    c2["e2e_loopback_fedavg" + ("" if streamed else "_no_streaming")] = e2e_run(
                        [FA_AGGREGATOR, "-i", "-1", "-d", "8", "-c", "1", "--rounds", str(C2_E2E_ROUNDS),
                         "--port-base", str(base)] + ([] if streamed else ["--stream-min-bytes", "0"]) +
                        os.environ.get("FA_BENCH_C2_AGG_ARGS", "").split(),
                        "fedavg", base, blobs, 8, C2_MODEL, C2_E2E_ROUNDS, timeout=180, owner_flags=["--routing-table"])
        except Exception as e:  # noqa: BLE001
            c2["e2e_error"] = repr(e)[:300]

    def one(key, s, desc):
        progress(key)
        torch.cuda.synchronize()
        _, ka, _ = timed_loop(torch, s, max(10, args.steps), 3, stream, dist, barrier)
        sec[key] = {"description": desc, "kernel_ms_avg": round(ka, 4),
                    "achieved_GBs": round(s.algo_bytes() / (ka * 1e-3) / 1e9, 1),
                    "frac": round(s.algo_bytes() / (ka * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                    "input_sets_rotated": s.nsets}
        if isinstance(s, SyncSetup) and s.in_dt == fa.F32 and not under_profiler():
            cp = rw_plain_peak(fa, torch, s, stream)  # before the parity check, which refills a set
            sec[key]["copy_ceiling_independent"] = cp
            sec[key]["frac_of_copy_independent"] = round(sec[key]["achieved_GBs"] / cp["GBs"], 4)
        sec[key]["parity"] = parity_guarded(lambda: s.parity(0))
        s.close()
        settle(s.nsets * s.input_bytes())
    # compute-node aggregation on the C2 shape: 8 client copies synced in place
    sD, sn, si, so, _ = WORKLOADS["c2"]
    one("sync_c2", SyncSetup(fa, torch, sD, sn, si, so, 0, device),
        "compute-node state sync, 8 client copies of the ResNet-18 buckets, fp32, in place "
        "(D reads + D writes per element)")
    # the same on a large part: 8 copies of VGG-19's FC part (119.6 M parameters, C4's split 3,19)
    one("sync_vgg_fc", SyncSetup(fa, torch, 8, 119_586_826, "f32", "f32", 0, device),
        "compute-node state sync, 8 client copies of VGG-19's FC part (119.6 M fp32 parameters), in place")
    # the reference's own semantics (aggregator.cpp:72-88, literal mode): fl(fl(x+x)/1000) of the last
    # receipt, on its largest bucket (VGG-19's FC part); per element one read + one write
    one("literal_vgg_fc", Setup(fa, torch, 1, 119_586_826, "f32", "f32", 0, device, mode=fa.LITERAL),
        "reference-literal mode fl(fl(x+x)/1000) of the last receipt, VGG-19's FC part (119.6 M fp32 parameters)")
    return sec


if __name__ == "__main__":
    main()
