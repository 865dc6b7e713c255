"""GPU tests of the aggregation context's layouts and round shapes through the C ABI, against the oracle.

* FA_SHARD_CLIENT_RS: clients dealt to the context's GPUs, fp32 partials summed by an RCCL reduce-scatter
  (ncclCommInitAll in-process), pieces overlapped with the reduction; bit-exact at one GPU (a one-rank
  reduce-scatter is a copy), within 1e-6 of sum_k |w_k x_k| at more.
* FA_ACCUMULATE_ON_ARRIVAL: the chain advances over the in-order prefix of receipts (same bits).
* fa_reduce_parts: every model-part bucket of a phase in one batched launch (segment table), the
  aggregator's own bucket sizes (tests/golden/layouts: ResNet-18 split 3,8), same bits as per part.
The reduction the reference performs here is aggregator.cpp:59-93 / :112-150.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def assert_bits(got, ref):
    ut = np.uint16 if got.dtype == np.uint16 else np.uint32
    bad = np.flatnonzero(got.view(ut) != ref.view(ut))
    assert bad.size == 0, "%d/%d mismatches, first at %s: got %s ref %s" % (
        bad.size, got.size, bad[:4], got[bad[:4]], ref[bad[:4]])


def host_clients(O, seed, D, n, bf16=False):
    return [O.gen(seed, k, n, dtype="bf16" if bf16 else "f32") for k in range(D)]


def rs_ctx(fa, G):
    """An rs context on G GPUs: real ones (RCCL communicators) when visible, else G shards on GPU 0
    (test-only FA_TEST_SHARED_DEVICE: RCCL refuses two ranks on one device -- "invalid usage", gpurun_out
    r02s06 -- so the reduce-scatter is replaced by its definition, the rest of the layout is the product's)."""
    if fa.device_count() >= G:
        return fa.Aggregator(G, rs=True)
    return fa.Aggregator(devices=[0] * G, rs=True, shared_device=True)


# ----------------------------------------------------------------- FA_SHARD_CLIENT_RS

@pytest.mark.gpu
def test_exchange_stream_only_in_rs_contexts(fa, torch_gpu):
    """Only the rs layout has an exchange, so only an rs context holds the (high-priority) exchange stream:
    a second high-priority stream on a device slowed every later launch there by ~2% (DESIGN.md 5,
    profiles/r05_order_effect.jsonl), e.g. a process that creates a context per workload."""
    with fa.Aggregator(1) as agg:
        assert agg.exchange_streams() == 0
    with fa.Aggregator(1, eager=True) as agg:
        assert agg.exchange_streams() == 0
    with fa.Aggregator(devices=[0, 0], shared_device=True) as agg:  # range layout on two shards
        assert agg.exchange_streams() == 0
    with rs_ctx(fa, 2) as agg:
        assert agg.exchange_streams() == 2


@pytest.mark.parametrize("n,D,chunks,bf16,out_bf16", [
    (1_000_003, 5, 1, False, False), (4_194_304, 8, 8, False, False), (333_333, 3, 4, True, False),
    (63, 2, 3, False, False), (2_000_000, 130, 2, False, False),
    (333_333, 3, 4, True, True), (1_000_003, 6, 3, False, True)])  # bf16 outputs: the shard rounded once
def test_rs_layout_one_gpu_bitexact(fa, O, torch_gpu, n, D, chunks, bf16, out_bf16):
    """One GPU: the reduce-scatter over a one-rank communicator is a copy, so the pieces' chains are the
    single chain -- bit-exact, whatever the piece count; the slot padding stays out of the result."""
    w = O.weights(D)
    xs = host_clients(O, 60 + D, D, n, bf16)
    ref = O.fedavg(xs, w, out_dtype="bf16") if bf16 and out_bf16 else \
        O.f32_to_bf16(O.fedavg(xs, w)) if out_bf16 else O.fedavg(xs, w)  # f32 chain, rounded once
    with fa.Aggregator(1, rs=True) as agg:
        agg.set_tuning(rs_chunks=chunks)
        assert agg.get_tuning()["rs_chunks"] == chunks
        agg.define(1, n, fa.BF16 if bf16 else fa.F32, fa.BF16 if out_bf16 else fa.F32, D, fa.FEDAVG)
        for k in reversed(range(D)):
            agg.submit(1, k, xs[k], w[k])
        assert_bits(agg.finalize(1), ref)
        # the device-resident round on the same slots
        agg.reduce(1, w)
        assert_bits(agg.copy_output(1), ref)


def test_rs_layout_literal_and_errors(fa, O, torch_gpu):
    n, D = 100_001, 3
    xs = host_clients(O, 70, D, n)
    with fa.Aggregator(1, rs=True) as agg:
        agg.define(1, n, fa.F32, fa.F32, D, fa.LITERAL)
        for k in [0, 2, 1]:
            agg.submit(1, k, xs[k])
        assert_bits(agg.finalize(1), O.literal(xs[1]))
        agg.define(2, n, fa.F32, fa.BF16, D, fa.LITERAL)  # the last client's GPU writes bf16 directly
        for k in [2, 0, 1]:
            agg.submit(2, k, xs[k])
        assert_bits(agg.finalize(2), O.f32_to_bf16(O.literal(xs[1])))  # fp32 literal, rounded once
        with pytest.raises(fa.FaError):
            agg.sync_states(1)


@pytest.mark.parametrize("G,D,chunks,bf16,out_bf16", [
    (2, 7, 8, False, False), (4, 7, 3, False, False), (3, 2, 5, False, False), (4, 9, 1, False, False),
    (2, 5, 4, True, False), (3, 6, 2, True, False), (3, 6, 2, True, True), (4, 7, 3, False, True)])
def test_rs_layout_multi_gpu_tolerance(fa, O, torch_gpu, record_property, G, D, chunks, bf16, out_bf16):
    """G shards: clients dealt to the GPUs (a GPU may hold none: D < G), every GPU's shard holds its
    cyclic blocks; the whole result within 1e-6 of sum_k |w_k x_k| of the oracle's ordered chain (the
    exchange adds per-GPU partials; bf16 inputs exchange fp32 partials too) -- for a bf16 output, plus
    the one bf16 rounding of that sum (half a bf16 ulp, 2^-8 relative); the device-resident round on the
    same slots agrees bit for bit.  The largest error, relative to sum_k |w_k x_k| and as a fraction of the
    bound, is reported ("parity by tolerance ... with the max error reported")."""
    n = 1_234_567
    w = O.weights(D)
    xs = host_clients(O, 71, D, n, bf16)
    with rs_ctx(fa, G) as agg:
        agg.set_tuning(rs_chunks=chunks)
        agg.define(1, n, fa.BF16 if bf16 else fa.F32, fa.BF16 if out_bf16 else fa.F32, D, fa.FEDAVG)
        for k in range(D):
            agg.submit(1, k, xs[k], w[k])
        got = agg.finalize(1)
        for _ in range(3):  # back-to-back device-resident rounds: each waits for the previous exchange
            agg.reduce(1, w)
        assert_bits(agg.copy_output(1), got)
    ref = O.fedavg(xs, w)
    vals = [O.bf16_to_f32(x) if bf16 else x for x in xs]
    absw = sum(abs(np.float64(wk)) * np.abs(x.astype(np.float64)) for wk, x in zip(w, vals))
    gotf = (O.bf16_to_f32(got) if out_bf16 else got).astype(np.float64)
    bound = 1e-6 * absw + (2.0 ** -8 * np.abs(ref.astype(np.float64)) if out_bf16 else 0.0) + 1e-30
    err = np.abs(gotf - ref) / bound
    rel = float((np.abs(gotf - ref) / (absw + 1e-30)).max())
    record_property("max_err_rel_to_sum_abs", rel)
    record_property("max_err_fraction_of_bound", float(err.max()))
    ulps = ""
    if out_bf16:  # against the oracle's fp32 chain rounded once to bf16: bf16 ulps apart (ordered bit patterns)
        def ordered(b):
            b = b.astype(np.int64)
            return np.where(b & 0x8000, 0x8000 - (b & 0x7FFF), 0x8000 + b)
        du = int(np.abs(ordered(got.view(np.uint16)) - ordered(O.f32_to_bf16(ref))).max())
        record_property("max_bf16_ulps_from_rounded_oracle", du)
        ulps = ", max %d bf16 ulp(s) from the oracle's rounded chain" % du
    print("rs tolerance G=%d D=%d chunks=%d bf16_in=%s bf16_out=%s: max |err| / sum|w x| = %.3g, "
          "max fraction of the bound = %.3g%s" % (G, D, chunks, bf16, out_bf16, rel, float(err.max()), ulps))
    assert np.all(err <= 1.0), float(err.max())


@pytest.mark.parametrize("G", [2, 4])
def test_rs_layout_large_pieces_no_persistent_grid(fa, O, torch_gpu, G):
    """VGG-19's FC bucket (C4's largest, 119.6 M elements) over 8 clients in the rs layout at G GPUs (G shards
    of the one GPU when only one is visible): every piece is several phases long, yet no launch of the
    round takes the phased grid (fa_diag_rs_plan; verdict r02 #1), no meeting times out, and sampled
    elements stay within 1e-6 of sum_k |w_k x_k| of the oracle's chain."""
    torch = torch_gpu
    n, D = 119_586_826, 8
    w = O.weights(D)
    launches, phased, _ = fa.rs_plan(n, G, D, 2)
    assert launches == 2 * G and phased == 0
    t0 = fa.phased_timeouts(0)
    with rs_ctx(fa, G) as agg:
        agg.set_tuning(rs_chunks=2)  # two pieces of ~60 M elements: 2-3 phases each, were it phased
        agg.define(1, n, fa.F32, fa.F32, D, fa.FEDAVG)
        for g in range(G):
            for k in range(D):
                try:
                    ptr, cnt, off = agg.slot(1, g, k)
                except fa.FaError:  # the client lives on another GPU
                    continue
                fa.fill_uniform(ptr, cnt, fa.F32, 0x5EED, k, idx0=off)
        torch.cuda.synchronize()
        for _ in range(2):
            agg.reduce(1, w)
        got = agg.copy_output(1)
    assert fa.phased_timeouts(0) - t0 == 0
    rng = np.random.default_rng(11)
    idx = np.unique(np.concatenate([[0, n - 1], rng.integers(0, n, 512)]))
    ref = O.fedavg_at(0x5EED, w, idx).astype(np.float64)
    absw = sum(abs(np.float64(w[k])) * np.abs(O.gen_at(0x5EED, k, idx).astype(np.float64)) for k in range(D))
    err = np.abs(got[idx].astype(np.float64) - ref) / (1e-6 * absw + 1e-30)
    assert np.all(err <= 1.0), float(err.max())


# ----------------------------------------------------------------- accumulate on arrival

@pytest.mark.parametrize("G", [1, 2])
def test_accumulate_on_arrival_same_bits(fa, O, torch_gpu, G):
    """Receipts in order advance the chain one launch at a time (the phase end then only copies);
    out of order they wait for the gap; a replaced receipt restarts the chain.  Every result equals
    the one ordered chain bit for bit."""
    n, D = 2_000_003, 6
    w = O.weights(D)
    xs = host_clients(O, 72, D, n)
    ref = O.fedavg(xs, w)
    ctx = fa.Aggregator(G, eager=True) if fa.device_count() >= G else \
        fa.Aggregator(devices=[0] * G, eager=True, shared_device=True)
    with ctx as agg:
        agg.define(1, n, fa.F32, fa.F32, D, fa.FEDAVG)
        for k in range(D):  # in order: the prefix grows with every receipt
            agg.submit(1, k, xs[k], w[k])
            assert agg.progress(1) == (k + 1, k + 1)
        assert_bits(agg.finalize(1), ref)
        assert agg.progress(1) == (0, 0)
        order = [1, 0, 3, 2, 5, 4]
        reduced = []
        for k in order:  # out of order: the prefix only moves past gaps once they are filled
            agg.submit(1, k, xs[k], w[k])
            reduced.append(agg.progress(1)[1])
        assert reduced == [0, 2, 2, 4, 4, 6]
        assert_bits(agg.finalize(1), ref)
        for k in range(D):
            agg.submit(1, k, xs[k], w[k])
        xs2 = list(xs)
        xs2[2] = O.gen(73, 2, n)
        agg.submit(1, 2, xs2[2], w[2])  # a replaced receipt: the chain restarts and catches up at once
        assert agg.progress(1) == (D, D)
        assert_bits(agg.finalize(1), O.fedavg(xs2, w))
        # bf16 output, a part defined with D > kMaxClients (two passes from the accumulator)
        agg.define(2, 50_001, fa.F32, fa.BF16, 130, fa.FEDAVG)
        w130 = O.weights(130)
        x130 = host_clients(O, 74, 130, 50_001)
        for k in range(130):
            agg.submit(2, k, x130[k], w130[k])
        assert_bits(agg.finalize(2), O.f32_to_bf16(O.fedavg(x130, w130)))


# ----------------------------------------------------------------- one launch per phase

@pytest.mark.parametrize("device_resident", [True, False])
def test_reduce_parts_batched_same_bits(fa, O, torch_gpu, device_resident):
    """ResNet-18's split-3,8 buckets (83,584 / 9,442,304 / 5,130 elements, D = 8, the reference builders'
    sizes) in one fa_reduce_parts call: the two last-part buckets are one segment-table launch; plus a
    bf16 bucket and a D = 32 bucket large enough for the phased kernel in the same call.  Each result
    equals the oracle (whole buckets up to 10 M elements)."""
    torch = torch_gpu
    D = 8
    parts = {1: (83_584, D, False), 2: (9_442_304, D, False), 3: (5_130, D, False), 4: (77_777, 5, True),
             5: (6_000_001, 32, False)}
    with fa.Aggregator(1) as agg:
        for pid, (n, d, bf16) in parts.items():
            agg.define(pid, n, fa.BF16 if bf16 else fa.F32, fa.F32, d, fa.FEDAVG)
        refs = {}
        for pid, (n, d, bf16) in parts.items():
            wd = O.weights(d)
            xs = host_clients(O, 80 + pid, d, n, bf16)
            refs[pid] = O.fedavg(xs, wd, threads=8)
            for k in range(d):
                if device_resident:
                    ptr, cnt, _ = agg.slot(pid, 0, k)
                    fa.fill_uniform(ptr, cnt, fa.BF16 if bf16 else fa.F32, 80 + pid, k)
                else:
                    agg.submit(pid, k, xs[k], wd[k])
        torch.cuda.synchronize()
        ids = list(parts)
        if device_resident:
            agg.reduce_parts(ids, weights=[O.weights(parts[p][1]) for p in ids])
            for pid in ids:
                assert_bits(agg.copy_output(pid), refs[pid])
        else:
            agg.reduce_parts(ids)
            for pid in ids:
                assert agg.progress(pid)[1] == parts[pid][1]  # ready: finalize only copies
                assert_bits(agg.finalize(pid), refs[pid])
        with pytest.raises(fa.FaError):
            agg.reduce_parts([1, 1])


def test_reduce_parts_two_gpus_and_literal(fa, O, torch_gpu):
    """Range shards of a two-GPU context (two shards on one GPU when only one is visible): each GPU's
    segment table holds its ranges; a literal part in the same call takes its own launch."""
    ctx = fa.Aggregator(2) if fa.device_count() >= 2 else fa.Aggregator(devices=[0, 0], shared_device=True)
    D = 4
    w = O.weights(D)
    with ctx as agg:
        sizes = {1: 100_003, 2: 64, 3: 1}
        for pid, n in sizes.items():
            agg.define(pid, n, fa.F32, fa.F32, D, fa.FEDAVG)
        agg.define(9, 5000, fa.F32, fa.F32, D, fa.LITERAL)
        refs = {}
        for pid, n in sizes.items():
            xs = host_clients(O, 90 + pid, D, n)
            refs[pid] = O.fedavg(xs, w)
            for k in range(D):
                agg.submit(pid, k, xs[k], w[k])
        lit = host_clients(O, 99, D, 5000)
        for k in [3, 1]:
            agg.submit(9, k, lit[k])
        agg.reduce_parts([1, 2, 3, 9])
        for pid in sizes:
            assert_bits(agg.finalize(pid), refs[pid])
        assert_bits(agg.finalize(9), O.literal(lit[1]))


def d2h(ptr, n):
    """n fp32 elements at a raw device address, copied to the host (hipMemcpy, device to host)."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    out = np.empty(n, np.float32)
    assert hip.hipMemcpy(ctypes.c_void_p(out.ctypes.data), ctypes.c_void_p(ptr), ctypes.c_size_t(4 * n), 2) == 0
    return out


def test_sync_part_waits_for_submits(fa, O, torch_gpu):
    """fa_submit then fa_sync_part with no fa_sync between: the state sync orders itself after the
    submits' H2D copies, so every slot holds the FedAvg of the submitted receipts."""
    n, D = 3_000_001, 5
    w = O.weights(D)
    xs = host_clients(O, 95, D, n)
    with fa.Aggregator(1) as agg:
        agg.define(1, n, fa.F32, fa.F32, D, fa.FEDAVG)
        for k in range(D):
            agg.submit(1, k, xs[k], w[k])
        agg.sync_states(1)
        agg.sync()
        ref = O.fedavg(xs, w)
        for k in (0, D - 1):
            ptr, cnt, _ = agg.slot(1, 0, k)
            assert_bits(d2h(ptr, cnt), ref)


def test_reduce_parts_device_table_and_reuse(fa, O, torch_gpu):
    """A batch beyond the kernel-argument table (more than 8 buckets, or more than 192 clients) goes
    through a device-side segment table, uploaded only when it changed: the same batch twice (no
    upload), then new weights (upload), every time bit-exact."""
    torch = torch_gpu
    sizes = [1, 4, 63, 64, 65, 1000, 4099, 77_777, 5, 300_001, 12]
    D = 6
    with fa.Aggregator(1) as agg:
        xs = {}
        for pid, n in enumerate(sizes, start=1):
            agg.define(pid, n, fa.F32, fa.F32, D, fa.FEDAVG)
            xs[pid] = host_clients(O, 200 + pid, D, n)
            for k in range(D):
                ptr, cnt, _ = agg.slot(pid, 0, k)
                fa.fill_uniform(ptr, cnt, fa.F32, 200 + pid, k)
        torch.cuda.synchronize()
        ids = list(range(1, len(sizes) + 1))
        for w in (O.weights(D), O.weights(D), O.weights(D, seed=99)):
            agg.reduce_parts(ids, weights=[w] * len(ids))
            for pid in ids:
                assert_bits(agg.copy_output(pid), O.fedavg(xs[pid], w))
        # many clients: 2 buckets x 130 clients (> 192 in the kernel arguments, and > 128 per bucket: those
        # take their own multi-pass launch) and 2 x 100 (device table)
        for pid, (n, d) in {20: (5000, 130), 21: (777, 100), 22: (4096, 100)}.items():
            agg.define(pid, n, fa.F32, fa.F32, d, fa.FEDAVG)
            xs[pid] = host_clients(O, 300 + pid, d, n)
            for k in range(d):
                ptr, cnt, _ = agg.slot(pid, 0, k)
                fa.fill_uniform(ptr, cnt, fa.F32, 300 + pid, k)
        torch.cuda.synchronize()
        ws = {pid: O.weights(len(xs[pid])) for pid in (20, 21, 22)}
        agg.reduce_parts([20, 21, 22], weights=[ws[20], ws[21], ws[22]])
        for pid in (20, 21, 22):
            assert_bits(agg.copy_output(pid), O.fedavg(xs[pid], ws[pid]))


def test_reduce_parts_device_tables_across_streams(fa, O, torch_gpu):
    """Device segment tables (batches of more than 8 buckets) used from two streams without a sync between:
    an explicit stream kept busy, then the context's compute stream.  Each batch's table
    lives in its own slot of the per-GPU ring until its launch is done, a reused table orders itself after
    the upload on the other stream, and every bucket ends bit-exact."""
    torch = torch_gpu
    D = 6
    P = {pid: n for pid, n in zip(range(1, 11), [3, 64, 65, 1000, 4099, 77_777, 5, 30_001, 12, 130])}
    Q = {pid: n for pid, n in zip(range(21, 31), [7, 63, 129, 999, 4097, 50_000, 9, 20_001, 16, 131])}
    A = torch.cuda.Stream()
    busy = torch.empty(1 << 27, dtype=torch.float32, device="cuda")
    with fa.Aggregator(1) as agg:
        xs = {}
        for pid, n in {**P, **Q}.items():
            agg.define(pid, n, fa.F32, fa.F32, D, fa.FEDAVG)
            xs[pid] = host_clients(O, 400 + pid, D, n)
            for k in range(D):
                ptr, cnt, _ = agg.slot(pid, 0, k)
                fa.fill_uniform(ptr, cnt, fa.F32, 400 + pid, k)
        torch.cuda.synchronize()
        for rep in range(3):
            wP, wQ = O.weights(D, seed=10 + rep), O.weights(D, seed=50 + rep)
            fa.fill_uniform(busy, busy.numel(), fa.F32, 1, rep, stream=A)  # stream A starts late
            agg.reduce_parts(list(P), weights=[wP] * len(P), stream=A)
            agg.reduce_parts(list(Q), weights=[wQ] * len(Q))  # a new table on the compute stream
            if rep == 2:  # the same table again, now on the compute stream: after its upload on A
                fa.fill_uniform(busy, busy.numel(), fa.F32, 2, rep, stream=A)
                agg.reduce_parts(list(P), weights=[wP] * len(P), stream=A)
                agg.reduce_parts(list(P), weights=[wP] * len(P))
            torch.cuda.synchronize()
            agg.sync()
            for pid in P:
                assert_bits(agg.copy_output(pid), O.fedavg(xs[pid], wP))
            for pid in Q:
                assert_bits(agg.copy_output(pid), O.fedavg(xs[pid], wQ))
