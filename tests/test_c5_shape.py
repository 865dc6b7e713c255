"""GPU: BASELINE config C5's shape -- 128 clients x 1 GiB fp32 buckets -- pinned against the oracle on one
MI355X (VERDICT r02 "next" #1 and #6).  The 8-GPU leg of C5 needs the driver's node; here its bucket shape
runs whole on one GPU through the three paths the aggregator uses (the reduction replaced is
aggregator.cpp:112-150):

* the range context, device-resident: a GPU holding 128 GiB of slots cuts them into 8 pieces of 16 GiB
  ("the address span") reduced one launch after another; sampled elements against the oracle's
  chain, the chain split over two launches per piece equal to the context's result in every bit, and no
  phased meeting that gave up waiting;
* the rs context at one GPU (FA_SHARD_CLIENT_RS: per-piece reductions + a one-rank reduce-scatter, i.e. a
  copy), whose launches never take the phased grid: bit-exact at the sampled elements, no timeout;
* host-inclusive: 128 fa_submit_pinned receipts (8 distinct host buckets, client k sends bucket k mod 8) and
  one fa_finalize into host memory, sampled against the oracle's chain over the same inputs.
Memory: 129-130 GiB of HBM at a time (one context after the other), 9 GiB pinned host memory.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N, D, SEED = 1 << 28, 128, 0x5EED


def sample_idx(n, m=1024):
    rng = np.random.default_rng(5)
    return np.unique(np.concatenate([[0, 1, 2, 3, n // 2, n - 4, n - 3, n - 2, n - 1], rng.integers(0, n, m)]))


def assert_bits(got, ref):
    bad = np.flatnonzero(np.asarray(got, np.float32).view(np.uint32) != np.asarray(ref, np.float32).view(np.uint32))
    assert bad.size == 0, "%d mismatches, first at %s: got %s ref %s" % (bad.size, bad[:4], got[bad[:4]], ref[bad[:4]])


def filled_ctx(fa, torch, rs):
    agg = fa.Aggregator(devices=[0], rs=rs)
    agg.define(1, N, fa.F32, fa.F32, D, fa.FEDAVG)
    for k in range(D):
        for ptr, cnt, off in agg.pieces(1, 0, k):
            fa.fill_uniform(ptr, cnt, fa.F32, SEED, k, idx0=off)
    torch.cuda.synchronize()
    return agg


def test_c5_range_context_sampled_split_and_no_timeouts(fa, O, torch_gpu):
    torch = torch_gpu
    w = O.weights(D)
    idx = sample_idx(N)
    ref = O.fedavg_at(SEED, w, idx)
    t0 = fa.phased_timeouts(0)
    with filled_ctx(fa, torch, rs=False) as agg:
        pcs = agg.pieces(1, 0, 0)
        assert len(pcs) == 8 and sum(c for _, c, _ in pcs) == N
        agg.reduce(1, w)
        out = agg.copy_output(1)  # waits for the reduction, D2H of the 1 GiB result
        assert_bits(out[idx], ref)
        # per piece, the same chain in two launches (first 50 clients, then 78 continuing it): the same bits
        acc = torch.empty(N, dtype=torch.float32, device="cuda")
        for j, (_, cnt, off) in enumerate(pcs):
            cl = [agg.pieces(1, 0, k)[j][0] for k in range(D)]
            a = acc[off:off + cnt]
            fa.reduce_device(cl[:50], w[:50], cnt, fa.F32, a, fa.F32)
            fa.reduce_device(cl[50:], w[50:], cnt, fa.F32, a, fa.F32, init=a)
        torch.cuda.synchronize()
        assert np.array_equal(out.view(np.uint32), acc.cpu().numpy().view(np.uint32))
        del out, acc
    assert fa.phased_timeouts(0) - t0 == 0


def test_c5_rs_context_one_gpu_bitexact_no_phased(fa, O, torch_gpu):
    torch = torch_gpu
    w = O.weights(D)
    idx = sample_idx(N)
    ref = O.fedavg_at(SEED, w, idx)
    assert fa.rs_plan(N, 1, D)[1] == 0  # no piece takes the persistent grid
    t0 = fa.phased_timeouts(0)
    with filled_ctx(fa, torch, rs=True) as agg:
        agg.reduce(1, w)
        out = agg.copy_output(1)  # the shard's segments, in bucket order
        assert_bits(out[idx], ref)
        del out
    assert fa.phased_timeouts(0) - t0 == 0


def test_c5_host_inclusive_round(fa, O, torch_gpu):
    torch = torch_gpu
    w = O.weights(D)
    idx = sample_idx(N)
    hosts = [fa.PinnedBuffer(N * 4) for _ in range(8)]
    try:
        tmp = torch.empty(N, dtype=torch.float32, device="cuda")
        for j, h in enumerate(hosts):  # bucket j = the generator's client j, made on the device
            fa.fill_uniform(tmp, N, fa.F32, SEED, j)
            torch.cuda.synchronize()
            h.view(np.float32)[:] = tmp.cpu().numpy()
        del tmp
        res = np.empty(N, np.float32)
        with fa.Aggregator(devices=[0]) as agg:
            agg.define(1, N, fa.F32, fa.F32, D, fa.FEDAVG)
            for k in range(D):
                agg.submit(1, k, hosts[k % 8].view(np.float32), w[k], pinned=True)
            agg.finalize(1, res)
        cols = [hosts[k % 8].view(np.float32)[idx] for k in range(D)]
        assert_bits(res[idx], O.fedavg(cols, w))
        assert_bits(hosts[3].view(np.float32)[idx[:64]], O.gen_at(SEED, 3, idx[:64]))  # the inputs themselves
    finally:
        for h in hosts:
            h.close()
