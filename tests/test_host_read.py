"""GPU: small receipts read where they arrived (csrc/fa_api.hip, host_keep / host_reduce).

A pinned receipt of a one-GPU range part whose D receipts total at most 1 MiB is not copied to its device
slot: the reduction's kernels read its segments over PCIe -- into the part's output, or at
fa_finalize_gather(FA_HOST_PINNED) straight into the pinned destination segments -- and every other path
that needs the slots first copies the kept receipts in.  These tests hold every path to the oracle's bits
(the ordered chain of aggregator.cpp:59-93 with FedAvg semantics, or the literal fl(fl(x+x)/1000) of the last
receipt), and check through fa_diag_host_reads that the in-place reads really ran where they should and not
where they must not (a misaligned segment, a pageable receipt, a bucket over the limit).
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def layout(n, es, cuts, gaps, rng):
    """A receipt of n elements split at element positions `cuts`, the pieces placed in one pinned buffer
    with `gaps` bytes before each (element-aligned, not 16-byte aligned): [(byte offset, elements)]."""
    edges = [0] + sorted(cuts) + [n]
    out, off = [], 0
    for i in range(len(edges) - 1):
        off += gaps[i % len(gaps)]
        cnt = edges[i + 1] - edges[i]
        out.append((off, cnt))
        off += cnt * es
    return out, off


def place(fa, values, segs, total, shift=0):
    """A PinnedBuffer holding `values` at the segments' offsets (+ shift bytes); the segment views."""
    es = values.itemsize
    buf = fa.PinnedBuffer(total + shift + 64)
    raw = buf.view(np.uint8)
    views, e = [], 0
    for off, cnt in segs:
        v = raw[shift + off: shift + off + cnt * es]
        v[:] = values[e:e + cnt].view(np.uint8)
        views.append(v)
        e += cnt
    return buf, views


def dst_views(fa, n, es, segs, total):
    buf = fa.PinnedBuffer(total + 64)
    raw = buf.view(np.uint8)
    raw[:] = 0xA5
    return buf, [raw[off: off + cnt * es] for off, cnt in segs]


def gathered(views, dtype):
    return np.concatenate([np.frombuffer(v.tobytes(), dtype) for v in views])


def expected(O, xs, w, in_bf16, out_bf16, literal=None):
    if literal is not None:
        return O.literal(xs[literal], out_dtype="bf16" if out_bf16 else "f32")
    if in_bf16:
        return O.fedavg(xs, w, out_dtype="bf16" if out_bf16 else "f32")
    ref = O.fedavg(xs, w)
    return O.f32_to_bf16(ref) if out_bf16 else ref  # the fp32 chain, rounded once (RNE)


@pytest.mark.parametrize("D,n,in_bf16,out_bf16", [(1, 777, False, False), (2, 50_536, False, False),
                                                 (5, 10_164, False, False), (3, 850, True, True),
                                                 (4, 20_003, True, False)])
def test_small_pinned_round_reads_in_place(fa, O, torch_gpu, D, n, in_bf16, out_bf16):
    """Receipts as four scattered pinned segments each (as archive records are), the reply as three other
    segments: one finalize reads them in place and writes the reply's segments directly, bit-exact."""
    rng = np.random.default_rng(n)
    es, eo = (2 if in_bf16 else 4), (2 if out_bf16 else 4)
    xs = [O.gen(0x5EED, k, n, dtype="bf16" if in_bf16 else "f32") for k in range(D)]
    w = O.weights(D)
    cuts = sorted(rng.choice(np.arange(1, n), 3, replace=False).tolist())
    with fa.Aggregator(1) as agg:
        agg.define(1, n, fa.BF16 if in_bf16 else fa.F32, fa.BF16 if out_bf16 else fa.F32, D, fa.FEDAVG)
        for rnd in range(2):  # twice: the second round reuses the part
            keep = []
            for k in reversed(range(D)):  # out of order
                segs, total = layout(n, es, cuts, [es * 3, 64 + es, 256 + 2 * es], rng)
                buf, views = place(fa, xs[k], segs, total)
                keep.append(buf)
                agg.submit_gather(1, k, views, w[k], pinned=True)
            dsegs, dtotal = layout(n, eo, [n // 3, 2 * n // 3] if n > 3 else [], [eo, 128 + eo], rng)
            dbuf, dviews = dst_views(fa, n, eo, dsegs, dtotal)
            before = agg.host_reads()
            agg.finalize_gather(1, dviews, pinned=True)
            assert agg.host_reads() == before + 1
            got = gathered(dviews, np.uint16 if out_bf16 else np.float32)
            want = expected(O, xs, w, in_bf16, out_bf16)
            assert np.array_equal(got.view(np.uint16 if out_bf16 else np.uint32),
                                  want.view(np.uint16 if out_bf16 else np.uint32))


@pytest.mark.parametrize("in_bf16,out_bf16", [(False, False), (True, True), (False, True), (True, False)])
def test_aligned_records_in_one_launch(fa, O, torch_gpu, in_bf16, out_bf16):
    """Records 64-byte aligned in the receipts and the reply (as fa_aggregator's frames hold them): all
    pieces of the phase in one segment launch -- bit-exact, f32 / bf16 in and out."""
    D, n = 3, 50_536
    es, eo = (2 if in_bf16 else 4), (2 if out_bf16 else 4)
    xs = [O.gen(0xA11, k, n, dtype="bf16" if in_bf16 else "f32") for k in range(D)]
    w = O.weights(D)
    cuts = [2400, 2416, 50_416]  # LeNet-5 part 1's records: 2400 / 16 / 48 000 / 120 elements
    def aligned_layout(es_):
        segs, off, edges = [], 0, [0] + cuts + [n]
        for a, b in zip(edges, edges[1:]):
            off = (off + 63) // 64 * 64
            segs.append((off, b - a))
            off += (b - a) * es_
        return segs, off
    with fa.Aggregator(1) as agg:
        agg.define(1, n, fa.BF16 if in_bf16 else fa.F32, fa.BF16 if out_bf16 else fa.F32, D, fa.FEDAVG)
        keep = []
        for k in range(D):
            segs, total = aligned_layout(es)
            buf, views = place(fa, xs[k], segs, total)
            keep.append(buf)
            agg.submit_gather(1, k, views, w[k], pinned=True)
        dsegs, dtotal = aligned_layout(eo)
        dbuf, dviews = dst_views(fa, n, eo, dsegs, dtotal)
        agg.finalize_gather(1, dviews, pinned=True)
        assert agg.host_reads() == 1
        got = gathered(dviews, np.uint16 if out_bf16 else np.float32)
        want = expected(O, xs, w, in_bf16, out_bf16)
        assert np.array_equal(got.view(np.uint16 if out_bf16 else np.uint32),
                              want.view(np.uint16 if out_bf16 else np.uint32))


def test_literal_last_receipt_in_place(fa, O, torch_gpu):
    n, D = 10_164, 3
    xs = [O.gen(0x1234, k, n) for k in range(D)]
    with fa.Aggregator(1) as agg:
        agg.define(2, n, fa.F32, fa.F32, D, fa.LITERAL)
        keep = []
        for k in (2, 0, 1):  # the last submitted is slot 1
            buf, views = place(fa, xs[k], [(0, n)], n * 4, shift=12)
            keep.append(buf)
            agg.submit_gather(2, k, views, 1.0, pinned=True)
        dbuf, dviews = dst_views(fa, n, 4, [(20, n)], 20 + n * 4)
        agg.finalize_gather(2, dviews, pinned=True)
        assert agg.host_reads() == 1
        assert np.array_equal(gathered(dviews, np.float32).view(np.uint32), O.literal(xs[1]).view(np.uint32))


def test_kept_receipts_into_output_then_copy(fa, O, torch_gpu):
    """A pageable destination: the kept receipts are reduced in place into the part's output, which the usual
    copy-out returns.  fa_reduce_parts before the finalize (and fa_copy_output after it) take the plain path:
    the kept receipts go to their slots first, since the caller keeps them only until the finalize."""
    D = 2
    sizes = {1: 50_536, 2: 10_164, 3: 850}
    xs = {mp: [O.gen(0x77 + mp, k, n) for k in range(D)] for mp, n in sizes.items()}
    w = O.weights(D)
    with fa.Aggregator(1) as agg:
        keep = []
        for mp, n in sizes.items():
            agg.define(mp, n, fa.F32, fa.F32, D, fa.FEDAVG)
            for k in range(D):
                segs, total = layout(n, 4, [n // 2], [4, 64], None)
                buf, views = place(fa, xs[mp][k], segs, total, shift=4)
                keep.append(buf)
                agg.submit_gather(mp, k, views, w[k], pinned=True)
        out1 = agg.finalize(1)  # pageable destination
        assert agg.host_reads() == 1
        agg.reduce_parts([2, 3])  # the batched phase 2: the kept receipts are copied in, one batched launch
        assert agg.host_reads() == 1
        out2 = agg.copy_output(2)
        dbuf, dviews = dst_views(fa, sizes[3], 4, [(0, sizes[3])], sizes[3] * 4)
        agg.finalize_gather(3, dviews, pinned=True)
        assert agg.host_reads() == 1  # phase 2 was already reduced: the finalize only copies
        out3 = gathered(dviews, np.float32)
        for mp, got in ((1, out1), (2, out2), (3, out3)):
            assert np.array_equal(got.view(np.uint32), O.fedavg(xs[mp], w).view(np.uint32)), mp


def test_host_read_query_and_no_stale_copy_output(fa, O, torch_gpu):
    """fa_bucket_host_read says whether a part's round is kept to be read in place (the drop-in's phase 2 asks
    it before batching); and once a round was reduced straight into a pinned reply, the part's
    device output was not written, so fa_copy_output refuses (FA_ERR_STATE) rather than return the previous
    round's result."""
    n, D = 10_164, 2
    w = O.weights(D)
    with fa.Aggregator(1) as agg:
        agg.define(2, n, fa.F32, fa.F32, D, fa.FEDAVG)
        # round 0 the plain way (pageable receipts): a device output exists afterwards
        xs0 = [O.gen(0x10, k, n) for k in range(D)]
        for k in range(D):
            agg.submit(2, k, xs0[k], w[k])
        assert not agg.host_read_kept(2)
        agg.finalize(2)
        assert np.array_equal(agg.copy_output(2).view(np.uint32), O.fedavg(xs0, w).view(np.uint32))
        # round 1: pinned receipts kept in place, reduced straight into the pinned reply
        xs1 = [O.gen(0x11, k, n) for k in range(D)]
        keep = []
        for k in range(D):
            assert not agg.host_read_kept(2)  # not every receipt yet
            buf, views = place(fa, xs1[k], [(0, n)], n * 4)
            keep.append(buf)
            agg.submit_gather(2, k, views, w[k], pinned=True)
        assert agg.host_read_kept(2)
        dbuf, dviews = dst_views(fa, n, 4, [(0, n)], n * 4)
        agg.finalize_gather(2, dviews, pinned=True)
        assert agg.host_reads() == 1
        assert np.array_equal(gathered(dviews, np.float32).view(np.uint32), O.fedavg(xs1, w).view(np.uint32))
        with pytest.raises(fa.FaError) as e:
            agg.copy_output(2)
        assert e.value.code == fa.ERR_STATE
        # a device reduction afterwards gives it an output again
        for k in range(D):
            agg.submit(2, k, xs1[k], w[k])
        agg.reduce(2)
        assert np.array_equal(agg.copy_output(2).view(np.uint32), O.fedavg(xs1, w).view(np.uint32))


@pytest.mark.parametrize("case", ["pageable_mix", "misaligned", "over_limit", "sync", "slot_read", "replaced"])
def test_paths_that_copy_kept_receipts_in(fa, O, torch_gpu, case):
    """Where the in-place read must not (or cannot) run, the kept receipts go to their slots first and the
    result is the plain path's: a pageable receipt beside kept ones, a source not element-aligned, a bucket
    over the 1 MiB limit, the in-place state sync, a caller reading a slot; and a receipt replaced by a
    second kept one (the second wins)."""
    D = 3
    n = 150_000 if case == "over_limit" else 4_099
    xs = [O.gen(0x99, k, n) for k in range(D)]
    w = O.weights(D)
    with fa.Aggregator(1) as agg:
        agg.define(1, n, fa.F32, fa.F32, D, fa.FEDAVG)
        keep = []
        for k in range(D):
            if case == "pageable_mix" and k == 1:
                agg.submit(1, k, xs[k], w[k])
                continue
            shift = 2 if case == "misaligned" and k == 2 else 8
            if case == "replaced" and k == 0:
                junk = O.gen(0xBAD, 0, n)
                buf, views = place(fa, junk, [(0, n)], n * 4, shift=shift)
                keep.append(buf)
                agg.submit_gather(1, k, views, w[k], pinned=True)
            buf, views = place(fa, xs[k], [(0, n)], n * 4, shift=shift)
            keep.append(buf)
            agg.submit_gather(1, k, views, w[k], pinned=True)
        want = O.fedavg(xs, w)
        if case == "sync":
            agg.sync_states(1, w)
            agg.sync()
            slot0 = agg.slot(1, 0, 0)[0]
            got = np.empty(n, np.float32)
            import ctypes
            hip = ctypes.CDLL("libamdhip64.so.7")
            assert hip.hipMemcpy(ctypes.c_void_p(got.ctypes.data), ctypes.c_void_p(slot0), ctypes.c_size_t(n * 4), 2) == 0
            assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
            assert agg.host_reads() == 0
            return
        if case == "slot_read":
            import ctypes
            hip = ctypes.CDLL("libamdhip64.so.7")
            ptr = agg.slot(1, 0, 1)[0]  # asking for a slot copies the kept receipts in
            agg.sync()
            got = np.empty(n, np.float32)
            assert hip.hipMemcpy(ctypes.c_void_p(got.ctypes.data), ctypes.c_void_p(ptr), ctypes.c_size_t(n * 4), 2) == 0
            assert np.array_equal(got.view(np.uint32), xs[1].view(np.uint32))  # the receipt is in its slot
        dbuf, dviews = dst_views(fa, n, 4, [(4, n)], n * 4 + 4)
        agg.finalize_gather(1, dviews, pinned=True)
        assert np.array_equal(gathered(dviews, np.float32).view(np.uint32), want.view(np.uint32))
        in_place = case == "replaced"
        assert agg.host_reads() == (1 if in_place else 0), case


_OFF_CHILD = r"""
import json, sys
import numpy as np
import torch
sys.path.insert(0, %(tests)r)
sys.path.insert(0, %(oracle)r)
from conftest import load_pkg
import oracle as O
fa = load_pkg()
fa.lib()
n, D = 50_536, 2
xs = [O.gen(5, k, n) for k in range(D)]
w = O.weights(D)
bufs = []
with fa.Aggregator(1) as agg:
    agg.define(1, n, fa.F32, fa.F32, D, fa.FEDAVG)
    for k in range(D):
        b = fa.PinnedBuffer(n * 4)
        b.view(np.float32)[:] = xs[k]
        bufs.append(b)
        agg.submit_gather(1, k, [b.view(np.uint8)], w[k], pinned=True)
    d = fa.PinnedBuffer(n * 4)
    agg.finalize_gather(1, [d.view(np.uint8)], pinned=True)
    print(json.dumps({"exact": bool(np.array_equal(d.view(np.uint32), O.fedavg(xs, w).view(np.uint32))),
                      "host_reads": agg.host_reads()}))
"""


def test_host_read_off_switch(fa, torch_gpu):
    """FA_HOST_READ=0 (read once per process): the plain DMA path, same bits."""
    from test_gpu_parity import _child
    r = _child(_OFF_CHILD, env={"FA_HOST_READ": "0"})
    assert r == {"exact": True, "host_reads": 0}
    r = _child(_OFF_CHILD)
    assert r == {"exact": True, "host_reads": 1}
