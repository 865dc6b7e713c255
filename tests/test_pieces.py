"""GPU: range-layout pieces (fa_api.hip piece_len_for; DESIGN.md 4, "the address span").  A GPU whose client
slots would span more than 48 GiB holds them piece-major -- piece j of every slot, then piece j+1 -- and
reduces one launch per piece, so that each launch's clients lie within 16 GiB.  The shapes that trigger it
(C5: 128 GiB) are checked by tests/test_c5_shape.py; here fa_tuning.piece_split_kib = -1 / piece_span_kib force pieces on
small buckets so that every round shape runs over them against the oracle, bit-exact: host receipts (staged
and pinned copies cut at piece boundaries), device-resident fills through fa_bucket_piece, accumulate on
arrival, bf16, literal mode, the state sync, fa_reduce_parts with a pieced part, two range shards.  The
reduction replaced is aggregator.cpp:59-93 / :112-150.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def assert_bits(got, ref):
    ut = np.uint16 if got.dtype == np.uint16 else np.uint32
    bad = np.flatnonzero(got.view(ut) != ref.view(ut))
    assert bad.size == 0, "%d/%d mismatches, first at %s: got %s ref %s" % (
        bad.size, got.size, bad[:4], got[bad[:4]], ref[bad[:4]])


@pytest.fixture
def pieces_env(monkeypatch):
    """Every range part defined inside the test is cut into pieces of <= 256 KiB of slots."""
    from conftest import load_pkg
    fa = load_pkg()
    before = fa.get_tuning()
    fa.set_tuning(piece_split_kib=-1, piece_span_kib=256)  # the process defaults new contexts start from
    yield
    fa.set_tuning(piece_split_kib=before["piece_split_kib"], piece_span_kib=before["piece_span_kib"])


def ctx_for(fa, G, **kw):
    if G == 1:
        return fa.Aggregator(1, **kw)
    if fa.device_count() >= G:
        return fa.Aggregator(G, **kw)
    return fa.Aggregator(devices=[0] * G, shared_device=True, **kw)


def d2h(ptr, n):
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    out = np.empty(n, np.float32)
    assert hip.hipMemcpy(ctypes.c_void_p(out.ctypes.data), ctypes.c_void_p(ptr), ctypes.c_size_t(4 * n), 2) == 0
    return out


@pytest.mark.parametrize("G", [1, 2])
@pytest.mark.parametrize("pinned", [False, True])
def test_pieced_host_rounds(fa, O, torch_gpu, pieces_env, G, pinned):
    n, D = 100_003, 5
    w = O.weights(D)
    xs = [O.gen(300, k, n) for k in range(D)]
    with ctx_for(fa, G) as agg:
        agg.define(1, n, fa.F32, fa.F32, D, fa.FEDAVG)
        for g in range(G):
            pcs = agg.pieces(1, g, 0)
            assert len(pcs) > 1, pcs
            assert pcs[0][2] + sum(c for _, c, _ in pcs) == pcs[-1][2] + pcs[-1][1]  # contiguous, in order
            with pytest.raises(fa.FaError) as e:
                agg.slot(1, g, 0)
            assert e.value.code == fa.ERR_STATE
        bufs = []
        for k in reversed(range(D)):
            if pinned:
                b = fa.PinnedBuffer(4 * n)
                b.view(np.float32)[:] = xs[k]
                bufs.append(b)
                agg.submit(1, k, b.view(np.float32), w[k], pinned=True)
            else:
                agg.submit(1, k, xs[k], w[k])
        assert_bits(agg.finalize(1), O.fedavg(xs, w))
        for b in bufs:
            b.close()


def test_pieced_device_resident_bf16_literal(fa, O, torch_gpu, pieces_env):
    torch = torch_gpu
    n, D = 333_335, 6
    w = O.weights(D)
    with fa.Aggregator(1) as agg:
        for pid, dt, out, mode in ((1, fa.F32, fa.F32, fa.FEDAVG), (2, fa.BF16, fa.BF16, fa.FEDAVG),
                                   (3, fa.F32, fa.BF16, fa.FEDAVG), (4, fa.F32, fa.F32, fa.LITERAL)):
            agg.define(pid, n, dt, out, D, mode)
            for k in range(D):
                pcs = agg.pieces(pid, 0, k)
                assert len(pcs) > 1
                for ptr, cnt, off in pcs:
                    fa.fill_uniform(ptr, cnt, dt, 310 + pid, k, idx0=off)
        torch.cuda.synchronize()
        xs = {pid: [O.gen(310 + pid, k, n, dtype="bf16" if pid == 2 else "f32") for k in range(D)] for pid in (1, 2, 3, 4)}
        agg.reduce(1, w)
        assert_bits(agg.copy_output(1), O.fedavg(xs[1], w))
        agg.reduce(2, w)
        assert_bits(agg.copy_output(2), O.fedavg(xs[2], w, out_dtype="bf16"))
        agg.reduce(3, w)
        assert_bits(agg.copy_output(3), O.f32_to_bf16(O.fedavg(xs[3], w)))
        agg.reduce(4)
        assert_bits(agg.copy_output(4), O.literal(xs[4][-1]))


@pytest.mark.parametrize("G", [1, 2])
def test_pieced_accumulate_on_arrival(fa, O, torch_gpu, pieces_env, G):
    n, D = 200_001, 6
    w = O.weights(D)
    xs = [O.gen(320, k, n) for k in range(D)]
    with ctx_for(fa, G, eager=True) as agg:
        agg.define(1, n, fa.F32, fa.F32, D, fa.FEDAVG)
        assert len(agg.pieces(1, 0, 0)) > 1
        reduced = []
        for k in [1, 0, 3, 2, 5, 4]:
            agg.submit(1, k, xs[k], w[k])
            reduced.append(agg.progress(1)[1])
        assert reduced == [0, 2, 2, 4, 4, 6]
        assert_bits(agg.finalize(1), O.fedavg(xs, w))


def test_pieced_state_sync_and_reduce_parts(fa, O, torch_gpu, pieces_env):
    n, D = 150_007, 5
    w = O.weights(D)
    xs = [O.gen(330, k, n) for k in range(D)]
    ref = O.fedavg(xs, w)
    with fa.Aggregator(1) as agg:
        agg.define(1, n, fa.F32, fa.F32, D, fa.FEDAVG)
        for k in range(D):
            agg.submit(1, k, xs[k], w[k])
        agg.sync_states(1)
        agg.sync()
        for k in (0, D - 1):
            got = np.concatenate([d2h(ptr, cnt) for ptr, cnt, _ in agg.pieces(1, 0, k)])
            assert_bits(got, ref)
        # a batch with a pieced part (its own launches) beside parts small enough to stay whole
        agg.define(2, n, fa.F32, fa.F32, D, fa.FEDAVG)
        agg.define(3, 5_000, fa.F32, fa.F32, D, fa.FEDAVG)
        agg.define(4, 64, fa.F32, fa.F32, D, fa.FEDAVG)
        assert len(agg.pieces(2, 0, 0)) > 1 and len(agg.pieces(3, 0, 0)) == 1
        refs = {}
        for pid, m in ((2, n), (3, 5_000), (4, 64)):
            ys = [O.gen(340 + pid, k, m) for k in range(D)]
            refs[pid] = O.fedavg(ys, w)
            for k in range(D):
                agg.submit(pid, k, ys[k], w[k])
        agg.reduce_parts([2, 3, 4])
        for pid in refs:
            assert agg.progress(pid)[1] == D
            assert_bits(agg.finalize(pid), refs[pid])
