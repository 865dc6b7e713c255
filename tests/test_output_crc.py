"""GPU: fa_output_crc32 -- the CRC-32 of a reply's zip records computed from the reduced bucket in HBM.

The drop-in aggregator seals every reply record with its CRC-32 (torch::save's zip, which the data owner's
torch::load checks, data_owner.cpp:232-253).  The record bytes are the part's device output, so
fa_output_crc32 computes the CRCs there (256-byte chunks per lane, shifted into place in GF(2), XOR-joined;
csrc/fa_kernels.hip crc32_pieces_kernel).  Every case compares with zlib's crc32 over the same bytes read
back with fa_copy_output: random byte segments (odd lengths, empty ones, one byte), f32 and bf16 outputs,
range shards and the client-sharded rs layout (runs split across GPUs, rehearsed as shards of one GPU), a
multi-hundred-MB bucket, and the state rule (no device output after a round read in place into a pinned
reply).
"""
import zlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _ctx(fa, G, **kw):
    if G == 1:
        return fa.Aggregator(1, **kw)
    if fa.device_count() >= G:
        return fa.Aggregator(G, **kw)
    return fa.Aggregator(devices=[0] * G, shared_device=True, **kw)


def _reduced(fa, O, agg, n, D, out_bf16=False, seed=0x77):
    agg.define(1, n, fa.F32, fa.BF16 if out_bf16 else fa.F32, D, fa.FEDAVG)
    w = O.weights(D)
    for k in range(D):
        agg.submit(1, k, O.gen(seed, k, n), w[k])
    agg.reduce(1)
    agg.sync()
    return agg.copy_output(1)


def _segments(total, rng, k):
    cuts = np.sort(rng.integers(0, total + 1, k - 1)) if k > 1 else np.array([], np.int64)
    edges = np.concatenate([[0], cuts, [total]]).astype(np.int64)
    return [int(b - a) for a, b in zip(edges[:-1], edges[1:])]


def _check(agg, got_bytes, seg):
    crcs = agg.output_crc32(1, seg)
    o = 0
    for c, L in zip(crcs, seg):
        assert c == zlib.crc32(got_bytes[o:o + L]) & 0xFFFFFFFF, (o, L)
        o += L


@pytest.mark.parametrize("G,rs,n,out_bf16", [(1, False, 1_000_003, False), (1, False, 77_777, True),
                                             (3, False, 2_000_011, False), (2, True, 500_000, False),
                                             (4, True, 300_001, True)])
def test_output_crc32_matches_zlib(fa, O, torch_gpu, G, rs, n, out_bf16):
    rng = np.random.default_rng(n)
    with _ctx(fa, G, rs=rs) as agg:
        got = _reduced(fa, O, agg, n, 5, out_bf16)
        raw = got.tobytes()
        for k in (1, 2, 17, 300):  # one segment = the whole bucket; random byte cuts, empty segments possible
            _check(agg, raw, _segments(len(raw), rng, k))
        # segments on element boundaries (what a reply's parameter records are), with tiny and 1-byte ones
        es = 2 if out_bf16 else 4
        seg = [1, 3, 0, es * 7, 255, 256, 257] + [es * int(x) for x in rng.integers(1, n // 20, 10)]
        seg.append(len(raw) - sum(seg))
        assert seg[-1] >= 0
        _check(agg, raw, seg)


def test_output_crc32_large_bucket(fa, O, torch_gpu):
    """A VGG-FC-sized bucket (119.6 M fp32 = 478 MB, the C4 reply's FC record) in its real record split."""
    n = 119_586_826
    with fa.Aggregator(1) as agg:
        agg.define(1, n, fa.F32, fa.F32, 2, fa.FEDAVG)
        for k in range(2):
            ptr, cnt, _ = agg.slot(1, 0, k)
            fa.fill_uniform(ptr, cnt, fa.F32, 0x5EED, k)
        agg.reduce(1, np.array([0.25, 0.75], np.float32))
        agg.sync()
        raw = agg.copy_output(1).tobytes()
        seg = [4 * x for x in (102_760_448, 4096, 16_777_216, 4096, 40_960, 10)]  # VGG-19's FC layers
        assert sum(seg) == len(raw)
        _check(agg, raw, seg)


def test_output_crc32_state_and_arguments(fa, O, torch_gpu):
    n, D = 10_164, 2
    w = O.weights(D)
    with fa.Aggregator(1) as agg:
        agg.define(1, n, fa.F32, fa.F32, D, fa.FEDAVG)
        with pytest.raises(fa.FaError) as e:  # never reduced
            agg.output_crc32(1, [4 * n])
        assert e.value.code == fa.ERR_STATE
        # a round read in place straight into a pinned reply leaves no device output
        keep = []
        for k in range(D):
            buf = fa.PinnedBuffer(4 * n)
            buf.view(np.float32, count=n)[:] = O.gen(0x42, k, n)
            keep.append(buf)
            agg.submit(1, k, buf.view(np.uint8, count=4 * n), w[k], pinned=True)
        out = fa.PinnedBuffer(4 * n)
        agg.finalize_gather(1, [out.view(np.uint8, count=4 * n)], pinned=True)
        assert agg.host_reads() == 1
        with pytest.raises(fa.FaError) as e:
            agg.output_crc32(1, [4 * n])
        assert e.value.code == fa.ERR_STATE
        for k in range(D):
            agg.submit(1, k, O.gen(0x42, k, n), w[k])
        agg.reduce(1)
        raw = agg.copy_output(1).tobytes()
        _check(agg, raw, [4 * n])
        with pytest.raises(fa.FaError) as e:  # the segments must cover the output exactly
            agg.output_crc32(1, [4 * n - 4])
        assert e.value.code == fa.ERR_ARG
