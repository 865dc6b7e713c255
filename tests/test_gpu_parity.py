"""GPU parity: libfa.so kernels vs the oracle (bit-exact) through the C ABI.

Inputs are produced on the device by fa_fill_uniform and on the host by the
oracle's generator (the two are checked equal first), so both sides reduce the
same bytes.  Small and ragged sizes are compared whole; the reference configs
(tests/golden) are compared at full size against the reference-generated
fixtures (file or SHA-256 + sampled bits); the north-star size is checked by
sampled elements plus a split-chain consistency property.
"""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, ROOT

pytestmark = pytest.mark.gpu


def to_np(t, bf16):
    a = t.cpu().numpy()
    return a.view(np.uint16) if bf16 else a


def dev_buf(torch, n, bf16, offset=0):
    """Device buffer of n elements starting `offset` elements into a fresh allocation."""
    base = torch.empty(n + 16, dtype=torch.int16 if bf16 else torch.float32, device="cuda")
    return base[offset:offset + n]


def filled(fa, torch, n, bf16, seed, client, offset=0):
    t = dev_buf(torch, n, bf16, offset)
    fa.fill_uniform(t, n, fa.BF16 if bf16 else fa.F32, seed, client)
    return t


def run_fedavg(fa, torch, clients, w, n, bf16_in, bf16_out, init=None, out_offset=0):
    out = dev_buf(torch, n, bf16_out, out_offset)
    fa.reduce_device(clients, w, n, fa.BF16 if bf16_in else fa.F32, out, fa.BF16 if bf16_out else fa.F32,
                     fa.FEDAVG, init=init)
    torch.cuda.synchronize()
    return to_np(out, bf16_out)


def host_clients(O, seed, D, n, bf16):
    xs = [O.gen(seed, k, n) for k in range(D)]
    return [O.f32_to_bf16(x) for x in xs] if bf16 else xs


def assert_bits(got, ref):
    ut = np.uint16 if got.dtype == np.uint16 else np.uint32
    bad = np.flatnonzero(got.view(ut) != ref.view(ut))
    assert bad.size == 0, "%d/%d mismatches, first at %s: got %s ref %s" % (
        bad.size, got.size, bad[:4], got[bad[:4]], ref[bad[:4]])


@pytest.mark.parametrize("bf16", [False, True])
def test_fill_matches_oracle_generator(fa, O, torch_gpu, bf16):
    torch = torch_gpu
    for n, client, idx0 in [(1, 0, 0), (4099, 5, 17), (1 << 20, 31, 1 << 33)]:
        t = dev_buf(torch, n, bf16)
        fa.fill_uniform(t, n, fa.BF16 if bf16 else fa.F32, 0x5EED, client, idx0)
        assert_bits(to_np(t, bf16), O.gen(0x5EED, client, n, idx0=idx0, dtype="bf16" if bf16 else "f32"))


@pytest.mark.parametrize("D", [1, 2, 3, 8, 33, 64, 65, 130])
def test_fedavg_f32_bitexact(fa, O, torch_gpu, D):
    torch = torch_gpu
    w = O.weights(D)
    for n in [1, 3, 5, 64, 1000, 4097, 262147]:
        xs = host_clients(O, 100 + n, D, n, False)
        clients = [filled(fa, torch, n, False, 100 + n, k) for k in range(D)]
        assert_bits(run_fedavg(fa, torch, clients, w, n, False, False), O.fedavg(xs, w))


@pytest.mark.parametrize("unroll", [4, 8, 16])
def test_fedavg_every_tail_width(fa, O, torch_gpu, unroll):
    """Every remainder of D modulo the unroll (the grouped chain tail: 0..U-1 clients after the full
    groups, in groups of up to 8), f32 and bf16, bit-exact."""
    torch = torch_gpu
    before = fa.get_tuning()
    try:
        fa.set_tuning(unroll=unroll)
        n = 4099
        for D in list(range(1, 2 * unroll + 2)) + [47]:
            w = O.weights(D)
            for bf16 in (False, True):
                xs = host_clients(O, 300 + D, D, n, bf16)
                clients = [filled(fa, torch, n, bf16, 300 + D, k) for k in range(D)]
                assert_bits(run_fedavg(fa, torch, clients, w, n, bf16, False), O.fedavg(xs, w))
    finally:
        fa.set_tuning(unroll=before["unroll"])


PHASE_ELEMS = 256 * 256 * 72 * 4  # one phase of walk 4 on a 256-CU MI355X (f32 and bf16 alike); walk 5: x 88/72


@pytest.mark.parametrize("in_bf16,out_bf16,D,phases,offset,use_init", [
    (False, False, 32, 2.3, 0, False),   # north-star shape, partial last phase
    (False, False, 3, 1.0, 1, False),    # exactly one phase (+ a misaligned head and a scalar tail)
    (True, True, 5, 1.6, 0, False),
    (True, False, 2, 1.2, 3, False),
    (False, True, 4, 1.1, 0, False),
    (False, False, 130, 1.05, 0, False),  # two passes: the second continues the chain (INIT)
    (False, False, 6, 1.4, 0, True),     # d_init given by the caller
    (False, False, 7, 1.25, 2, False),   # just over one phase of walk 5
    (True, True, 32, 2.5, 0, False),     # bf16 -> bf16: two phases of bf16 LDS rows (33.5 M elements each)
])
def test_phased_walk_same_bits(fa, O, torch_gpu, in_bf16, out_bf16, D, phases, offset, use_init):
    """The phased kernel (walk 4: persistent grid, reads and writes separated in time) against the
    one-shot XCD walk on the same device inputs, full buckets compared bit for bit, at sizes that
    make whole phases, a partial last phase and a wave chunk that crosses the end of the bucket;
    plus sampled elements against the oracle."""
    torch = torch_gpu
    n = int(PHASE_ELEMS * phases) + 12_345 + offset
    w = O.weights(D)
    seed = 900 + D
    clients = [filled(fa, torch, n, in_bf16, seed, k, offset=offset) for k in range(D)]
    init = None
    if use_init:
        init = dev_buf(torch, n, False, offset)
        fa.fill_uniform(init, n, fa.F32, seed, 999)
    before = fa.get_tuning()
    outs = {}
    try:
        for walk in (2, 4, 5, 6):
            fa.set_tuning(walk=walk)
            out = dev_buf(torch, n, out_bf16, offset)
            ctx = fa.Aggregator(1) if (out_bf16 and D > 128) else None
            fa.reduce_device(clients, w, n, fa.BF16 if in_bf16 else fa.F32, out, fa.BF16 if out_bf16 else fa.F32,
                             fa.FEDAVG, init=init, ctx=ctx)
            torch.cuda.synchronize()
            outs[walk] = out
    finally:
        fa.set_tuning(walk=before["walk"])
    dt = torch.int16 if out_bf16 else torch.int32
    for walk in (4, 5, 6):
        assert torch.equal(outs[2].view(dt), outs[walk].view(dt)), "phased walk %d differs from walk 2" % walk
    # sampled elements against the oracle (f32 in, no init: the oracle's closed form)
    if not in_bf16 and not use_init:
        rng = np.random.default_rng(D)
        idx = np.unique(np.concatenate([[0, 1, 2, n - 3, n - 2, n - 1], rng.integers(0, n, 1024)]))
        got = outs[4][torch.as_tensor(idx, device="cuda")].cpu().numpy()
        ref = O.fedavg_at(seed, w, idx)
        if out_bf16:
            assert_bits(got.view(np.uint16), O.f32_to_bf16(ref))
        else:
            assert_bits(got, ref)
    del clients


LANES_F32, LANES_BF16 = 256 * 256, 256 * 512  # phased grid lanes (256 CUs): f32 256-thread, bf16 512-thread


@pytest.mark.parametrize("in_bf16,D,q,frac,out_bf16", [
    # buckets below one phase, D >= 16: one phase sized to the bucket, q vectors per lane
    (False, 16, 9, 0.3, False), (False, 16, 20, 0.9, False), (False, 20, 26, 0.5, False),
    (False, 16, 40, 0.1, False), (False, 32, 64, 0.0, False), (False, 17, 87, 0.7, False),
    (True, 16, 5, 0.5, False), (True, 16, 9, 0.2, False), (True, 18, 20, 0.9, False),
    # several phases whose last one is balanced: q_last in (RL, RR) -> registers only, > RR -> both
    (False, 32, 88 + 44, 0.5, False), (False, 16, 88 * 2 + 70, 0.3, False), (True, 16, 22 + 15, 0.4, False),
    # bf16 outputs: LDS rows hold bf16 (bf16 -> bf16: RL 20 + RR 12 per phase; f32 -> bf16: RL 80 + RR 48)
    (True, 16, 30, 0.3, True), (True, 32, 32 + 20, 0.4, True), (True, 16, 11, 0.6, True),
    (False, 16, 100, 0.5, True), (False, 16, 128 + 30, 0.2, True),
])
def test_sized_phase_same_bits(fa, O, torch_gpu, in_bf16, D, q, frac, out_bf16):
    """Phases sized to the bucket (launch_phased_sized) and the balanced last phase (phased_rl_last)
    against the one-shot walk on the same device inputs, whole buckets bit for bit, plus sampled
    elements against the oracle.  n = q vectors per lane minus a fraction of one lane-vector row, so
    the last register chunk crosses the end of the bucket."""
    torch = torch_gpu
    lanes, V = (LANES_BF16, 8) if in_bf16 else (LANES_F32, 4)
    n = q * lanes * V - int(frac * lanes * V) - 3
    w = O.weights(D)
    seed = 1300 + q
    clients = [filled(fa, torch, n, in_bf16, seed, k) for k in range(D)]
    before = fa.get_tuning()
    outs = {}
    try:
        for walk in (2, 5):
            fa.set_tuning(walk=walk)
            out = dev_buf(torch, n, out_bf16)
            fa.reduce_device(clients, w, n, fa.BF16 if in_bf16 else fa.F32, out, fa.BF16 if out_bf16 else fa.F32,
                             fa.FEDAVG)
            torch.cuda.synchronize()
            outs[walk] = out
    finally:
        fa.set_tuning(walk=before["walk"])
    dt = torch.int16 if out_bf16 else torch.int32
    assert torch.equal(outs[2].view(dt), outs[5].view(dt))
    if not in_bf16:
        rng = np.random.default_rng(q)
        idx = np.unique(np.concatenate([[0, n - 1], rng.integers(0, n, 512)]))
        ref = O.fedavg_at(seed, w, idx)
        got = outs[5][torch.as_tensor(idx, device="cuda")].cpu().numpy()
        if out_bf16:
            assert_bits(got.view(np.uint16), O.f32_to_bf16(ref))
        else:
            assert_bits(got, ref)
    del clients


def test_fedavg_zero_elements_is_noop(fa, O, torch_gpu):
    torch = torch_gpu
    c = [dev_buf(torch, 4, False)]
    fa.reduce_device(c, [1.0], 0, fa.F32, dev_buf(torch, 4, False), fa.F32)
    torch.cuda.synchronize()


@pytest.mark.parametrize("offsets", [(1, 1, 1, 1), (2, 2, 2, 2), (3, 3, 3, 3), (0, 1, 2, 3), (3, 0, 0, 1)])
def test_fedavg_misaligned_pointers(fa, O, torch_gpu, offsets):
    """Same 16-B phase -> vector body + scalar head; mixed phases -> general path. Same bits either way."""
    torch = torch_gpu
    n, D = 100_003, len(offsets) - 1
    w = O.weights(D)
    xs = host_clients(O, 77, D, n, False)
    clients = [filled(fa, torch, n, False, 77, k, offset=offsets[k]) for k in range(D)]
    assert_bits(run_fedavg(fa, torch, clients, w, n, False, False, out_offset=offsets[-1]), O.fedavg(xs, w))


def test_fedavg_init_continues_the_chain(fa, O, torch_gpu):
    """Clients split over two launches with d_init == one ordered chain (used for multi-GPU chains)."""
    torch = torch_gpu
    n, D = 300_001, 10
    w = O.weights(D)
    xs = host_clients(O, 5, D, n, False)
    clients = [filled(fa, torch, n, False, 5, k) for k in range(D)]
    acc = dev_buf(torch, n, False)
    fa.reduce_device(clients[:4], w[:4], n, fa.F32, acc, fa.F32)
    out = run_fedavg(fa, torch, clients[4:], w[4:], n, False, False, init=acc)
    assert_bits(out, O.fedavg(xs, w))


@pytest.mark.parametrize("n", [300_001, int(PHASE_ELEMS * 1.3) + 7])  # one-shot and phased kernels
def test_fedavg_init_in_place(fa, O, torch_gpu, n):
    """d_init and the output may be the same buffer (shard.reduce_chain continues a rank's chain in
    place): every lane reads its init elements before it writes them.  Same bits as a separate output,
    and as the oracle on sampled elements."""
    torch = torch_gpu
    D = 10
    w = O.weights(D)
    clients = [filled(fa, torch, n, False, 6, k) for k in range(D)]
    acc = dev_buf(torch, n, False)
    fa.reduce_device(clients[:4], w[:4], n, fa.F32, acc, fa.F32)
    sep = dev_buf(torch, n, False)
    fa.reduce_device(clients[4:], w[4:], n, fa.F32, sep, fa.F32, fa.FEDAVG, init=acc)
    fa.reduce_device(clients[4:], w[4:], n, fa.F32, acc, fa.F32, fa.FEDAVG, init=acc)
    torch.cuda.synchronize()
    assert torch.equal(acc.view(torch.int32), sep.view(torch.int32))
    idx = np.unique(np.concatenate([[0, 1, n - 2, n - 1], np.random.default_rng(n).integers(0, n, 1024)]))
    assert_bits(acc[torch.as_tensor(idx, device="cuda")].cpu().numpy(), O.fedavg_at(6, w, idx))


@pytest.mark.parametrize("out_bf16", [False, True])
@pytest.mark.parametrize("D", [1, 7, 32, 70, 130])
def test_fedavg_bf16_inputs(fa, O, torch_gpu, D, out_bf16):
    torch = torch_gpu
    n = 100_003
    w = O.weights(D)
    xs = host_clients(O, 9, D, n, True)
    clients = [filled(fa, torch, n, True, 9, k) for k in range(D)]
    ref = O.fedavg(xs, w, out_dtype="bf16" if out_bf16 else "f32")
    if out_bf16 and D > 128:
        ctx = fa.Aggregator(1)  # bf16 output across passes needs ctx scratch
        out = dev_buf(torch, n, True)
        fa.reduce_device(clients, w, n, fa.BF16, out, fa.BF16, ctx=ctx)
        torch.cuda.synchronize()
        assert_bits(to_np(out, True), ref)
        ctx.close()
    else:
        assert_bits(run_fedavg(fa, torch, clients, w, n, True, out_bf16), ref)


def test_fedavg_f32_in_bf16_out(fa, O, torch_gpu):
    torch = torch_gpu
    n, D = 65_537, 6
    w = O.weights(D)
    xs = host_clients(O, 3, D, n, False)
    clients = [filled(fa, torch, n, False, 3, k) for k in range(D)]
    ref = O.f32_to_bf16(O.fedavg(xs, w))
    assert_bits(run_fedavg(fa, torch, clients, w, n, False, True), ref)


@pytest.mark.parametrize("bf16", [False, True])
def test_literal_mode(fa, O, torch_gpu, bf16):
    """aggregator.cpp:63-88 semantics: only the last client survives, fl(fl(2x)/1000)."""
    torch = torch_gpu
    n, D = 70_001, 4
    xs = host_clients(O, 21, D, n, bf16)
    clients = [filled(fa, torch, n, bf16, 21, k, offset=1) for k in range(D)]
    for out_bf16 in ([False, True] if bf16 else [False]):
        out = dev_buf(torch, n, out_bf16, offset=1)
        fa.reduce_device(clients, np.zeros(D), n, fa.BF16 if bf16 else fa.F32, out,
                         fa.BF16 if out_bf16 else fa.F32, fa.LITERAL)
        torch.cuda.synchronize()
        assert_bits(to_np(out, out_bf16), O.literal(xs[-1], out_dtype="bf16" if out_bf16 else "f32"))


@pytest.mark.parametrize("tuning", [dict(block=64, unroll=4, load_policy=1, store_policy=1),
                                    dict(block=128, unroll=16, load_policy=2, store_policy=2),
                                    dict(block=256, unroll=8, load_policy=1, store_policy=3, max_blocks=7),
                                    dict(block=256, unroll=16, load_policy=2, store_policy=4, max_blocks=1),
                                    dict(block=128, unroll=8, load_policy=2, store_policy=3, max_blocks=-1),
                                    dict(block=64, unroll=16, load_policy=1, store_policy=4, max_blocks=5),
                                    dict(block=128, unroll=16, load_policy=2, store_policy=3, max_blocks=-1, walk=2),
                                    dict(block=256, unroll=8, load_policy=2, store_policy=3, max_blocks=-1, walk=3),
                                    dict(block=64, unroll=4, load_policy=1, store_policy=2, max_blocks=9, walk=3)])
def test_tuning_variants_same_bits(fa, O, torch_gpu, tuning):
    torch = torch_gpu
    before = fa.get_tuning()
    try:
        fa.set_tuning(**tuning)
        for n, D, bf16, bf16_out in [(200_003, 19, False, False), (1_048_573, 33, False, False), (3001, 3, False, False),
                                     (250_001, 21, True, True), (250_001, 21, True, False), (99_999, 5, False, True)]:
            w = O.weights(D)
            xs = host_clients(O, 8, D, n, bf16)
            clients = [filled(fa, torch, n, bf16, 8, k) for k in range(D)]
            if bf16_out and not bf16:  # f32 inputs, bf16 output: one rounding of the fp32 chain
                ref = O.f32_to_bf16(O.fedavg(xs, w))
            else:
                ref = O.fedavg(xs, w, out_dtype="bf16" if bf16_out else "f32")
            assert_bits(run_fedavg(fa, torch, clients, w, n, bf16, bf16_out), ref)
    finally:
        restore = dict(before)
        restore["max_blocks"] = restore["max_blocks"] or -1
        restore["slot_skew"] = restore["slot_skew"] or -1
        fa.set_tuning(**restore)


# ----------------------------------------------------------------- reference golden configs, full size

CONFIGS = ["lenet5_c1", "resnet18_c2", "resnet101_c3", "vgg19_c4"]


def check_golden(cfg, rec, got):
    if "file" in rec:
        ref = np.fromfile(os.path.join(GOLDEN, cfg, rec["file"]), dtype=got.dtype)
        assert_bits(got, ref)
    else:
        idx = np.asarray(rec["sample_idx"])
        bits = got.view(np.uint32 if got.dtype == np.float32 else np.uint16)[idx]
        assert np.array_equal(bits, np.asarray(rec["sample_bits"], bits.dtype))
        assert hashlib.sha256(got.tobytes()).hexdigest() == rec["sha256"]


@pytest.mark.parametrize("cfg", CONFIGS)
def test_reference_golden_on_gpu(fa, O, torch_gpu, cfg):
    torch = torch_gpu
    with open(os.path.join(GOLDEN, cfg, "manifest.json")) as f:
        m = json.load(f)
    D = m["D"]
    w = O.weights(D)
    for b in m["buckets"]:
        n, s = b["numel"], b["bucket_seed"]
        cf = [filled(fa, torch, n, False, s, k) for k in range(D)]
        check_golden(cfg, b["outputs"]["fedavg.f32"], run_fedavg(fa, torch, cf, w, n, False, False))
        out = dev_buf(torch, n, False)
        fa.reduce_device(cf, w, n, fa.F32, out, fa.F32, fa.LITERAL)
        torch.cuda.synchronize()
        check_golden(cfg, b["outputs"]["literal.f32"], to_np(out, False))
        del cf
        cb = [filled(fa, torch, n, True, s, k) for k in range(D)]
        check_golden(cfg, b["outputs"]["fedavg_bf16.bf16"], run_fedavg(fa, torch, cb, w, n, True, True))
        check_golden(cfg, b["outputs"]["fedavg_bf16.f32"], run_fedavg(fa, torch, cb, w, n, True, False))
        del cb


def test_north_star_size_sampled_and_split_consistent(fa, O, torch_gpu):
    """256 MiB fp32 x 32 clients: sampled elements vs the oracle, and a split chain == one chain."""
    torch = torch_gpu
    n, D = 64 << 20, 32
    w = O.weights(D)
    clients = [filled(fa, torch, n, False, 0x5EED, k) for k in range(D)]
    out = dev_buf(torch, n, False)
    fa.reduce_device(clients, w, n, fa.F32, out, fa.F32)
    acc = dev_buf(torch, n, False)
    fa.reduce_device(clients[:13], w[:13], n, fa.F32, acc, fa.F32)
    fa.reduce_device(clients[13:], w[13:], n, fa.F32, acc, fa.F32, init=acc)
    torch.cuda.synchronize()
    assert torch.equal(out.view(torch.int32), acc.view(torch.int32))
    rng = np.random.default_rng(0)
    idx = np.unique(np.concatenate([[0, 1, 2, 3, n - 4, n - 3, n - 2, n - 1], rng.integers(0, n, 2048)]))
    got = out[torch.as_tensor(idx, device="cuda")].cpu().numpy()
    assert_bits(got, O.fedavg_at(0x5EED, w, idx))


# ----------------------------------------------------------------- aggregation context (host buckets)

def test_context_fedavg_out_of_order_submits(fa, O, torch_gpu):
    n, D = 1_000_003, 5
    w = O.weights(D)
    xs = host_clients(O, 44, D, n, False)
    with fa.Aggregator(1) as agg:
        agg.define(2, n, fa.F32, fa.F32, D, fa.FEDAVG)
        for k in [3, 0, 4, 1, 2]:
            agg.submit(2, k, xs[k], w[k])
        assert_bits(agg.finalize(2), O.fedavg(xs, w))
        # next round reuses the bucket
        xs2 = host_clients(O, 45, D, n, False)
        for k in range(D):
            agg.submit(2, k, xs2[k], w[k])
        assert_bits(agg.finalize(2), O.fedavg(xs2, w))


def test_context_literal_takes_last_submitted(fa, O, torch_gpu):
    n, D = 50_000, 3
    xs = host_clients(O, 46, D, n, False)
    with fa.Aggregator(1) as agg:
        agg.define(1, n, fa.F32, fa.F32, D, fa.LITERAL)
        for k in [2, 0, 1]:
            agg.submit(1, k, xs[k])
        assert_bits(agg.finalize(1), O.literal(xs[1]))
        agg.set_divisor(7.0, part_id=1)
        agg.submit(1, 2, xs[2])
        assert_bits(agg.finalize(1), O.literal(xs[2], divisor=7.0))


def test_context_large_bucket_multi_chunk_and_bf16(fa, O, torch_gpu):
    n, D = 20_000_001, 3  # 80 MB per client: several pinned staging chunks
    w = O.weights(D)
    xs = host_clients(O, 47, D, n, True)
    with fa.Aggregator(1) as agg:
        agg.define(1, n, fa.BF16, fa.BF16, D, fa.FEDAVG)
        for k in range(D):
            agg.submit(1, k, xs[k], w[k])
        assert_bits(agg.finalize(1), O.fedavg(xs, w, out_dtype="bf16", threads=8))


def test_context_pinned_submit(fa, O, torch_gpu):
    torch = torch_gpu
    n, D = 333_333, 4
    w = O.weights(D)
    xs = host_clients(O, 48, D, n, False)
    pinned = [torch.empty(n, dtype=torch.float32, pin_memory=True) for _ in range(D)]
    for p, x in zip(pinned, xs):
        p.numpy()[:] = x
    with fa.Aggregator(1) as agg:
        agg.define(1, n, fa.F32, fa.F32, D, fa.FEDAVG)
        for k in range(D):
            agg.submit(1, k, pinned[k].numpy(), w[k], pinned=True)
        assert_bits(agg.finalize(1), O.fedavg(xs, w))


def test_context_errors(fa, O, torch_gpu):
    with fa.Aggregator(1) as agg:
        agg.define(1, 1000, fa.F32, fa.F32, 3, fa.FEDAVG)
        agg.submit(1, 0, np.zeros(1000, np.float32), 0.5)
        with pytest.raises(fa.FaError) as e:
            agg.finalize(1)
        assert e.value.code == fa.ERR_STATE
        with pytest.raises(fa.FaError) as e:
            agg.submit(1, 3, np.zeros(1000, np.float32), 0.5)
        assert e.value.code == fa.ERR_ARG
        with pytest.raises(fa.FaError):
            agg.finalize(9)


def multi_gpu_ctx(fa, G, **kw):
    """A G-GPU context: real GPUs when visible, else G shards of one context on GPU 0 (test-only
    FA_TEST_SHARED_DEVICE), so the multi-GPU host logic (ranges, per-GPU staging, split gather/scatter,
    per-GPU done events) runs on the one-GPU box."""
    if fa.device_count() >= G:
        return fa.Aggregator(G, **kw)
    return fa.Aggregator(devices=[0] * G, shared_device=True, **kw)


@pytest.mark.parametrize("G", [2, 3])
def test_context_multi_gpu_range_shards(fa, O, torch_gpu, G):
    n, D = 1_000_001, 4
    w = O.weights(D)
    xs = host_clients(O, 49, D, n, False)
    with multi_gpu_ctx(fa, G) as agg:
        agg.define(1, n, fa.F32, fa.F32, D, fa.FEDAVG)
        for k in range(D):
            agg.submit(1, k, xs[k], w[k])
        assert_bits(agg.finalize(1), O.fedavg(xs, w))


def test_device_resident_part_round(fa, O, torch_gpu):
    """fa_bucket_slot + fa_reduce_part + fa_copy_output: receipts written straight into the pooled slots."""
    n, D = 777_777, 6
    w = O.weights(D)
    xs = host_clients(O, 50, D, n, False)
    with fa.Aggregator(1) as agg:
        agg.define(3, n, fa.F32, fa.F32, D, fa.FEDAVG)
        ptrs = []
        for k in range(D):
            ptr, cnt, off = agg.slot(3, 0, k)
            assert (cnt, off) == (n, 0) and ptr % 16 == 0
            ptrs.append(ptr)
            fa.fill_uniform(ptr, cnt, fa.F32, 50, k)
        gaps = {b - a for a, b in zip(ptrs, ptrs[1:])}
        skew = fa.get_tuning()["slot_skew"]
        assert len(gaps) == 1 and gaps.pop() % 4096 == (2048 if skew == -2 else skew % 4096)
        agg.reduce(3, w)
        assert_bits(agg.copy_output(3), O.fedavg(xs, w))
        # literal mode on the same layout: the last slot when nothing was submitted
        agg.define(4, n, fa.F32, fa.F32, D, fa.LITERAL)
        for k in range(D):
            fa.fill_uniform(agg.slot(4, 0, k)[0], n, fa.F32, 50, k)
        agg.reduce(4)
        assert_bits(agg.copy_output(4), O.literal(xs[-1]))


def test_slot_skew_by_slot_size(fa, torch_gpu):
    """The default skew (-2) is 2048 B below 48 MiB slots and 512 B from 48 MiB up (fa_api.hip
    slot_skew_for); an explicit skew applies at every size."""
    assert fa.get_tuning()["slot_skew"] == -2
    with fa.Aggregator(1) as agg:
        for part, n, want in ((1, (48 << 20) // 4 - 1024, 2048), (2, (48 << 20) // 4, 512), (3, (48 << 20) // 2, 512)):
            dt = fa.BF16 if part == 3 else fa.F32
            agg.define(part, n, dt, dt, 3, fa.FEDAVG)
            p = [agg.slot(part, 0, k)[0] for k in range(3)]
            assert p[1] - p[0] == p[2] - p[1] == (48 << 20) - (4096 if part == 1 else 0) + want
    before = fa.get_tuning()
    try:
        fa.set_tuning(slot_skew=2048)
        with fa.Aggregator(1) as agg:
            agg.define(1, (64 << 20) // 4, fa.F32, fa.F32, 2, fa.FEDAVG)
            assert agg.slot(1, 0, 1)[0] - agg.slot(1, 0, 0)[0] == (64 << 20) + 2048
    finally:
        fa.set_tuning(slot_skew=before["slot_skew"] or -1)


@pytest.mark.parametrize("skew", [-1, -2, 256, 512, 4096 + 512])
def test_slot_skew_does_not_change_bits(fa, O, torch_gpu, skew):
    before = fa.get_tuning()
    try:
        fa.set_tuning(slot_skew=skew)
        n, D = 300_007, 9
        w = O.weights(D)
        xs = host_clients(O, 51, D, n, False)
        with fa.Aggregator(1) as agg:
            agg.define(1, n, fa.F32, fa.F32, D, fa.FEDAVG)
            for k in range(D):
                agg.submit(1, k, xs[k], w[k])
            assert_bits(agg.finalize(1), O.fedavg(xs, w))
    finally:
        fa.set_tuning(slot_skew=before["slot_skew"] or -1)


def test_context_submit_gather_matches_flat(fa, O, torch_gpu):
    """fa_submit_gather: a receipt split into ragged pieces (archive records) == the flat submit."""
    n, D = 2_000_003, 3
    w = O.weights(D)
    xs = host_clients(O, 52, D, n, False)
    cuts = [0, 1, 7, 1000, 65_536, 1_234_567, n]
    with fa.Aggregator(1) as agg:
        agg.define(1, n, fa.F32, fa.F32, D, fa.FEDAVG)
        for k in range(D):
            agg.submit_gather(1, k, [xs[k][a:b] for a, b in zip(cuts, cuts[1:])], w[k])
        assert_bits(agg.finalize(1), O.fedavg(xs, w))
        with pytest.raises(fa.FaError):
            agg.submit_gather(1, 0, [xs[0][:10]], w[0])  # wrong total size


@pytest.mark.parametrize("gpus", [1, 2])
@pytest.mark.parametrize("pinned", [False, True])
def test_context_zero_copy_gather_in_and_out(fa, O, torch_gpu, pinned, gpus):
    """fa_submit_gather_pinned + fa_finalize_gather: receipts as ragged records at odd byte offsets of one
    pinned frame buffer (how the network layer hands them over), the result scattered into the records
    of a reply buffer; == the flat path, bit for bit.  gpus=2 splits the ranges across record pieces
    (two shards on one GPU when only one is visible)."""
    n, D = 3_000_017, 3
    w = O.weights(D)
    xs = host_clients(O, 53, D, n, False)
    cuts = [0, 5, 4096, 777_777, 2_000_000, n]
    hdr = 13  # the archive starts after a text header: records are not 16-byte aligned in host memory
    frames = [fa.PinnedBuffer(hdr + 4 * n + 64 * len(cuts)) for _ in range(D)] if pinned else None
    pieces = []
    for k in range(D):
        raw = frames[k].view() if pinned else np.empty(hdr + 4 * n + 64 * len(cuts), np.uint8)
        ps, off = [], hdr
        for a, b in zip(cuts, cuts[1:]):
            seg = raw[off:off + 4 * (b - a)]
            seg[:] = xs[k][a:b].view(np.uint8)
            ps.append(seg)
            off += 4 * (b - a) + 64 - (4 * (b - a)) % 64 + 3
        pieces.append(ps)
    reply = fa.PinnedBuffer(4 * n + 100) if pinned else None
    rraw = reply.view() if pinned else np.zeros(4 * n + 100, np.uint8)
    out_cuts = [0, 1, 333_333, n]
    outs = [rraw[7 + 4 * a: 7 + 4 * b] for a, b in zip(out_cuts, out_cuts[1:])]
    with multi_gpu_ctx(fa, gpus) as agg:
        agg.define(1, n, fa.F32, fa.F32, D, fa.FEDAVG)
        for k in range(D):
            agg.submit_gather(1, k, pieces[k], w[k], pinned=pinned)
        agg.finalize_gather(1, outs, pinned=pinned)
        got = np.concatenate([o.view(np.float32) if o.ctypes.data % 4 == 0 else o.copy().view(np.float32)
                              for o in outs])
        assert_bits(got, O.fedavg(xs, w))
        assert not rraw[:7].any()  # nothing written outside the pieces
        with pytest.raises(fa.FaError):
            agg.finalize_gather(1, outs[:1], pinned=pinned)  # nothing submitted / wrong size
    for f in frames or []:
        f.close()
    if reply:
        reply.close()


# ----------------------------------------------------------------- IEEE special values

def _special_clients(D, n, seed):
    """Client buckets mixing ordinary values with +-0, +-Inf, NaNs, subnormals and values whose
    weighted sums land in the subnormal range or overflow (a diverged or a vanishing parameter)."""
    rng = np.random.default_rng(seed)
    specials = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 1e-45, -1e-45, 1.1754942e-38, 1e-39, -3e-39,
                         1.17549435e-38, 3.4e38, -3.4e38, 1e-30, 1e30], np.float32)
    xs = []
    for k in range(D):
        x = rng.uniform(-1, 1, n).astype(np.float32)
        pick = rng.random(n) < 0.3
        x[pick] = specials[rng.integers(0, specials.size, int(pick.sum()))]
        xs.append(x)
    return xs


def _assert_bits_nan_aware(got, ref):
    """Bit-exact, except that a NaN only has to be a NaN (x86 and CDNA FMAs may pick different NaN payloads)."""
    gn, rn = np.isnan(got), np.isnan(ref)
    assert np.array_equal(gn, rn), "NaN positions differ: %d vs %d" % (gn.sum(), rn.sum())
    assert_bits(got[~gn], ref[~rn])


@pytest.mark.parametrize("D", [3, 17])
def test_special_values_fedavg_and_literal(fa, O, torch_gpu, D):
    torch = torch_gpu
    n = 50_003
    xs = _special_clients(D, n, 41 + D)
    for w in (O.weights(D), np.array([1e-30 if k % 2 else 0.75 for k in range(D)], np.float32)):
        ref = O.fedavg(xs, w)
        clients = [torch.from_numpy(x).to("cuda") for x in xs]
        out = torch.empty(n, dtype=torch.float32, device="cuda")
        fa.reduce_device(clients, w, n, fa.F32, out, fa.F32)
        torch.cuda.synchronize()
        _assert_bits_nan_aware(out.cpu().numpy(), ref)
        # bf16 output of the same chain (one rounding at the end)
        outb = torch.empty(n, dtype=torch.int16, device="cuda")
        fa.reduce_device(clients, w, n, fa.F32, outb, fa.BF16)
        torch.cuda.synchronize()
        gb = outb.cpu().numpy().view(np.uint16)
        rb = O.f32_to_bf16(ref)
        nan_b = ((gb & 0x7FFF) > 0x7F80)
        assert np.array_equal(nan_b, (rb & 0x7FFF) > 0x7F80)
        assert np.array_equal(gb[~nan_b], rb[~nan_b])
    lit = torch.empty(n, dtype=torch.float32, device="cuda")
    fa.reduce_device(clients, np.zeros(D, np.float32), n, fa.F32, lit, fa.F32, fa.LITERAL)
    torch.cuda.synchronize()
    _assert_bits_nan_aware(lit.cpu().numpy(), O.literal(xs[-1]))


# ----------------------------------------------------------------- beyond 2^31 / 2^32 elements

def _big_idx(n, rng):
    edges = [0, 1, 2, 3, (1 << 31) - 1, 1 << 31, (1 << 31) + 1, (1 << 32) - 1, 1 << 32, (1 << 32) + 1,
             n - 5, n - 4, n - 3, n - 2, n - 1]
    return np.unique(np.array([i for i in edges if 0 <= i < n] + list(rng.integers(0, n, 2048)), np.int64))


@pytest.mark.parametrize("in_bf16,n,D,walk", [
    (False, (1 << 31) + 1027, 3, 5),   # 8 GiB per client, 94 phases of the phased kernel
    (False, (1 << 31) + 1027, 3, 2),   # the one-shot kernel over the same bucket
    (True, (1 << 32) + 4099, 2, 5),    # bf16: element offsets past 2^32, byte offsets past 2^33
])
def test_buckets_past_32bit_indices(fa, O, torch_gpu, in_bf16, n, D, walk):
    """Maximum-size buckets: element indices past 2^31 / 2^32 reduce like the small ones (sampled vs the
    oracle), literal mode at the same size, and the in-place state sync."""
    torch = torch_gpu
    before = fa.get_tuning()
    clients = []
    try:
        fa.set_tuning(walk=walk)
        w = O.weights(D)
        dt = fa.BF16 if in_bf16 else fa.F32
        clients = [filled(fa, torch, n, in_bf16, 0x5EED, k) for k in range(D)]
        idx = _big_idx(n, np.random.default_rng(n))
        tidx = torch.as_tensor(idx, device="cuda")
        ref = O.fedavg_at(0x5EED, w, idx, bf16=in_bf16)
        ref = O.f32_to_bf16(ref) if in_bf16 else ref
        out = torch.empty(n, dtype=torch.int16 if in_bf16 else torch.float32, device="cuda")
        fa.reduce_device(clients, w, n, dt, out, dt)
        torch.cuda.synchronize()
        got = out[tidx].cpu().numpy()
        assert_bits(got.view(np.uint16) if in_bf16 else got, ref)
        # literal mode of the last client, into the same output
        fa.reduce_device(clients, np.zeros(D, np.float32), n, dt, out, dt, fa.LITERAL)
        torch.cuda.synchronize()
        last = O.gen_at(0x5EED, D - 1, idx)
        if in_bf16:
            assert_bits(out[tidx].cpu().numpy().view(np.uint16), O.literal(O.f32_to_bf16(last), out_dtype="bf16"))
        else:
            assert_bits(out[tidx].cpu().numpy(), O.literal(last))
        del out
        # compute-node sync in place: every slot becomes the chain, rounded to the slot dtype
        fa.sync_device(clients, w, n, dt)
        torch.cuda.synchronize()
        for k in (0, D - 1):
            got = clients[k][tidx].cpu().numpy()
            assert_bits(got.view(np.uint16) if in_bf16 else got, ref)
    finally:
        fa.set_tuning(walk=before["walk"])
        clients = None
        torch.cuda.empty_cache()


# Run in a fresh child process, so that which counter slot a stream gets does not depend on what earlier tests
# left: the first 48 streams that launch the phased kernel in a process own a slot each (until their context is
# destroyed), later ones share the 16 hashed slots (fa_kernels.hip, PhasedDevice::slot_of).
_SHARED_SLOT_CHILD = r"""
import json, sys
import numpy as np
import torch
sys.path.insert(0, %(tests)r)
sys.path.insert(0, %(oracle)r)
from conftest import load_pkg
import oracle as O
fa = load_pkg()
fa.lib()
fa.set_tuning(walk=5)
n, D = 30_000_005, 4  # 1.3 phases of the default f32 form: a meeting, so both streams count on the slot
assert fa.plan_chain(fa.F32, fa.F32, n, D)[0] == fa.PLAN_PHASED
assert fa.phased_owned_slots(0) == 0
w = O.weights(D)
sets = []
for s in range(2):
    clients = []
    for k in range(D):
        t = torch.empty(n, dtype=torch.float32, device="cuda")
        fa.fill_uniform(t, n, fa.F32, 0x5EED + s, k)
        clients.append(t)
    sets.append((clients, torch.empty(n, dtype=torch.float32, device="cuda")))
# distinct HIP streams: torch.cuda.Stream() hands out its pool's 32 streams round-robin, so it cannot give 65
import ctypes
hip = ctypes.CDLL("libamdhip64.so.7")  # the runtime torch already loaded


def new_stream():
    p = ctypes.c_void_p()
    assert hip.hipStreamCreateWithFlags(ctypes.byref(p), 1) == 0  # hipStreamNonBlocking
    return torch.cuda.ExternalStream(p.value)


streams, hashed, pair = [], {}, None
while pair is None:  # 48 owned, then pigeonhole: two of 17 more streams share one of the 16 hashed slots
    st = new_stream()
    streams.append(st)
    slot, own = fa.phased_slot(st)
    assert own == (len(streams) <= 48) and (slot < 48) == own, (len(streams), slot, own)
    if not own:
        if slot in hashed:
            pair = (hashed[slot], st)
        hashed[slot] = st
    assert len(streams) <= 48 + 17
assert fa.phased_owned_slots(0) == 48 and fa.phased_slot(pair[0]) == fa.phased_slot(pair[1])
ref = []
for clients, out in sets:  # each set alone, on an owned stream
    with torch.cuda.stream(streams[0]):
        fa.reduce_device(clients, w, n, fa.F32, out, fa.F32, stream=streams[0])
    torch.cuda.synchronize()
    ref.append(out.clone())
idx = np.unique(np.concatenate([[0, n - 1], np.random.default_rng(1).integers(0, n, 1024)]))
for s in range(2):  # the lone results against the oracle
    assert np.array_equal(ref[s].cpu().numpy()[idx].view(np.uint32),
                          O.sampled_chain(0x5EED + s, w, idx)[0].view(np.uint32))

def median_ms(st):
    evs = []
    clients, out = sets[0]
    for _ in range(7):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        fa.reduce_device(clients, w, n, fa.F32, out, fa.F32, stream=st)
        b.record(st)
        evs.append((a, b))
    torch.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in evs[2:]]))

t0 = median_ms(pair[0])
for _ in range(6):  # overlapping launches of the two sets on the two streams that share the slot
    for k in range(2):
        clients, out = sets[k]
        with torch.cuda.stream(pair[k]):
            out.zero_()
        fa.reduce_device(clients, w, n, fa.F32, out, fa.F32, stream=pair[k])
torch.cuda.synchronize()
same = [bool(torch.equal(sets[k][1].view(torch.int32), ref[k].view(torch.int32))) for k in range(2)]
t1, t2 = median_ms(pair[0]), median_ms(pair[1])
same_after = bool(torch.equal(sets[0][1].view(torch.int32), ref[0].view(torch.int32)))
print(json.dumps({"same": same, "same_after": same_after, "t0": t0, "t1": t1, "t2": t2, "streams": len(streams),
                  "timeouts": fa.phased_timeouts(0)}))
"""


def _child(script, timeout=180, env=None):
    import subprocess
    import sys
    r = subprocess.run([sys.executable, "-c", script % {"tests": os.path.join(ROOT, "tests"),
                                                        "oracle": os.path.join(ROOT, "oracle")}],
                       capture_output=True, text=True, timeout=timeout, env=dict(os.environ, **(env or {})))
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_phased_streams_sharing_a_counter(fa, torch_gpu):
    """Two streams forced onto one hashed counter slot (a fresh process: 48 streams take the owned slots, then
    two of the next 17 share one of the 16 hashed ones), launched so they overlap: both results stay bit-exact
    with each set reduced alone (itself checked against the oracle), and later launches on either stream stay
    bit-exact.  The launch times before and after (t0 / t1 / t2: a skewed counter would show as slower later
    launches) are reported, not asserted: a noisy neighbour must not fail a parity test."""
    r = _child(_SHARED_SLOT_CHILD)
    assert r["same"] == [True, True], r
    assert r["same_after"], r
    print("shared counter slot: t0 %.3f ms, after the overlapped launches t1 %.3f / t2 %.3f ms" %
          (r["t0"], r["t1"], r["t2"]))
    assert r["streams"] <= 65


_RELEASE_CHILD = r"""
import json, sys
import numpy as np
import torch
sys.path.insert(0, %(tests)r)
from conftest import load_pkg
fa = load_pkg()
fa.lib()
n, D = 4 << 20, 16  # below one phase with 16 clients: one sized phase of the phased kernel
assert fa.plan_chain(fa.F32, fa.F32, n, D)[0] == fa.PLAN_PHASED
w = np.full(D, 1.0 / D, np.float32)
counts = []
for i in range(60):  # more contexts than owned slots
    with fa.Aggregator(1) as agg:
        agg.define(1, n, fa.F32, fa.F32, D, fa.FEDAVG)
        for k in range(D):
            fa.fill_uniform(agg.slot(1, 0, k)[0], n, fa.F32, 0x5EED, k)
        agg.reduce(1, w)  # on the context's compute stream: it takes an owned slot
        agg.sync()
        during = fa.phased_owned_slots(0)
    counts.append((during, fa.phased_owned_slots(0)))
import ctypes
p = ctypes.c_void_p()
assert ctypes.CDLL("libamdhip64.so.7").hipStreamCreateWithFlags(ctypes.byref(p), 1) == 0  # a new HIP stream
print(json.dumps({"counts": counts, "fresh_stream_owns": fa.phased_slot(p.value)[1]}))
"""


def test_destroyed_context_releases_its_counter_slot(fa, torch_gpu):
    """fa_destroy gives its streams' owned counter slots back: 60 contexts one after another each hold one
    owned slot while alive and none after, so a stream created after them still gets a slot of its own."""
    r = _child(_RELEASE_CHILD)
    assert all(c == [1, 0] for c in r["counts"]), r["counts"]
    assert r["fresh_stream_owns"]


_CALLER_STREAM_CHILD = r"""
import ctypes, gc, json, sys
import numpy as np
import torch
sys.path.insert(0, %(tests)r)
sys.path.insert(0, %(oracle)r)
from conftest import load_pkg
import oracle as O
fa = load_pkg()
fa.lib()
n, D = 4 << 20, 16  # below one phase with 16 clients: one sized phase of the phased kernel
assert fa.plan_chain(fa.F32, fa.F32, n, D)[0] == fa.PLAN_PHASED
w = O.weights(D)
clients = []
for k in range(D):
    t = torch.empty(n, dtype=torch.float32, device="cuda")
    fa.fill_uniform(t, n, fa.F32, 0x5EED, k)
    clients.append(t)
out = torch.empty(n, dtype=torch.float32, device="cuda")
hip = ctypes.CDLL("libamdhip64.so.7")  # the runtime torch already loaded
idx = np.unique(np.concatenate([[0, n - 1], np.random.default_rng(3).integers(0, n, 512)]))
want = O.sampled_chain(0x5EED, w, idx)[0].view(np.uint32)
base = fa.phased_owned_slots(0)
owned, exact, during, after = [], [], [], []
for i in range(60):  # more caller streams than owned slots, one after another
    p = ctypes.c_void_p()
    assert hip.hipStreamCreateWithFlags(ctypes.byref(p), 1) == 0
    out.zero_()
    torch.cuda.synchronize()
    fa.reduce_device(clients, w, n, fa.F32, out, fa.F32, stream=p.value)  # its first phased launch takes a slot
    assert hip.hipStreamSynchronize(p) == 0
    owned.append(fa.phased_slot(p.value)[1])
    during.append(fa.phased_owned_slots(0) - base)
    exact.append(bool(np.array_equal(out.cpu().numpy()[idx].view(np.uint32), want)))
    fa.release_stream(p.value, 0)
    after.append(fa.phased_owned_slots(0) - base)
    assert hip.hipStreamDestroy(p) == 0
# torch stream objects are released when collected (the binding tracks what it was handed)
for i in range(60):
    st = torch.cuda.Stream()
    fa.reduce_device(clients, w, n, fa.F32, out, fa.F32, stream=st)
    st.synchronize()
    during.append(fa.phased_owned_slots(0) - base)
    del st
    gc.collect()
    after.append(fa.phased_owned_slots(0) - base)
print(json.dumps({"owned": owned, "exact": exact, "during": during, "after": after,
                  "bad_device": fa.lib().fa_release_stream(999, None)}))
"""


def test_caller_streams_release_their_counter_slots(fa, torch_gpu):
    """fa_release_stream: 60 raw caller streams one after another, each launching one phased reduction (its
    first launch takes an owned counter slot) and releasing it before hipStreamDestroy -- every one of them gets
    an owned slot (48 would be the limit without the release) and a bit-exact result against the oracle; then
    60 torch.cuda.Stream objects, whose slots the binding gives back when they are collected."""
    r = _child(_CALLER_STREAM_CHILD)
    assert all(r["owned"]) and len(r["owned"]) == 60, r["owned"]
    assert all(r["exact"]), r["exact"]
    assert all(d == 1 for d in r["during"]), str(r["during"])
    assert all(a == 0 for a in r["after"]), str(r["after"])
    assert r["bad_device"] == fa.ERR_ARG


_TIMELINE_CHILD = r"""
import ctypes, json, sys
import numpy as np
import torch
sys.path.insert(0, %(tests)r)
from conftest import load_pkg
fa = load_pkg()
fa.lib()
n, D = 30_000_005, 4
assert fa.plan_chain(fa.F32, fa.F32, n, D)[0] == fa.PLAN_PHASED
clients = [torch.zeros(n, dtype=torch.float32, device="cuda:0") for _ in range(D)]
out = torch.empty(n, dtype=torch.float32, device="cuda:0")
fa.reduce_device(clients, np.full(D, 0.25, np.float32), n, fa.F32, out, fa.F32)  # enqueued, not synchronized
buf = (ctypes.c_ulonglong * 4096)()
L = fa.lib()
got = L.fa_diag_phased_timeline(0, buf, 4096)  # synchronizes device 0 itself before the copy
starts = [buf[8 * i] for i in range(max(0, got) // 8)]
print(json.dumps({"words": got, "stamped": sum(1 for x in starts if x), "none": L.fa_diag_phased_timeline(63, buf, 8)}))
"""


def test_phased_timeline_reads_its_own_device(fa, torch_gpu):
    """fa_diag_phased_timeline (FA_TIMELINE=1, tools/timeline.py) synchronizes and copies on the device it is
    asked about, not the caller's current one: right after an enqueued phased launch on device 0 every
    workgroup's start stamp is there (8 words per CU); a device that never ran one reports 0 words."""
    r = _child(_TIMELINE_CHILD, env={"FA_TIMELINE": "1"})
    assert r["words"] > 0 and r["words"] % 8 == 0 and r["stamped"] == r["words"] // 8, r
    assert r["none"] == 0


def test_phased_meeting_timeouts_counter(fa, O, torch_gpu):
    """fa_phased_timeouts: on a quiet GPU a phased launch never runs out of its bounded wait (the grid is
    co-resident), so the counter does not move; the call itself synchronizes and reads the device table."""
    torch = torch_gpu
    n, D = int(PHASE_ELEMS * 1.2), 16
    w = O.weights(D)
    clients = [filled(fa, torch, n, False, 77, k) for k in range(D)]
    out = dev_buf(torch, n, False)
    before = fa.phased_timeouts(0)
    for _ in range(3):
        fa.reduce_device(clients, w, n, fa.F32, out, fa.F32)
    torch.cuda.synchronize()
    assert fa.phased_timeouts(0) == before
    assert fa.phased_timeouts(63) == 0  # a device that never ran a phased launch


def test_phased_graph_replays(fa, O, torch_gpu):
    """A phased launch captured in a graph and replayed: each replay is one epoch of the counter ring,
    results stay bit-exact, and eager launches afterwards stay bit-exact too.  Their speed before and after is
    reported, not asserted (a noisy neighbour must not fail a parity test)."""
    torch = torch_gpu
    n, D = 30_000_005, 3
    w = O.weights(D)
    clients = [filled(fa, torch, n, False, 0x5EED, k) for k in range(D)]
    out = torch.empty(n, dtype=torch.float32, device="cuda")
    st = torch.cuda.Stream()

    def eager_ms():
        evs = []
        for _ in range(6):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(st)
            fa.reduce_device(clients, w, n, fa.F32, out, fa.F32, stream=st)
            b.record(st)
            evs.append((a, b))
        torch.cuda.synchronize()
        return float(np.median([a.elapsed_time(b) for a, b in evs[1:]]))

    t0 = eager_ms()
    ref = out.clone()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=st):
        fa.reduce_device(clients, w, n, fa.F32, out, fa.F32, stream=torch.cuda.current_stream())
    for _ in range(11):  # more replays than ring entries
        out.zero_()
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(out.view(torch.int32), ref.view(torch.int32))
    out.zero_()
    t1 = eager_ms()
    assert torch.equal(out.view(torch.int32), ref.view(torch.int32))
    print("graph replays: eager launch %.3f ms before, %.3f ms after" % (t0, t1))


@pytest.mark.parametrize("n,D", [(1_000_000, 8), (4_000_000, 16), (2_000_000, 20), (16_000_000, 16),
                                 (int(PHASE_ELEMS * 88 / 72 * 1.5), 6)])
def test_read_stream_probe_reads_only(fa, O, torch_gpu, n, D):
    """fa_diag_read_stream (bench's roofline.read_stream_peak): the simple probe below one phase with few
    clients, the phased kernel with its output stream switched off where an f32 chain takes it (a sized
    phase below one phase from 16 clients: register stage + LDS, and LDS only; full phases above); it writes
    nothing -- every client buffer keeps its bits and the kernel's output pointer stays null (put() returns
    before any store)."""
    torch = torch_gpu
    clients = [filled(fa, torch, n, False, 55, k) for k in range(D)]
    before = [c.clone() for c in clients]
    s = torch.cuda.Stream()
    for _ in range(2):
        fa.diag_read_stream(clients, n, stream=s)
    s.synchronize()
    for a, b in zip(clients, before):
        assert torch.equal(a.view(torch.int32), b.view(torch.int32))
    with pytest.raises(fa.FaError):
        fa.diag_read_stream(clients, n + 1, stream=s)  # not a multiple of 4


@pytest.mark.parametrize("n,D,grid,unroll,nt", [(1_000_000, 8, 2048, 8, False), (4_000_004, 3, 8192, 16, True),
                                                (12, 2, 16384, 16, False), (2_000_000, 20, 4096, 16, True)])
def test_rw_plain_probe_leaves_values(fa, O, torch_gpu, n, D, grid, unroll, nt):
    """fa_diag_rw_plain (the sync legs' copy_ceiling_independent): every slot is read and written back where
    it lies, x * 1 -- every client buffer keeps its bits (full strides, the strided tail and a buffer smaller
    than one stride), so the bench's sync parity check after it sees the slots as they were."""
    torch = torch_gpu
    clients = [filled(fa, torch, n, False, 57, k) for k in range(D)]
    before = [c.clone() for c in clients]
    s = torch.cuda.Stream()
    for _ in range(2):
        fa.diag_rw_plain(clients, n, grid=grid, unroll=unroll, nt=nt, stream=s)
    s.synchronize()
    for a, b in zip(clients, before):
        assert torch.equal(a.view(torch.int32), b.view(torch.int32))
    with pytest.raises(fa.FaError):
        fa.diag_rw_plain(clients, n, grid=grid, unroll=12, stream=s)  # unroll 8 or 16 only


def test_context_misuse(fa, O, torch_gpu):
    """Misuse of a context is an error code, never a wrong result: gather pieces that do not add up to
    the bucket, a slot out of range, a finalize into pieces of the wrong total; redefining a bucket
    replaces it (new size, new client count) and the next round is bit-exact; a receipt submitted
    twice counts once (the later one replaces it, as a retransmitted owner would)."""
    n, D = 10_007, 3
    w = O.weights(D)
    xs = host_clients(O, 81, D, n, False)
    with fa.Aggregator(1) as agg:
        agg.define(1, n, fa.F32, fa.F32, D, fa.FEDAVG)
        with pytest.raises(fa.FaError) as e:
            agg.submit_gather(1, 0, [xs[0][:100], xs[0][100:-1]], w[0])  # one element short
        assert e.value.code == fa.ERR_ARG
        with pytest.raises(fa.FaError):
            agg.submit(1, -1, xs[0], w[0])
        junk = np.full(n, 7.0, np.float32)
        agg.submit(1, 1, junk, 0.25)      # replaced below
        for k in range(D):
            agg.submit(1, k, xs[k], w[k])
        with pytest.raises(fa.FaError) as e:
            agg.finalize_gather(1, [np.empty(n - 1, np.float32)])
        assert e.value.code == fa.ERR_ARG
        assert_bits(agg.finalize(1), O.fedavg(xs, w))
        # redefine: more elements and clients, then a full round
        n2, D2 = 20_011, 5
        w2 = O.weights(D2)
        xs2 = host_clients(O, 82, D2, n2, False)
        agg.define(1, n2, fa.F32, fa.F32, D2, fa.FEDAVG)
        for k in range(D2):
            agg.submit(1, k, xs2[k], w2[k])
        assert_bits(agg.finalize(1), O.fedavg(xs2, w2))
