"""Compute-node client states: the per-client intermediate parts of
systemAPI::init_state_vector (systemAPI.cpp:3-15) packed into flat slots and aggregated in place.

CPU tests cover the packing/binding with the oracle as the in-place sync; GPU tests compare
fa_sync_device / fa_sync_part with the oracle bit for bit."""
import ctypes
import importlib

import numpy as np
import pytest

from conftest import load_pkg


def _compute():
    load_pkg()
    return importlib.import_module("mhfsl_amd.compute")


def _mods(torch, ids, dtype=None, seed=0):
    torch.manual_seed(seed)
    out = {}
    for c in ids:
        m = torch.nn.Sequential(torch.nn.Conv2d(3, 8, 3), torch.nn.BatchNorm2d(8), torch.nn.ReLU(),
                                torch.nn.Flatten(), torch.nn.Linear(8 * 6 * 6, 10))
        out[c] = m.to(dtype) if dtype is not None else m
    return out


def _oracle_sync(O):
    def sync(slots, w, n):
        xs = [s.detach().cpu().numpy().copy() for s in slots]
        r = O.fedavg(xs, w)
        for s in slots:
            s.copy_(s.new_tensor(r))
    return sync


def test_states_pack_bind_and_aggregate_cpu(O):
    import torch
    C = _compute()
    ids = [7, 0, 3]
    mods = _mods(torch, ids)
    before = {c: torch.cat([p.detach().reshape(-1).clone() for p in mods[c].parameters()]) for c in ids}
    st = C.ClientStates(mods, sync_fn=_oracle_sync(O))
    assert st.ids == [0, 3, 7] and st.n == sum(p.numel() for p in mods[0].parameters())
    assert (st.stride * 4) % 16 == 0 and st.stride * 4 >= st.n * 4 + C.SKEW_BYTES
    for c in ids:  # parameters are views of their slot, values unchanged
        slot = st.slot(c)
        assert torch.equal(slot, before[c])
        for p in mods[c].parameters():
            assert slot.data_ptr() <= p.data_ptr() < slot.data_ptr() + slot.numel() * 4
    # a training step of one client updates only its slot (optimizers keep their Parameters)
    opt = torch.optim.SGD(mods[3].parameters(), lr=0.1)
    mods[3](torch.randn(2, 3, 8, 8)).sum().backward()
    opt.step()
    assert not torch.equal(st.slot(3), before[3]) and torch.equal(st.slot(0), before[0])
    cur = [st.slot(c).detach().numpy().copy() for c in st.ids]
    w = st.weights({0: 100, 3: 300, 7: 600})
    st.aggregate(w)
    want = O.fedavg(cur, w)
    for c in ids:
        got = torch.cat([p.detach().reshape(-1) for p in mods[c].parameters()]).numpy()
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32))


def test_states_reject_mixed_architectures():
    import torch
    C = _compute()
    mods = {0: torch.nn.Linear(4, 4), 1: torch.nn.Linear(4, 5)}
    with pytest.raises(ValueError):
        C.ClientStates(mods)


@pytest.mark.gpu
@pytest.mark.parametrize("D,bf16", [(1, False), (2, True), (5, False), (3, True), (8, False), (8, True), (9, False), (13, False), (13, True), (64, False), (70, False), (70, True), (130, False), (130, True)])
def test_sync_device_bitexact(fa, O, torch_gpu, D, bf16):
    torch = torch_gpu
    n = 100_003
    w = O.weights(D)
    xs = [O.gen(61, k, n) for k in range(D)]
    if bf16:
        xs = [O.f32_to_bf16(x) for x in xs]
    want = O.fedavg(xs, w, out_dtype="bf16" if bf16 else "f32")
    dev = [torch.from_numpy(x.view(np.int16) if bf16 else x).cuda() for x in xs]
    ctx = fa.Aggregator(1) if D > 128 else None
    fa.sync_device(dev, w, n, fa.BF16 if bf16 else fa.F32, ctx=ctx)
    torch.cuda.synchronize()
    for d in dev:
        got = d.cpu().numpy()
        assert np.array_equal(got.view(np.uint16 if bf16 else np.uint32), want.view(np.uint16 if bf16 else np.uint32))
    if ctx:
        ctx.close()


@pytest.mark.gpu
def test_sync_device_misaligned_slots(fa, O, torch_gpu):
    torch = torch_gpu
    n, D = 4099, 4
    w = O.weights(D)
    xs = [O.gen(62, k, n) for k in range(D)]
    want = O.fedavg(xs, w)
    for offs in [(1, 1, 1, 1), (0, 1, 2, 3)]:
        bufs = [torch.zeros(n + 8, dtype=torch.float32, device="cuda") for _ in range(D)]
        views = [b[o:o + n] for b, o in zip(bufs, offs)]
        for v, x in zip(views, xs):
            v.copy_(torch.from_numpy(x))
        fa.sync_device(views, w, n, fa.F32)
        torch.cuda.synchronize()
        for b, o in zip(bufs, offs):
            got = b.cpu().numpy()
            assert np.array_equal(got[o:o + n].view(np.uint32), want.view(np.uint32))
            assert not got[:o].any() and not got[o + n:].any()  # nothing outside the slot


def _read_device(torch, ptr, n, device):
    """n fp32 at a raw device address (a ctx slot), through the HIP runtime torch has loaded."""
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    t = torch.empty(n, dtype=torch.float32, device=device)
    torch.cuda.synchronize()
    assert hip.hipMemcpy(ctypes.c_void_p(t.data_ptr()), ctypes.c_void_p(ptr), n * 4, 3) == 0  # D2D
    return t.cpu().numpy()


@pytest.mark.gpu
def test_sync_part_on_context_slots(fa, O, torch_gpu):
    """fa_sync_part over a ctx part's own slots (range-sharded when 2 GPUs are visible): every slot
    of every GPU holds its range of the FedAvg afterwards."""
    torch = torch_gpu
    n, D = 300_001, 6
    w = O.weights(D)
    xs = [O.gen(63, k, n) for k in range(D)]
    want = O.fedavg(xs, w)
    gpus = min(2, fa.device_count())
    with fa.Aggregator(gpus) as agg:
        agg.define(5, n, fa.F32, fa.F32, D, fa.FEDAVG)
        for k in range(D):
            agg.submit(5, k, xs[k], w[k])
        fa.check(fa.lib().fa_sync(agg.handle))
        agg.sync_states(5)
        fa.check(fa.lib().fa_sync(agg.handle))
        for g in range(gpus):
            for k in range(D):
                ptr, cnt, off = agg.slot(5, g, k)
                got = _read_device(torch, ptr, cnt, "cuda:%d" % agg.devices[g])
                assert np.array_equal(got.view(np.uint32), want[off:off + cnt].view(np.uint32))
        with pytest.raises(fa.FaError):
            agg.sync_states(99)


@pytest.mark.gpu
def test_client_states_on_gpu(fa, O, torch_gpu):
    torch = torch_gpu
    C = _compute()
    ids = [0, 2, 3, 5]
    mods = {c: m.cuda() for c, m in _mods(torch, ids, seed=3).items()}
    st = C.ClientStates(mods)
    cur = [st.slot(c).cpu().numpy().copy() for c in st.ids]
    w = st.weights({0: 1, 2: 2, 3: 3, 5: 4})
    st.aggregate(w)
    torch.cuda.synchronize()
    want = O.fedavg(cur, w)
    for c in ids:
        got = torch.cat([p.detach().reshape(-1) for p in mods[c].parameters()]).cpu().numpy()
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("D,bf16,phases", [(4, False, 1.3), (3, True, 2.2), (9, False, 1.05)])
def test_sync_phased_same_bits(fa, O, torch_gpu, D, bf16, phases):
    """The phased kernel in state-sync form (walk 5) against the one-shot sync (walk 2): every slot of
    buckets of one to a few phases, bit for bit, plus sampled elements against the oracle."""
    torch = torch_gpu
    n = int(256 * 256 * 88 * 4 * phases) + 4_321
    w = O.weights(D)
    dt = fa.BF16 if bf16 else fa.F32
    tdt = torch.int16 if bf16 else torch.float32
    before = fa.get_tuning()
    res = {}
    try:
        for walk in (2, 5, 6):
            fa.set_tuning(walk=walk)
            dev = [torch.empty(n, dtype=tdt, device="cuda") for _ in range(D)]
            for k, d in enumerate(dev):
                fa.fill_uniform(d, n, dt, 62, k)
            fa.sync_device(dev, w, n, dt)
            torch.cuda.synchronize()
            res[walk] = dev
    finally:
        fa.set_tuning(walk=before["walk"])
    for k in range(D):
        assert torch.equal(res[2][k], res[5][k]), "slot %d differs" % k
        assert torch.equal(res[2][k], res[6][k]), "slot %d differs (walk 6)" % k
        if k:
            assert torch.equal(res[5][0], res[5][k])
    idx = np.unique(np.concatenate([[0, 1, n - 2, n - 1], np.random.default_rng(D).integers(0, n, 512)]))
    got = res[5][0][torch.as_tensor(idx, device="cuda")].cpu().numpy()
    ref = O.fedavg_at(62, w, idx, bf16=bf16)
    if bf16:
        assert np.array_equal(got.view(np.uint16), O.f32_to_bf16(ref))
    else:
        assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
