"""CPU tests of the launch planner (fa::plan_chain through fa_diag_plan_chain / fa_diag_rs_plan, pure host
arithmetic): which kernel each bucket shape takes on a 256-CU MI355X, and that the client-sharded rs layout
(FA_SHARD_CLIENT_RS) never launches the phased persistent grid -- its launches run beside RCCL's exchange,
whose blocks the grid would keep off the CUs (VERDICT r02 "next" #1)."""
import pytest

C4_FC, C4_ALL, C5 = 119_586_826, 139_611_210, 1 << 28


@pytest.mark.parametrize("gpus", [1, 2, 4, 8])
@pytest.mark.parametrize("n,clients", [(C4_FC, 64), (C4_ALL, 64), (C5, 128), (64 << 20, 32)])
@pytest.mark.parametrize("out_bf16", [False, True])
def test_rs_layout_never_takes_the_phased_grid(fa, gpus, n, clients, out_bf16):
    out = fa.BF16 if out_bf16 else fa.F32
    for chunks in (0, 1, 8, 16):
        launches, phased, most = fa.rs_plan(n, gpus, clients, chunks, fa.F32, out)
        pieces = len(fa.rs_segments(n, gpus, chunks or fa.get_tuning()["rs_chunks"], 0))
        assert launches == gpus * (pieces + (1 if out_bf16 else 0))
        assert phased == 0 and most == 0, (launches, phased, most)


def test_range_layout_plans(fa):
    ph = fa.PLAN_PHASED
    # the north star: three phases of the 256-thread f32 form (two meetings)
    assert fa.plan_chain(fa.F32, fa.F32, 64 << 20, 32) == (ph, 3)
    # C4 on one GPU: seven phases; C5 (1 GiB x 128): twelve
    assert fa.plan_chain(fa.F32, fa.F32, C4_ALL, 64) == (ph, 7)
    assert fa.plan_chain(fa.F32, fa.F32, C5, 128) == (ph, 12)
    # below one phase with >= 16 clients: one phase sized to the bucket (no meeting)
    assert fa.plan_chain(fa.F32, fa.F32, 16 << 20, 32) == (ph, 1)
    assert fa.plan_chain(fa.F32, fa.F32, 8 << 20, 32) == (ph, 1)
    # ... fewer clients, or too few vectors per lane: the one-shot grid
    assert fa.plan_chain(fa.F32, fa.F32, 12_557_962, 8)[0] == fa.PLAN_ONE_SHOT
    assert fa.plan_chain(fa.F32, fa.F32, 1 << 20, 64)[0] == fa.PLAN_ONE_SHOT
    # C3 (bf16 in and out): the 512-thread form, 33.5 M elements per phase
    assert fa.plan_chain(fa.BF16, fa.BF16, 42_737_546, 32) == (ph, 2)
    assert fa.plan_chain(fa.BF16, fa.BF16, 29_511_680, 32) == (ph, 1)
    # walk 2 (the one-shot XCD walk) and no device (0 CUs) never plan the phased grid
    assert fa.plan_chain(fa.F32, fa.F32, 64 << 20, 32, walk=2)[0] == fa.PLAN_ONE_SHOT
    assert fa.plan_chain(fa.F32, fa.F32, 64 << 20, 32, cus=0)[0] == fa.PLAN_ONE_SHOT
    # a partitioned chip (fewer CUs): smaller phases
    assert fa.plan_chain(fa.F32, fa.F32, 64 << 20, 32, cus=128)[1] > 3


def test_plan_arguments_checked(fa):
    with pytest.raises(fa.FaError):
        fa.plan_chain(7, fa.F32, 100, 2)
    with pytest.raises(fa.FaError):
        fa.rs_plan(100, 0, 2)


def test_range_pieces(fa):
    """Range layout pieces (fa_api.hip piece_len_for, DESIGN.md 4 "the address span"): a GPU whose held slots
    span more than 48 GiB cuts them into pieces of <= 16 GiB of slots (a multiple of 64 elements)."""
    before = fa.get_tuning()
    assert before["piece_span_kib"] == 16 << 20 and before["piece_split_kib"] == 48 << 20
    assert fa.piece_plan(C5, 128) == (8, 1 << 25)            # C5 on one GPU: 128 GiB -> 8 x 16 GiB
    assert fa.piece_plan(C5 // 2, 128) == (4, 1 << 25)       # ... its range shard at 2 GPUs: 64 GiB
    assert fa.piece_plan(C5 // 4, 128) == (1, C5 // 4)       # ... at 4 GPUs: 32 GiB, one piece
    assert fa.piece_plan(C4_ALL, 64) == (1, C4_ALL)          # C4: 33 GiB, one piece (no gain measured)
    assert fa.piece_plan(C5, 128, fa.BF16) == (4, 1 << 26)   # bf16: 64 GiB
    assert fa.piece_plan(0, 128) == (1, 1) and fa.piece_plan(C5, 0) == (1, C5)
    n, pl = fa.piece_plan(12 << 30, 5)                        # 240 GiB of slots in 5 slots: 15 pieces
    assert n == 15 and pl % 64 == 0 and (n - 1) * pl < 12 << 30 <= n * pl
    try:
        fa.set_tuning(piece_span_kib=-1)                      # never cut
        assert fa.piece_plan(C5, 128) == (1, C5)
        fa.set_tuning(piece_span_kib=1 << 10, piece_split_kib=-1)
        n, pl = fa.piece_plan(100_003, 5)                     # 2 MB of slots at 1 MiB per piece
        assert (n, pl) == (2, 50_048)
    finally:
        fa.set_tuning(piece_span_kib=before["piece_span_kib"], piece_split_kib=before["piece_split_kib"])
