"""CPU: the client-sharded reduce-scatter layout passes its 1e-6 bound in ANY order RCCL may sum in.

FA_SHARD_CLIENT_RS (and shard.reduce_rs / reduce_rs_cyclic) deal the D clients to G GPUs; GPU g reduces its
clients into an fp32 partial with the ordered chain, and RCCL's reduce-scatter adds the G partials.  Which
order RCCL adds them in is its own choice (a ring that starts at rank g + 1, several channels each with its
own ring position, or a tree), and the one-GPU box can only run the exchange's definition in one ring order
(FA_TEST_SHARED_DEVICE).  The layout's parity check is |got - oracle| <= 1e-6 * sum_k |w_k x_k| per element
(BASELINE.json north_star: "within 1e-6 relative fp32"; bench.py RS_REL_TOL).  Here the partials are the
oracle's own chains over each GPU's clients (what the kernels compute, bit for bit) and they are combined in
every order of G = 2 and 4 (sequential and balanced-tree), and in 300 random orders of G = 8 plus its 8 ring
orders, at the shapes of the configs that use the layout: C4 (64 clients, 4 GPUs), the north star (32
clients on 2 / 4 / 8) and C5 (128 clients on 8).  Every order has to stay within the bound -- so the driver's
first 8-GPU run cannot fail the check on summation order alone.
"""
import importlib
import itertools

import numpy as np
import pytest

from conftest import load_pkg


def seq_sum(parts):
    acc = parts[0].copy()
    for p in parts[1:]:
        acc = (acc + p).astype(np.float32)
    return acc


def tree_sum(parts):
    parts = list(parts)
    while len(parts) > 1:
        nxt = [(parts[i] + parts[i + 1]).astype(np.float32) for i in range(0, len(parts) - 1, 2)]
        if len(parts) % 2:
            nxt.append(parts[-1])
        parts = nxt
    return parts[0]


@pytest.mark.parametrize("D,G", [(64, 4), (32, 2), (32, 4), (32, 8), (128, 8), (64, 8)])
def test_any_summation_order_stays_within_the_bound(O, D, G):
    load_pkg()
    shard = importlib.import_module("mhfsl_amd.shard")
    n = 200_003
    xs = [O.gen(0x5EED + D, k, n) for k in range(D)]
    w = O.weights(D)
    ref = O.fedavg(xs, w)  # the single-GPU ordered chain (bit-exact with the kernels)
    sabs = np.zeros(n, np.float64)
    for k in range(D):
        sabs += np.abs(np.float64(w[k]) * xs[k].astype(np.float64))
    parts = []
    for g in range(G):  # each GPU's partial: the ordered chain over its clients, from +0
        c0, c1 = shard.client_bounds(D, G, g)
        parts.append(O.fedavg(xs[c0:c1], w[c0:c1]))
    if G <= 4:
        orders = list(itertools.permutations(range(G)))
    else:
        rng = np.random.default_rng(7)
        orders = [tuple((g + 1 + i) % G for i in range(G)) for g in range(G)]  # ring orders, block g
        orders += [tuple(rng.permutation(G)) for _ in range(300)]
    worst = 0.0
    for order in orders:
        ps = [parts[i] for i in order]
        for got in (seq_sum(ps), tree_sum(ps)):
            ok, ratio = shard.tolerance_ok(got, ref, sabs)
            assert ok, (order, ratio)
            worst = max(worst, ratio)
    print("D=%d G=%d: %d orders, worst |err| = %.3f of the 1e-6 bound" % (D, G, len(orders), worst))
    assert worst < 0.5  # well inside: no order comes near the bound
