"""Multi-GPU layouts of the aggregation round, one process per GPU.

The reference has one aggregator process reducing every receipt itself
(pipeline_simulation/aggregator.cpp:59-150); on a node of G GPUs the buckets
are partitioned instead:

* ``range``  -- rank r owns elements [lo_r, hi_r) of EVERY client bucket and
  reduces them locally.  No collective; bit-exact with the oracle.
* ``rs``     -- rank r owns clients [c_r, c_{r+1}) (whole buckets), reduces them
  into an fp32 partial of the full bucket, and an RCCL reduce-scatter
  (``torch.distributed.reduce_scatter_tensor``, backend "nccl" = RCCL over
  xGMI) sums the partials so rank r ends with elements [lo_r, hi_r).  The
  summation order changes: parity is by tolerance (1e-6 relative to
  sum_k |w_k x_k|).  ``reduce_rs_cyclic`` is the same exchange with
  block-cyclic ownership, so every chunk is one launch (what bench.py times).
* ``chain``  -- client-sharded like ``rs`` but bit-exact: the ordered FMA chain
  is passed rank to rank (rank r continues from rank r-1's fp32 accumulator via
  fa_reduce_device's d_init), pipelined over element chunks with point-to-point
  send/recv, and the last rank scatters each rank's range to it.

The local reduction is a callable so the exchange logic runs unchanged on CPU
tensors under gloo in tests; on the GPU it is ``fa_reducer`` (libfa.so).

Overlap: in ``rs`` and ``chain`` the local reductions run while RCCL's kernels
move the previous chunk.  RCCL's blocks need CUs and LDS that the phased
persistent grid (the default walk for large buckets) holds on every CU for its
whole launch, so run these layouts with the one-shot walk:
``fa.set_tuning(walk=OVERLAP_WALK)`` (bench.py does; the in-process
FA_SHARD_CLIENT_RS layout of libfa.so does the same by itself).
"""
import numpy as np

UNIT = 64  # shard boundaries in elements (keeps every shard's 16-byte phase)
OVERLAP_WALK = 2  # fa_tuning.walk of reductions that run beside a collective: the one-shot XCD walk


def range_bounds(n, world, rank, unit=UNIT):
    """[lo, hi) of bucket elements owned by `rank` (shards are multiples of `unit` except the last)."""
    per_rank = (n + world - 1) // world
    per = (per_rank + unit - 1) // unit * unit
    lo = min(n, rank * per)
    return lo, min(n, lo + per)


def client_bounds(n_clients, world, rank):
    """[c0, c1) of client slots held by `rank` (contiguous, balanced, client order preserved)."""
    base, extra = divmod(n_clients, world)
    c0 = rank * base + min(rank, extra)
    return c0, c0 + base + (1 if rank < extra else 0)


def fa_reducer(fa, in_dtype, stream=None):
    """Local reduction on the GPU through libfa.so: (clients, weights, n, init) -> fp32 tensor."""
    import torch

    def reduce(clients, weights, n, init=None, out=None):
        if out is None:
            out = torch.empty(n, dtype=torch.float32, device="cuda")
        fa.reduce_device(clients, weights, n, in_dtype, out, fa.F32, fa.FEDAVG, init=init, stream=stream)
        return out
    return reduce


def reduce_range(reduce, clients, weights, lo, hi):
    """`clients` are this rank's slices [lo, hi) of every bucket."""
    return reduce(clients, weights, hi - lo)


def reduce_rs(reduce, dist, clients, weights, n, device, chunks=1, itemsize=4):
    """Client-sharded partial + reduce-scatter; returns this rank's [lo, hi) of the sum.

    `n` must be a multiple of world * UNIT (pad the bucket) so that reduce-scatter
    shards are equal and line up with range_bounds.  With chunks > 1 the ranges are
    cut into chunks: chunk c of EVERY rank's range is reduced into one contiguous
    buffer (one launch per rank range) and reduce-scattered asynchronously while
    chunk c+1 is reduced, so the RCCL transfer over xGMI overlaps the HBM-bound
    local reduction (~G*min(1, D/39) instead of G*D/(D+39)).
    `clients` are tensors or raw device addresses (itemsize bytes per element).
    """
    import torch
    world, rank = dist.get_world_size(), dist.get_rank()
    assert n % (world * UNIT) == 0, "pad the bucket to a multiple of world * %d" % UNIT
    per = n // world
    lo, hi = range_bounds(n, world, rank)
    assert (lo, hi) == (rank * per, (rank + 1) * per)
    shard = torch.empty(per, dtype=torch.float32, device=device)
    edges = sorted({min(per, (per * c // chunks) // UNIT * UNIT) for c in range(max(1, chunks))} | {per})
    q_max = max(b - a for a, b in zip(edges, edges[1:]))
    bufs = [torch.empty(world * q_max, dtype=torch.float32, device=device) for _ in range(min(2, len(edges) - 1))]
    pending = [None] * len(bufs)
    for c, (a, b) in enumerate(zip(edges, edges[1:])):
        q = b - a
        i = c % len(bufs)
        if pending[i] is not None:  # the buffer's previous reduce-scatter must be done before it is refilled
            pending[i].wait()
        buf = bufs[i][:world * q]
        for r in range(world):
            out = buf[r * q:(r + 1) * q]
            if clients:
                o0 = r * per + a
                reduce([_piece(x, o0, o0 + q, itemsize) for x in clients], weights, q, out=out)
            else:  # a rank without clients contributes zeros
                out.zero_()
        pending[i] = dist.reduce_scatter_tensor(shard[a:b], buf, op=dist.ReduceOp.SUM, async_op=True)
    for p in pending:
        if p is not None:
            p.wait()
    return shard


def cyclic_pieces(n, world, chunks):
    """[A, B) bucket pieces of the block-cyclic rs layout: `chunks` contiguous pieces, each a multiple of
    world * UNIT elements (n must be a multiple of world * UNIT), so each splits into `world` equal blocks."""
    g = world * UNIT
    assert n % g == 0, "pad the bucket to a multiple of world * %d" % UNIT
    m = n // g
    edges = sorted({m * c // max(1, chunks) * g for c in range(max(1, chunks))} | {n})
    return list(zip(edges, edges[1:]))


def cyclic_bounds(n, world, rank, chunks):
    """The [lo, hi) segments rank `rank` owns under reduce_rs_cyclic, in the order of its shard."""
    out = []
    for a, b in cyclic_pieces(n, world, chunks):
        q = (b - a) // world
        out.append((a + rank * q, a + (rank + 1) * q))
    return out


def reduce_rs_cyclic(reduce, dist, clients, weights, n, device, chunks=16, itemsize=4):
    """Client-sharded partial + reduce-scatter with block-cyclic ownership: ONE launch per chunk.

    reduce_rs with chunks > 1 reduces every rank's range separately (chunks * world launches per round:
    128 small ones at 8 ranks x 16 chunks, each a ctypes call).  Here chunk c is one contiguous piece of
    the bucket (cyclic_pieces), reduced by a single launch into a buffer whose reduce-scatter hands rank
    r the r-th block of the piece.  The reduce-scatter of piece c overlaps the reduction of piece c+1.
    Rank r ends with the segments cyclic_bounds(n, world, r, chunks), concatenated.  Same summation as
    reduce_rs: parity by tolerance (1e-6 relative to sum_k |w_k x_k|).
    """
    import torch
    world = dist.get_world_size()
    pieces = cyclic_pieces(n, world, chunks)
    shard = torch.empty(n // world, dtype=torch.float32, device=device)
    if not pieces:
        return shard
    q_max = max(b - a for a, b in pieces)
    bufs = [torch.empty(q_max, dtype=torch.float32, device=device) for _ in range(min(2, len(pieces)))]
    pending = [None] * len(bufs)
    off = 0
    for c, (a, b) in enumerate(pieces):
        i = c % len(bufs)
        if pending[i] is not None:  # the buffer's previous reduce-scatter must be done before it is refilled
            pending[i].wait()
        buf = bufs[i][:b - a]
        if clients:
            reduce([_piece(x, a, b, itemsize) for x in clients], weights, b - a, out=buf)
        else:  # a rank without clients contributes zeros
            buf.zero_()
        q = (b - a) // world
        pending[i] = dist.reduce_scatter_tensor(shard[off:off + q], buf, op=dist.ReduceOp.SUM, async_op=True)
        off += q
    for p in pending:
        if p is not None:
            p.wait()
    return shard


def _piece(x, a, b, itemsize):
    """Elements [a, b) of a client bucket given as a tensor or a raw device address."""
    return x + a * itemsize if isinstance(x, int) else x[a:b]


def _staged(dist, t):
    """gloo's send/recv take host tensors only (a device tensor's pointer would be read as host memory):
    device tensors go through a host copy there.  RCCL moves device buffers directly."""
    return t.is_cuda and dist.get_backend() == "gloo"


def _send(dist, t, dst):
    """Send `t` to `dst`; returns a handle to wait() on (the send is blocking when staged through host)."""
    if _staged(dist, t):
        dist.send(t.cpu(), dst=dst)
        return None
    return dist.isend(t, dst=dst)


def _recv(dist, t, src):
    if _staged(dist, t):
        import torch
        h = torch.empty(t.shape, dtype=t.dtype)
        dist.recv(h, src=src)
        t.copy_(h)
    else:
        dist.recv(t, src=src)


def reduce_chain(reduce, dist, clients, weights, n, device, chunks=8, itemsize=4):
    """Bit-exact client-sharded reduction: the fp32 chain is handed rank r -> r+1 chunk by chunk.

    Rank r holds clients in global order after rank r-1's.  Returns this rank's
    [lo, hi) of the ordered chain over ALL clients (== the single-GPU result).
    """
    import torch
    world, rank = dist.get_world_size(), dist.get_rank()
    edges = sorted({min(n, (n * c // chunks) // UNIT * UNIT) for c in range(chunks)} | {n})
    acc = torch.empty(n, dtype=torch.float32, device=device)
    sends = []
    for a, b in zip(edges, edges[1:]):
        init = None
        if rank > 0:
            _recv(dist, acc[a:b], rank - 1)
            init = acc[a:b]
        if clients:  # in place: each lane reads its init elements before it writes them
            reduce([_piece(x, a, b, itemsize) for x in clients], weights, b - a, init=init, out=acc[a:b])
        elif rank == 0:
            acc[a:b].zero_()  # the chain starts at +0
        if rank < world - 1:
            sends.append(_send(dist, acc[a:b], rank + 1))
    for r in sends:
        if r is not None:
            r.wait()
    # the last rank holds the full chain: it sends every rank its range
    lo, hi = range_bounds(n, world, rank)
    mine = torch.empty(hi - lo, dtype=torch.float32, device=device)
    last = world - 1
    if rank == last:
        outs = []
        for r in range(world - 1):
            rlo, rhi = range_bounds(n, world, r)
            if rhi > rlo:
                outs.append(_send(dist, acc[rlo:rhi].contiguous(), r))
        mine.copy_(acc[lo:hi])
        for o in outs:
            if o is not None:
                o.wait()
    elif hi > lo:
        _recv(dist, mine, last)
    return mine


def tolerance_ok(got, ref, xs_abs_weighted, rel=1e-6):
    """|got - ref| <= rel * sum_k |w_k x_k| elementwise (the rs layout's parity bound)."""
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    bound = rel * np.asarray(xs_abs_weighted, np.float64) + 1e-30
    return bool(np.all(np.abs(got - ref) <= bound)), float(np.max(np.abs(got - ref) / bound))
