"""Compute-node client states, laid out for in-place aggregation on the MI355X.

A compute node of the reference holds one State per client:
``systemAPI::init_state_vector`` (pipeline_simulation/systemAPI.cpp:3-15) builds
``clients_state`` (client id -> State: the layers of the intermediate model part
plus one SGD optimizer per layer), and ``compute_node.cpp:16-84`` trains them
per client.  The paper aggregates these intermediate parts across clients; the
code never does.

``ClientStates`` is that map, MI355X-first:

* one device allocation holds every client's part as a flat bucket (slot k at
  ``k * stride`` elements, stride = the bucket rounded up to 4 KiB plus a 512 B
  skew, the same placement as the aggregator's context slots);
* each module parameter is rebound to a view of its client's slot
  (``param.data = view``), so training updates the slot in place and the
  optimizers keep their Parameter objects;
* aggregation is one in-place launch over all slots (``fa_sync_device``: the
  ordered fp32 FMA chain, rounded once to the parameter dtype and written back
  to every slot) instead of a per-tensor loop.

Buffers (BatchNorm running statistics) stay per client, as in the reference,
where only parameters are trained state.
"""
import numpy as np

SKEW_BYTES = 512


def _round_up(x, m):
    return (x + m - 1) // m * m


class ClientStates:
    """client id -> module, parameters packed into one flat slot per client.

    modules:  {client_id: torch.nn.Module}, same architecture, on one device.
    The client order of the FMA chain is ascending client id (``ids``).
    sync_fn:  (slot_tensors, weights, n) -> None, in place; default = libfa's fa_sync_device.
    """

    def __init__(self, modules, sync_fn=None, stream=None):
        import torch
        if not modules:
            raise ValueError("need at least one client")
        self.ids = sorted(modules)
        self.modules = {c: modules[c] for c in self.ids}
        first = self.modules[self.ids[0]]
        self.names = [n for n, _ in first.named_parameters()]
        self.shapes = [tuple(p.shape) for _, p in first.named_parameters()]
        dtypes = {p.dtype for _, p in first.named_parameters()}
        if len(dtypes) != 1 or next(iter(dtypes)) not in (torch.float32, torch.bfloat16):
            raise ValueError("parameters must all be fp32 or all bf16, got %s" % dtypes)
        self.dtype = next(iter(dtypes))
        self.device = next(first.parameters()).device
        self.n = sum(int(np.prod(s)) for s in self.shapes)
        esize = 4 if self.dtype == torch.float32 else 2
        self.stride = (_round_up(self.n * esize, 4096) + SKEW_BYTES) // esize
        self.flat = torch.empty(len(self.ids) * self.stride, dtype=self.dtype, device=self.device)
        for k, cid in enumerate(self.ids):
            params = list(self.modules[cid].named_parameters())
            if [n for n, _ in params] != self.names or [tuple(p.shape) for _, p in params] != self.shapes:
                raise ValueError("client %r has a different architecture" % cid)
            off = k * self.stride
            for _, p in params:
                view = self.flat[off:off + p.numel()].view(p.shape)
                view.copy_(p.data)
                p.data = view
                off += p.numel()
        self._sync = sync_fn
        self.stream = stream

    def slot(self, client_id):
        """The flat bucket of one client (a view: named_parameters() order, concatenated)."""
        k = self.ids.index(client_id)
        return self.flat[k * self.stride:k * self.stride + self.n]

    def slots(self):
        return [self.slot(c) for c in self.ids]

    def weights(self, samples=None):
        """FedAvg weights n_k / sum n in client order (uniform when samples is None)."""
        D = len(self.ids)
        if samples is None:
            return np.full(D, 1.0 / D, np.float32)
        n = np.array([samples[c] for c in self.ids], np.float64)
        return (n / n.sum()).astype(np.float32)

    def aggregate(self, weights=None):
        """Every client's part := sum_k w_k part_k, in place (enqueued on the stream)."""
        w = self.weights() if weights is None else np.asarray(weights, np.float32)
        if w.size != len(self.ids):
            raise ValueError("need one weight per client")
        if self._sync is not None:
            self._sync(self.slots(), w, self.n)
            return
        import importlib
        import sys
        fa = sys.modules.get(__name__.rpartition(".")[0]) or importlib.import_module(__name__.rpartition(".")[0])
        import torch
        dt = fa.F32 if self.dtype == torch.float32 else fa.BF16
        fa.sync_device(self.slots(), w, self.n, dt, stream=self.stream)
