"""MI355X FedAvg aggregation path -- Python view of the C ABI in include/fedavg/fa.h.

The product is ``lib/libfa.so`` (HIP kernels + C ABI, built by this directory's
Makefile).  This module only binds it with ctypes so tests, bench.py and the
multi-GPU driver (``shard.py``) can call it; there is no CPU fallback: if the
library or a gfx950 device is missing, calls raise ``FaError``.

Names mirror the reference aggregator (pipeline_simulation/aggregator.cpp):
a *part* is one model part bucket (``model_part`` 1 = parts[0].layers[0],
m >= 2 = parts[1].layers[m-2]), a *client slot* is one data owner's receipt.
"""
import ctypes
import os
import threading

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PKG_DIR, "lib", "libfa.so")

F32, BF16 = 0, 1
FEDAVG, LITERAL = 0, 1
SHARD_RANGE, SHARD_CLIENT_RS, ACCUMULATE_ON_ARRIVAL, TEST_SHARED_DEVICE = 0x1, 0x2, 0x4, 0x100
OK, ERR_ARG, ERR_HIP, ERR_NOMEM, ERR_STATE, ERR_NODEV, ERR_ALIGN, ERR_NCCL = 0, -1, -2, -3, -4, -5, -6, -7
DTYPE_SIZE = {F32: 4, BF16: 2}

_lib = None


class FaError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("fa error %d: %s" % (code, msg))
        self.code = code


class _Tuning(ctypes.Structure):
    _fields_ = [("block", ctypes.c_int), ("max_blocks", ctypes.c_int), ("unroll", ctypes.c_int),
                ("load_policy", ctypes.c_int), ("store_policy", ctypes.c_int), ("slot_skew", ctypes.c_int),
                ("walk", ctypes.c_int), ("rs_chunks", ctypes.c_int), ("piece_span_kib", ctypes.c_int),
                ("piece_split_kib", ctypes.c_int)]


def build():
    """Compile libfa.so in-tree (hipcc, gfx950)."""
    import subprocess
    subprocess.run(["make", "-C", PKG_DIR, "-j8"], check=True)
    return LIB_PATH


def lib():
    """Load libfa.so (torch, when used, must be imported first: both share libamdhip64.so.7)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise FaError(ERR_NODEV, "libfa.so not built at %s (run make -C %s)" % (LIB_PATH, PKG_DIR))
    L = ctypes.CDLL(LIB_PATH)
    P, S, I, F, U64, U32 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_float, ctypes.c_uint64, ctypes.c_uint32
    sig = {
        "fa_version": (I, []),
        "fa_last_error": (ctypes.c_char_p, []),
        "fa_device_count": (I, [ctypes.POINTER(I)]),
        "fa_create": (I, [ctypes.POINTER(P), I, I]),
        "fa_create_ex": (I, [ctypes.POINTER(P), ctypes.POINTER(I), I, I]),
        "fa_reduce_part": (I, [P, I, P, P]),
        "fa_bucket_slot": (I, [P, I, I, I, ctypes.POINTER(P), ctypes.POINTER(S), ctypes.POINTER(S)]),
        "fa_bucket_pieces": (I, [P, I, I, ctypes.POINTER(I)]),
        "fa_bucket_piece": (I, [P, I, I, I, I, ctypes.POINTER(P), ctypes.POINTER(S), ctypes.POINTER(S)]),
        "fa_bucket_output": (I, [P, I, I, ctypes.POINTER(P)]),
        "fa_sync": (I, [P]),
        "fa_copy_output": (I, [P, I, P]),
        "fa_destroy": (None, [P]),
        "fa_bucket_define": (I, [P, I, S, I, I, I, I]),
        "fa_set_literal_divisor": (I, [P, I, F]),
        "fa_submit": (I, [P, I, I, P, F]),
        "fa_submit_pinned": (I, [P, I, I, P, F]),
        "fa_submit_gather": (I, [P, I, I, I, P, P, F]),
        "fa_submit_gather_pinned": (I, [P, I, I, I, P, P, F]),
        "fa_finalize": (I, [P, I, P]),
        "fa_finalize_gather": (I, [P, I, I, P, P, I]),
        "fa_host_alloc": (I, [S, ctypes.POINTER(P)]),
        "fa_host_free": (I, [P]),
        "fa_sync_device": (I, [P, I, P, P, I, S, I, P]),
        "fa_sync_part": (I, [P, I, P, P]),
        "fa_bucket_progress": (I, [P, I, ctypes.POINTER(I), ctypes.POINTER(I)]),
        "fa_bucket_host_read": (I, [P, I, ctypes.POINTER(I)]),
        "fa_output_crc32": (I, [P, I, I, ctypes.POINTER(S), ctypes.POINTER(U32)]),
        "fa_reduce_parts": (I, [P, I, ctypes.POINTER(I), P, P]),
        "fa_ctx_set_tuning": (I, [P, ctypes.POINTER(_Tuning)]),
        "fa_ctx_get_tuning": (I, [P, ctypes.POINTER(_Tuning)]),
        "fa_rs_segments": (I, [S, I, I, I, ctypes.POINTER(S), I]),
        "fa_phased_timeouts": (I, [I, ctypes.POINTER(U64)]),
        "fa_release_stream": (I, [I, P]),
        "fa_reduce_device": (I, [P, I, P, P, I, S, I, P, I, I, P, P]),
        "fa_fill_uniform": (I, [P, S, I, U64, U32, U64, P]),
        "fa_diag_read_stream": (I, [P, I, S, P]),  # diagnostics (outside fa.h)
        "fa_diag_read_plain": (I, [P, I, S, I, I, P]),
        "fa_diag_rw_plain": (I, [P, I, S, I, I, I, P]),
        "fa_diag_plan_chain": (I, [I, I, S, I, I, I, ctypes.POINTER(I), ctypes.POINTER(ctypes.c_longlong)]),
        "fa_diag_rs_plan": (I, [S, I, I, I, I, I, I, ctypes.POINTER(I), ctypes.POINTER(I),
                                ctypes.POINTER(ctypes.c_longlong)]),
        "fa_diag_pieces": (I, [S, I, I, ctypes.POINTER(I), ctypes.POINTER(S)]),
        "fa_diag_phased_slot": (I, [I, P, ctypes.POINTER(I)]),
        "fa_diag_phased_owned": (I, [I]),
        "fa_diag_host_reads": (ctypes.c_longlong, [P]),
        "fa_diag_exchange_streams": (I, [P]),
        "fa_set_tuning": (I, [ctypes.POINTER(_Tuning)]),
        "fa_get_tuning": (I, [ctypes.POINTER(_Tuning)]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def check(rc):
    if rc != OK:
        raise FaError(rc, lib().fa_last_error().decode(errors="replace"))
    return rc


def last_error():
    return lib().fa_last_error().decode(errors="replace")


def device_count():
    n = ctypes.c_int(0)
    check(lib().fa_device_count(ctypes.byref(n)))
    return n.value


def _addr(x):
    """Device/host address of a torch tensor, numpy array or raw int."""
    if x is None:
        return None
    if isinstance(x, int):
        return x
    if hasattr(x, "data_ptr"):
        return x.data_ptr()
    if isinstance(x, np.ndarray):
        return x.ctypes.data
    raise TypeError("need a tensor, array or int address, got %r" % type(x))


# Caller streams handed to the library as torch stream objects: (device, hipStream_t) -> live Python objects
# wrapping it.  When the last one is collected the stream is retired and its phased counter slot goes back
# (fa_release_stream); torch's pooled streams are wrapped again later, and simply take a slot anew.  Torch
# stream objects take no weak references, so the tracker rides in the object's __dict__ and goes with it.
_tracked = {}
_tracked_mu = threading.Lock()


class _StreamSlot:
    __slots__ = ("key",)

    def __init__(self, key):
        self.key = key
        with _tracked_mu:
            _tracked[key] = _tracked.get(key, 0) + 1

    def __del__(self):
        try:
            key = self.key
            with _tracked_mu:
                _tracked[key] -= 1
                if _tracked[key]:
                    return
                del _tracked[key]
            if _lib is not None:
                _lib.fa_release_stream(key[0], key[1])
        except Exception:  # interpreter shutdown: module globals may be gone
            pass


def _stream(stream):
    if stream is None:
        return None
    if isinstance(stream, int):
        return stream
    h = stream.cuda_stream  # torch.cuda.Stream on ROCm wraps a hipStream_t
    if h and getattr(stream, "_fa_slot", None) is None:
        dev = stream.device.index if getattr(stream, "device", None) is not None else 0
        try:
            stream._fa_slot = _StreamSlot((dev or 0, h))
        except AttributeError:  # an object without a __dict__: release_stream() by hand
            pass
    return h


def release_stream(stream, device=None):
    """fa_release_stream: give back the phased kernel's owned counter slot of a caller stream (a torch stream
    object or a raw hipStream_t address) before destroying it.  Torch stream objects passed to this module
    are released by themselves when collected; raw handles need this call."""
    if device is None:
        device = stream.device.index if hasattr(stream, "device") and stream.device.index is not None else 0
    h = stream if isinstance(stream, int) else stream.cuda_stream
    check(lib().fa_release_stream(device, h))


def reduce_device(clients, weights, n, in_dtype, out, out_dtype=F32, mode=FEDAVG, init=None, stream=None, gpu=0,
                  ctx=None):
    """fa_reduce_device: D device-resident client buckets -> out (enqueued, not synchronized)."""
    D = len(clients)
    arr = (ctypes.c_void_p * D)(*[_addr(c) for c in clients])
    w = np.ascontiguousarray(np.asarray(weights, np.float32).reshape(-1))
    if w.size != D:
        raise ValueError("need one weight per client")
    check(lib().fa_reduce_device(ctx.handle if ctx is not None else None, gpu, arr, w.ctypes.data, D, n, in_dtype,
                                 _addr(out), out_dtype, mode, _addr(init), _stream(stream)))


def sync_device(clients, weights, n, dtype, stream=None, gpu=0, ctx=None):
    """fa_sync_device: every device bucket in `clients` := sum_k w_k clients[k] (in place, enqueued)."""
    D = len(clients)
    arr = (ctypes.c_void_p * D)(*[_addr(c) for c in clients])
    w = np.ascontiguousarray(np.asarray(weights, np.float32).reshape(-1))
    if w.size != D:
        raise ValueError("need one weight per client")
    check(lib().fa_sync_device(ctx.handle if ctx is not None else None, gpu, arr, w.ctypes.data, D, n, dtype,
                               _stream(stream)))


def fill_uniform(dst, n, dtype, seed, client, idx0=0, stream=None):
    check(lib().fa_fill_uniform(_addr(dst), n, dtype, seed, client, idx0, _stream(stream)))


def diag_read_stream(buffers, n, stream=None):
    """fa_diag_read_stream (diagnostic, outside fa.h): one read-only launch over the fp32 device buffers
    (n elements each, n % 4 == 0, 16-byte aligned) on `stream`; time it with events on that stream."""
    arr = (ctypes.c_void_p * len(buffers))(*[_addr(b) for b in buffers])
    check(lib().fa_diag_read_stream(arr, len(buffers), n, _stream(stream)))


def diag_read_plain(buffers, n, grid=8192, unroll=16, stream=None):
    """fa_diag_read_plain (diagnostic, outside fa.h): the independent read ceiling -- one plain grid-stride
    launch (`grid` workgroups of 256 lanes, `unroll` nt 16-byte loads in flight) reading the fp32 device
    buffers (n elements each) one after another, on `stream`."""
    arr = (ctypes.c_void_p * len(buffers))(*[_addr(b) for b in buffers])
    check(lib().fa_diag_read_plain(arr, len(buffers), n, grid, unroll, _stream(stream)))


def diag_rw_plain(buffers, n, grid=8192, unroll=16, nt=False, stream=None):
    """fa_diag_rw_plain (diagnostic, outside fa.h): the independent in-place read+write ceiling -- one plain
    grid-stride launch reading every fp32 device buffer (n elements each) and writing it back where it lies
    (values unchanged), buffer after buffer, nt loads and plain (or nt) stores, on `stream`."""
    arr = (ctypes.c_void_p * len(buffers))(*[_addr(b) for b in buffers])
    check(lib().fa_diag_rw_plain(arr, len(buffers), n, grid, unroll, 1 if nt else 0, _stream(stream)))


PLAN_ONE_SHOT, PLAN_SCALAR, PLAN_PHASED = 0, 1, 2


def plan_chain(in_dtype, out_dtype, n, n_clients, walk=0, cus=256):
    """fa_diag_plan_chain (diagnostic, host arithmetic): (kind, phases) of the launch one FedAvg chain over a
    16-byte aligned bucket of n elements takes under fa_tuning.walk `walk` (0 = the process default) on `cus`
    CUs; kind PLAN_PHASED with phases > 1 means chip-wide meetings."""
    k, ph = ctypes.c_int(), ctypes.c_longlong()
    check(lib().fa_diag_plan_chain(in_dtype, out_dtype, n, n_clients, walk, cus, ctypes.byref(k), ctypes.byref(ph)))
    return k.value, ph.value


def rs_plan(n, n_gpus, n_clients, chunks=0, in_dtype=F32, out_dtype=F32, cus=256):
    """fa_diag_rs_plan (diagnostic): (launches, phased launches, most phases of one launch) that one
    FA_SHARD_CLIENT_RS round enqueues for a bucket of n elements (the process-default tuning)."""
    a, b, c = ctypes.c_int(), ctypes.c_int(), ctypes.c_longlong()
    check(lib().fa_diag_rs_plan(n, n_gpus, n_clients, chunks, in_dtype, out_dtype, cus, ctypes.byref(a),
                                ctypes.byref(b), ctypes.byref(c)))
    return a.value, b.value, c.value


def piece_plan(n, held, in_dtype=F32):
    """fa_diag_pieces (diagnostic): (pieces, elements per piece) of a range-layout GPU holding `held` slots of
    n elements (under the process-default piece_span_kib / piece_split_kib, set_tuning)."""
    a, b = ctypes.c_int(), ctypes.c_size_t()
    check(lib().fa_diag_pieces(n, held, in_dtype, ctypes.byref(a), ctypes.byref(b)))
    return a.value, b.value


def _tuning_dict(t):
    return {"block": t.block, "max_blocks": t.max_blocks, "unroll": t.unroll, "load_policy": t.load_policy,
            "store_policy": t.store_policy, "slot_skew": t.slot_skew, "walk": t.walk, "rs_chunks": t.rs_chunks,
            "piece_span_kib": t.piece_span_kib, "piece_split_kib": t.piece_split_kib}


def get_tuning():
    """fa_get_tuning: the process defaults (new contexts and context-less calls start from them)."""
    t = _Tuning()
    check(lib().fa_get_tuning(ctypes.byref(t)))
    return _tuning_dict(t)


LOAD_DEFAULT, LOAD_NT = 1, 2
STORE_PLAIN, STORE_NT, STORE_SC1, STORE_SC01 = 1, 2, 3, 4


def set_tuning(block=0, max_blocks=0, unroll=0, load_policy=0, store_policy=0, slot_skew=0, walk=0, rs_chunks=0,
               piece_span_kib=0, piece_split_kib=0):
    """fa_set_tuning (process defaults); every argument 0 = keep.  max_blocks -1 = one-shot grid,
    slot_skew -1 = none, -2 = by slot size (the default: 512 B from 48 MiB slots up, else 2048);
    piece_span_kib -1 = never cut a GPU's slots into range pieces, piece_split_kib -1 = always cut them."""
    t = _Tuning(block, max_blocks, unroll, load_policy, store_policy, slot_skew, walk, rs_chunks, piece_span_kib,
                piece_split_kib)
    check(lib().fa_set_tuning(ctypes.byref(t)))


def phased_timeouts(device=0):
    """fa_phased_timeouts: phased-kernel meetings on `device` whose bounded wait ran out (grid not
    co-resident) since the process started."""
    c = ctypes.c_uint64()
    check(lib().fa_phased_timeouts(device, ctypes.byref(c)))
    return c.value


def phased_slot(stream, device=0):
    """fa_diag_phased_slot (diagnostic): (counter slot, owned) of the phased kernel for `stream` on `device`,
    assigned now if the stream has none yet -- owned: the slot is the stream's alone (the first 48 streams,
    until their context is destroyed), else a hashed slot shared with other streams."""
    own = ctypes.c_int()
    slot = lib().fa_diag_phased_slot(device, _stream(stream), ctypes.byref(own))
    if slot < 0:
        check(slot)
    return slot, bool(own.value)


def phased_owned_slots(device=0):
    """fa_diag_phased_owned (diagnostic): how many of the 48 owned counter slots are taken on `device`."""
    n = lib().fa_diag_phased_owned(device)
    if n < 0:
        check(n)
    return n


def rs_segments(n, n_gpus, chunks, gpu):
    """fa_rs_segments: [(lo, hi), ...] of bucket elements GPU `gpu` holds after the rs layout's
    reduce-scatter (block-cyclic over `chunks` pieces), in the order of its shard."""
    cnt = lib().fa_rs_segments(n, n_gpus, chunks, gpu, None, 0)
    if cnt < 0:
        check(cnt)
    buf = (ctypes.c_size_t * (2 * max(1, cnt)))()
    lib().fa_rs_segments(n, n_gpus, chunks, gpu, buf, cnt)
    return [(buf[2 * i], buf[2 * i + 1]) for i in range(cnt)]


HOST_PINNED = 0x1


class PinnedBuffer:
    """fa_host_alloc'd page-locked host memory, viewed as a numpy array (freed on close / GC)."""

    def __init__(self, nbytes):
        p = ctypes.c_void_p()
        check(lib().fa_host_alloc(nbytes, ctypes.byref(p)))
        self.ptr, self.nbytes = p.value, nbytes

    def view(self, dtype=np.uint8, count=-1, offset=0):
        if not self.ptr:
            return np.empty(0, dtype)
        raw = (ctypes.c_char * self.nbytes).from_address(self.ptr)
        return np.frombuffer(raw, dtype=dtype, count=count, offset=offset)

    def close(self):
        if self.ptr:
            check(lib().fa_host_free(self.ptr))
            self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _segments(pieces):
    pieces = [np.ascontiguousarray(x) for x in pieces]
    ptrs = (ctypes.c_void_p * len(pieces))(*[x.ctypes.data for x in pieces])
    sizes = (ctypes.c_size_t * len(pieces))(*[x.nbytes for x in pieces])
    return pieces, ptrs, sizes


class Aggregator:
    """fa_ctx: the aggregator's global parts on 1..G GPUs (range-sharded when G > 1).

    Usage mirrors one aggregation phase of aggregator.cpp: define the bucket
    once (refactor), submit every receipt, finalize to obtain the reduced part.
    """

    def __init__(self, n_gpus=1, flags=None, devices=None, rs=False, eager=False, shared_device=False):
        if devices is None:
            devices = list(range(n_gpus))
        n_gpus = len(devices)
        if flags is None:
            flags = SHARD_CLIENT_RS if rs else SHARD_RANGE if n_gpus > 1 else 0
            flags |= (ACCUMULATE_ON_ARRIVAL if eager else 0) | (TEST_SHARED_DEVICE if shared_device else 0)
        h = ctypes.c_void_p()
        ids = (ctypes.c_int * n_gpus)(*devices)
        check(lib().fa_create_ex(ctypes.byref(h), ids, n_gpus, flags))
        self.devices = list(devices)
        self.handle = h
        self.parts = {}

    def define(self, part_id, n, in_dtype=F32, out_dtype=F32, n_clients=1, mode=FEDAVG):
        check(lib().fa_bucket_define(self.handle, part_id, n, in_dtype, out_dtype, n_clients, mode))
        self.parts[part_id] = (n, in_dtype, out_dtype, n_clients, mode)

    def set_divisor(self, divisor, part_id=-1):
        check(lib().fa_set_literal_divisor(self.handle, part_id, divisor))

    def submit(self, part_id, slot, host, weight=1.0, pinned=False):
        host = np.ascontiguousarray(host)
        if part_id not in self.parts:
            check(lib().fa_submit(self.handle, part_id, slot, host.ctypes.data, float(weight)))
        n, in_dtype = self.parts[part_id][:2]
        if host.nbytes != n * DTYPE_SIZE[in_dtype]:
            raise ValueError("bucket %d expects %d bytes, got %d" % (part_id, n * DTYPE_SIZE[in_dtype], host.nbytes))
        fn = lib().fa_submit_pinned if pinned else lib().fa_submit
        check(fn(self.handle, part_id, slot, host.ctypes.data, float(weight)))

    def submit_gather(self, part_id, slot, pieces, weight=1.0, pinned=False):
        """fa_submit_gather(_pinned): `pieces` (host arrays) concatenate to the bucket.  pinned: views of
        PinnedBuffers the caller keeps unchanged until finalize returns."""
        pieces, ptrs, sizes = _segments(pieces)
        fn = lib().fa_submit_gather_pinned if pinned else lib().fa_submit_gather
        check(fn(self.handle, part_id, slot, len(pieces), ptrs, sizes, float(weight)))

    def sync_states(self, part_id, weights=None, stream=None):
        """fa_sync_part: every client slot of the part := the FedAvg of all slots (in place, async)."""
        wp = None
        if weights is not None:
            w = np.ascontiguousarray(np.asarray(weights, np.float32))
            self._w_keep = w
            wp = w.ctypes.data
        check(lib().fa_sync_part(self.handle, part_id, wp, _stream(stream)))

    def finalize_gather(self, part_id, pieces, pinned=False):
        """fa_finalize_gather: the reduced bucket scattered over `pieces` (writable host arrays)."""
        for x in pieces:
            if not (isinstance(x, np.ndarray) and x.flags.c_contiguous and x.flags.writeable):
                raise ValueError("finalize_gather needs writable contiguous arrays")
        _, ptrs, sizes = _segments(pieces)
        check(lib().fa_finalize_gather(self.handle, part_id, len(pieces), ptrs, sizes, HOST_PINNED if pinned else 0))

    def finalize(self, part_id, out=None):
        if part_id not in self.parts:  # let the library report it (FA_ERR_ARG)
            check(lib().fa_finalize(self.handle, part_id, None))
        n, _, out_dtype = self.parts[part_id][:3]
        if out is None:
            out = np.empty(n, np.float32 if out_dtype == F32 else np.uint16)
        check(lib().fa_finalize(self.handle, part_id, out.ctypes.data))
        return out

    def slot(self, part_id, gpu, client_slot):
        """(device address, n_elems, elem_offset) of a client slot."""
        ptr, n, off = ctypes.c_void_p(), ctypes.c_size_t(), ctypes.c_size_t()
        check(lib().fa_bucket_slot(self.handle, part_id, gpu, client_slot, ctypes.byref(ptr), ctypes.byref(n),
                                   ctypes.byref(off)))
        return ptr.value, n.value, off.value

    def pieces(self, part_id, gpu, client_slot):
        """[(device address, n_elems, elem_offset)] of every piece of a client slot, in element order (one
        entry unless the GPU's slots span more than the piece threshold, fa_bucket_pieces)."""
        npc = ctypes.c_int()
        check(lib().fa_bucket_pieces(self.handle, part_id, gpu, ctypes.byref(npc)))
        out = []
        for j in range(npc.value):
            ptr, n, off = ctypes.c_void_p(), ctypes.c_size_t(), ctypes.c_size_t()
            check(lib().fa_bucket_piece(self.handle, part_id, gpu, j, client_slot, ctypes.byref(ptr),
                                        ctypes.byref(n), ctypes.byref(off)))
            out.append((ptr.value, n.value, off.value))
        return out

    def progress(self, part_id):
        """fa_bucket_progress: (receipts submitted this round, leading slots already reduced)."""
        a, b = ctypes.c_int(), ctypes.c_int()
        check(lib().fa_bucket_progress(self.handle, part_id, ctypes.byref(a), ctypes.byref(b)))
        return a.value, b.value

    def host_read_kept(self, part_id):
        """fa_bucket_host_read: True when the part's round so far is kept host-side to be read in place."""
        k = ctypes.c_int()
        check(lib().fa_bucket_host_read(self.handle, part_id, ctypes.byref(k)))
        return bool(k.value)

    def reduce_parts(self, part_ids, weights=None, stream=None):
        """fa_reduce_parts: one batched reduction of several parts (async); weights: None or one array per
        part (None entries = the submitted weights)."""
        ids = (ctypes.c_int * len(part_ids))(*part_ids)
        wp = None
        if weights is not None:
            keep = [None if w is None else np.ascontiguousarray(np.asarray(w, np.float32)) for w in weights]
            self._w_keep = keep
            wp = (ctypes.c_void_p * len(part_ids))(*[None if w is None else w.ctypes.data for w in keep])
        check(lib().fa_reduce_parts(self.handle, len(part_ids), ids, wp, _stream(stream)))

    def set_tuning(self, **kw):
        """fa_ctx_set_tuning: this context's tuning (same keys as set_tuning; 0 = keep)."""
        t = _Tuning(*[kw.get(k, 0) for k, _ in _Tuning._fields_])
        check(lib().fa_ctx_set_tuning(self.handle, ctypes.byref(t)))

    def get_tuning(self):
        t = _Tuning()
        check(lib().fa_ctx_get_tuning(self.handle, ctypes.byref(t)))
        return _tuning_dict(t)

    def output(self, part_id, gpu=0):
        ptr = ctypes.c_void_p()
        check(lib().fa_bucket_output(self.handle, part_id, gpu, ctypes.byref(ptr)))
        return ptr.value

    def reduce(self, part_id, weights=None, stream=None):
        """fa_reduce_part: device-resident reduction of the part's slots (async)."""
        wp = None
        if weights is not None:
            w = np.ascontiguousarray(np.asarray(weights, np.float32))
            self._w_keep = w
            wp = w.ctypes.data
        check(lib().fa_reduce_part(self.handle, part_id, wp, _stream(stream)))

    def copy_output(self, part_id, out=None):
        n, _, out_dtype = self.parts[part_id][:3]
        if out is None:
            out = np.empty(n, np.float32 if out_dtype == F32 else np.uint16)
        check(lib().fa_copy_output(self.handle, part_id, out.ctypes.data))
        return out

    def output_crc32(self, part_id, seg_bytes):
        """fa_output_crc32: zlib CRC-32 of consecutive byte segments of the part's device output (GPU-side)."""
        n = len(seg_bytes)
        b = (ctypes.c_size_t * max(1, n))(*seg_bytes)
        out = (ctypes.c_uint32 * max(1, n))()
        check(lib().fa_output_crc32(self.handle, part_id, n, b, out))
        return [out[i] for i in range(n)]

    def sync(self):
        check(lib().fa_sync(self.handle))

    def host_reads(self):
        """fa_diag_host_reads (diagnostic): reductions of this context that read their receipts where they
        arrived (small pinned receipts of a one-GPU range part)."""
        return lib().fa_diag_host_reads(self.handle)

    def exchange_streams(self):
        """fa_diag_exchange_streams (diagnostic): GPUs of this context holding an exchange stream (rs only)."""
        return lib().fa_diag_exchange_streams(self.handle)

    def close(self):
        if self.handle:
            lib().fa_destroy(self.handle)
            self.handle = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
