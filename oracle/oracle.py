"""numpy/ctypes front-end to liboracle.so (oracle/fa_oracle.c).

TEST INFRASTRUCTURE ONLY -- imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg as the checker.  The product (libfa.so) never
imports or calls this module.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")
SEED = 0x5EED
WSEED = 7

_lib = None


def build(force=False):
    """Compile liboracle.so (gcc, x86-64-v3 for the FMA instruction; -ffp-contract=off)."""
    src = os.path.join(HERE, "fa_oracle.c")
    if not force and os.path.exists(LIB_PATH) and os.path.getmtime(LIB_PATH) >= os.path.getmtime(src):
        return LIB_PATH
    subprocess.run(["gcc", "-O3", "-march=x86-64-v3", "-ffp-contract=off", "-fPIC", "-shared", "-pthread",
                    src, "-o", LIB_PATH], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        P, S, U64, U32, I, F = (ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_uint32,
                                ctypes.c_int, ctypes.c_float)
        L.fa_oracle_splitmix64.restype = U64
        L.fa_oracle_splitmix64.argtypes = [U64]
        L.fa_oracle_gen_value.restype = F
        L.fa_oracle_gen_value.argtypes = [U64, U32, U64]
        L.fa_oracle_fill_f32.argtypes = [U64, U32, U64, S, P]
        L.fa_oracle_fill_bf16.argtypes = [U64, U32, U64, S, P]
        L.fa_oracle_gen_at.argtypes = [U64, U32, P, S, P]
        L.fa_oracle_weights.argtypes = [U64, I, P]
        L.fa_oracle_fedavg_f32.argtypes = [P, P, I, S, P, P, I]
        L.fa_oracle_fedavg_bf16.argtypes = [P, P, I, S, P, P, I, I]
        L.fa_oracle_literal_f32.argtypes = [P, S, F, P]
        L.fa_oracle_literal_bf16.argtypes = [P, S, F, P, I]
        _lib = L
    return _lib


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def gen(seed, client, n, idx0=0, dtype="f32"):
    """Synthetic bucket of `n` elements for `client` (fp32 or bf16 bits as uint16)."""
    if dtype == "f32":
        out = np.empty(n, np.float32)
        lib().fa_oracle_fill_f32(seed, client, idx0, n, _ptr(out))
    else:
        out = np.empty(n, np.uint16)
        lib().fa_oracle_fill_bf16(seed, client, idx0, n, _ptr(out))
    return out


def gen_at(seed, client, idx):
    """Generator values at arbitrary indices (for sampled checks at full size)."""
    idx = np.ascontiguousarray(idx, np.uint64)
    out = np.empty(idx.size, np.float32)
    lib().fa_oracle_gen_at(seed, client, _ptr(idx), idx.size, _ptr(out))
    return out


def weights(n_clients, seed=WSEED):
    w = np.empty(n_clients, np.float32)
    lib().fa_oracle_weights(seed, n_clients, _ptr(w))
    return w


def _ptr_array(xs):
    return (ctypes.c_void_p * len(xs))(*[x.ctypes.data for x in xs])


def fedavg(xs, w, init=None, out_dtype="f32", threads=1):
    """Ordered fmaf chain over the client list `xs` (all f32 or all bf16-as-uint16)."""
    n = xs[0].size
    w = np.ascontiguousarray(w, np.float32)
    init_p = _ptr(np.ascontiguousarray(init, np.float32)) if init is not None else None
    arr = _ptr_array(xs)
    if xs[0].dtype == np.float32:
        assert out_dtype == "f32"
        out = np.empty(n, np.float32)
        lib().fa_oracle_fedavg_f32(arr, _ptr(w), len(xs), n, init_p, _ptr(out), threads)
    else:
        out = np.empty(n, np.uint16 if out_dtype == "bf16" else np.float32)
        lib().fa_oracle_fedavg_bf16(arr, _ptr(w), len(xs), n, init_p, _ptr(out), int(out_dtype == "bf16"), threads)
    return out


def literal(x_last, divisor=1000.0, out_dtype="f32"):
    n = x_last.size
    if x_last.dtype == np.float32:
        out = np.empty(n, np.float32)
        lib().fa_oracle_literal_f32(_ptr(x_last), n, divisor, _ptr(out))
    else:
        out = np.empty(n, np.uint16 if out_dtype == "bf16" else np.float32)
        lib().fa_oracle_literal_bf16(_ptr(x_last), n, divisor, _ptr(out), int(out_dtype == "bf16"))
    return out


def fedavg_at(seed, w, idx, bf16=False):
    """Oracle chain evaluated only at the indices `idx` (inputs regenerated per index)."""
    idx = np.asarray(idx, np.uint64)
    xs = []
    for k in range(len(w)):
        v = gen_at(seed, k, idx)
        if bf16:
            v = bf16_to_f32(f32_to_bf16(v))
        xs.append(v)
    return fedavg(xs, w)


def sampled_chain(seed, w, idx, clients=None, bf16=False):
    """The FedAvg chain at the indices `idx` only, for parity checks of full-size results: chain position k
    holds generator client clients[k] (default k) of `seed`, rounded to bf16 first when `bf16`.
    Returns (ref fp32, sum_k |w_k x_k| in fp64 -- the scale of the rs layout's 1e-6 tolerance)."""
    idx = np.asarray(idx, np.uint64)
    xs, sabs = [], np.zeros(idx.size, np.float64)
    for k in range(len(w)):
        v = gen_at(seed, k if clients is None else clients[k], idx)
        if bf16:
            v = bf16_to_f32(f32_to_bf16(v))
        xs.append(v)
        sabs += np.abs(np.float64(w[k]) * v.astype(np.float64))
    return fedavg(xs, w), sabs


def f32_to_bf16(a):
    u = np.ascontiguousarray(a, np.float32).view(np.uint32).astype(np.uint64)
    nan = (u & 0x7FFFFFFF) > 0x7F800000
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)
    r[nan] = ((u[nan] >> 16) | 0x40).astype(np.uint16)
    return r


def bf16_to_f32(h):
    return (np.asarray(h, np.uint16).astype(np.uint32) << 16).view(np.float32)
