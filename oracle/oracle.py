"""ctypes wrapper of oracle/liboracle.so — the CPU restatement of flac-py's hot path.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, as the checker and the timed CPU baseline.  The product never
imports this module.
"""
import ctypes as C
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
if REPO not in sys.path:
    sys.path.insert(0, REPO)

from flac_amd import abi  # noqa: E402  (struct layouts of include/flacmi.h)

LIB_PATH = os.path.join(HERE, "liboracle.so")
_lib = None


def build(force: bool = False) -> str:
    """Compile liboracle.so with oracle/Makefile (gcc, -ffp-contract=off)."""
    if force or not os.path.exists(LIB_PATH) or _stale():
        subprocess.run(["make", "-s", "-C", HERE, "-B" if force else "all"], check=True)
    return LIB_PATH


def _stale() -> bool:
    t = os.path.getmtime(LIB_PATH)
    srcs = [os.path.join(HERE, f) for f in ("flac_oracle.c", "flac_oracle.h")]
    srcs.append(os.path.join(REPO, "include", "flacmi.h"))
    return any(os.path.getmtime(s) > t for s in srcs)


def lib():
    global _lib
    if _lib is None:
        build()
        L = C.CDLL(LIB_PATH)
        P = C.POINTER
        L.oracle_analyze_unit.argtypes = [P(C.c_int64), C.c_int32, P(abi.Params), P(abi.UnitMeta),
                                          P(C.c_int32), P(C.c_uint64), P(C.c_double), P(C.c_int64),
                                          P(C.c_int64), P(C.c_int32)]
        L.oracle_analyze_unit.restype = C.c_int
        L.oracle_analyze_batch.argtypes = [P(abi.Batch), P(abi.Params), C.c_void_p, C.c_void_p,
                                           C.c_int64, C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p,
                                           C.c_void_p, C.c_void_p, C.c_int]
        L.oracle_analyze_batch.restype = C.c_int
        L.oracle_tukey.argtypes = [C.c_int32, P(C.c_double)]
        L.oracle_tukey.restype = C.c_int
        L.oracle_autocorrelation.argtypes = [P(C.c_double), C.c_int32, C.c_int32]
        L.oracle_autocorrelation.restype = C.c_double
        L.oracle_levinson.argtypes = [P(C.c_double), C.c_int32, P(C.c_double), P(C.c_int32)]
        L.oracle_levinson.restype = C.c_int
        L.oracle_quantize.argtypes = [P(C.c_double), C.c_int32, C.c_int32, P(C.c_int32),
                                      P(C.c_int32), P(C.c_int32), P(C.c_int32)]
        L.oracle_quantize.restype = C.c_int
        L.oracle_pypow2.argtypes = [C.c_double, P(C.c_int32)]
        L.oracle_pypow2.restype = C.c_double
        L.oracle_floor_log2.argtypes = [C.c_double, P(C.c_int32)]
        L.oracle_floor_log2.restype = C.c_int32
        L.oracle_synth_unit.argtypes = [C.c_int64, C.c_int32, C.c_int32, C.c_uint64, P(C.c_int32)]
        L.oracle_synth_unit.restype = None
        L.oracle_synth_unit_mix.argtypes = [C.c_int64, C.c_int32, C.c_int32, C.c_uint64, C.c_int32, P(C.c_int32)]
        L.oracle_synth_unit_mix.restype = None
        _lib = L
    return _lib


def _ptr(a, ctype):
    return a.ctypes.data_as(C.POINTER(ctype))


def make_params(max_lpc_order=12, qlp_precision=5, rice_min=0, rice_max=5,
                mode=abi.MODE_REFERENCE) -> abi.Params:
    p = abi.Params()
    p.max_lpc_order, p.qlp_precision = max_lpc_order, qlp_precision
    p.rice_min, p.rice_max, p.mode = rice_min, rice_max, mode
    return p


def analyze_unit(samples, params: abi.Params) -> dict:
    """One unit through the oracle; returns meta fields + intermediates."""
    x = np.ascontiguousarray(np.asarray(samples, dtype=np.int64))
    n = len(x)
    meta = abi.UnitMeta()
    rice = np.zeros((1 << abi.MAX_RICE_ORDER) + 2, dtype=np.int32)
    res = np.zeros(max(n, 1), dtype=np.uint64)
    acf = np.zeros(33, dtype=np.float64)
    fs = np.zeros(5, dtype=np.int64)
    ls = np.zeros(32, dtype=np.int64)
    rec = np.zeros(abi.lpc_rec_words(32), dtype=np.int32)
    lib().oracle_analyze_unit(_ptr(x, C.c_int64), n, C.byref(params), C.byref(meta),
                              _ptr(rice, C.c_int32), _ptr(res, C.c_uint64), _ptr(acf, C.c_double),
                              _ptr(fs, C.c_int64), _ptr(ls, C.c_int64), _ptr(rec, C.c_int32))
    out = {f: getattr(meta, f) for f, _ in abi.UnitMeta._fields_ if f != "coefs"}
    out["coefs"] = list(meta.coefs)[: meta.ncoefs]
    out["rice_params"] = rice[: meta.n_parts].copy()
    out["residual"] = res[meta.res_offset: meta.res_offset + meta.res_len].copy()
    out["acf"] = acf
    out["fixed_sums"] = fs
    out["lpc_sums"] = ls
    out["lpc_record"] = rec
    return out


def analyze_batch(samples2d: np.ndarray, params: abi.Params, block_len: int, tail_len: int = 0,
                  n_tail_units: int = 0, sample_bits: int = 16, threads: int = 1) -> dict:
    """Batch through the oracle with the flacmi_batch layout (rows of samples2d)."""
    s = np.ascontiguousarray(samples2d)
    assert s.dtype in (np.int16, np.int32)
    n_units, stride = s.shape
    b = abi.Batch()
    b.samples = s.ctypes.data
    b.sample_bytes = s.dtype.itemsize
    b.sample_bits = sample_bits
    b.unit_stride = stride
    b.n_units = n_units
    b.block_len = block_len
    b.tail_len = tail_len
    b.n_tail_units = n_tail_units
    pstride = (1 << max(params.rice_max, 0)) + 1
    meta = np.zeros(n_units, dtype=abi.META_DTYPE)
    rice = np.zeros((n_units, pstride), dtype=np.int32)
    res = np.zeros((n_units, stride), dtype=np.uint64)
    acf = np.zeros((n_units, 33), dtype=np.float64)
    fs = np.zeros((n_units, 5), dtype=np.int64)
    ls = np.zeros((n_units, 32), dtype=np.int64)
    rec = np.zeros((n_units, abi.lpc_rec_words(32)), dtype=np.int32)
    lib().oracle_analyze_batch(C.byref(b), C.byref(params), meta.ctypes.data, rice.ctypes.data,
                               pstride, res.ctypes.data, stride, acf.ctypes.data, fs.ctypes.data,
                               ls.ctypes.data, rec.ctypes.data, threads)
    return {"meta": meta, "rice_params": rice, "residual": res, "acf": acf, "fixed_sums": fs,
            "lpc_sums": ls, "lpc_records": rec}


def meta_mismatches(dev, ora) -> list:
    """Fields of a device meta row (abi.META_DTYPE) that differ from the oracle's row.  A
    device row with lpc_order == abi.LPC_PRUNED (the analysis proved every LPC candidate
    loses, include/flacmi.h FLACMI_LPC_PRUNED) must have lpc_sum == LPC_PRUNED, and the
    oracle must agree that LPC loses strictly: its best LPC sum above its best fixed sum."""
    bad = []
    pruned = int(dev["lpc_order"]) == abi.LPC_PRUNED
    for f in abi.META_DTYPE.names:
        if f in ("coefs", "lpc_tiers") or (pruned and f in ("lpc_order", "lpc_sum")):
            continue
        if dev[f] != ora[f]:
            bad.append((f, dev[f], ora[f]))
    k = int(ora["ncoefs"])
    if list(dev["coefs"][:k]) != list(ora["coefs"][:k]):
        bad.append(("coefs", list(dev["coefs"][:k]), list(ora["coefs"][:k])))
    if pruned:
        if int(dev["lpc_sum"]) != abi.LPC_PRUNED:
            bad.append(("lpc_sum (pruned)", int(dev["lpc_sum"]), abi.LPC_PRUNED))
        if int(ora["status"]) == 0 and not int(ora["lpc_sum"]) > int(ora["fixed_sum"]):
            bad.append(("pruned but LPC does not lose", int(ora["lpc_sum"]), int(ora["fixed_sum"])))
    return bad


def tukey(n: int):
    w = np.zeros(max(n, 1), dtype=np.float64)
    st = lib().oracle_tukey(n, _ptr(w, C.c_double))
    return st, w[:n]


def autocorrelation(x, lag: int) -> float:
    a = np.ascontiguousarray(np.asarray(x, dtype=np.float64))
    return lib().oracle_autocorrelation(_ptr(a, C.c_double), len(a), lag)


def levinson(r, order: int):
    a = np.ascontiguousarray(np.asarray(r, dtype=np.float64))
    out = np.zeros(max(order, 1), dtype=np.float64)
    site = C.c_int32()
    st = lib().oracle_levinson(_ptr(a, C.c_double), order, _ptr(out, C.c_double), C.byref(site))
    return st, site.value, out[:order]


def quantize(c, precision: int):
    a = np.ascontiguousarray(np.asarray(c, dtype=np.float64))
    q = np.zeros(max(len(a), 1), dtype=np.int32)
    nq, sh, site = C.c_int32(), C.c_int32(), C.c_int32()
    st = lib().oracle_quantize(_ptr(a, C.c_double), len(a), precision, _ptr(q, C.c_int32),
                               C.byref(nq), C.byref(sh), C.byref(site))
    return st, site.value, list(q[: nq.value]), sh.value


def pypow2(x: float):
    st = C.c_int32()
    r = lib().oracle_pypow2(x, C.byref(st))
    return r, st.value


def floor_log2(x: float):
    st = C.c_int32()
    r = lib().oracle_floor_log2(x, C.byref(st))
    return r, st.value


def synth_unit(unit: int, length: int, bits: int, seed: int, open_eighths: int = 0) -> np.ndarray:
    out = np.zeros(length, dtype=np.int32)
    if open_eighths:
        lib().oracle_synth_unit_mix(unit, length, bits, seed, open_eighths, _ptr(out, C.c_int32))
    else:
        lib().oracle_synth_unit(unit, length, bits, seed, _ptr(out, C.c_int32))
    return out


def synth_batch(first_unit: int, n_units: int, length: int, bits: int, seed: int,
                dtype=np.int16, stride: int = None, open_eighths: int = 0) -> np.ndarray:
    stride = stride or length
    a = np.zeros((n_units, stride), dtype=dtype)
    for i in range(n_units):
        a[i, :length] = synth_unit(first_unit + i, length, bits, seed, open_eighths)
    return a
