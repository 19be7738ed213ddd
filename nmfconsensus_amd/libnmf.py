"""Python view of the libnmf drop-in entry points (include/libnmf_compat.h) in libnmf.so.

These mirror how nmf.r drives the library: `.C("nmf_mu", a, w0, h0, m, n, k, maxiter, TolX, TolFun)`
(nmf.r:42-45) copies its arguments and returns them; nmf_mu below does the same (numpy in, numpy out).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib

_dp = ctypes.POINTER(ctypes.c_double)


def _f(a):
    return np.array(a, dtype=np.float64, order="F", copy=True)


def nmf_mu(a, w0, h0, maxiter: int, TolX: float = 1e-4, TolFun: float = 1e-4):
    """.C('nmf_mu', ...) semantics: returns dict(a, w0, h0, pm, pn, pk, maxiter, pTolX, pTolFun, ret)."""
    a, w0, h0 = _f(a), _f(w0), _f(h0)
    m, n = a.shape
    k = w0.shape[1]
    if w0.shape != (m, k) or h0.shape != (k, n):
        raise ValueError("shape mismatch between a, w0 and h0")
    c = ctypes.c_int
    mi = c(int(maxiter))
    tx, tf = ctypes.c_double(TolX), ctypes.c_double(TolFun)
    ret = _lib.lib().nmf_mu(a.ctypes.data_as(_dp), w0.ctypes.data_as(_dp), h0.ctypes.data_as(_dp),
                            ctypes.byref(c(m)), ctypes.byref(c(n)), ctypes.byref(c(k)), ctypes.byref(mi),
                            ctypes.byref(tx), ctypes.byref(tf))
    return {"a": a, "w0": w0, "h0": h0, "pm": m, "pn": n, "pk": k, "maxiter": mi.value, "pTolX": TolX,
            "pTolFun": TolFun, "ret": ret}


def set_default_opts() -> _lib.OptionsT:
    o = _lib.OptionsT()
    _lib.lib().set_default_opts(ctypes.byref(o))
    return o


def checkArguments(a: bytes | None, k: int, iter: int, w0: bytes | None, h0: bytes | None, opts) -> int:
    return _lib.lib().checkArguments(a, k, iter, w0, h0, ctypes.byref(opts))


def checkMatrices(a, w, h) -> int:
    a, w, h = _f(a), _f(w), _f(h)
    m, n = a.shape
    k = w.shape[1]
    return _lib.lib().checkMatrices(a.ctypes.data_as(_dp), w.ctypes.data_as(_dp), h.ctypes.data_as(_dp), m, n, k)


def randnumber(lo: int, hi: int) -> float:
    return _lib.lib().randnumber(lo, hi)


def generateMatrix(m: int, n: int, k: int, init: int = 0, lo: int = 0, hi: int = 1):
    W = np.zeros((m, k), order="F")
    H = np.zeros((k, n), order="F")
    c = ctypes.c_int
    _lib.lib().generateMatrix(ctypes.byref(c(m)), ctypes.byref(c(n)), ctypes.byref(c(k)), ctypes.byref(c(init)),
                              ctypes.byref(c(lo)), ctypes.byref(c(hi)), W.ctypes.data_as(_dp), H.ctypes.data_as(_dp),
                              None, None)
    return W, H


def calculateNorm(a, w, h):
    a, w, h = _f(a), _f(w), _f(h)
    m, n = a.shape
    k = w.shape[1]
    d = np.zeros((m, n), order="F")
    v = _lib.lib().calculateNorm(a.ctypes.data_as(_dp), w.ctypes.data_as(_dp), h.ctypes.data_as(_dp),
                                 d.ctypes.data_as(_dp), m, n, k)
    return v, d


def calculateMaxchange(mat, mat0, sqrteps: float = 2.0 ** -26.5):
    mat, mat0 = _f(mat), _f(mat0)
    m, n = mat.shape
    v = _lib.lib().calculateMaxchange(mat.ctypes.data_as(_dp), mat0.ctypes.data_as(_dp), m, n, sqrteps)
    return v, mat0
