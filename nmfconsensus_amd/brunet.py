"""Brunet KL-divergence MU consensus (BASELINE.json configs[4]) on the HIP engine.

Host mirror of the BROAD `nmfconsensus(...)` R script that the reference names (commented-out call at
test_nmf.r:29) but does not ship.  Names and argument meaning follow that script:

  NMF_div(V, k, maxniter, seed, stopconv, stopfreq)      NMF.div: one Brunet KL-divergence restart
  nmfconsensus(input_ds, k_init, k_final, num_clusterings, maxniter, error_function="divergence",
               rseed=123456789, stopconv=40, stopfreq=10)  the k sweep + consensus + cophenetic

Every compute step calls nmfconsensus_amd/libnmf.so (nmfc_brunet_*, HIP gfx950); there is no CPU
fallback.  Restart i (1-based) of every k runs set.seed(rseed + i) then W <- runif(m k), H <- runif(k n)
(R's Mersenne-Twister, bit-exact).  NMF.div's error.v trace (a per-iteration log-sum over A, not used
by the consensus) is not computed.  Parity vs the reference is unpinned (the script is not in the
reference); the oracle is oracle/brunet_oracle.c.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from ._lib import BrunetOpts, Result
from .nmf import SweepResult, computeConsensusAndSaveFiles

__all__ = ["BrunetEngine", "NMF_div", "nmfconsensus"]

_dp = ctypes.POINTER(ctypes.c_double)
_ip = ctypes.POINTER(ctypes.c_int32)


def _f64(a) -> np.ndarray:
    return np.asfortranarray(np.asarray(a, dtype=np.float64))


class BrunetEngine:
    """A resident data matrix on one MI355X plus the batched Brunet restart engine (nmfc_brunet_*)."""

    def __init__(self, A=None, device: int = -1, *, a_device_ptr: int | None = None, shape=None):
        self.L = _lib.lib()
        if a_device_ptr is not None:
            m, n = shape
            h = self.L.nmfc_brunet_create(device, ctypes.c_void_p(a_device_ptr), m, n, 1)
        else:
            A = _f64(A)
            m, n = A.shape
            self._A = A
            h = self.L.nmfc_brunet_create(device, A.ctypes.data_as(ctypes.c_void_p), m, n, 0)
        if not h:
            raise RuntimeError(f"nmfc_brunet_create failed: {_lib.last_error()}")
        self.h = h
        self.m, self.n = m, n
        self.device = self.L.nmfc_brunet_device(h)   # HIP ordinal resolved at creation (device -1: the current one)

    def close(self):
        if getattr(self, "h", None):
            self.L.nmfc_brunet_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def set_timing(self, on: bool):
        self.L.nmfc_brunet_set_timing(self.h, 1 if on else 0)

    def kernel_time(self, kid: int):
        """(launches, accumulated event ms, algorithmic flop per launch) of kernel kid (_lib.BK_*)."""
        ms, fl = ctypes.c_double(0.0), ctypes.c_double(0.0)
        cnt = self.L.nmfc_brunet_kernel_time(self.h, kid, ctypes.byref(ms), ctypes.byref(fl))
        return cnt, ms.value, fl.value

    def run(self, ks, R: int, *, maxiter: int = 2000, seed: int = 123456789, stopconv: int = 40, stopfreq: int = 10,
            restart_begin: int = 0, restart_end: int = -1, W_init=None, H_init=None, want_factors: bool = False,
            want_counts: bool = True, counts_device_ptr: int | None = None, verbose: bool = False,
            lanes: int = 0) -> SweepResult:
        """Jobs in nmfconsensus order (for k in ks: for i in restart shard); per-job arrays follow it."""
        ks = [int(k) for k in ks]
        nk = len(ks)
        rb = max(0, restart_begin)
        re = R if restart_end < 0 else min(restart_end, R)
        B = re - rb
        if B <= 0:
            raise ValueError("empty restart range")
        jk = [k for k in ks for _ in range(B)]
        nj = len(jk)
        o = BrunetOpts()
        self.L.nmfc_brunet_default_opts(ctypes.byref(o))
        o.maxiter, o.stopconv, o.stopfreq, o.seed = maxiter, stopconv, stopfreq, seed & 0xFFFFFFFF
        o.restart_begin, o.restart_end, o.verbose, o.lanes = rb, re, 1 if verbose else 0, lanes
        m, n = self.m, self.n
        res = Result()
        iters = np.zeros(nj, dtype=np.int32)
        early = np.zeros(nj, dtype=np.int32)
        labels = np.zeros((nj, n), dtype=np.int32)
        res.iters = iters.ctypes.data_as(_ip)
        res.stopped_early = early.ctypes.data_as(_ip)
        res.labels = labels.ctypes.data_as(_ip)
        counts = consensus = None
        if counts_device_ptr is not None:
            res.counts = ctypes.cast(ctypes.c_void_p(counts_device_ptr), _ip)
            res.counts_on_device = 1
        elif want_counts:
            counts = np.zeros((nk, n, n), dtype=np.int32)
            consensus = np.zeros((nk, n, n), dtype=np.float64)
            res.counts = counts.ctypes.data_as(_ip)
            res.consensus = consensus.ctypes.data_as(_dp)
        wflat = hflat = None
        if want_factors:
            wflat = np.zeros(sum(m * k for k in jk), dtype=np.float64)
            hflat = np.zeros(sum(k * n for k in jk), dtype=np.float64)
            res.W = wflat.ctypes.data_as(_dp)
            res.H = hflat.ctypes.data_as(_dp)
        wi = hi = None
        if W_init is not None or H_init is not None:
            if W_init is None or H_init is None:
                raise ValueError("W_init and H_init must be given together")
            wi = np.concatenate([_f64(w).reshape(-1, order="F") for w in W_init])
            hi = np.concatenate([_f64(h).reshape(-1, order="F") for h in H_init])
            if wi.size != sum(m * k for k in jk) or hi.size != sum(k * n for k in jk):
                raise ValueError("W_init/H_init sizes do not match the job shard")
        ks_arr = np.array(ks, dtype=np.int32)
        rc = self.L.nmfc_brunet_run(self.h, ks_arr.ctypes.data_as(_ip), nk, R, ctypes.byref(o),
                                    wi.ctypes.data_as(_dp) if wi is not None else None,
                                    hi.ctypes.data_as(_dp) if hi is not None else None, ctypes.byref(res))
        if rc != 0:
            raise RuntimeError(f"nmfc_brunet_run failed: {_lib.last_error()}")
        Ws = Hs = None
        if want_factors:
            Ws, Hs = [], []
            wo = ho = 0
            for k in jk:
                Ws.append(wflat[wo:wo + m * k].reshape((m, k), order="F"))
                Hs.append(hflat[ho:ho + k * n].reshape((k, n), order="F"))
                wo += m * k
                ho += k * n
        return SweepResult(ks=ks, R=R, n=n, counts=counts, consensus=consensus, labels=labels, iters=iters,
                           stopped_early=early, W=Ws, H=Hs, seconds_total=res.seconds_total,
                           seconds_iterate=res.seconds_iterate, restart_iterations=res.restart_iterations,
                           max_iter_run=res.max_iter_run, job_begin=rb, job_end=re)


def NMF_div(V, k: int, maxniter: int = 2000, seed: int = 123456, stopconv: int = 40, stopfreq: int = 10,
            device: int = -1) -> dict:
    """NMF.div: one Brunet KL-divergence restart from set.seed(seed).  Returns dict(W, H, t)."""
    with BrunetEngine(V, device) as eng:
        # restart i = 1 of a one-restart sweep runs set.seed(rseed + 1)
        r = eng.run([k], 1, maxiter=maxniter, seed=seed - 1, stopconv=stopconv, stopfreq=stopfreq,
                    want_factors=True, want_counts=False)
    return {"W": r.W[0], "H": r.H[0], "t": int(r.iters[0])}


def nmfconsensus(input_ds, k_init: int, k_final: int, num_clusterings: int, maxniter: int,
                 error_function: str = "divergence", rseed: int = 123456789, directory: str | None = None,
                 stopconv: int = 40, stopfreq: int = 10, doc_string: str = "", device: int = -1) -> dict:
    """The BROAD consensus sweep: for k in k_init..k_final, num_clusterings Brunet restarts, membership
    = argmax of each H column, connectivity summed and divided by num_clusterings, then the cophenetic
    correlation, ordering and cutree membership (computeConsensusAndSaveFiles).  input_ds is an m x n
    array or a .gct path."""
    if error_function != "divergence":
        raise NotImplementedError("only error_function='divergence' (Brunet KL MU) is implemented")
    if k_init < 2 or k_final < k_init:
        raise ValueError("need 2 <= k_init <= k_final")
    if isinstance(input_ds, str):
        from .gct import read_gct
        A = read_gct(input_ds)[0]
    else:
        A = input_ds
    ks = list(range(k_init, k_final + 1))
    with BrunetEngine(A, device) as eng:
        sw = eng.run(ks, num_clusterings, maxiter=maxniter, seed=rseed, stopconv=stopconv, stopfreq=stopfreq)
    result = {str(k): sw.consensus[i] for i, k in enumerate(ks)}
    out = computeConsensusAndSaveFiles(result, save_dir=directory, doc_string=doc_string)
    out["sweep"] = sw
    return out
