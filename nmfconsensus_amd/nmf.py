"""Host-side mirror of the reference's R driver (nmf.r), running on the HIP engine.

Same names, argument meaning and error behaviour as nmf.r, so code written against the reference's
workflow reads the same:

  doNMF(A, k, maxniter, seed, tolerance)                        nmf.r:23-51
  createJobArray(A, k, num_clusterings, maxniter, seed)          nmf.r:53-70
  runNMFinJobs(A, k, num_clusterings, maxniter, seed, njobs)     nmf.r:106-119
  computeConsensusMatrixFromClusterings(listOfResults)           nmf.r:121-144
  computeConsensusAndSaveFiles(resultList)                       nmf.r:146-253 (cophenetic, order,
                                                                  membership, GCT outputs; no plots)

Every compute step calls nmfconsensus_amd/libnmf.so (HIP, gfx950); there is no CPU fallback.
Differences from nmf.r, all documented in DESIGN.md:
  * per-job init defaults to libnmf's generateMatrix(ran) stream (glibc rand, job seed = seed + job_id - 1,
    the north star's choice); init_stream=INIT_R_RUNIF gives nmf.r:37-38's runif under the BatchJobs job
    seed (R's Mersenne-Twister restated, bit-exact; BatchJobs' seed rule itself is unpinned);
  * the consensus is built from the FINAL H of every restart (what nmf.r intends; with R >= 3.2 the
    literal nmf.r:47-50 returns the initial H);
  * label_rule selects nmf.r:128's literal `order()[1]` (argmin, LABEL_R_ORDER) or the documented
    intent (argmax, LABEL_ARGMAX, default).
"""
from __future__ import annotations

import ctypes
import os
import threading
from dataclasses import dataclass, field

import numpy as np

from . import _lib
from ._lib import (INIT_LIBNMF, INIT_R_RUNIF, LABEL_ARGMAX, LABEL_R_ORDER, STOP_ARGMAX_STABLE, STOP_FIXED, STOP_REF_COMPAT, STOP_TOLX, Result,
                   SweepOpts)

__all__ = [
    "Engine", "SweepResult", "doNMF", "createJobArray", "runNMFinJobs", "computeConsensusMatrixFromClusterings",
    "computeConsensusAndSaveFiles", "cophenetic", "cophenetic_batch", "cutree", "job_grid",
    "STOP_FIXED", "STOP_REF_COMPAT", "STOP_ARGMAX_STABLE", "STOP_TOLX", "LABEL_ARGMAX", "LABEL_R_ORDER",
    "INIT_LIBNMF", "INIT_R_RUNIF", "release_doNMF_engine",
]

_dp = ctypes.POINTER(ctypes.c_double)
_ip = ctypes.POINTER(ctypes.c_int32)


def _f64(a) -> np.ndarray:
    return np.asfortranarray(np.asarray(a, dtype=np.float64))


def job_grid(ks, num_clusterings: int):
    """batchExpandGrid(k=ks, num.clusterings=1:R) job order (nmf.r:64-68): k varies fastest.
    Returns a list of (job_id, k, r) with 1-based job_id and r."""
    ks = list(ks)
    out = []
    jid = 0
    for r in range(1, num_clusterings + 1):
        for k in ks:
            jid += 1
            out.append((jid, k, r))
    return out


@dataclass
class SweepResult:
    ks: list
    R: int
    n: int
    counts: np.ndarray | None          # (nk, n, n) int32
    consensus: np.ndarray | None       # (nk, n, n) float64 = counts / R
    labels: np.ndarray | None          # (njobs, n) int32, 1-based
    iters: np.ndarray                  # (njobs,) int32
    stopped_early: np.ndarray          # (njobs,) int32
    W: list | None = None              # per job (m x k)
    H: list | None = None              # per job (k x n)
    seconds_total: float = 0.0
    seconds_iterate: float = 0.0
    restart_iterations: int = 0
    max_iter_run: int = 0
    job_begin: int = 0
    job_end: int = 0
    extras: dict = field(default_factory=dict)


class Engine:
    """A resident data matrix on one MI355X plus the batched restart engine (nmfc_engine_*).

    A is either a host array (m x n) or an integer device pointer (`a_device_ptr`) to a column-major
    m x n fp64 buffer already in HBM (e.g. torch_tensor.data_ptr() of a Fortran-ordered tensor)."""

    def __init__(self, A=None, device: int = -1, *, a_device_ptr: int | None = None, shape=None):
        self.L = _lib.lib()
        if a_device_ptr is not None:
            m, n = shape
            h = self.L.nmfc_engine_create(device, ctypes.c_void_p(a_device_ptr), m, n, 1)
        else:
            A = _f64(A)
            m, n = A.shape
            self._A = A
            h = self.L.nmfc_engine_create(device, A.ctypes.data_as(ctypes.c_void_p), m, n, 0)
        if not h:
            raise RuntimeError(f"nmfc_engine_create failed: {_lib.last_error()}")
        self.h = h
        self.m, self.n = m, n
        self.device = self.L.nmfc_engine_device(h)   # HIP ordinal resolved at creation (device -1: the current one)

    def close(self):
        if getattr(self, "h", None):
            self.L.nmfc_engine_destroy(self.h)
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

    def set_timing(self, on: bool, stride: int = 1):
        """Event-time the launches of every `stride`-th MU iteration (nmfc_engine_set_timing)."""
        self.L.nmfc_engine_set_timing(self.h, max(1, int(stride)) if on else 0)

    def kernel_time(self, kid: int):
        ms = ctypes.c_double(0.0)
        cnt = self.L.nmfc_engine_kernel_time(self.h, kid, ctypes.byref(ms))
        return cnt, ms.value

    def kernel_flops(self, kid: int) -> float:
        return self.L.nmfc_engine_kernel_flops(self.h, kid)

    def kernel_bytes(self, kid: int):
        """(design bytes, algorithmic bytes) per launch of kernel `kid` in the last run."""
        algo = ctypes.c_double(0.0)
        b = self.L.nmfc_engine_kernel_bytes(self.h, kid, ctypes.byref(algo))
        return b, algo.value

    def mu1(self, W0, H0, *, maxiter: int = 10000, stop_rule: int = STOP_REF_COMPAT):
        """One restart from caller factors (W0 m x k, H0 k x n) on the small-shape team kernel: the per-call path
        of the nmf_mu drop-in (nmfc_engine_mu1; m rounded up to 128 <= 1024, n <= 64).  Returns (W, H, iters,
        stopped_early)."""
        W = np.array(W0, dtype=np.float64, order="F", copy=True)
        H = np.array(H0, dtype=np.float64, order="F", copy=True)
        k = W.shape[1]
        if W.shape != (self.m, k) or H.shape != (k, self.n):
            raise ValueError(f"W0 {W.shape} / H0 {H.shape} do not match A {self.m}x{self.n}")
        it, early = ctypes.c_int(0), ctypes.c_int(0)
        dp = ctypes.POINTER(ctypes.c_double)
        w, h = W.ctypes.data_as(dp), H.ctypes.data_as(dp)
        if self.L.nmfc_engine_mu1(self.h, k, int(maxiter), int(stop_rule), w, h, w, h, ctypes.byref(it),
                                  ctypes.byref(early)) != 0:
            raise RuntimeError(f"nmfc_engine_mu1 failed: {_lib.last_error()}")
        return W, H, it.value, bool(early.value)

    def run(self, ks, R: int, *, maxiter: int = 10000, seed: int = 123, stop_rule: int = STOP_REF_COMPAT,
            label_rule: int = LABEL_ARGMAX, job_begin: int = 0, job_end: int = -1, W_init=None, H_init=None,
            want_factors: bool = False, want_counts: bool = True, counts_device_ptr: int | None = None,
            check_every: int = 4, min_init: int = 0, max_init: int = 1, verbose: bool = False,
            TolX: float = 1e-4, TolFun: float = 1e-4, init_stream: int = INIT_LIBNMF, want_h: bool = False) -> SweepResult:
        """One sweep of the (k, restart) job grid (or its shard [job_begin, job_end)).  want_factors: final W and
        H of every job; want_h: final H only (the C3-sized checks: W of 1800 jobs is 1.7 GB of host memory)."""
        ks = [int(k) for k in ks]
        nk = len(ks)
        njobs_all = nk * R
        je = njobs_all if job_end < 0 else min(job_end, njobs_all)
        jb = max(0, job_begin)
        nj = je - jb
        if nj <= 0:
            raise ValueError("empty job range")
        jk = [ks[(jb + s) % nk] for s in range(nj)]
        o = SweepOpts()
        self.L.nmfc_default_opts(ctypes.byref(o))
        o.maxiter, o.stop_rule, o.label_rule, o.seed = maxiter, stop_rule, label_rule, seed & 0xFFFFFFFF
        o.job_begin, o.job_end, o.check_every, o.verbose = jb, je, check_every, 1 if verbose else 0
        o.min_init, o.max_init = min_init, max_init
        o.TolX, o.TolFun = TolX, TolFun
        o.init_stream = init_stream
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
            res.W = wflat.ctypes.data_as(_dp)
        if want_factors or want_h:
            hflat = np.zeros(sum(k * n for k in jk), dtype=np.float64)
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
        rc = self.L.nmfc_engine_run(self.h, ks_arr.ctypes.data_as(_ip), nk, R, ctypes.byref(o),
                                    wi.ctypes.data_as(_dp) if wi is not None else None,
                                    hi.ctypes.data_as(_dp) if hi is not None else None, ctypes.byref(res))
        if rc != 0:
            raise RuntimeError(f"nmfc_engine_run failed: {_lib.last_error()}")
        Ws = Hs = None
        if want_factors or want_h:
            Ws = [] if want_factors else None
            Hs = []
            wo = ho = 0
            for k in jk:
                if want_factors:
                    Ws.append(wflat[wo:wo + m * k].reshape((m, k), order="F"))
                Hs.append(hflat[ho:ho + k * n].reshape((k, n), order="F"))
                wo += m * k
                ho += k * n
        return SweepResult(ks=ks, R=R, n=n, counts=counts, consensus=consensus, labels=labels, iters=iters,
                           stopped_early=early, W=Ws, H=Hs, seconds_total=res.seconds_total,
                           seconds_iterate=res.seconds_iterate, restart_iterations=res.restart_iterations,
                           max_iter_run=res.max_iter_run, job_begin=jb, job_end=je)


_DONMF = {"A": None, "eng": None, "device": None}
_DONMF_LOCK = threading.Lock()


def _donmf_engine(A: np.ndarray, device: int) -> "Engine":
    """The Engine doNMF reuses across calls (nmf.r calls doNMF once per restart on one matrix): kept while A is
    byte-identical to the cached host copy and the device is the same; anything else builds a new one.  device -1
    is resolved to the calling thread's current HIP device first, so a change of current device between calls
    builds a new engine instead of reusing the one on the old device."""
    from . import _lib

    if device < 0:
        device = _lib.lib().nmfc_current_device()
    c = _DONMF
    if c["eng"] is not None and c["device"] == device and c["A"].shape == A.shape and np.array_equal(c["A"], A):
        return c["eng"]
    release_doNMF_engine_locked()
    c["eng"] = Engine(A, device)
    c["A"], c["device"] = A.copy(order="F"), c["eng"].device
    return c["eng"]


def release_doNMF_engine_locked():
    c = _DONMF
    if c["eng"] is not None:
        c["eng"].close()
    c["eng"] = c["A"] = c["device"] = None


def release_doNMF_engine():
    """Frees the engine (HBM, A's layouts) that doNMF keeps between calls."""
    with _DONMF_LOCK:
        release_doNMF_engine_locked()


def doNMF(A, k: int, maxniter: int, seed: int = 123, tolerance: float = 1e-4, num_clusterings=None,
          *, job_id: int = 1, stop_rule: int = STOP_REF_COMPAT, init_stream: int = INIT_LIBNMF, device: int = -1):
    """nmf.r:23-51 -- one restart: init W, H (generateMatrix(ran) stream, seed + job_id - 1), run the
    MU loop on the GPU, return dict(W=m x k, H=k x n, iter=iterations).  `tolerance` is accepted and
    unused, like the reference (nmf_mu.c:92-93).  The engine (A resident in HBM in its layouts) is kept for
    the next call with the same A (release_doNMF_engine() frees it)."""
    del tolerance, num_clusterings
    A = _f64(A)
    with _DONMF_LOCK:
        eng = _donmf_engine(A, device)
        # a single-job "grid" whose job seed is seed + job_id - 1
        r = eng.run([k], 1, maxiter=maxniter, seed=seed + job_id - 1, stop_rule=stop_rule, want_factors=True,
                    want_counts=False, init_stream=init_stream)
    return {"W": r.W[0], "H": r.H[0], "iter": int(r.iters[0])}


@dataclass
class JobArray:
    """The registry of nmf.r:53-70: A, the (k, r) grid, and the job parameters."""
    A: np.ndarray
    k: list
    num_clusterings: int
    maxniter: int
    seed: int
    tolerance: float = 1e-4

    @property
    def jobs(self):
        return job_grid(self.k, self.num_clusterings)


def createJobArray(A, k, num_clusterings: int, maxniter: int, seed: int, tolerance: float = 1e-4) -> JobArray:
    """nmf.r:53-70."""
    return JobArray(_f64(A), list(k), int(num_clusterings), int(maxniter), int(seed), tolerance)


def runNMFinJobs(A, k, num_clusterings: int, maxniter: int, seed: int, njobs: int = 1, *,
                 stop_rule: int = STOP_REF_COMPAT, label_rule: int = LABEL_ARGMAX, save_dir: str | None = None,
                 device: int = -1, init_stream: int = INIT_LIBNMF):
    """nmf.r:106-119: run every (k, restart) job, reduce per k to a consensus matrix, then cophenetic,
    ordering and membership (computeConsensusAndSaveFiles).  `njobs` (BatchJobs chunks) has no effect:
    all jobs run as one batched sweep on the GPU (use nmfconsensus_amd.distributed for several GPUs).
    Returns the dict produced by computeConsensusAndSaveFiles, plus the raw SweepResult under 'sweep'."""
    del njobs
    ks = list(k)
    if 1 in ks:
        raise ValueError("Need at least two clusters to compute standard deviation")   # nmf.r:107-108
    reg = createJobArray(A, ks, num_clusterings, maxniter, seed)
    with Engine(reg.A, device) as eng:
        sw = eng.run(ks, num_clusterings, maxiter=maxniter, seed=seed, stop_rule=stop_rule, label_rule=label_rule,
                     init_stream=init_stream)
    result = {str(kk): sw.consensus[i] for i, kk in enumerate(ks)}
    out = computeConsensusAndSaveFiles(result, save_dir=save_dir)
    out["sweep"] = sw
    return out


def computeConsensusMatrixFromClusterings(listOfResults, label_rule: int = LABEL_ARGMAX) -> np.ndarray:
    """nmf.r:121-144: labels per result, connectivity = sum of outer(l, l, ==), divided by the number of
    results.  listOfResults: sequence of dicts with an 'H' (k x n) entry (doNMF's return value)."""
    Hs = [_f64(x["H"]) for x in listOfResults]
    if not Hs:
        raise ValueError("empty listOfResults")
    k, n = Hs[0].shape
    flat = np.concatenate([h.reshape(-1, order="F") for h in Hs])
    R = len(Hs)
    cons = np.zeros((n, n), dtype=np.float64, order="F")
    rc = _lib.lib().nmfc_consensus(flat.ctypes.data_as(_dp), k, n, R, label_rule, None, None, cons.ctypes.data_as(_dp))
    if rc != 0:
        raise RuntimeError(f"nmfc_consensus failed: {_lib.last_error()}")
    return np.ascontiguousarray(cons)


def cophenetic(C: np.ndarray):
    """nmf.r:165-172 (+ HC$order, merge, heights): returns (rho_unrounded, order 1-based, merge, height)."""
    C = np.asfortranarray(np.asarray(C, dtype=np.float64))
    n = C.shape[0]
    order = np.zeros(n, dtype=np.int32)
    merge = np.zeros((n - 1, 2), dtype=np.int32)
    height = np.zeros(n - 1, dtype=np.float64)
    rho = _lib.lib().nmfc_cophenetic(C.ctypes.data_as(_dp), n, order.ctypes.data_as(_ip), merge.ctypes.data_as(_ip),
                                     height.ctypes.data_as(_dp))
    return rho, order, merge, height


def cophenetic_batch(Cs: np.ndarray, nthreads: int = 0, symmetric: bool = False):
    """cophenetic() for a stack of consensus matrices (nk, n, n), the k's on parallel host threads.
    symmetric=True: the caller guarantees Cs[q] == Cs[q].T (consensus matrices are), so the row-major
    stack is passed as is (no column-major copy).
    Returns (rho[nk], order[nk, n] 1-based, merge[nk, n-1, 2], height[nk, n-1])."""
    Cs = np.asarray(Cs, dtype=np.float64)
    nk, n, _ = Cs.shape
    if symmetric:
        flat = np.ascontiguousarray(Cs)
    else:
        flat = np.ascontiguousarray(np.transpose(Cs, (0, 2, 1)))   # each matrix column-major
    rho = np.zeros(nk, dtype=np.float64)
    order = np.zeros((nk, n), dtype=np.int32)
    merge = np.zeros((nk, n - 1, 2), dtype=np.int32)
    height = np.zeros((nk, n - 1), dtype=np.float64)
    rc = _lib.lib().nmfc_cophenetic_batch(flat.ctypes.data_as(_dp), nk, n, nthreads, rho.ctypes.data_as(_dp),
                                          order.ctypes.data_as(_ip), merge.ctypes.data_as(_ip),
                                          height.ctypes.data_as(_dp))
    if rc != 0:
        raise ValueError("cophenetic_batch: bad arguments")
    return rho, order, merge, height


def cutree(merge: np.ndarray, k: int) -> np.ndarray:
    """cutree(HC, k) (nmf.r:177): 1-based memberships numbered by first appearance."""
    merge = np.ascontiguousarray(merge, dtype=np.int32)
    n = merge.shape[0] + 1
    out = np.zeros(n, dtype=np.int32)
    if _lib.lib().nmfc_cutree(merge.ctypes.data_as(_ip), n, k, out.ctypes.data_as(_ip)) != 0:
        raise ValueError("cutree: bad arguments")
    return out


def _signif(x: float, digits: int = 4) -> float:
    if not np.isfinite(x) or x == 0:
        return x
    return float(f"{x:.{digits - 1}e}")


def computeConsensusAndSaveFiles(resultList: dict, save_dir: str | None = None, doc_string: str = "") -> dict:
    """nmf.r:146-253 without the plots: per k, hclust/cophenetic rho (signif 4), ordered consensus,
    cutree membership; optionally the GCT/txt outputs of nmf.r:197-198, 241-242, 251-252."""
    from .gct import write_gct

    k_vec = list(resultList.keys())
    rho, ordered, membership, orders = {}, {}, {}, {}
    Cs = np.stack([np.asarray(resultList[kk], dtype=np.float64) for kk in k_vec])
    rhos, order_all, merge_all, _ = cophenetic_batch(Cs)   # the k's on parallel host threads
    for q, kk in enumerate(k_vec):
        C = Cs[q]
        order = order_all[q]
        rho[kk] = _signif(float(rhos[q]), 4)
        o = order - 1
        ordered[kk] = C[np.ix_(o, o)]
        membership[kk] = cutree(merge_all[q], int(kk))
        orders[kk] = order
    if save_dir:
        os.makedirs(save_dir, exist_ok=True)
        n = len(next(iter(membership.values())))
        col_names = [str(i + 1) for i in range(n)]
        for kk in k_vec:
            o = orders[kk] - 1
            write_gct(membership[kk][o], [col_names[i] for i in o], ["membership.ordered"],
                      os.path.join(save_dir, f"{doc_string}.consensus.k.{kk}.gct"))
        allm = np.stack([membership[kk] for kk in k_vec], axis=1)
        write_gct(allm, col_names, [f"k={kk}" for kk in k_vec], os.path.join(save_dir, f"{doc_string}.membership.gct"))
        with open(os.path.join(save_dir, f"{doc_string}.cophenetic.txt"), "w") as f:
            # R's write(cbind(k.vector, rho)) writes column-major, 5 values per line
            vals = [kk for kk in k_vec] + [str(rho[kk]) for kk in k_vec]
            for i in range(0, len(vals), 5):
                f.write(" ".join(str(v) for v in vals[i:i + 5]) + "\n")
    return {"rho": rho, "consensus_ordered": ordered, "membership": membership, "order": orders,
            "consensus": {kk: np.asarray(resultList[kk]) for kk in k_vec}}
