"""oracle/pyoracle.py -- TEST INFRASTRUCTURE ONLY.

ctypes bindings for
  * oracle/liboracle.so   : our plain-C restatement of the reference hot path (nmf_oracle.c), and
  * oracle/_ref/libnmf_ref.so : the reference's own libnmf sources compiled out-of-tree (Makefile `ref`).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.
It is the checker, never the thing measured or shipped.
"""
from __future__ import annotations

import ctypes
import os
import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "liboracle.so")
REF_SO = os.path.join(HERE, "_ref", "libnmf_ref.so")

STOP_FIXED, STOP_REF_COMPAT, STOP_ARGMAX_STABLE, STOP_TOLX = 0, 1, 2, 3
LABEL_ARGMAX, LABEL_R_ORDER = 0, 1

_dp = ctypes.POINTER(ctypes.c_double)
_ip = ctypes.POINTER(ctypes.c_int32)


def _d(a: np.ndarray):
    assert a.dtype == np.float64 and (a.flags["C_CONTIGUOUS"] or a.flags["F_CONTIGUOUS"])
    return a.ctypes.data_as(_dp)


def _i(a: np.ndarray):
    assert a.dtype == np.int32
    return a.ctypes.data_as(_ip)


class _RandState(ctypes.Structure):
    _fields_ = [("ring", ctypes.c_uint32 * 34), ("pos", ctypes.c_uint64)]


class _RMTState(ctypes.Structure):
    _fields_ = [("mt", ctypes.c_uint32 * 624), ("mti", ctypes.c_int)]


class Oracle:
    """Restatement (port) of libnmf nmf_mu + init stream + consensus (nmf_oracle.c), and of the
    Brunet KL-divergence MU with R's set.seed/runif init (brunet_oracle.c)."""

    def __init__(self, path: str = ORACLE_SO):
        if not os.path.exists(path):
            raise FileNotFoundError(f"{path} missing: run `make -C oracle`")
        L = ctypes.CDLL(path)
        L.orc_srand.argtypes = [ctypes.POINTER(_RandState), ctypes.c_uint32]
        L.orc_rand.argtypes = [ctypes.POINTER(_RandState)]
        L.orc_rand.restype = ctypes.c_int32
        L.orc_init_restart.argtypes = [ctypes.c_uint32, ctypes.c_int, ctypes.c_int, ctypes.c_int, _dp, _dp]
        L.orc_nmf_mu.argtypes = [_dp, _dp, _dp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.orc_nmf_mu.restype = ctypes.c_int
        L.orc_labels.argtypes = [_dp, ctypes.c_int, ctypes.c_int, ctypes.c_int, _ip]
        L.orc_counts.argtypes = [_ip, ctypes.c_int, ctypes.c_int, _ip]
        L.orc_calculate_norm.argtypes = [_dp, _dp, _dp, _dp, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.orc_calculate_norm.restype = ctypes.c_double
        L.orc_calculate_maxchange.argtypes = [_dp, _dp, ctypes.c_int, ctypes.c_int, ctypes.c_double]
        L.orc_calculate_maxchange.restype = ctypes.c_double
        L.orc_nmf_mu_tol.argtypes = [_dp, _dp, _dp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_double, ctypes.c_double]
        L.orc_nmf_mu_tol.restype = ctypes.c_int
        # Brunet KL-divergence MU (brunet_oracle.c; parity unpinned vs the reference, see its header)
        L.orc_rmt_seed.argtypes = [ctypes.POINTER(_RMTState), ctypes.c_uint32]
        L.orc_rmt_unif.argtypes = [ctypes.POINTER(_RMTState)]
        L.orc_rmt_unif.restype = ctypes.c_double
        L.orc_brunet_init.argtypes = [ctypes.c_uint32, ctypes.c_int, ctypes.c_int, ctypes.c_int, _dp, _dp]
        L.orc_brunet.argtypes = [_dp, _dp, _dp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                 ctypes.c_int, ctypes.c_void_p]
        L.orc_brunet.restype = ctypes.c_int
        self.L = L

    def runif(self, seed: int, count: int) -> np.ndarray:
        """set.seed(seed); runif(count) (R's Mersenne-Twister restated)."""
        st = _RMTState()
        self.L.orc_rmt_seed(ctypes.byref(st), seed & 0xFFFFFFFF)
        return np.array([self.L.orc_rmt_unif(ctypes.byref(st)) for _ in range(count)], dtype=np.float64)

    def brunet_init(self, seed: int, m: int, n: int, k: int):
        W = np.zeros((m, k), dtype=np.float64, order="F")
        H = np.zeros((k, n), dtype=np.float64, order="F")
        self.L.orc_brunet_init(seed & 0xFFFFFFFF, m, n, k, _d(W), _d(H))
        return W, H

    def brunet(self, A, W, H, maxiter: int, stopconv: int = 40, stopfreq: int = 10, want_error: bool = False):
        """NMF.div (Brunet KL MU) -> (W, H, t[, error.v])."""
        A = np.asfortranarray(A, dtype=np.float64)
        W = np.array(W, dtype=np.float64, order="F", copy=True)
        H = np.array(H, dtype=np.float64, order="F", copy=True)
        m, n = A.shape
        k = W.shape[1]
        err = np.zeros(maxiter, dtype=np.float64) if want_error else None
        t = self.L.orc_brunet(_d(A), _d(W), _d(H), m, n, k, maxiter, stopconv, stopfreq,
                              err.ctypes.data_as(ctypes.c_void_p) if want_error else None)
        return (W, H, t, err[:t]) if want_error else (W, H, t)

    def rand_stream(self, seed: int, count: int) -> np.ndarray:
        st = _RandState()
        self.L.orc_srand(ctypes.byref(st), seed)
        return np.array([self.L.orc_rand(ctypes.byref(st)) for _ in range(count)], dtype=np.int64)

    def init_restart(self, seed: int, m: int, n: int, k: int):
        W = np.zeros((m, k), dtype=np.float64, order="F")
        H = np.zeros((k, n), dtype=np.float64, order="F")
        self.L.orc_init_restart(seed, m, n, k, _d(W), _d(H))
        return W, H

    def nmf_mu(self, A: np.ndarray, W: np.ndarray, H: np.ndarray, maxiter: int, stop_rule: int = STOP_REF_COMPAT):
        A = np.asfortranarray(A, dtype=np.float64)
        W = np.array(W, dtype=np.float64, order="F", copy=True)
        H = np.array(H, dtype=np.float64, order="F", copy=True)
        m, n = A.shape
        k = W.shape[1]
        it = self.L.orc_nmf_mu(_d(A), _d(W), _d(H), m, n, k, maxiter, stop_rule)
        return W, H, it

    def nmf_mu_tol(self, A, W, H, maxiter: int, TolX: float = 1e-4, TolFun: float = 1e-4):
        """MU under the nmf_als.c:304-349 TolX/TolFun test -> (W, H, iterations)."""
        A = np.asfortranarray(A, dtype=np.float64)
        W = np.array(W, dtype=np.float64, order="F", copy=True)
        H = np.array(H, dtype=np.float64, order="F", copy=True)
        m, n = A.shape
        k = W.shape[1]
        it = self.L.orc_nmf_mu_tol(_d(A), _d(W), _d(H), m, n, k, maxiter, TolX, TolFun)
        return W, H, it

    def labels(self, H: np.ndarray, rule: int = LABEL_ARGMAX) -> np.ndarray:
        H = np.asfortranarray(H, dtype=np.float64)
        k, n = H.shape
        out = np.zeros(n, dtype=np.int32)
        self.L.orc_labels(_d(H), k, n, rule, _i(out))
        return out

    def counts(self, labels: np.ndarray) -> np.ndarray:
        labels = np.ascontiguousarray(labels, dtype=np.int32)
        R, n = labels.shape
        out = np.zeros((n, n), dtype=np.int32, order="F")
        self.L.orc_counts(_i(labels), R, n, _i(out))
        return out

    def calculate_norm(self, A, W, H):
        A = np.asfortranarray(A, dtype=np.float64)
        W = np.asfortranarray(W, dtype=np.float64)
        H = np.asfortranarray(H, dtype=np.float64)
        m, n = A.shape
        k = W.shape[1]
        d = np.zeros((m, n), dtype=np.float64, order="F")
        v = self.L.orc_calculate_norm(_d(A), _d(W), _d(H), _d(d), m, n, k)
        return v, d

    def calculate_maxchange(self, mat, mat0, sqrteps=2.0 ** -26.5):
        mat = np.asfortranarray(mat, dtype=np.float64)
        mat0 = np.array(mat0, dtype=np.float64, order="F", copy=True)
        m, n = mat.shape
        v = self.L.orc_calculate_maxchange(_d(mat), _d(mat0), m, n, sqrteps)
        return v, mat0


class RefLib:
    """The reference's own libnmf (compiled from /root/reference sources by `make -C oracle ref`)."""

    def __init__(self, path: str = REF_SO):
        if not os.path.exists(path):
            raise FileNotFoundError(f"{path} missing: run `make -C oracle ref` (needs /root/reference)")
        # use_errno: the reference's generateMatrix returns early, leaving W/H untouched, whenever errno is
        # non-zero on entry (generatematrix.c:86-90 under ERROR_CHECKING, common.h:25); generate_ran clears
        # the ctypes-private errno before every call and checks that W/H came back filled.
        L = ctypes.CDLL(path, mode=os.RTLD_LAZY, use_errno=True)
        ip = ctypes.POINTER(ctypes.c_int)
        L.nmf_mu.argtypes = [_dp, _dp, _dp, ip, ip, ip, ip, _dp, _dp]
        L.nmf_mu.restype = ctypes.c_double
        L.randnumber.argtypes = [ctypes.c_int, ctypes.c_int]
        L.randnumber.restype = ctypes.c_double
        L.generateMatrix.argtypes = [ip, ip, ip, ip, ip, ip, _dp, _dp, _dp, ctypes.c_void_p]
        L.generateMatrix.restype = None
        L.calculateNorm.argtypes = [_dp, _dp, _dp, _dp, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.calculateNorm.restype = ctypes.c_double
        L.calculateMaxchange.argtypes = [_dp, _dp, ctypes.c_int, ctypes.c_int, ctypes.c_double]
        L.calculateMaxchange.restype = ctypes.c_double
        self.L = L
        self.libc = ctypes.CDLL(None)
        self.libc.srand.argtypes = [ctypes.c_uint]
        # randnumber() calls srand(time(NULL)) on its first use (randnumber.c:29-33): trip it once so
        # that an explicit srand(seed) afterwards defines the stream.
        self.L.randnumber(0, 1)

    def seed(self, seed: int):
        self.libc.srand(seed)

    def generate_ran(self, seed: int, m: int, n: int, k: int, lo: int = 0, hi: int = 1):
        self.seed(seed)
        W = np.zeros((m, k), dtype=np.float64, order="F")
        H = np.zeros((k, n), dtype=np.float64, order="F")
        c = ctypes.c_int
        init = c(0)  # ran
        ctypes.set_errno(0)
        self.L.generateMatrix(ctypes.byref(c(m)), ctypes.byref(c(n)), ctypes.byref(c(k)), ctypes.byref(init),
                              ctypes.byref(c(lo)), ctypes.byref(c(hi)), _d(W), _d(H), None, None)
        if not (W.any() and H.any()):
            raise RuntimeError(f"reference generateMatrix left W/H unfilled (errno {ctypes.get_errno()} on return; "
                               "generatematrix.c:86-90 returns early when errno is set on entry)")
        return W, H

    def nmf_mu(self, A, W, H, maxiter: int, tol: float = 1e-4):
        """Calls the reference nmf_mu.  maxiter must be even (nmf_mu.c:241-242 pointer swap) and the
        h0 buffer is padded with zeros to max(k*n, n*n) so that the stability check's reads past k*n
        (nmf_mu.c:259) are defined.  Returns (W, H, iterations)."""
        assert maxiter % 2 == 0
        A = np.asfortranarray(A, dtype=np.float64)
        m, n = A.shape
        k = W.shape[1]
        w0 = np.array(W, dtype=np.float64, order="F", copy=True)
        hbuf = np.zeros(max(k * n, n * n), dtype=np.float64)
        hbuf[: k * n] = np.asarray(H, dtype=np.float64).reshape(-1, order="F")
        c = ctypes.c_int
        mi = c(maxiter)
        tx = ctypes.c_double(tol)
        tf = ctypes.c_double(tol)
        self.L.nmf_mu(_d(A), _d(w0), _d(hbuf), ctypes.byref(c(m)), ctypes.byref(c(n)), ctypes.byref(c(k)),
                      ctypes.byref(mi), ctypes.byref(tx), ctypes.byref(tf))
        Hout = hbuf[: k * n].reshape((k, n), order="F").copy(order="F")
        return w0, Hout, mi.value
