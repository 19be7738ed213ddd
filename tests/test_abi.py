"""The C-ABI library (nmfconsensus_amd/libnmf.so) loads and exports every symbol include/*.h declares;
host-only entry points behave like the reference's.  No GPU compute here."""
import ctypes
import errno
import os
import re

import numpy as np
import pytest

from conftest import ROOT

HEADERS = [os.path.join(ROOT, "include", h) for h in ("libnmf_compat.h", "nmfc.h")]


def declared_functions():
    names = []
    for h in HEADERS:
        txt = open(h).read()
        txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
        txt = re.sub(r"//[^\n]*", "", txt)
        for mt in re.finditer(r"^[A-Za-z_][\w\s\*]*?\b([A-Za-z_]\w*)\s*\(([^;{}]*)\)\s*;", txt, flags=re.M):
            if mt.group(0).lstrip().startswith("typedef"):
                continue
            names.append(mt.group(1))
    return sorted(set(names))


@pytest.fixture(scope="module")
def L():
    from nmfconsensus_amd import _lib
    return _lib.lib()


def test_headers_parse():
    names = declared_functions()
    for must in ("nmf_mu", "set_default_opts", "checkArguments", "generateMatrix", "randnumber", "calculateNorm",
                 "calculateMaxchange", "checkMatrices", "nmfc_engine_run", "nmfc_cophenetic"):
        assert must in names


def test_exports_every_declared_symbol(L):
    for name in declared_functions():
        assert hasattr(L, name), name
    from nmfconsensus_amd import _lib
    assert set(declared_functions()) == set(_lib.EXPORTED)


def test_soname_is_libnmf(L):
    out = os.popen(f"readelf -d {os.path.join(ROOT, 'nmfconsensus_amd', 'lib', 'libnmf.so')}").read()
    assert "Library soname: [libnmf.so]" in out


def test_set_default_opts_and_check_arguments():
    from nmfconsensus_amd import libnmf
    o = libnmf.set_default_opts()
    assert (o.rep, o.init, o.min_init, o.max_init) == (1, 0, 0, 1)
    assert o.w_out == b"final_w.matrix" and o.h_out == b"final_h.matrix"
    assert o.TolX == 1e-4 and o.TolFun == 1e-4
    assert (o.nndsvd_maxiter, o.nndsvd_blocksize, o.nndsvd_tol, o.nndsvd_ncv) == (-1, 64, 2e-16, -1)
    assert libnmf.checkArguments(b"a.matrix", 3, 100, None, None, o) == 0
    assert libnmf.checkArguments(None, 3, 100, None, None, o) == 1
    # checkarguments.c:61-65 sets errno = EDOM: read it through a use_errno handle of the same library
    from nmfconsensus_amd import _lib
    Le = ctypes.CDLL(_lib.LIB_PATH, use_errno=True)
    Le.checkArguments.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_char_p, ctypes.c_char_p,
                                  ctypes.POINTER(_lib.OptionsT)]
    ctypes.set_errno(0)
    assert Le.checkArguments(None, 3, 100, None, None, ctypes.byref(o)) == 1
    assert ctypes.get_errno() == errno.EDOM
    ctypes.set_errno(0)
    assert Le.checkArguments(b"a.matrix", 3, 100, None, None, ctypes.byref(o)) == 0
    assert ctypes.get_errno() == 0
    o.TolX = -1.0
    assert libnmf.checkArguments(b"a.matrix", 3, 100, None, None, o) == 1


def test_check_matrices():
    from nmfconsensus_amd import libnmf
    a = np.ones((4, 3))
    w = np.ones((4, 2))
    h = np.ones((2, 3))
    assert libnmf.checkMatrices(a, w, h) == 0
    w[2, 1] = -1.0
    assert libnmf.checkMatrices(a, w, h) == 1


@pytest.mark.parametrize("k", [0, 21])
def test_nmf_mu_rank_limit(capfd, k):
    # libnmf_compat.h: k outside 1..min(m, n) is refused before any device work, factors untouched
    from nmfconsensus_amd import libnmf
    rng = np.random.default_rng(0)
    a = rng.random((40, 20)) + 0.1
    w0, h0 = rng.random((40, k)), rng.random((k, 20))
    w_in, h_in = w0.copy(), h0.copy()
    out = libnmf.nmf_mu(a, w0, h0, 100)
    assert out["ret"] == -1 and out["maxiter"] == 100
    assert np.array_equal(out["w0"], w_in) and np.array_equal(out["h0"], h_in)
    err = capfd.readouterr().err
    assert f"Error in nmf_mu: k={k} unsupported (need 1 <= k <= min(m, n))" in err


def test_generate_matrix_follows_libc_stream(golden):
    # generateMatrix(ran) draws W then H from libc rand() (generatematrix.c:131-137): after the first
    # randnumber call trips srand(time) (randnumber.c:29-33), srand(123) reproduces the golden init.
    from nmfconsensus_amd import libnmf
    libc = ctypes.CDLL(None)
    libc.srand.argtypes = [ctypes.c_uint]
    libnmf.randnumber(0, 1)
    libc.srand(123)
    W, H = libnmf.generateMatrix(1000, 40, 3)
    assert np.array_equal(W, golden["init_k3_W"]) and np.array_equal(H, golden["init_k3_H"])


def test_cophenetic_vs_scipy():
    from scipy.cluster.hierarchy import cophenet, fcluster, linkage
    from scipy.spatial.distance import squareform
    from nmfconsensus_amd.nmf import cophenetic, cutree
    rng = np.random.default_rng(11)
    for n, groups in ((40, 2), (57, 3), (120, 5)):
        lab = rng.integers(0, groups, size=n)
        C = (lab[:, None] == lab[None, :]).astype(float) * 0.8 + rng.random((n, n)) * 0.2
        C = (C + C.T) / 2
        np.fill_diagonal(C, 1.0)
        rho, order, merge, height = cophenetic(C)
        D = squareform(1.0 - C, checks=False)
        Z = linkage(D, "average")
        ref, _ = cophenet(Z, D)
        assert abs(rho - ref) < 1e-12
        assert np.allclose(np.sort(height), np.sort(Z[:, 2]), rtol=0, atol=1e-12)
        assert sorted(order) == list(range(1, n + 1))
        mem = cutree(merge, groups)
        ref_mem = fcluster(Z, groups, criterion="maxclust")
        # same partition up to relabelling
        pairs = {(a, b) for a, b in zip(mem, ref_mem)}
        assert len(pairs) == groups
        assert mem[0] == 1


def test_cutree_numbering():
    from nmfconsensus_amd.nmf import cophenetic, cutree
    C = np.array([[1, 1, 0, 0], [1, 1, 0, 0], [0, 0, 1, 1], [0, 0, 1, 1]], dtype=float)
    rho, order, merge, height = cophenetic(C)
    assert rho == pytest.approx(1.0)
    assert list(cutree(merge, 2)) == [1, 1, 2, 2]
    assert list(cutree(merge, 4)) == [1, 2, 3, 4]
    assert list(cutree(merge, 1)) == [1, 1, 1, 1]


def test_cophenetic_batch_equals_single():
    from nmfconsensus_amd.nmf import cophenetic, cophenetic_batch
    rng = np.random.default_rng(3)
    n, nk = 61, 5
    Cs = []
    for q in range(nk):
        lab = rng.integers(0, q + 2, size=(20, n))
        C = np.mean(lab[:, :, None] == lab[:, None, :], axis=0)   # quantised to 1/20: many ties
        Cs.append(C)
    Cs = np.array(Cs)
    rho, order, merge, height = cophenetic_batch(Cs, nthreads=3)
    for q in range(nk):
        r1, o1, m1, h1 = cophenetic(Cs[q])
        assert rho[q] == r1 and np.array_equal(order[q], o1) and np.array_equal(merge[q], m1)
        assert np.array_equal(height[q], h1)

def test_cophenetic_batch_symmetric_fast_path():
    # consensus matrices are symmetric: the row-major stack passed as is gives the same results
    from nmfconsensus_amd.nmf import cophenetic_batch
    rng = np.random.default_rng(5)
    n, nk = 47, 3
    lab = rng.integers(0, 4, size=(nk, 25, n))
    Cs = np.array([np.mean(l[:, :, None] == l[:, None, :], axis=0) for l in lab])
    a = cophenetic_batch(Cs, nthreads=2)
    b = cophenetic_batch(Cs, nthreads=2, symmetric=True)
    for x, y in zip(a, b):
        assert np.array_equal(x, y)


def test_solo_path_shape_limits():
    """The solo path's range (nmfc_mu_solo_fits) and its refusal of shapes outside it."""
    import ctypes
    from nmfconsensus_amd import _lib
    L = _lib.lib()   # no device work: the range check comes first
    for m, n, k in ((1000, 40, 2), (1024, 40, 3), (1000, 40, 4), (1000, 40, 5), (1024, 40, 8), (8, 8, 8)):
        assert L.nmfc_mu_solo_fits(m, n, k), (m, n, k)
    for m, n, k in ((1000, 41, 2), (1025, 40, 2), (1000, 41, 3), (1000, 41, 4), (1000, 40, 9), (1000, 41, 8),
                    (1025, 40, 6), (1000, 40, 1), (3, 2, 3), (7, 40, 8)):
        assert not L.nmfc_mu_solo_fits(m, n, k), (m, n, k)
    dp = ctypes.POINTER(ctypes.c_double)
    A = np.ones((1000, 41), order="F")
    W, H = np.ones((1000, 2), order="F"), np.ones((2, 41), order="F")
    it, early = ctypes.c_int(0), ctypes.c_int(0)
    rc = L.nmfc_mu_solo(A.ctypes.data_as(dp), 1000, 41, 2, 10, 1, W.ctypes.data_as(dp), H.ctypes.data_as(dp),
                        W.ctypes.data_as(dp), H.ctypes.data_as(dp), ctypes.byref(it), ctypes.byref(early))
    assert rc == -1 and "bad arguments" in _lib.last_error()


def test_generate_matrix_fills_despite_stale_errno(golden, monkeypatch):
    """The reference's generateMatrix returns early, W/H unfilled, when errno is set on entry (generatematrix.c:86-90);
    the drop-in fills them anyway, NMFC_GENERATE_ERRNO_COMPAT=1 restores the early return."""
    import errno
    from nmfconsensus_amd import _lib
    L = ctypes.CDLL(os.path.join(ROOT, "nmfconsensus_amd", "lib", "libnmf.so"), use_errno=True)
    libc = ctypes.CDLL(None)
    libc.srand.argtypes = [ctypes.c_uint]
    L.randnumber.argtypes = [ctypes.c_int, ctypes.c_int]
    L.randnumber.restype = ctypes.c_double
    L.randnumber(0, 1)
    dp = ctypes.POINTER(ctypes.c_double)
    c = ctypes.c_int

    def gen():
        W = np.zeros((1000, 3), order="F")
        H = np.zeros((3, 40), order="F")
        libc.srand(123)
        ctypes.set_errno(errno.EISDIR)
        L.generateMatrix(ctypes.byref(c(1000)), ctypes.byref(c(40)), ctypes.byref(c(3)), ctypes.byref(c(0)),
                         ctypes.byref(c(0)), ctypes.byref(c(1)), W.ctypes.data_as(dp), H.ctypes.data_as(dp), None, None)
        return W, H

    W, H = gen()
    assert np.array_equal(W, golden["init_k3_W"]) and np.array_equal(H, golden["init_k3_H"])
    monkeypatch.setenv("NMFC_GENERATE_ERRNO_COMPAT", "1")
    W, H = gen()
    assert not W.any() and not H.any()
    assert _lib.lib() is not None
