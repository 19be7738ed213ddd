"""The R bindings of INTEGRATION.md sections 2 and 6 as code (examples/r_nmfc.c, built by build() into
examples/r_nmfc.so), driven through ctypes with R's .C convention: EVERY argument a pointer to a vector -- integer
vectors as int32 arrays, double vectors as float64 arrays, outputs preallocated (integer(nk*n*n), double(nk*n*n),
...) and filled in place.  What they replace: runNMFinJobs' fan-out + consensus (nmf.r:106-144) and the BROAD
nmfconsensus() per-k loop (test_nmf.r:29).

Checked against the reference: runExample()'s grid (nmf.r:6-14: k = 2:5, 10 restarts, seed 123; golden_runexample.npz,
the reference's own nmf_mu on all 40 jobs) and test_nmf.r's C1 job (k = 2:5, 5 restarts, seed 123: the first 20 jobs
of golden.npz's C1 sweep) -- iterations, labels, counts and consensus bit for bit under both label rules.  Brunet:
against the oracle restatement (oracle/brunet_oracle.c; the BROAD script is not in the reference).
"""
import ctypes
import os

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

SO = os.path.join(ROOT, "examples", "r_nmfc.so")
I32P = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
F64P = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")


@pytest.fixture(scope="module")
def rlib():
    assert os.path.exists(SO), "examples/r_nmfc.so missing: build() builds it (make -C examples r_nmfc.so)"
    lib = ctypes.CDLL(SO)
    lib.r_nmfc_sweep.argtypes = [F64P] + [I32P] * 9 + [I32P, F64P, I32P, I32P, I32P]
    lib.r_nmfc_sweep.restype = None
    lib.r_nmfc_brunet.argtypes = [F64P] + [I32P] * 9 + [I32P, F64P, I32P, I32P]
    lib.r_nmfc_brunet.restype = None
    return lib


def iv(*x):
    """as.integer(...): an R integer vector"""
    return np.array(x, dtype=np.int32)


def r_sweep(lib, A, ks, R, seed, label_rule, maxiter=10000, init_stream=0):
    m, n = A.shape
    nk = len(ks)
    a = np.ascontiguousarray(np.asfortranarray(A).ravel(order="F"))   # as.double(A): column-major
    counts = np.zeros(nk * n * n, dtype=np.int32)
    cons = np.zeros(nk * n * n)
    labels = np.zeros(nk * R * n, dtype=np.int32)
    iters = np.zeros(nk * R, dtype=np.int32)
    rc = iv(-7)
    lib.r_nmfc_sweep(a, iv(m), iv(n), iv(*ks), iv(nk), iv(R), iv(maxiter), iv(seed), iv(label_rule), iv(init_stream),
                     counts, cons, labels, iters, rc)
    assert rc[0] == 0
    # R reads them back as array(res$counts, c(n, n, nk)): k-major blocks of n x n
    return counts.reshape(nk, n, n), cons.reshape(nk, n, n), labels.reshape(nk * R, n), iters


@pytest.mark.parametrize("rule", [0, 1])
def test_r_sweep_runexample_vs_reference(rlib, golden, rule):
    """runExample(): runNMFinJobs(gct, k = 2:5, num.clusterings = 10, maxniter = 10000, seed = 123, njobs = 4)."""
    with np.load(os.path.join(ROOT, "tests", "golden", "golden_runexample.npz"), allow_pickle=False) as z:
        g = {k: z[k] for k in z.files}
    counts, cons, labels, iters = r_sweep(rlib, golden["A_gct"], [2, 3, 4, 5], 10, 123, rule)
    name = "argmax" if rule == 0 else "rorder"
    assert np.array_equal(iters, g["rx_iters"])
    assert np.array_equal(labels, g[f"rx_labels_{name}"])
    assert np.array_equal(counts, g[f"rx_counts_{name}"])
    assert np.array_equal(cons, g[f"rx_consensus_{name}"])


@pytest.mark.parametrize("rule", [0, 1])
def test_r_sweep_test_nmf_r_job_vs_reference(rlib, golden, rule):
    """test_nmf.r:27: runNMFinJobs(gct, k = 2:5, num.clusterings = 5, maxniter = 10000, seed = 123, njobs = 1) -- the
    first 20 jobs of the reference's C1 sweep (same job ids, same seeds)."""
    ks, R = [2, 3, 4, 5], 5
    counts, cons, labels, iters = r_sweep(rlib, golden["A_gct"], ks, R, 123, rule)
    name = "argmax" if rule == 0 else "rorder"
    nj = len(ks) * R
    assert np.array_equal(iters, golden["c1_iters"][:nj])
    L = golden[f"c1_labels_{name}"][:nj]
    assert np.array_equal(labels, L)
    jk = golden["c1_job_k"][:nj]
    for i, k in enumerate(ks):
        C = sum((l[:, None] == l[None, :]).astype(np.int32) for l in L[jk == k])
        assert np.array_equal(counts[i], C)
        assert np.array_equal(cons[i], C / R)


def test_r_sweep_bad_rank_reports_error(rlib, golden):
    A = golden["A_gct"]
    m, n = A.shape
    out = [np.zeros(n * n, dtype=np.int32), np.zeros(n * n), np.zeros(n, dtype=np.int32), np.zeros(1, dtype=np.int32)]
    rc = iv(0)
    rlib.r_nmfc_sweep(np.ascontiguousarray(A.ravel(order="F")), iv(m), iv(n), iv(1), iv(1), iv(1), iv(10), iv(1),
                      iv(0), iv(0), *out, rc)
    assert rc[0] != 0   # nmf.r:107-108 rejects k = 1; the sweep reports it through rc


def test_r_brunet_vs_oracle(rlib, golden, oracle):
    """nmfconsensus(eset, k.init = 2, k.final = 4, num.clusterings = 4, maxniter = 300, stopconv = 40, stopfreq = 10)
    through r_nmfc_brunet: iterations, counts and consensus against the restated NMF.div run job by job."""
    A = golden["A_gct"]
    m, n = A.shape
    ks, R, rseed, maxiter = [2, 3, 4], 4, 123456789, 300
    nk = len(ks)
    counts = np.zeros(nk * n * n, dtype=np.int32)
    cons = np.zeros(nk * n * n)
    iters = np.zeros(nk * R, dtype=np.int32)
    rc = iv(-7)
    rlib.r_nmfc_brunet(np.ascontiguousarray(A.ravel(order="F")), iv(m), iv(n), iv(*ks), iv(nk), iv(R), iv(maxiter),
                       iv(rseed), iv(40), iv(10), counts, cons, iters, rc)
    assert rc[0] == 0
    counts, cons = counts.reshape(nk, n, n), cons.reshape(nk, n, n)
    for ki, k in enumerate(ks):
        labs = []
        for i in range(R):
            W0, H0 = oracle.brunet_init(rseed + i + 1, m, n, k)
            _W, H, t = oracle.brunet(A, W0, H0, maxiter, 40, 10)
            assert iters[ki * R + i] == t, (k, i)
            labs.append(oracle.labels(H, 0))
        C = oracle.counts(np.array(labs, dtype=np.int32))
        assert np.array_equal(counts[ki], C)
        assert np.array_equal(cons[ki], C / R)
