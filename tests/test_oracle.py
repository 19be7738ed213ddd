"""The oracle (our C restatement, oracle/nmf_oracle.c) pinned against the reference's golden vectors
(tests/golden/golden.npz, produced by the reference's own C code) and against libc itself."""
import ctypes
import os

import numpy as np
import pytest

from conftest import ROOT, relfro

TOL = 1e-9


def test_rand_stream_matches_libc_and_golden(golden, oracle):
    libc = ctypes.CDLL(None)
    libc.srand.argtypes = [ctypes.c_uint]
    for s, draws in zip(golden["rand_seeds"], golden["rand_draws"]):
        ours = oracle.rand_stream(int(s), draws.size)
        assert np.array_equal(ours, draws), int(s)
        libc.srand(int(s))
        assert [libc.rand() for _ in range(50)] == list(draws[:50])


def test_randnumber_values(golden, oracle):
    # randnumber(0, 1) = rand() / (double)RAND_MAX (randnumber.c:34), bit-exact
    W, H = oracle.init_restart(123, 64, 0, 1)
    assert np.array_equal(W[:, 0], golden["randnumber_seed123"])


@pytest.mark.parametrize("k", [2, 3, 4, 5])
def test_init_bitexact(golden, oracle, k):
    W, H = oracle.init_restart(123, 1000, 40, k)
    assert np.array_equal(W, golden[f"init_k{k}_W"])
    assert np.array_equal(H, golden[f"init_k{k}_H"])
    W, H = oracle.init_restart(123, 5, 4, 2)
    assert np.array_equal(W, golden["init_small_W"]) and np.array_equal(H, golden["init_small_H"])


@pytest.mark.parametrize("k", [2, 3, 4, 5])
def test_fixed_iterations(golden, oracle, k):
    A = golden["A_gct"]
    for T in (2, 10, 200, 398):
        W, H, it = oracle.nmf_mu(A, golden[f"init_k{k}_W"], golden[f"init_k{k}_H"], T, 0)
        assert it == T
        assert relfro(W, golden[f"fixed_k{k}_T{T}_W"]) < TOL
        assert relfro(H, golden[f"fixed_k{k}_T{T}_H"]) < TOL


@pytest.mark.parametrize("k", [2, 3, 4, 5])
def test_ref_compat_exit(golden, oracle, k):
    A = golden["A_gct"]
    W, H, it = oracle.nmf_mu(A, golden[f"init_k{k}_W"], golden[f"init_k{k}_H"], 10000, 1)
    assert it == int(golden[f"refc_k{k}_iter"])
    assert relfro(W, golden[f"refc_k{k}_W"]) < TOL
    assert relfro(H, golden[f"refc_k{k}_H"]) < TOL


def test_c1_sweep(golden, oracle):
    """runNMFinJobs semantics (nmf.r:106-143) on the bundled gct: per-job seeds, exits, labels, counts."""
    A = golden["A_gct"]
    m, n = A.shape
    iters, Lam, Lro = [], [], []
    for jk, js in zip(golden["c1_job_k"], golden["c1_job_seed"]):
        W0, H0 = oracle.init_restart(int(js), m, n, int(jk))
        W, H, it = oracle.nmf_mu(A, W0, H0, 10000, 1)
        iters.append(it)
        Lam.append(oracle.labels(H, 0))
        Lro.append(oracle.labels(H, 1))
    assert np.array_equal(np.array(iters), golden["c1_iters"])
    Lam, Lro = np.array(Lam), np.array(Lro)
    assert np.array_equal(Lam, golden["c1_labels_argmax"])
    assert np.array_equal(Lro, golden["c1_labels_rorder"])
    jk = golden["c1_job_k"]
    for k in golden["c1_ks"]:
        assert np.array_equal(oracle.counts(Lam[jk == k]), golden[f"c1_counts_argmax_k{k}"])
        assert np.array_equal(oracle.counts(Lro[jk == k]), golden[f"c1_counts_rorder_k{k}"])


def test_norm_maxchange(golden, oracle):
    v, d = oracle.calculate_norm(golden["norm_a"], golden["norm_w"], golden["norm_h"])
    assert abs(v - float(golden["norm_value"])) < 1e-14
    assert relfro(d, golden["norm_d"]) < 1e-14
    v, m0 = oracle.calculate_maxchange(golden["maxchange_mat"], golden["maxchange_mat0"])
    assert v == float(golden["maxchange_value"])
    assert np.array_equal(m0, golden["maxchange_mat0_after"])


def test_golden_labels_have_margin(golden):
    # labels are only meaningful as a bit-exact target when no column is a near-tie
    assert golden["c1_margin_argmax"].min() > 1e-6


def test_tolx_rule_oracle(oracle, golden):
    """orc_nmf_mu_tol: the nmf_als.c:304-349 convergence test around the MU update."""
    A = golden["A_gct"]
    W0, H0 = oracle.init_restart(123, A.shape[0], A.shape[1], 3)
    # TolX = 0 never fires and TolFun < 1 only on an exactly-zero residual: plain fixed iterations
    W, H, it = oracle.nmf_mu_tol(A, W0, H0, 20, 0.0, 1e-4)
    Wf, Hf, _ = oracle.nmf_mu(A, W0, H0, 20, 0)
    assert it == 20 and np.array_equal(W, Wf) and np.array_equal(H, Hf)
    # TolFun >= 1: dnorm <= TolFun * dnorm0 with dnorm0 == dnorm holds at the first check (iteration 2)
    assert oracle.nmf_mu_tol(A, W0, H0, 100, 0.0, 1.0)[2] == 2
    # a real TolX stop: even, and the max-change at that iteration is below TolX (NumPy restatement)
    W, H, it = oracle.nmf_mu_tol(A, W0, H0, 5000, 1e-3, 1e-4)
    assert 2 < it < 5000 and it % 2 == 0
    Wp, Hp, _ = oracle.nmf_mu(A, W0, H0, it - 1, 0)
    sq = 2.0 ** -26.5
    dw = np.max(np.abs(Wp - W)) / (sq + np.max(np.abs(Wp)))
    dh = np.max(np.abs(Hp - H)) / (sq + np.max(np.abs(Hp)))
    assert max(dw, dh) < 1e-3


@pytest.mark.parametrize("tag", ["c2", "c1r"])
def test_c2_and_runif_sweeps_subset(golden, golden_c2, oracle, tag):
    """The restatement against the reference's own nmf_mu on BASELINE configs[1] (C2, libnmf init) and on
    the C1 sweep under nmf.r:37-38's runif init (tests/golden/make_golden_c2.py): the first 2 jobs of
    every k -- exits, labels and H."""
    g = golden_c2
    A = g["c2_A"] if tag == "c2" else golden["A_gct"]
    A = np.asfortranarray(A)
    m, n = A.shape
    ks = [int(k) for k in g[f"{tag}_ks"]]
    seed = int(g[f"{tag}_seed"])
    for k in ks:
        for q, j in enumerate(g[f"{tag}_Hjobs_k{k}"]):
            s = seed + int(j)
            W0, H0 = oracle.init_restart(s, m, n, k) if tag == "c2" else oracle.brunet_init(s, m, n, k)
            W, H, it = oracle.nmf_mu(A, W0, H0, 10000, 1)
            assert it == int(g[f"{tag}_iters"][j]), (k, j)
            assert np.array_equal(oracle.labels(H, 0), g[f"{tag}_labels_argmax"][j])
            assert np.array_equal(oracle.labels(H, 1), g[f"{tag}_labels_rorder"][j])
            assert relfro(H, g[f"{tag}_H_k{k}"][q]) < TOL


@pytest.mark.skipif(not os.path.exists(os.path.join(ROOT, "oracle", "_ref", "libnmf_ref.so")),
                    reason="oracle/_ref not built (needs /root/reference)")
def test_reflib_generate_ran_is_errno_safe(golden):
    """The reference's generateMatrix returns early, W/H untouched, whenever errno is set on entry
    (generatematrix.c:86-90, ERROR_CHECKING at common.h:25).  RefLib.generate_ran clears errno first, so a
    stale EISDIR from an earlier call still gives the golden init; the raw call with errno set shows the
    early return (and generate_ran would raise on an unfilled W/H)."""
    import ctypes
    import errno
    from pyoracle import RefLib, _d
    ref = RefLib()
    ctypes.set_errno(errno.EISDIR)
    W, H = ref.generate_ran(123, 1000, 40, 3)
    assert np.array_equal(W, golden["init_k3_W"]) and np.array_equal(H, golden["init_k3_H"])
    # the reference's own behaviour, called raw with errno set on entry: nothing is written
    ref.seed(123)
    W2 = np.zeros((1000, 3), order="F")
    H2 = np.zeros((3, 40), order="F")
    c = ctypes.c_int
    ctypes.set_errno(errno.EISDIR)
    ref.L.generateMatrix(ctypes.byref(c(1000)), ctypes.byref(c(40)), ctypes.byref(c(3)), ctypes.byref(c(0)),
                         ctypes.byref(c(0)), ctypes.byref(c(1)), _d(W2), _d(H2), None, None)
    assert not W2.any() and not H2.any()


def test_golden_c4_covers_every_shard():
    """Every shard of the 8-GPU C4 job (distributed.shard_range(14000, r, 8)) holds reference jobs of every k in
    tests/golden/golden_c4.npz (make_golden_c4.py), and the rank-3 shard's golden jobs carry their final H."""
    import os

    from nmfconsensus_amd.distributed import shard_range
    path = os.path.join(os.path.dirname(__file__), "golden", "golden_c4.npz")
    with np.load(path, allow_pickle=False) as z:
        ids, ks, job_k = z["c4_job_id"], z["c4_ks"], z["c4_job_k"]
        hjobs = np.concatenate([z[f"c4_Hjobs_k{int(k)}"] for k in ks])
        R = int(z["c4_R_total"])
    nk = len(ks)
    assert np.array_equal(job_k, ks[ids % nk])
    for r in range(8):
        jb, je = shard_range(nk * R, r, 8)
        inside = (ids >= jb) & (ids < je)
        assert set(job_k[inside].tolist()) == set(ks.tolist()), r
    jb, je = shard_range(nk * R, 3, 8)
    pos3 = set(np.where((ids >= jb) & (ids < je))[0].tolist())
    assert pos3 and pos3 <= set(hjobs.tolist())
