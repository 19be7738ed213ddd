"""GPU parity of the Brunet KL-divergence engine (nmfc_brunet_*, brunet.hip) against the C oracle
(oracle/brunet_oracle.c; parity vs the reference unpinned, see that file's header).

Bars as for the MU path: init bit-exact; W/H within 1e-9 relative Frobenius after a fixed count;
stop iterations, labels, connectivity counts and consensus bit-exact; results independent of the
restart shard and of the group a restart is batched in.
"""
import numpy as np
import pytest

from conftest import relfro

pytestmark = pytest.mark.gpu

TOL = 1e-9
NOSTOP = 10 ** 6   # stopconv no restart reaches: fixed iteration count


def oracle_job(O, A, k, seed, maxiter, stopconv=40, stopfreq=10):
    m, n = A.shape
    W0, H0 = O.brunet_init(seed, m, n, k)
    return O.brunet(A, W0, H0, maxiter, stopconv, stopfreq)


@pytest.fixture(scope="module")
def gct_brunet(golden):
    from nmfconsensus_amd.brunet import BrunetEngine
    eng = BrunetEngine(golden["A_gct"])
    yield eng
    eng.close()


@pytest.mark.parametrize("k", [2, 3, 4, 5, 10, 16])
def test_init_bitexact(gct_brunet, oracle, golden, k):
    m, n = golden["A_gct"].shape
    r = gct_brunet.run([k], 3, maxiter=1, seed=1000, want_factors=True, want_counts=False, stopconv=NOSTOP)
    # one iteration from the init: compare the init through the oracle at T=1 and directly via W_init
    for i in range(3):
        W0, H0 = oracle.brunet_init(1000 + i + 1, m, n, k)
        Wo, Ho, _ = oracle.brunet(golden["A_gct"], W0, H0, 1, NOSTOP)
        assert relfro(r.W[i], Wo) < TOL and relfro(r.H[i], Ho) < TOL


def test_init_stream_exact_via_caller_roundtrip(oracle):
    # the device init must equal the runif stream bit for bit: compare against caller-provided init
    # after 1 iteration (identical inputs => identical bits)
    from nmfconsensus_amd.brunet import BrunetEngine
    rng = np.random.default_rng(3)
    A = np.asfortranarray(rng.random((130, 17)) + 0.1)
    k = 4
    W0, H0 = oracle.brunet_init(123456789 + 1, 130, 17, k)
    with BrunetEngine(A) as eng:
        a = eng.run([k], 1, maxiter=3, stopconv=NOSTOP, want_factors=True, want_counts=False)
        b = eng.run([k], 1, maxiter=3, stopconv=NOSTOP, want_factors=True, want_counts=False, W_init=[W0], H_init=[H0])
    assert np.array_equal(a.W[0], b.W[0]) and np.array_equal(a.H[0], b.H[0])


@pytest.mark.parametrize("k", [2, 3, 4, 5])
@pytest.mark.parametrize("T", [1, 10, 100])
def test_fixed_iterations(gct_brunet, oracle, golden, k, T):
    A = golden["A_gct"]
    r = gct_brunet.run([k], 2, maxiter=T, seed=7, stopconv=NOSTOP, want_factors=True, want_counts=False)
    for i in range(2):
        Wo, Ho, t = oracle_job(oracle, A, k, 7 + i + 1, T, NOSTOP)
        assert r.iters[i] == T == t
        assert relfro(r.W[i], Wo) < TOL and relfro(r.H[i], Ho) < TOL, (k, T, i)


def test_consensus_sweep_matches_oracle(gct_brunet, oracle, golden):
    """C1-sized nmfconsensus run: k = 2..5, 6 restarts, default stop rule (stopconv 40 / stopfreq 10)."""
    A = golden["A_gct"]
    ks, R = [2, 3, 4, 5], 6
    r = gct_brunet.run(ks, R, maxiter=2000, seed=123456789, want_factors=True)
    n = A.shape[1]
    for ki, k in enumerate(ks):
        labs = []
        for i in range(R):
            Wo, Ho, t = oracle_job(oracle, A, k, 123456789 + i + 1, 2000)
            j = ki * R + i
            assert r.iters[j] == t, (k, i)
            assert relfro(r.W[j], Wo) < TOL and relfro(r.H[j], Ho) < TOL
            lo = oracle.labels(Ho, 0)
            assert np.array_equal(r.labels[j], lo)
            labs.append(lo)
        cnt = oracle.counts(np.array(labs, dtype=np.int32))
        assert np.array_equal(r.counts[ki], cnt)
        assert np.array_equal(r.consensus[ki], cnt / R)
    assert r.counts.shape == (len(ks), n, n)


def test_shard_and_group_invariance(gct_brunet):
    ks, R = [3, 7], 9
    full = gct_brunet.run(ks, R, maxiter=60, seed=11, stopconv=2, stopfreq=10, want_factors=True)
    a = gct_brunet.run(ks, R, maxiter=60, seed=11, stopconv=2, stopfreq=10, restart_end=4, want_factors=True)
    b = gct_brunet.run(ks, R, maxiter=60, seed=11, stopconv=2, stopfreq=10, restart_begin=4, want_factors=True)
    for ki in range(len(ks)):
        for i in range(R):
            src, s = (a, ki * 4 + i) if i < 4 else (b, ki * 5 + i - 4)
            j = ki * R + i
            assert np.array_equal(full.W[j], src.W[s]) and np.array_equal(full.H[j], src.H[s])
            assert full.iters[j] == src.iters[s]
        assert np.array_equal(full.counts[ki], a.counts[ki] + b.counts[ki])


@pytest.mark.parametrize("m,n,k", [(333, 77, 7), (130, 300, 13), (64, 5, 2), (1, 3, 2), (257, 256, 16)])
def test_ragged_shapes(oracle, m, n, k):
    from nmfconsensus_amd.brunet import BrunetEngine
    rng = np.random.default_rng(m * 1000 + n)
    A = np.asfortranarray(rng.random((m, n)) * 3.0)
    A[0, :] = 0.0   # a zero row
    T = 20
    with BrunetEngine(A) as eng:
        r = eng.run([k], 3, maxiter=T, seed=99, stopconv=NOSTOP, want_factors=True)
    for i in range(3):
        Wo, Ho, _ = oracle_job(oracle, A, k, 99 + i + 1, T, NOSTOP)
        assert relfro(r.W[i], Wo) < TOL and relfro(r.H[i], Ho) < TOL, (m, n, k, i)


def test_c3_shape_vs_oracle(oracle):
    """The full BASELINE configs[4] matrix shape (20000 x 500) at k = 10 for a few iterations."""
    from nmfconsensus_amd.brunet import BrunetEngine
    from nmfconsensus_amd.synthetic import planted_matrix
    A = planted_matrix(20000, 500)
    T = 3
    with BrunetEngine(A) as eng:
        r = eng.run([10], 2, maxiter=T, seed=5, stopconv=NOSTOP, want_factors=True, want_counts=False)
    Wo, Ho, _ = oracle_job(oracle, A, 10, 5 + 2, T, NOSTOP)
    assert relfro(r.W[1], Wo) < TOL and relfro(r.H[1], Ho) < TOL


def test_nmfconsensus_api(golden):
    from nmfconsensus_amd.brunet import NMF_div, nmfconsensus
    A = golden["A_gct"]
    out = nmfconsensus(A, 2, 3, 4, 500)
    assert set(out["rho"]) == {"2", "3"}
    for k in ("2", "3"):
        C = out["consensus"][k]
        assert np.allclose(np.diag(C), 1.0) and np.allclose(C, C.T)
    one = NMF_div(A, 3, maxniter=50, seed=42, stopconv=NOSTOP)
    assert one["t"] == 50 and one["W"].shape == (A.shape[0], 3) and one["H"].shape == (3, A.shape[1])


def test_bad_arguments():
    from nmfconsensus_amd.brunet import BrunetEngine
    A = np.ones((10, 4))
    with BrunetEngine(A) as eng:
        with pytest.raises(RuntimeError):
            eng.run([17], 1)
        with pytest.raises(RuntimeError):
            eng.run([2], 1, stopfreq=0)
        # caller factors outside [2^-60, 2^60] (the batched reciprocals' domain, brunet.hip recip_batch)
        W0, H0 = np.full((10, 2), 0.5), np.full((2, 4), 0.5)
        W0[3, 1] = 0.0
        with pytest.raises(RuntimeError, match="caller factors"):
            eng.run([2], 1, maxiter=2, W_init=[W0], H_init=[H0])
    # A: finite, non-negative, at most 2^64
    for bad in (-1.0, np.nan, np.inf, 1e30):
        B = np.ones((10, 4))
        B[7, 2] = bad
        with pytest.raises(RuntimeError, match="non-negative"):
            BrunetEngine(B)


def test_c5_full_size_stop_rule_vs_oracle():
    """BASELINE configs[4] at full size under the real NMF.div stop rule (tests/golden/golden_c5.npz, made by
    tests/golden/make_golden_c5.py from the Brunet oracle): 20000 x 500, k = 2..10, one restart per k
    (set.seed(rseed + 1)), stopconv 40 / stopfreq 10, maxniter 2000.  Iterations, labels and counts bit-exact;
    H within 1e-9; W within 1e-9 on its first W_ROWS rows for every k and on the whole of k = 10."""
    import hashlib
    import os
    from conftest import ROOT
    from nmfconsensus_amd.brunet import BrunetEngine
    from nmfconsensus_amd.synthetic import planted_matrix
    path = os.path.join(ROOT, "tests", "golden", "golden_c5.npz")
    if not os.path.exists(path):
        pytest.skip("golden_c5.npz not generated")
    with np.load(path, allow_pickle=False) as z:
        g = {k: z[k] for k in z.files}
    A = planted_matrix(int(g["c5_m"]), int(g["c5_n"]))
    assert hashlib.sha256(np.ascontiguousarray(A).tobytes(order="F")).hexdigest() == str(g["c5_A_sha256"])
    ks = [int(k) for k in g["c5_ks"]]
    n = A.shape[1]
    with BrunetEngine(A) as eng:
        r = eng.run(ks, 1, maxiter=int(g["c5_maxiter"]), seed=int(g["c5_rseed"]), stopconv=int(g["c5_stopconv"]),
                    stopfreq=int(g["c5_stopfreq"]), want_factors=True)
    assert np.array_equal(r.iters, g["c5_iters"]), (r.iters, g["c5_iters"])
    assert np.array_equal(r.labels, g["c5_labels_argmax"].astype(np.int32))
    rows = int(g["c5_W_rows"])
    for i, k in enumerate(ks):
        assert relfro(r.H[i], g[f"c5_H_k{k}"]) < TOL, k
        assert relfro(r.W[i][:rows], g[f"c5_Wtop_k{k}"]) < TOL, k
        lab = g["c5_labels_argmax"][i].astype(np.int32)
        assert np.array_equal(r.counts[i], (lab[:, None] == lab[None, :]).astype(np.int32)), k
        assert np.array_equal(r.consensus[i], r.counts[i] / 1.0)
    kf = int(g["c5_W_full_k"])
    assert relfro(r.W[ks.index(kf)], g["c5_W_full"]) < TOL
    assert r.counts.shape == (len(ks), n, n)


def test_c5_four_restarts_per_k_multilane_vs_oracle():
    """BASELINE configs[4] at full size, R = 4 restarts of every k = 2..10 (36 jobs: tests/golden/golden_c5.npz c5_*_all,
    the Brunet oracle on every job, make_golden_c5.py) run as ONE multi-lane sweep (the default 4 lanes: k batches on
    four host threads and streams, as the C5 bench runs): iterations, labels, the consensus counts of the 4 restarts
    and the consensus bit-exact for every k, every job's H within 1e-9.  (9 -> 36 pinned jobs.)"""
    import hashlib
    import os
    from conftest import ROOT
    from nmfconsensus_amd.brunet import BrunetEngine
    from nmfconsensus_amd.synthetic import planted_matrix
    path = os.path.join(ROOT, "tests", "golden", "golden_c5.npz")
    with np.load(path, allow_pickle=False) as z:
        g = {k: z[k] for k in z.files}
    if "c5_R" not in g:
        pytest.skip("golden_c5.npz without the R = 4 set")
    A = planted_matrix(int(g["c5_m"]), int(g["c5_n"]))
    assert hashlib.sha256(np.ascontiguousarray(A).tobytes(order="F")).hexdigest() == str(g["c5_A_sha256"])
    ks = [int(k) for k in g["c5_ks"]]
    R = int(g["c5_R"])
    with BrunetEngine(A) as eng:
        r = eng.run(ks, R, maxiter=int(g["c5_maxiter"]), seed=int(g["c5_rseed"]), stopconv=int(g["c5_stopconv"]),
                    stopfreq=int(g["c5_stopfreq"]), want_factors=True)
    assert np.array_equal(r.iters.reshape(len(ks), R), g["c5_iters_all"]), (r.iters, g["c5_iters_all"])
    for i, k in enumerate(ks):
        L = g["c5_labels_all"][i].astype(np.int32)
        assert np.array_equal(r.labels[i * R:(i + 1) * R], L), k
        C = sum((l[:, None] == l[None, :]).astype(np.int32) for l in L)
        assert np.array_equal(r.counts[i], C), k
        assert np.array_equal(r.consensus[i], C / R), k
        for q in range(R):
            assert relfro(r.H[i * R + q], g[f"c5_Hall_k{k}"][q]) < TOL, (k, q)
