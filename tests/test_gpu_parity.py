"""GPU parity: the HIP engine (libnmf.so) against the reference's golden vectors and the oracle.

Bars (BASELINE.json north_star): init, iteration counts, labels, connectivity and consensus
bit-exact; W/H within 1e-9 relative Frobenius error after a fixed iteration count.
"""
import numpy as np
import pytest

from conftest import relfro

pytestmark = pytest.mark.gpu

TOL = 1e-9   # north_star: per-restart W/H within 1e-9 relative Frobenius error


@pytest.fixture(scope="module")
def gct_engine(golden):
    from nmfconsensus_amd.nmf import Engine
    eng = Engine(golden["A_gct"])
    yield eng
    eng.close()


def test_mfma_layout_and_small_gemm(golden):
    # a tiny case through the whole path: m=5, n=4, k=2 with the reference's generateMatrix init
    from nmfconsensus_amd.nmf import Engine
    from pyoracle import Oracle, STOP_FIXED
    A = np.asfortranarray(np.arange(1, 21, dtype=np.float64).reshape(5, 4) % 7 + 0.5)
    O = Oracle()
    with Engine(A) as eng:
        r0 = eng.run([2], 1, maxiter=0, seed=123, want_factors=True, want_counts=False)
        assert np.array_equal(r0.W[0], golden["init_small_W"])
        assert np.array_equal(r0.H[0], golden["init_small_H"])
        for T in (1, 2, 7, 50):
            r = eng.run([2], 1, maxiter=T, seed=123, stop_rule=0, want_factors=True, want_counts=False)
            Wo, Ho, it = O.nmf_mu(A, golden["init_small_W"], golden["init_small_H"], T, STOP_FIXED)
            assert r.iters[0] == T
            assert relfro(r.W[0], Wo) < TOL and relfro(r.H[0], Ho) < TOL, T


@pytest.mark.parametrize("k", [2, 3, 4, 5])
def test_init_stream_bitexact(gct_engine, golden, k):
    r = gct_engine.run([k], 1, maxiter=0, seed=123, want_factors=True, want_counts=False)
    assert np.array_equal(r.W[0], golden[f"init_k{k}_W"])
    assert np.array_equal(r.H[0], golden[f"init_k{k}_H"])


@pytest.mark.parametrize("k", [2, 3, 4, 5])
@pytest.mark.parametrize("T", [2, 10, 200, 398])
def test_fixed_iterations(gct_engine, golden, k, T):
    r = gct_engine.run([k], 1, maxiter=T, seed=123, stop_rule=0, want_factors=True, want_counts=False)
    assert r.iters[0] == T
    assert relfro(r.W[0], golden[f"fixed_k{k}_T{T}_W"]) < TOL
    assert relfro(r.H[0], golden[f"fixed_k{k}_T{T}_H"]) < TOL


@pytest.mark.parametrize("k", [2, 3, 4, 5])
def test_engine_mu1_vs_reference(gct_engine, golden, k):
    """The nmf_mu per-call path (one restart on a k_team_mu team with one upload / launch / download,
    nmfc_engine_mu1) against the reference-built golden: fixed counts within 1e-9, the REF_COMPAT exit exact.
    Repeated calls also exercise the team counter carried across calls."""
    W0, H0 = golden[f"init_k{k}_W"], golden[f"init_k{k}_H"]
    for T in (2, 10, 200, 398):
        W, H, it, early = gct_engine.mu1(W0, H0, maxiter=T, stop_rule=0)
        assert it == T and not early
        assert relfro(W, golden[f"fixed_k{k}_T{T}_W"]) < TOL and relfro(H, golden[f"fixed_k{k}_T{T}_H"]) < TOL, T
    W, H, it, early = gct_engine.mu1(W0, H0, maxiter=10000, stop_rule=1)
    assert it == int(golden[f"refc_k{k}_iter"]) and early
    r = gct_engine.run([k], 1, maxiter=10000, seed=123, stop_rule=1, want_factors=True, want_counts=False)
    # the batched entry runs the one-workgroup kernel (another fixed summation order): same exit, W/H to rounding
    assert r.iters[0] == it and relfro(r.W[0], W) < 1e-11 and relfro(r.H[0], H) < 1e-11


@pytest.mark.parametrize("m,n,k", [(5, 4, 2), (300, 50, 16), (1024, 64, 7), (129, 17, 3), (2000, 38, 3),
                                   (5000, 38, 5), (8192, 64, 16), (8100, 33, 2)])
def test_engine_mu1_shapes_vs_oracle(oracle, m, n, k):
    """Team shapes at the edges: P = 2..128 workgroups (partials summed in batches of 16), 1..4 sample blocks,
    k up to 16, ragged m and n."""
    from nmfconsensus_amd.nmf import Engine
    rng = np.random.default_rng(m * 1000 + n + k)
    A = np.asfortranarray(rng.random((m, n)) + 0.05)
    W0 = np.asfortranarray(rng.random((m, k)) + 0.01)
    H0 = np.asfortranarray(rng.random((k, n)) + 0.01)
    with Engine(A) as eng:
        for T in (1, 2, 31):
            W, H, it, _ = eng.mu1(W0, H0, maxiter=T, stop_rule=0)
            Wo, Ho, _ = oracle.nmf_mu(A, W0, H0, T, 0)
            assert it == T
            assert relfro(W, Wo) < TOL and relfro(H, Ho) < TOL, (m, n, k, T)
        W, H, it, _ = eng.mu1(W0, H0, maxiter=3000, stop_rule=1)
        _, _, ito = oracle.nmf_mu(A, W0, H0, 3000, 1)
        assert it == ito


@pytest.mark.parametrize("k", [2, 3, 4, 5])
def test_ref_compat_exit(gct_engine, golden, k):
    r = gct_engine.run([k], 1, maxiter=10000, seed=123, stop_rule=1, want_factors=True, want_counts=False)
    assert r.iters[0] == int(golden[f"refc_k{k}_iter"])
    assert r.stopped_early[0] == 1
    assert relfro(r.W[0], golden[f"refc_k{k}_W"]) < TOL
    assert relfro(r.H[0], golden[f"refc_k{k}_H"]) < TOL


def test_user_init_path(gct_engine, golden):
    # caller-provided W0/H0 (the .C("nmf_mu") path) gives the same result as the generated init
    k, T = 3, 10
    r = gct_engine.run([k], 1, maxiter=T, stop_rule=0, W_init=[golden[f"init_k{k}_W"]],
                       H_init=[golden[f"init_k{k}_H"]], want_factors=True, want_counts=False)
    assert relfro(r.W[0], golden[f"fixed_k{k}_T{T}_W"]) < TOL
    assert relfro(r.H[0], golden[f"fixed_k{k}_T{T}_H"]) < TOL


@pytest.mark.parametrize("rule,key", [(0, "argmax"), (1, "rorder")])
def test_c1_sweep_consensus_bitexact(gct_engine, golden, rule, key):
    ks = [int(x) for x in golden["c1_ks"]]
    R = int(golden["c1_R"])
    r = gct_engine.run(ks, R, maxiter=10000, seed=int(golden["c1_seed"]), stop_rule=1, label_rule=rule,
                       want_factors=True)
    assert np.array_equal(r.iters, golden["c1_iters"])
    assert np.array_equal(r.labels, golden[f"c1_labels_{key}"])
    for i, k in enumerate(ks):
        assert np.array_equal(r.counts[i], golden[f"c1_counts_{key}_k{k}"])
        assert np.array_equal(r.consensus[i], golden[f"c1_counts_{key}_k{k}"] / R)
    jk = golden["c1_job_k"]
    for k in ks:
        idx = np.where(jk == k)[0]
        for q, j in enumerate(idx):
            assert relfro(r.H[j], golden[f"c1_H_k{k}"][q]) < TOL


def test_shard_and_batch_invariance(gct_engine, golden):
    ks = [2, 3, 4, 5]
    R = 20
    full = gct_engine.run(ks, R, maxiter=600, seed=7, stop_rule=1, want_factors=True)
    a = gct_engine.run(ks, R, maxiter=600, seed=7, stop_rule=1, job_begin=0, job_end=37, want_factors=True)
    b = gct_engine.run(ks, R, maxiter=600, seed=7, stop_rule=1, job_begin=37, job_end=80, want_factors=True)
    assert np.array_equal(a.counts + b.counts, full.counts)
    assert np.array_equal(np.concatenate([a.iters, b.iters]), full.iters)
    for j in range(80):
        src = a if j < 37 else b
        jj = j if j < 37 else j - 37
        assert np.array_equal(src.W[jj], full.W[j])   # bit-identical: arithmetic independent of placement
        assert np.array_equal(src.H[jj], full.H[j])
    # the same job alone in a batch of one
    one = gct_engine.run(ks, R, maxiter=600, seed=7, stop_rule=1, job_begin=41, job_end=42, want_factors=True)
    assert np.array_equal(one.W[0], full.W[41]) and np.array_equal(one.H[0], full.H[41])


def test_argmax_stable_rule(gct_engine, golden, oracle):
    A = golden["A_gct"]
    for k in (2, 4):
        W0, H0 = golden[f"init_k{k}_W"], golden[f"init_k{k}_H"]
        Wo, Ho, ito = oracle.nmf_mu(A, W0, H0, 10000, 2)
        r = gct_engine.run([k], 1, maxiter=10000, seed=123, stop_rule=2, want_factors=True, want_counts=False)
        assert r.iters[0] == ito
        assert relfro(r.W[0], Wo) < TOL and relfro(r.H[0], Ho) < TOL


def test_nmf_mu_abi(golden):
    from nmfconsensus_amd import libnmf
    A = golden["A_gct"]
    k = 4
    out = libnmf.nmf_mu(A, golden[f"init_k{k}_W"], golden[f"init_k{k}_H"], 10000)
    assert out["maxiter"] == int(golden[f"refc_k{k}_iter"])
    assert relfro(out["w0"], golden[f"refc_k{k}_W"]) < TOL
    assert relfro(out["h0"], golden[f"refc_k{k}_H"]) < TOL
    assert out["ret"] == 0
    # cap reached: *maxiter unchanged; odd counts still leave the result in the caller's buffers
    out = libnmf.nmf_mu(A, golden[f"init_k{k}_W"], golden[f"init_k{k}_H"], 10)
    assert out["maxiter"] == 10
    assert relfro(out["h0"], golden[f"fixed_k{k}_T10_H"]) < TOL


def test_nmf_mu_cache_follows_content(golden, monkeypatch):
    """The engine nmf_mu keeps across calls is reused only for the same A: A then A' (same shape, one entry
    changed) then A again must each give what an uncached call gives (NMFC_NMF_MU_CACHE=0).  NMFC_SOLO=0 keeps
    k = 3 off the solo kernel, so the engine path and its cache (compat.hip mu_cache_drop) are the ones tested."""
    from nmfconsensus_amd import _lib, libnmf
    _lib.lib().nmfc_nmf_mu_release()
    monkeypatch.setenv("NMFC_SOLO", "0")
    A = golden["A_gct"]
    A2 = A.copy(order="F")
    A2[517, 23] += 0.25
    W0, H0 = golden["init_k3_W"], golden["init_k3_H"]
    cached = [libnmf.nmf_mu(X, W0, H0, 40) for X in (A, A2, A)]
    monkeypatch.setenv("NMFC_NMF_MU_CACHE", "0")
    fresh = [libnmf.nmf_mu(X, W0, H0, 40) for X in (A, A2)]
    for c, f in zip(cached, fresh + fresh[:1]):
        assert np.array_equal(c["w0"], f["w0"]) and np.array_equal(c["h0"], f["h0"])
    assert not np.array_equal(cached[0]["h0"], cached[1]["h0"])
    _lib.lib().nmfc_nmf_mu_release()
    monkeypatch.delenv("NMFC_NMF_MU_CACHE")
    again = libnmf.nmf_mu(A, W0, H0, 40)   # a fresh engine after the release
    assert np.array_equal(again["h0"], fresh[0]["h0"])
    _lib.lib().nmfc_nmf_mu_release()       # later tests get an engine made without NMFC_SOLO=0


def test_nmf_mu_solo_cache_follows_content(golden):
    """The solo path (k = 2 on the gct) keeps its device copy of A across calls only for the same A: A, A' (one
    entry changed), A again give what a call after nmfc_nmf_mu_release (nothing cached) gives."""
    from nmfconsensus_amd import _lib, libnmf
    A = golden["A_gct"]
    A2 = A.copy(order="F")
    A2[517, 23] += 0.25
    W0, H0 = golden["init_k2_W"], golden["init_k2_H"]
    assert _lib.lib().nmfc_mu_solo_fits(A.shape[0], A.shape[1], 2)
    cached = [libnmf.nmf_mu(X, W0, H0, 40) for X in (A, A2, A)]
    fresh = []
    for X in (A, A2):
        _lib.lib().nmfc_nmf_mu_release()
        fresh.append(libnmf.nmf_mu(X, W0, H0, 40))
    for c, f in zip(cached, fresh + fresh[:1]):
        assert np.array_equal(c["w0"], f["w0"]) and np.array_equal(c["h0"], f["h0"])
    assert not np.array_equal(cached[0]["h0"], cached[1]["h0"])


def test_nmf_mu_odd_iterations(golden, oracle):
    from nmfconsensus_amd import libnmf
    A = golden["A_gct"]
    W0, H0 = golden["init_k3_W"], golden["init_k3_H"]
    out = libnmf.nmf_mu(A, W0, H0, 7)
    Wo, Ho, _ = oracle.nmf_mu(A, W0, H0, 7, 0)
    assert out["maxiter"] == 7
    assert relfro(out["w0"], Wo) < TOL and relfro(out["h0"], Ho) < TOL


def test_norm_and_maxchange(golden):
    from nmfconsensus_amd import libnmf
    v, d = libnmf.calculateNorm(golden["norm_a"], golden["norm_w"], golden["norm_h"])
    assert abs(v - float(golden["norm_value"])) <= 1e-12 * abs(float(golden["norm_value"]))
    assert relfro(d, golden["norm_d"]) < 1e-13
    v, m0 = libnmf.calculateMaxchange(golden["maxchange_mat"], golden["maxchange_mat0"])
    assert v == float(golden["maxchange_value"])
    assert np.array_equal(m0, golden["maxchange_mat0_after"])


@pytest.mark.parametrize("k", [1, 3, 10, 16, 20])
def test_norm_rank_templated_pass(k):
    """calculateNorm's rank-templated pass (k <= 16) and the generic pass (k > 16) against numpy: d = a - w h
    per element with the q-ordered fma sum, the norm within 1e-12."""
    from nmfconsensus_amd import libnmf
    rng = np.random.default_rng(100 + k)
    m, n = 3001, 151
    a, w, h = rng.random((m, n)), rng.random((m, k)), rng.random((k, n))
    v, d = libnmf.calculateNorm(np.asfortranarray(a), np.asfortranarray(w), np.asfortranarray(h))
    ref = a - w @ h
    assert relfro(d, ref) < 1e-13
    assert abs(v - np.linalg.norm(ref) / np.sqrt(m * n)) <= 1e-12 * v


def test_consensus_entry_matches_sweep(gct_engine, golden):
    from nmfconsensus_amd.nmf import computeConsensusMatrixFromClusterings
    k = 3
    C = computeConsensusMatrixFromClusterings([{"H": h} for h in golden[f"c1_H_k{k}"]])
    assert np.array_equal(C, golden[f"c1_counts_argmax_k{k}"] / 20)


@pytest.mark.parametrize("m,n,ks", [(3001, 150, [2, 7, 10, 16]), (64, 64, [2, 16]), (97, 33, [5]),
                                    (130, 17, [2, 3])])
def test_ragged_shapes_vs_oracle(oracle, m, n, ks):
    from nmfconsensus_amd.nmf import Engine
    rng = np.random.default_rng(m * 1000 + n)
    A = np.asfortranarray(rng.random((m, n)) * 3.0)
    A[5, :] = 0.0   # a zero gene row
    A[:, 3] = 0.0   # a zero sample column
    T = 12
    with Engine(A) as eng:
        r = eng.run(ks, 2, maxiter=T, seed=99, stop_rule=0, want_factors=True)
    for j in range(len(ks) * 2):
        k = ks[j % len(ks)]
        W0, H0 = oracle.init_restart(99 + j, m, n, k)
        Wo, Ho, _ = oracle.nmf_mu(A, W0, H0, T, 0)
        assert relfro(r.W[j], Wo) < TOL and relfro(r.H[j], Ho) < TOL, (m, n, k)
        assert np.all(r.H[j][:, 3] == 0.0)


# 2 and 1 sample tiles of 128 (the Gram blocks spread differently); 4 and 16: the big tiles take their diagonal Gram
# blocks from the W fragment registers (GTile GREG) while the other shapes stage them through LDS
@pytest.mark.parametrize("n", [150, 100, 500, 2000])
def test_tile_shapes_bit_identical(oracle, n):
    # every W^T A / A h^T tile shape the engine picks by grid size sums in the same canonical K order:
    # forcing each shape gives the same bits (so results never depend on how many restarts are live)
    import os
    from nmfconsensus_amd.nmf import Engine
    rng = np.random.default_rng(11)
    m, ks, T = 3001, [2, 7, 10, 16], 12
    A = np.asfortranarray(rng.random((m, n)) * 3.0)
    runs = {}
    try:
        for wta in ("big", "mid", "small", "tiny"):
            for ahtw in ("128", "64"):
                os.environ["NMFC_WTA_TILE"], os.environ["NMFC_AHTW_TILE"] = wta, ahtw
                with Engine(A) as eng:
                    runs[(wta, ahtw)] = eng.run(ks, 3, maxiter=T, seed=5, stop_rule=0, want_factors=True)
    finally:
        os.environ.pop("NMFC_WTA_TILE", None)
        os.environ.pop("NMFC_AHTW_TILE", None)
    ref = runs[("big", "128")]
    for key, r in runs.items():
        for j in range(len(ks) * 3):
            assert np.array_equal(r.W[j], ref.W[j]) and np.array_equal(r.H[j], ref.H[j]), (key, j)
    W0, H0 = oracle.init_restart(5 + 3, m, n, 16)
    Wo, Ho, _ = oracle.nmf_mu(A, W0, H0, T, 0)
    assert relfro(ref.W[3], Wo) < TOL and relfro(ref.H[3], Ho) < TOL


@pytest.mark.parametrize("m,R,lastsum,tile", [(4200, 160, "0", "big"), (2000, 310, "0", "big"), (4200, 160, "1", "big"),
                                              (4200, 160, "0", "mid"), (2000, 160, "0", "mid")])
def test_wta_stream_k_bit_identical(oracle, m, R, lastsum, tile):
    """The big (and the 2-panel, tile = mid) W^T A tile in its stream-K form (k_wta2_sk: whole rounds of items, then the rest split at stage boundaries
    over every CU with the MFMA chains handed over) gives the bits of the one-item-per-workgroup kernel: W and H after
    fixed iterations equal bit for bit with NMFC_WTA_SK=0.  m = 4200: three gene chunks, the last 128 genes long;
    m = 2000: one chunk.  Both grids are large enough for the stream-K launch (>= one round of items, every share at
    least one item long)."""
    import os
    from nmfconsensus_amd.nmf import Engine
    rng = np.random.default_rng(m)
    n, ks, T = 500, list(range(2, 11)), 6
    A = np.asfortranarray(rng.random((m, n)) * 3.0)
    runs = {}
    try:
        os.environ["NMFC_WTA_TILE"] = tile
        for sk in ("1", "0"):
            os.environ["NMFC_WTA_SK"] = sk
            os.environ["NMFC_WTA_LASTSUM"] = lastsum if sk == "1" else "0"   # the split-K combine probe arm (round 6)
            with Engine(A) as eng:
                runs[sk] = eng.run(ks, R, maxiter=T, seed=9, stop_rule=0, want_factors=True, want_counts=False)
    finally:
        os.environ.pop("NMFC_WTA_TILE", None)
        os.environ.pop("NMFC_WTA_SK", None)
        os.environ.pop("NMFC_WTA_LASTSUM", None)
    a, b = runs["1"], runs["0"]
    for j in range(len(ks) * R):
        assert np.array_equal(a.W[j], b.W[j]) and np.array_equal(a.H[j], b.H[j]), j
    j = 5   # one restart against the oracle too
    k = ks[j % len(ks)]
    W0, H0 = oracle.init_restart(9 + j, m, n, k)
    Wo, Ho, _ = oracle.nmf_mu(A, W0, H0, T, 0)
    assert relfro(a.W[j], Wo) < TOL and relfro(a.H[j], Ho) < TOL


def test_full_size_c3_shape_vs_oracle(oracle):
    # BASELINE config C3 shape (20000 x 500), k = 10, a few fixed iterations against the oracle
    from nmfconsensus_amd.nmf import Engine
    rng = np.random.default_rng(3)
    m, n, k, T = 20000, 500, 10, 4
    A = np.asfortranarray(rng.random((m, n)) * 5.0)
    with Engine(A) as eng:
        r = eng.run([k], 1, maxiter=T, seed=20261015, stop_rule=0, want_factors=True, want_counts=False)
    W0, H0 = oracle.init_restart(20261015, m, n, k)
    Wo, Ho, _ = oracle.nmf_mu(A, W0, H0, T, 0)
    assert relfro(r.W[0], Wo) < TOL and relfro(r.H[0], Ho) < TOL


@pytest.mark.parametrize("k", [2, 3, 4, 5])
def test_tolx_stop_rule(gct_engine, golden, k):
    """NMFC_STOP_TOLX: calculateMaxchange-based stop, nmf_als.c:304-349 pattern."""
    from pyoracle import Oracle
    O = Oracle()
    A = golden["A_gct"]
    r = gct_engine.run([k], 1, maxiter=5000, seed=123, stop_rule=3, TolX=1e-3, want_factors=True, want_counts=False)
    W0, H0 = O.init_restart(123, A.shape[0], A.shape[1], k)
    Wo, Ho, it = O.nmf_mu_tol(A, W0, H0, 5000, 1e-3, 1e-4)
    assert r.iters[0] == it and r.stopped_early[0] == (it < 5000)
    assert relfro(r.W[0], Wo) < TOL and relfro(r.H[0], Ho) < TOL


def test_tolx_tolfun_ge_one_stops_at_first_check(gct_engine):
    r = gct_engine.run([2, 3], 2, maxiter=100, seed=9, stop_rule=3, TolX=0.0, TolFun=1.0, want_counts=False)
    assert list(r.iters) == [2, 2, 2, 2]


def test_full_size_c4_shape_vs_oracle(oracle):
    """BASELINE config C4 shape (60000 x 2000), k = 2..15 batched, two fixed iterations: the k = 15 job
    against the oracle, and every job bit-identical to its single-job run (batch invariance at size)."""
    from nmfconsensus_amd.nmf import Engine
    rng = np.random.default_rng(4)
    m, n, T = 60000, 2000, 2
    ks = list(range(2, 16))
    A = np.asfortranarray(rng.random((m, n)) * 5.0)
    with Engine(A) as eng:
        r = eng.run(ks, 1, maxiter=T, seed=77, stop_rule=0, want_factors=True, want_counts=False)
        single = eng.run([15], 1, maxiter=T, seed=77 + 13, stop_rule=0, want_factors=True, want_counts=False)
    assert np.array_equal(r.W[13], single.W[0]) and np.array_equal(r.H[13], single.H[0])
    W0, H0 = oracle.init_restart(77 + 13, m, n, 15)
    Wo, Ho, _ = oracle.nmf_mu(A, W0, H0, T, 0)
    assert relfro(r.W[13], Wo) < TOL and relfro(r.H[13], Ho) < TOL


@pytest.mark.parametrize("m,n,k", [(1000, 40, 2), (1000, 40, 5), (1000, 40, 8), (3001, 150, 16), (97, 33, 3)])
def test_r_runif_init_bitexact(oracle, golden, m, n, k):
    """init_stream = R_RUNIF (nmf.r:37-38): set.seed(job seed); W <- runif(m*k); H <- runif(k*n), bit-exact
    against the R Mersenne-Twister restatement (pinned to R's published values, test_brunet_oracle.py)."""
    from nmfconsensus_amd.nmf import Engine, INIT_R_RUNIF
    A = golden["A_gct"] if (m, n) == (1000, 40) else np.asfortranarray(np.random.default_rng(m).random((m, n)))
    with Engine(A) as eng:
        r = eng.run([k, 2], 2, maxiter=0, seed=321, init_stream=INIT_R_RUNIF, want_factors=True, want_counts=False)
    for j, kk in enumerate([k, 2, k, 2]):
        W, H = oracle.brunet_init(321 + j, m, n, kk)   # job seed = seed + job_id - 1
        assert np.array_equal(r.W[j], W) and np.array_equal(r.H[j], H), j


@pytest.mark.parametrize("rule,key", [(0, "argmax"), (1, "rorder")])
def test_c1_runif_sweep_vs_reference(gct_engine, golden_c2, rule, key):
    """The C1 sweep under the R-path init against the reference's own nmf_mu run job by job
    (tests/golden/make_golden_c2.py): exits, labels, counts bit-exact; H within 1e-9."""
    from nmfconsensus_amd.nmf import INIT_R_RUNIF
    g = golden_c2
    ks = [int(k) for k in g["c1r_ks"]]
    R = int(g["c1r_R"])
    r = gct_engine.run(ks, R, maxiter=10000, seed=int(g["c1r_seed"]), stop_rule=1, label_rule=rule,
                       init_stream=INIT_R_RUNIF, want_factors=True)
    assert np.array_equal(r.iters, g["c1r_iters"])
    assert np.array_equal(r.labels, g[f"c1r_labels_{key}"])
    for i, k in enumerate(ks):
        assert np.array_equal(r.counts[i], g[f"c1r_counts_{key}_k{k}"])
        for q, j in enumerate(g[f"c1r_Hjobs_k{k}"]):
            assert relfro(r.H[j], g[f"c1r_H_k{k}"][q]) < TOL


@pytest.mark.parametrize("rule,key,kernel", [(0, "argmax", "auto"), (1, "rorder", "auto"), (1, "rorder", "team"),
                                             (0, "argmax", "nosolo")])
def test_c2_sweep_vs_reference(golden_c2, rule, key, kernel, monkeypatch):
    """BASELINE configs[1] (C2): synthetic 1000 x 40, k = 2..8, R = 100 (700 jobs) in one sweep against the
    reference's own nmf_mu run job by job: exits, labels, counts and consensus bit-exact; H within 1e-9.
    kernel "auto": every rank on the one-workgroup solo kernels (one restart per workgroup: k_solo_mu for rank
    2..4, k_solo8_mu for 5..8, one launch per kernel rank, concurrently); "nosolo" (NMFC_SOLO=0) every rank on the
    one-workgroup-per-block kernel; "team" (with NMFC_SOLO=0) forces the team kernel for the blocks, whose teams
    then run ~10 blocks one after another (tag and buffer continuity across blocks)."""
    from nmfconsensus_amd.nmf import Engine
    g = golden_c2
    ks = [int(k) for k in g["c2_ks"]]
    R = int(g["c2_R"])
    if kernel == "team":
        monkeypatch.setenv("NMFC_SMALL_KERNEL", kernel)
        monkeypatch.setenv("NMFC_SOLO", "0")
    elif kernel == "nosolo":
        monkeypatch.setenv("NMFC_SOLO", "0")
    with Engine(g["c2_A"]) as eng:
        r = eng.run(ks, R, maxiter=10000, seed=int(g["c2_seed"]), stop_rule=1, label_rule=rule, want_factors=True)
    assert np.array_equal(r.iters, g["c2_iters"])
    assert np.array_equal(r.labels, g[f"c2_labels_{key}"])
    for i, k in enumerate(ks):
        assert np.array_equal(r.counts[i], g[f"c2_counts_{key}_k{k}"])
        assert np.array_equal(r.consensus[i], g[f"c2_counts_{key}_k{k}"] / R)
        for q, j in enumerate(g[f"c2_Hjobs_k{k}"]):
            assert relfro(r.H[j], g[f"c2_H_k{k}"][q]) < TOL


@pytest.mark.parametrize("m,n,ks,R", [(1000, 40, [2, 3, 5], 1), (3001, 150, [7, 9], 1), (97, 33, [5], 2),
                                      (2500, 300, [16], 1), (2000, 120, [16, 16, 8, 8], 1)])
def test_narrow_end_kernels_bit_identical(oracle, golden, m, n, ks, R):
    """The narrow end-of-sweep kernels (the restarts inside the first 1..3 16-column blocks, none straddling a
    block) accumulate in the same canonical K order as the 64-row tiles: W/H bit-identical with them disabled
    (NMFC_NARROW=0).  The last case spans three blocks."""
    import os
    from nmfconsensus_amd.nmf import Engine
    A = golden["A_gct"] if (m, n) == (1000, 40) else np.asfortranarray(np.random.default_rng(m + n).random((m, n)))
    runs = []
    try:
        os.environ["NMFC_SMALL"] = "0"   # keep the 1000 x 40 case on the batched kernels
        for flag in ("1", "0"):
            os.environ["NMFC_NARROW"] = flag
            with Engine(A) as eng:
                runs.append(eng.run(ks, R, maxiter=14, seed=3, stop_rule=0, want_factors=True))
    finally:
        for v in ("NMFC_NARROW", "NMFC_SMALL"):
            os.environ.pop(v, None)
    for run in runs[1:]:
        for j in range(len(ks) * R):
            assert np.array_equal(runs[0].W[j], run.W[j]) and np.array_equal(runs[0].H[j], run.H[j]), j
    k = ks[0]
    W0, H0 = oracle.init_restart(3, m, n, k)
    Wo, Ho, _ = oracle.nmf_mu(A, W0, H0, 14, 0)
    assert relfro(runs[0].W[0], Wo) < TOL and relfro(runs[0].H[0], Ho) < TOL


def test_block_packed_tail_bit_identical():
    """A REF_COMPAT sweep whose tail is repacked into 16-column blocks and run by the narrow kernels gives the
    same exits, labels, counts and bit-identical W/H as the same sweep on the 64-row panel kernels."""
    import os
    from nmfconsensus_amd.nmf import Engine
    A = np.asfortranarray(np.random.default_rng(7).random((3001, 150)))
    runs = []
    try:
        for flag in ("1", "0"):
            os.environ["NMFC_NARROW"] = flag
            with Engine(A) as eng:
                runs.append(eng.run([2, 3, 4, 5, 6], 4, maxiter=3000, seed=11, stop_rule=1, want_factors=True))
    finally:
        os.environ.pop("NMFC_NARROW", None)
    a, b = runs
    assert np.array_equal(a.iters, b.iters) and np.array_equal(a.labels, b.labels)
    assert np.array_equal(a.counts, b.counts)
    assert len(set(a.iters.tolist())) > 3   # restarts stop at different iterations: the tail is repacked
    for j in range(20):
        assert np.array_equal(a.W[j], b.W[j]) and np.array_equal(a.H[j], b.H[j]), j


@pytest.mark.parametrize("ks,R,shape", [([2, 3, 4, 5], 5, None), ([4, 2], 3, None), ([8, 6, 5, 7, 9], 3, None),
                                        ([2, 3, 4, 5, 8], 2, (700, 30)), ([3, 7, 2], 2, (129, 13))])
def test_solo_batch_bitidentical_to_drop_in(golden, oracle, ks, R, shape):
    """A sweep's rank 2..8 restarts run on the solo kernels, one workgroup each (batched launches, one per kernel
    rank, beside k_small_mu, which takes k = 9): every such job's W/H, exit and labels are bit-identical to the same
    job through the single-restart drop-in (nmfc_mu_solo with the job's own generateMatrix(ran) init), so a job's
    bits do not depend on the batch.  The gct has n = 40, so k = 3 runs padded to the 4-row kernel (its zero row
    never mixes in); ranks 5..8 share one kernel (rows past k zero).  A batch whose every job is a solo job runs them
    all in ONE fused launch (k_solo_batch, one workgroup per job); with k = 9 beside them (a k_small_mu block) the
    per-rank launches run instead.  The synthetic shapes reach the fused kernel's other column-group forms (n = 30:
    the rank-3 body; n = 13, m = 129: a ragged short matrix)."""
    import ctypes
    from nmfconsensus_amd import _lib
    from nmfconsensus_amd.nmf import Engine
    if shape is None:
        A = np.asfortranarray(golden["A_gct"])   # the C ABI takes column-major A
    else:
        A = np.asfortranarray(np.random.default_rng(shape[0] + shape[1]).random(shape) + 0.05)
    m, n = A.shape
    seed = 123
    with Engine(A) as eng:
        r = eng.run(ks, R, maxiter=10000, seed=seed, stop_rule=1, want_factors=True)
    L = _lib.lib()
    dp = ctypes.POINTER(ctypes.c_double)
    checked = 0
    for j in range(len(ks) * R):
        k = ks[j % len(ks)]
        if not L.nmfc_mu_solo_fits(m, n, k):
            continue
        W0, H0 = oracle.init_restart(seed + j, m, n, k)
        W, H = np.zeros_like(W0, order="F"), np.zeros_like(H0, order="F")
        it, early = ctypes.c_int(0), ctypes.c_int(0)
        rc = L.nmfc_mu_solo(A.ctypes.data_as(dp), m, n, k, 10000, 1, W0.ctypes.data_as(dp), H0.ctypes.data_as(dp),
                            W.ctypes.data_as(dp), H.ctypes.data_as(dp), ctypes.byref(it), ctypes.byref(early))
        assert rc == 0, _lib.last_error()
        assert r.iters[j] == it.value, (j, k)
        assert np.array_equal(r.W[j], W) and np.array_equal(r.H[j], H), (j, k)
        checked += 1
    assert checked == sum(1 for j in range(len(ks) * R) if ks[j % len(ks)] <= 8)


def test_small_path_agrees_with_batched_engine(golden):
    """The small-shape persistent kernel (m_pad <= 1024, n <= 64) and the batched three-kernel engine sum in
    different fixed orders: on the C1 sweep they agree to rounding (W/H) and exactly (exits, labels)."""
    import os
    from nmfconsensus_amd.nmf import Engine
    runs = []
    try:
        for flag in ("1", "0"):
            os.environ["NMFC_SMALL"] = flag
            with Engine(golden["A_gct"]) as eng:
                runs.append(eng.run([2, 3, 4, 5], 6, maxiter=10000, seed=123, stop_rule=1, want_factors=True))
    finally:
        os.environ.pop("NMFC_SMALL", None)
    a, b = runs
    assert np.array_equal(a.iters, b.iters) and np.array_equal(a.labels, b.labels)
    assert np.array_equal(a.counts, b.counts)
    for j in range(24):
        assert relfro(a.W[j], b.W[j]) < 1e-11 and relfro(a.H[j], b.H[j]) < 1e-11


@pytest.mark.gpu
def test_full_c3_sweep_properties():
    # The full C3 shape (planted 20000 x 500, k = 2..10, reference stop rule) as a batched sweep, checked through
    # size-independent properties (the oracle is too slow at this size for whole sweeps): every stop iteration is
    # a check iteration >= 400 (200 unchanged checks, nmf_mu.c:253-271); labels = first argmax of the final H
    # (nmf.r:128); counts = sum over restarts of label equality (nmf.r:140-141), symmetric with diagonal R; and the
    # job-grid shards reproduce the whole sweep bit for bit (the multi-GPU split).
    from nmfconsensus_amd.nmf import Engine
    from nmfconsensus_amd.synthetic import planted_matrix
    m, n, ks, R = 20000, 500, list(range(2, 11)), 2
    A = planted_matrix(m, n)
    with Engine(A) as eng:
        full = eng.run(ks, R, maxiter=10000, seed=123, stop_rule=1, want_factors=True)
        a = eng.run(ks, R, maxiter=10000, seed=123, stop_rule=1, job_begin=0, job_end=7, want_factors=True)
        b = eng.run(ks, R, maxiter=10000, seed=123, stop_rule=1, job_begin=7, job_end=18, want_factors=True)
    nj = len(ks) * R
    assert np.all(full.iters >= 400) and np.all(full.iters % 2 == 0) and np.all(full.iters < 10000)
    assert np.array_equal(a.counts + b.counts, full.counts)
    assert np.array_equal(np.concatenate([a.iters, b.iters]), full.iters)
    assert np.array_equal(np.concatenate([a.labels, b.labels]), full.labels)
    for j in range(nj):
        src, jj = (a, j) if j < 7 else (b, j - 7)
        assert np.array_equal(src.H[jj], full.H[j]) and np.array_equal(src.W[jj], full.W[j])
        Hj = full.H[j]
        assert Hj.shape == (ks[j % len(ks)], n) and np.all(Hj >= 0)
        assert np.array_equal(full.labels[j], np.argmax(Hj, axis=0) + 1)
    for i, k in enumerate(ks):
        lab = full.labels[i::len(ks)]
        cnt = np.sum(lab[:, :, None] == lab[:, None, :], axis=0)
        assert np.array_equal(full.counts[i], cnt)
        assert np.array_equal(full.counts[i], full.counts[i].T) and np.all(np.diag(full.counts[i]) == R)
        assert np.array_equal(full.consensus[i], full.counts[i] / R)


@pytest.mark.parametrize("m,n,k", [(300, 60, 20), (1000, 40, 17), (129, 33, 1), (500, 50, 24), (1000, 40, 5)])
def test_generic_rank_path_vs_oracle(oracle, m, n, k):
    """nmf_mu for ranks outside the MFMA engine's 2..16 (nmfc_mu_generic, csrc/generic.hip; also k = 5 as a
    cross-check of the path itself): fixed counts within 1e-9, the REF_COMPAT exit exact."""
    import ctypes
    from nmfconsensus_amd import _lib
    L = _lib.lib()
    rng = np.random.default_rng(7 * m + n + k)
    A = np.asfortranarray(rng.random((m, n)) + 0.05)
    W0 = np.asfortranarray(rng.random((m, k)) + 0.01)
    H0 = np.asfortranarray(rng.random((k, n)) + 0.01)
    dp = ctypes.POINTER(ctypes.c_double)
    for T, rule in ((1, 0), (2, 0), (37, 0), (3000, 1)):
        W, H = W0.copy(order="F"), H0.copy(order="F")
        it, early = ctypes.c_int(0), ctypes.c_int(0)
        rc = L.nmfc_mu_generic(A.ctypes.data_as(dp), m, n, k, T, rule, W.ctypes.data_as(dp), H.ctypes.data_as(dp),
                               ctypes.byref(it), ctypes.byref(early))
        assert rc == 0, _lib.last_error()
        Wo, Ho, ito = oracle.nmf_mu(A, W0, H0, T, rule)
        assert it.value == ito, (T, rule)
        assert relfro(W, Wo) < TOL and relfro(H, Ho) < TOL, (m, n, k, T)


def test_nmf_mu_abi_rank_above_16(golden):
    """The drop-in takes ranks above 16 (the reference's nmf_mu takes any k): k = 20 on the gct through .C semantics."""
    from nmfconsensus_amd import libnmf
    from pyoracle import Oracle
    A = golden["A_gct"]
    rng = np.random.default_rng(20)
    W0, H0 = rng.random((A.shape[0], 20)), rng.random((20, A.shape[1]))
    out = libnmf.nmf_mu(A, W0, H0, 10000)
    Wo, Ho, ito = Oracle().nmf_mu(A, W0, H0, 10000, 1)
    assert out["ret"] == 0 and out["maxiter"] == ito
    assert relfro(out["w0"], Wo) < TOL and relfro(out["h0"], Ho) < TOL


def test_nmf_mu_team_failure_falls_back(golden, monkeypatch):
    """A drop-in call whose team cannot meet (e.g. many processes sharing the GPU) runs on the batched engine
    instead: the same exit and W/H to rounding (NMFC_TEAM_FAIL simulates the failure).  NMFC_SOLO=0 (set before
    the cached engine is made) keeps k = 3 on the gct off the solo kernel in both the drop-in and the fallback, so
    the team and then k_small_mu run."""
    from nmfconsensus_amd import _lib, libnmf
    _lib.lib().nmfc_nmf_mu_release()
    monkeypatch.setenv("NMFC_SOLO", "0")
    A, W0, H0 = golden["A_gct"], golden["init_k3_W"], golden["init_k3_H"]
    team = libnmf.nmf_mu(A, W0, H0, 10000)
    monkeypatch.setenv("NMFC_TEAM_FAIL", "1")
    fb = libnmf.nmf_mu(A, W0, H0, 10000)
    _lib.lib().nmfc_nmf_mu_release()   # later tests get an engine made without NMFC_SOLO=0
    assert team["ret"] == 0 and fb["ret"] == 0
    assert fb["maxiter"] == team["maxiter"] == int(golden["refc_k3_iter"])
    assert relfro(fb["w0"], team["w0"]) < 1e-11 and relfro(fb["h0"], team["h0"]) < 1e-11


@pytest.mark.parametrize("m,n,k", [(1000, 40, 2), (1024, 37, 2), (1000, 32, 3), (700, 24, 4), (640, 16, 2),
                                   (37, 5, 4), (300, 29, 3), (129, 21, 4), (2, 9, 2),
                                   (1000, 40, 3), (517, 37, 3), (1000, 40, 4), (1024, 30, 4), (3, 40, 3),
                                   (1000, 40, 5), (1024, 40, 8), (1000, 37, 6), (700, 32, 7), (640, 24, 5),
                                   (300, 16, 8), (129, 21, 6), (9, 8, 8), (37, 5, 5)])
def test_solo_path_vs_oracle(oracle, m, n, k):
    """nmf_mu on one workgroup (nmfc_mu_solo, csrc/solo.hip: rank 2..8 on gct-sized matrices, A in one CU's
    registers, its last gene steps in LDS for k = 4 at n > 24 and for ranks 5..8 at n > 16, k = 3 at n > 32 run
    padded to 4 rows, ranks 5..8 on the two-row-group kernel with zero rows past k): fixed counts within 1e-9, the
    REF_COMPAT and ARGMAX_STABLE exits exact, ragged m and n, every column-group form (n <= 16 / 24 / 32 / 40)."""
    import ctypes
    from nmfconsensus_amd import _lib
    L = _lib.lib()
    assert L.nmfc_mu_solo_fits(m, n, k) == 1
    rng = np.random.default_rng(11 * m + n + k)
    A = np.asfortranarray(rng.random((m, n)) + 0.05)
    W0 = np.asfortranarray(rng.random((m, k)) + 0.01)
    H0 = np.asfortranarray(rng.random((k, n)) + 0.01)
    dp = ctypes.POINTER(ctypes.c_double)
    for T, rule in ((1, 0), (2, 0), (37, 0), (3000, 1), (3000, 2)):
        W, H = np.zeros_like(W0, order="F"), np.zeros_like(H0, order="F")
        it, early = ctypes.c_int(0), ctypes.c_int(0)
        rc = L.nmfc_mu_solo(A.ctypes.data_as(dp), m, n, k, T, rule, W0.ctypes.data_as(dp), H0.ctypes.data_as(dp),
                            W.ctypes.data_as(dp), H.ctypes.data_as(dp), ctypes.byref(it), ctypes.byref(early))
        assert rc == 0, _lib.last_error()
        Wo, Ho, ito = oracle.nmf_mu(A, W0, H0, T, rule)
        assert it.value == ito, (T, rule, it.value, ito)
        assert bool(early.value) == (rule != 0 and ito < T), (T, rule)
        assert relfro(W, Wo) < TOL and relfro(H, Ho) < TOL, (m, n, k, T, relfro(W, Wo), relfro(H, Ho))



@pytest.mark.parametrize("m,n", [(200, 40), (500, 24), (700, 33), (1000, 64), (300, 16)])
def test_small_kernel_wave_forms_vs_oracle(oracle, m, n, monkeypatch):
    """k_small_mu runs eight waves where m_pad is a multiple of 256 (m = 200 / 500 / 700 / 1000: 2 / 4 / 6 / 8 gene
    blocks per wave) and four otherwise (m = 300 -> m_pad 384): rank 5..8 restarts in batches (NMFC_SOLO=0: the
    solo kernel would take those with n <= 40) against the oracle -- fixed counts within 1e-9, and the REF_COMPAT
    exits exact."""
    from nmfconsensus_amd.nmf import Engine
    monkeypatch.setenv("NMFC_SOLO", "0")
    rng = np.random.default_rng(31 * m + n)
    A = np.asfortranarray(rng.random((m, n)) * 2.0 + 0.05)
    ks, R, T = [5, 6, 8], 2, 24
    with Engine(A) as eng:
        r = eng.run(ks, R, maxiter=T, seed=41, stop_rule=0, want_factors=True)
        s = eng.run(ks, R, maxiter=10000, seed=41, stop_rule=1)
    for j in range(len(ks) * R):
        k = ks[j % len(ks)]
        W0, H0 = oracle.init_restart(41 + j, m, n, k)
        Wo, Ho, _ = oracle.nmf_mu(A, W0, H0, T, 0)
        assert relfro(r.W[j], Wo) < TOL and relfro(r.H[j], Ho) < TOL, (m, n, k)
        _, _, it = oracle.nmf_mu(A, W0, H0, 10000, 1)
        assert s.iters[j] == it, (m, n, k, j)
