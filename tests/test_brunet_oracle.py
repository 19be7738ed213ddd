"""CPU: the Brunet KL-divergence oracle (oracle/brunet_oracle.c) and its R runif restatement.

The Brunet algorithm (BROAD nmfconsensus NMF.div, BASELINE configs[4]) is not in /root/reference
(only named at test_nmf.r:29), so its parity vs the reference is UNPINNED.  What is pinned here:
  * R's set.seed()/runif() Mersenne-Twister restatement, against R's published outputs;
  * the C oracle against an independent NumPy restatement of NMF.div (different code, same
    algorithm), W/H to 1e-12 and identical stop iterations and memberships.
"""
import numpy as np
import pytest

from conftest import relfro

# R >= 1.7 (Mersenne-Twister, Inversion):  set.seed(s); runif(n)  -- values as R prints them (7 digits)
R_RUNIF = {
    1: [0.2655087, 0.3721239, 0.5728534, 0.9082078, 0.2016819],
    42: [0.9148060, 0.9370754, 0.2861395],
    123: [0.2875775, 0.7883051, 0.4089769],
}


@pytest.mark.parametrize("seed", sorted(R_RUNIF))
def test_runif_matches_r(oracle, seed):
    got = oracle.runif(seed, len(R_RUNIF[seed]))
    assert np.allclose(got, R_RUNIF[seed], rtol=0, atol=5e-8), got


def test_runif_range_and_regeneration(oracle):
    # 2000 draws cross three state regenerations; every draw in (0, 1), 32-bit resolution
    u = oracle.runif(123456790, 2000)
    assert np.all(u > 0) and np.all(u < 1)
    y = u * 2.0 ** 32
    assert np.allclose(y, np.round(y), rtol=0, atol=1e-6)
    assert len(np.unique(u)) == 2000


def test_brunet_init_is_runif_stream(oracle):
    m, n, k = 37, 11, 3
    W, H = oracle.brunet_init(77, m, n, k)
    u = oracle.runif(77, m * k + k * n)
    assert np.array_equal(W.reshape(-1, order="F"), u[: m * k])
    assert np.array_equal(H.reshape(-1, order="F"), u[m * k:])


def nmf_div_numpy(V, W, H, maxniter, stopconv=40, stopfreq=10):
    """Independent NumPy restatement of GenePattern's NMF.div (Brunet et al. 2004)."""
    eps = np.finfo(np.float64).eps
    W, H = W.copy(), H.copy()
    m, n = V.shape
    old = np.zeros(n, dtype=np.int64)
    nochange = 0
    t = 0
    for t in range(1, maxniter + 1):
        VP = W @ H
        H = H * (W.T @ (V / VP)) + eps
        H = H / W.sum(axis=0)[:, None]
        VP = W @ H
        W = W * ((V / VP) @ H.T) + eps
        W = W / H.sum(axis=1)[None, :]
        if t % stopfreq == 0:
            new = np.argmax(H, axis=0) + 1
            nochange = nochange + 1 if np.array_equal(new, old) else 0
            if nochange == stopconv:
                break
            old = new
    return W, H, t


@pytest.mark.parametrize("k", [2, 3, 5])
def test_oracle_vs_numpy_restatement(oracle, golden, k):
    A = np.asfortranarray(golden["A_gct"][:300])
    W0, H0 = oracle.brunet_init(123456789 + 1, A.shape[0], A.shape[1], k)
    W, H, t = oracle.brunet(A, W0, H0, 3000)
    Wn, Hn, tn = nmf_div_numpy(A, W0, H0, 3000)
    assert t == tn and t < 3000
    assert relfro(W, Wn) < 1e-12 and relfro(H, Hn) < 1e-12
    assert np.array_equal(oracle.labels(H, 0), np.argmax(Hn, axis=0) + 1)


def test_oracle_fixed_iterations_and_error_trace(oracle, golden):
    A = np.asfortranarray(golden["A_gct"][:200, :20])
    W0, H0 = oracle.brunet_init(5, 200, 20, 4)
    W, H, t, err = oracle.brunet(A, W0, H0, 25, stopconv=10 ** 6, want_error=True)
    Wn, Hn, _ = nmf_div_numpy(A, W0, H0, 25, stopconv=10 ** 6)
    assert t == 25 and relfro(W, Wn) < 1e-12 and relfro(H, Hn) < 1e-12
    assert err.shape == (25,) and np.all(np.isfinite(err))
    # the KL divergence of this multiplicative update is non-increasing (Lee & Seung 2001)
    assert np.all(np.diff(err) <= 1e-12 * np.abs(err[:-1]))
