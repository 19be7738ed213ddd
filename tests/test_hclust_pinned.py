"""HC$order, merge, heights and cutree membership (nmf.r:166-180) of the host C++ (hclust.cpp) against
tests/rhclust.py, a line-by-line restatement of R's hclust.f (HCLUST, HCASS2) and hclust-utils.c
(cutree).  The inputs are consensus matrices as the sweep produces them -- entries quantised to 1/R, so
exact ties everywhere -- plus tie-free matrices (also checked against scipy).  R itself is absent from
the image: these pin the C++ to R's published algorithm and tie rules, not to a running R."""
import numpy as np
import pytest

from rhclust import cutree as r_cutree
from rhclust import r_hclust_consensus


def quantised_consensus(rng, n, k, R, noise):
    grp = rng.integers(0, k, size=n)
    C = np.zeros((n, n))
    for _ in range(R):
        lab = grp.copy()
        flip = rng.random(n) < noise
        lab[flip] = rng.integers(0, k + 1, size=int(flip.sum()))
        C += lab[:, None] == lab[None, :]
    return C / R


CASES = [(n, k, R, noise, seed) for seed, (n, k, R, noise) in enumerate(
    [(7, 2, 3, 0.3), (12, 3, 5, 0.2), (20, 2, 20, 0.1), (33, 4, 10, 0.15), (40, 5, 25, 0.05), (57, 3, 4, 0.4),
     (64, 6, 8, 0.25), (25, 1, 6, 0.5)])]


@pytest.mark.parametrize("n,k,R,noise,seed", CASES)
def test_order_merge_height_cutree_on_tied_consensus(n, k, R, noise, seed):
    from nmfconsensus_amd.nmf import cophenetic, cutree
    rng = np.random.default_rng(seed + 100)
    C = quantised_consensus(rng, n, k, R, noise)
    rho, order, merge, height = cophenetic(C)
    r_order, r_merge, r_height = r_hclust_consensus(C)
    assert np.array_equal(merge, r_merge)
    assert np.array_equal(order, r_order)
    assert np.array_equal(height, r_height)   # identical arithmetic order: bit-exact
    for kk in sorted({1, 2, max(1, k), min(n, k + 2), n}):
        assert list(cutree(merge, kk)) == r_cutree(n, r_merge, kk), kk


def test_all_ties_and_tiny():
    from nmfconsensus_amd.nmf import cophenetic, cutree
    for n in (2, 3, 5, 9):
        for C in (np.ones((n, n)), np.eye(n), np.full((n, n), 0.5) + 0.5 * np.eye(n)):
            _, order, merge, height = cophenetic(C)
            r_order, r_merge, r_height = r_hclust_consensus(C)
            assert np.array_equal(merge, r_merge) and np.array_equal(order, r_order)
            assert np.array_equal(height, r_height)
            for kk in range(1, n + 1):
                assert list(cutree(merge, kk)) == r_cutree(n, r_merge, kk)


def test_tie_free_matches_scipy_merges():
    """Without ties the agglomeration sequence is unique: same heights and merged sets as scipy."""
    from scipy.cluster.hierarchy import linkage
    from scipy.spatial.distance import squareform
    from nmfconsensus_amd.nmf import cophenetic
    rng = np.random.default_rng(5)
    n = 30
    X = rng.random((n, n))
    C = 1.0 - (X + X.T) / 4.0
    np.fill_diagonal(C, 1.0)
    _, order, merge, height = cophenetic(C)
    r_order, r_merge, r_height = r_hclust_consensus(C)
    assert np.array_equal(merge, r_merge) and np.array_equal(order, r_order)
    Z = linkage(squareform(1.0 - C, checks=False), "average")
    assert np.allclose(height, Z[:, 2], rtol=0, atol=1e-12)

    def members(m, step, memo={}):
        out = set()
        for x in m[step]:
            out |= {int(-x)} if x < 0 else members(m, x - 1)
        return out

    ours = [frozenset(members(merge, s)) for s in range(n - 1)]
    cl = {i: {i + 1} for i in range(n)}
    theirs = []
    for s, (a, b, _, _) in enumerate(Z):
        cl[n + s] = cl[int(a)] | cl[int(b)]
        theirs.append(frozenset(cl[n + s]))
    assert ours == theirs
    # HC$order lists every leaf once and keeps each merged cluster contiguous
    pos = {int(v): i for i, v in enumerate(order)}
    for grp in ours:
        idx = sorted(pos[v] for v in grp)
        assert idx[-1] - idx[0] + 1 == len(idx)
