"""C4 against the REFERENCE (tests/golden/golden_c4.npz, tests/golden/make_golden_c4.py).

BASELINE configs[3]: synthetic 60000 x 2000 fp64, k = 2..15, seed 123, the reference's generateMatrix(ran)
init and REF_COMPAT stop rule (nmf_mu.c:253-282), maxiter 10000.  The golden holds the first 2 restarts of every
k (jobs 0..27 of the C4 grid) and the last restart of every k (jobs 13986..13999, the end of rank 7's shard of
the 8-GPU job), each run through the reference's own nmf_mu (oracle/_ref).  The engine must give, per
north_star, bit-exact iteration counts, labels (nmf.r:128 under both rules) and connectivity counts
(nmf.r:140-143), and final H within 1e-9 relative Frobenius error.

Round 5 added the first restart of every k inside each of shards 1..6 of the 8-GPU job (84 more reference jobs), so
every shard holds reference jobs (test_golden_c4_covers_every_shard, CPU).

Batches: the 28 first jobs on their own (small grids, both label rules through the engine's label kernel), and three
1750-job shards as the benches and the 8-GPU job run them -- `bench.py --config C4` (125 restarts of every k: jobs
0..1749, which is also rank 0's shard), rank 3's shard (jobs 5250..6999) and rank 7's shard (jobs 12250..13999 of the
whole 1000-restart grid) -- with their real tile shapes, repacks and tail kernels.
"""
import os

import numpy as np
import pytest

from conftest import ROOT, relfro

pytestmark = pytest.mark.gpu

GOLDEN_C4 = os.path.join(ROOT, "tests", "golden", "golden_c4.npz")
TOL = 1e-9


@pytest.fixture(scope="module")
def c4():
    if not os.path.exists(GOLDEN_C4):
        pytest.skip("golden_c4.npz not generated")
    with np.load(GOLDEN_C4, allow_pickle=False) as z:
        g = {k: z[k] for k in z.files}
    import hashlib
    from nmfconsensus_amd.synthetic import planted_matrix
    A = planted_matrix(int(g["c4_m"]), int(g["c4_n"]))
    sha = hashlib.sha256(np.ascontiguousarray(A).tobytes(order="F")).hexdigest()
    assert sha == str(g["c4_A_sha256"]), "this host's synthetic C4 matrix differs from the golden's"
    return g, A


@pytest.fixture(scope="module")
def c4_engine(c4):
    from nmfconsensus_amd.nmf import Engine
    eng = Engine(c4[1], device=0)
    yield eng
    eng.close()


def _report(name, ours, ref, margins):
    bad = np.where(np.any(ours.reshape(len(ours), -1) != ref.reshape(len(ref), -1), axis=1))[0]
    if len(bad):
        info = ", ".join(f"golden job {j} (label margin {margins[j]:.2e})" for j in bad[:10])
        return f"{name}: {len(bad)} of {len(ref)} jobs differ: {info}"
    return ""


def _golden_h(g):
    """golden position -> final H (the first and last golden job of every k)"""
    out = {}
    for k in g["c4_ks"]:
        for q, p in enumerate(g[f"c4_Hjobs_k{int(k)}"]):
            out[int(p)] = g[f"c4_H_k{int(k)}"][q]
    return out


def test_c4_restarts_vs_reference(c4, c4_engine):
    g, _ = c4
    ks = [int(k) for k in g["c4_ks"]]
    R = int(g["c4_R"])
    n = int(g["c4_n"])
    pos = np.where(g["c4_job_id"] < len(ks) * R)[0]   # the first R restarts of every k: jobs 0 .. 14 R - 1
    assert np.array_equal(g["c4_job_id"][pos], np.arange(len(ks) * R))
    runs = {key: c4_engine.run(ks, R, maxiter=10000, seed=int(g["c4_seed"]), stop_rule=1, label_rule=rule, want_h=True)
            for rule, key in ((0, "argmax"), (1, "rorder"))}
    job_k = g["c4_job_k"][pos]
    for key, r in runs.items():
        msg = _report("iterations", r.iters, g["c4_iters"][pos], g[f"c4_margin_{key}"][pos])
        msg += _report(" labels", r.labels, g[f"c4_labels_{key}"][pos].astype(np.int32), g[f"c4_margin_{key}"][pos])
        assert not msg, f"{key}: {msg}"
        for i, k in enumerate(ks):
            L = g[f"c4_labels_{key}"][pos][job_k == k].astype(np.int32)
            ref = np.zeros((n, n), dtype=np.int32)
            for lab in L:
                ref += lab[:, None] == lab[None, :]
            assert np.array_equal(r.counts[i], ref), (key, k)
    hs = _golden_h(g)
    for p in pos:
        if int(p) in hs:
            assert relfro(runs["argmax"].H[p], hs[int(p)]) < TOL, p


@pytest.mark.timeout(600)
@pytest.mark.parametrize("shard", ["bench_rank0", "rank3", "rank7"])
def test_c4_gpu_shard_vs_reference(c4, c4_engine, shard):
    """A whole 1750-job per-GPU shard, as the bench / the 8-GPU job runs it: the golden jobs inside it bit-exact
    (iterations; argmax labels from the engine's label kernel, R-order labels as argmin of the engine's final H;
    H within 1e-9), every job's labels = the first argmax of its own final H, and the shard's counts rebuilt from
    its labels."""
    g, _ = c4
    ks = [int(k) for k in g["c4_ks"]]
    nk, n = len(ks), int(g["c4_n"])
    if shard == "bench_rank0":     # bench.py --config C4 at N = 1: R = 1000 / 8 = 125 restarts of every k
        R, jb, je = 125, 0, 125 * nk
    else:                          # rank 3 / 7 of the whole C4 job (R = 1000): distributed.shard_range(14000, r, 8)
        from nmfconsensus_amd.distributed import shard_range
        R = int(g["c4_R_total"])
        jb, je = shard_range(nk * R, int(shard[4:]), 8)
    r = c4_engine.run(ks, R, maxiter=10000, seed=int(g["c4_seed"]), stop_rule=1, label_rule=0, job_begin=jb,
                      job_end=je, want_h=True)
    ids = g["c4_job_id"]
    pos = np.where((ids >= jb) & (ids < je))[0]
    assert len(pos) >= nk, f"shard [{jb}, {je}) holds {len(pos)} golden jobs"
    loc = ids[pos] - jb
    msg = _report("iterations", r.iters[loc], g["c4_iters"][pos], g["c4_margin_argmax"][pos])
    msg += _report(" labels", r.labels[loc], g["c4_labels_argmax"][pos].astype(np.int32), g["c4_margin_argmax"][pos])
    ro = np.stack([np.argmin(r.H[j], axis=0) + 1 for j in loc]).astype(np.int32)
    msg += _report(" R-order labels", ro, g["c4_labels_rorder"][pos].astype(np.int32), g["c4_margin_rorder"][pos])
    assert not msg, msg
    hs = _golden_h(g)
    for p, j in zip(pos, loc):
        if int(p) in hs:
            assert relfro(r.H[j], hs[int(p)]) < TOL, (p, j)
    # every job of the shard: labels are its H's first argmax (nmf.r:127-128), counts rebuilt from them
    for j in range(je - jb):
        assert np.array_equal(r.labels[j], np.argmax(r.H[j], axis=0) + 1), j
    job_k = np.array([ks[(jb + s) % nk] for s in range(je - jb)])
    for i, k in enumerate(ks):
        # counts = X^T X for X the (restart, cluster) x sample indicator matrix: exact integers in fp64
        L = r.labels[job_k == k]
        X = np.zeros((len(L) * k, n))
        X[np.arange(len(L))[:, None] * k + (L - 1), np.arange(n)[None, :]] = 1.0
        ref = X.T @ X
        assert np.array_equal(r.counts[i], ref.astype(np.int32)), k
