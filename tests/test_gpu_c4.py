"""C4 against the REFERENCE (tests/golden/golden_c4.npz, tests/golden/make_golden_c4.py).

BASELINE configs[3]: synthetic 60000 x 2000 fp64, k = 2..15, seed 123, the reference's generateMatrix(ran)
init and REF_COMPAT stop rule (nmf_mu.c:253-282), maxiter 10000.  The golden holds the first R restarts of
every k (jobs 0..14R-1 of the C4 grid: the start of rank 0's shard of the 8-GPU job and of the bench's
per-GPU C4 shard), each run through the reference's own nmf_mu (oracle/_ref).  The engine must give, per
north_star, bit-exact iteration counts, labels (nmf.r:128 under both rules) and connectivity counts
(nmf.r:140-143), and final H within 1e-9 relative Frobenius error.  A batch of 28 jobs takes other tile
shapes than the bench's 1750-job shard; every shape sums in the canonical K order, so these are the bits the
shard computes for the same jobs.
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


def _report(name, ours, ref, margins):
    bad = np.where(np.any(ours.reshape(len(ours), -1) != ref.reshape(len(ref), -1), axis=1))[0]
    if len(bad):
        info = ", ".join(f"job {j} (label margin {margins[j]:.2e})" for j in bad[:10])
        return f"{name}: {len(bad)} of {len(ref)} jobs differ: {info}"
    return ""


def test_c4_restarts_vs_reference(c4):
    from nmfconsensus_amd.nmf import Engine
    g, A = c4
    ks = [int(k) for k in g["c4_ks"]]
    R = int(g["c4_R"])
    n = int(g["c4_n"])
    with Engine(A, device=0) as eng:
        runs = {key: eng.run(ks, R, maxiter=10000, seed=int(g["c4_seed"]), stop_rule=1, label_rule=rule, want_h=True)
                for rule, key in ((0, "argmax"), (1, "rorder"))}
    job_k = g["c4_job_k"]
    for key, r in runs.items():
        msg = _report("iterations", r.iters, g["c4_iters"], g[f"c4_margin_{key}"])
        msg += _report(" labels", r.labels, g[f"c4_labels_{key}"].astype(np.int32), g[f"c4_margin_{key}"])
        assert not msg, f"{key}: {msg}"
        for i, k in enumerate(ks):
            L = g[f"c4_labels_{key}"][job_k == k].astype(np.int32)
            ref = np.zeros((n, n), dtype=np.int32)
            for lab in L:
                ref += lab[:, None] == lab[None, :]
            assert np.array_equal(r.counts[i], ref), (key, k)
    r = runs["argmax"]
    for k in ks:
        for q, j in enumerate(g[f"c4_Hjobs_k{k}"]):
            assert relfro(r.H[j], g[f"c4_H_k{k}"][q]) < TOL, (k, j)
