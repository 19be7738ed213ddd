"""C3, the north-star workload, against the REFERENCE (tests/golden/golden_c3.npz, tests/golden/make_golden_c3.py).

BASELINE configs[2]: synthetic 20000 x 500 fp64, k = 2..10, R = 200 restarts (1800 jobs), seed 123, the
reference's generateMatrix(ran) init and REF_COMPAT stop rule (nmf_mu.c:253-282), maxiter 10000.  The golden
was produced by the reference's own nmf_mu (oracle/_ref, compiled from /root/reference), job by job.  The
engine runs the WHOLE sweep as the bench does (4-panel W^T A tiles, the repacks, the 2-/1-panel and narrow
tail kernels) and must give, per north_star, bit-exact iteration counts, labels (nmf.r:128 under both rules),
connectivity counts and consensus (nmf.r:140-143), and final H within 1e-9 relative Frobenius error.
"""
import os

import numpy as np
import pytest

from conftest import ROOT, relfro

pytestmark = pytest.mark.gpu

GOLDEN_C3 = os.path.join(ROOT, "tests", "golden", "golden_c3.npz")
TOL = 1e-9


@pytest.fixture(scope="module")
def c3():
    with np.load(GOLDEN_C3, allow_pickle=False) as z:
        g = {k: z[k] for k in z.files}
    import hashlib
    from nmfconsensus_amd.synthetic import planted_matrix
    A = planted_matrix(int(g["c3_m"]), int(g["c3_n"]))
    sha = hashlib.sha256(np.ascontiguousarray(A).tobytes(order="F")).hexdigest()
    assert sha == str(g["c3_A_sha256"]), "this host's synthetic C3 matrix differs from the golden's"
    return g, A


@pytest.fixture(scope="module")
def c3_engine(c3):
    from nmfconsensus_amd.nmf import Engine
    eng = Engine(c3[1], device=0)
    yield eng
    eng.close()


def _counts(labels, job_k, k, n):
    L = labels[job_k == k].astype(np.int32)
    C = np.zeros((n, n), dtype=np.int32)
    for l in L:
        C += l[:, None] == l[None, :]
    return C


def _report(name, ours, ref, margins):
    bad = np.where(np.any(ours.reshape(len(ours), -1) != ref.reshape(len(ref), -1), axis=1))[0]
    if len(bad):
        info = ", ".join(f"job {j} (label margin {margins[j]:.2e})" for j in bad[:10])
        return f"{name}: {len(bad)} of {len(ref)} jobs differ: {info}"
    return ""


@pytest.mark.parametrize("rule,key", [(0, "argmax"), (1, "rorder")])
def test_c3_sweep_vs_reference(c3, c3_engine, rule, key):
    g, _ = c3
    ks = [int(k) for k in g["c3_ks"]]
    R = int(g["c3_R"])
    n = int(g["c3_n"])
    r = c3_engine.run(ks, R, maxiter=10000, seed=int(g["c3_seed"]), stop_rule=1, label_rule=rule, want_h=True)
    job_k = g["c3_job_k"]
    msg = _report("iterations", r.iters, g["c3_iters"], g[f"c3_margin_{key}"])
    msg += _report(" labels", r.labels, g[f"c3_labels_{key}"].astype(np.int32), g[f"c3_margin_{key}"])
    assert not msg, msg
    for i, k in enumerate(ks):
        ref = _counts(g[f"c3_labels_{key}"], job_k, k, n)
        assert np.array_equal(r.counts[i], ref), k
        assert np.array_equal(r.consensus[i], ref / R), k
    for k in ks:
        for q, j in enumerate(g[f"c3_Hjobs_k{k}"]):
            assert relfro(r.H[j], g[f"c3_H_k{k}"][q]) < TOL, (k, j)


def test_c3_sharded_groups_equal_reference_counts(c3):
    """The N = 8 strong-scaling layout (8 shards x 2 restart groups) on one GPU sums to the reference counts."""
    import torch
    from nmfconsensus_amd.distributed import RestartGroups, run_sharded_sweep

    g, A = c3
    ks = [int(k) for k in g["c3_ks"]]
    R = int(g["c3_R"])
    n = int(g["c3_n"])
    total = torch.zeros((len(ks), n, n), dtype=torch.int32, device="cuda:0")
    part = torch.zeros_like(total)
    iters = []
    with RestartGroups(A, device=0, groups=2) as grp:
        for rank in range(8):
            _, res = run_sharded_sweep(grp, ks, R, rank=rank, world=8, counts_tensor=part, reduce=False,
                                       maxiter=10000, seed=int(g["c3_seed"]))
            total += part
            iters.append(res.iters)
    assert np.array_equal(np.concatenate(iters), g["c3_iters"])
    host = total.cpu().numpy()
    for i, k in enumerate(ks):
        assert np.array_equal(host[i], _counts(g["c3_labels_argmax"], g["c3_job_k"], k, n)), k
