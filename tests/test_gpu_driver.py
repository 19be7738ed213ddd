"""The nmf.r mirror (nmfconsensus_amd.nmf) end to end on the GPU, and the multi-GPU host path on one GPU."""
import os

import numpy as np
import pytest

from conftest import relfro

pytestmark = pytest.mark.gpu


def test_runNMFinJobs_matches_golden(golden, tmp_path):
    from nmfconsensus_amd.nmf import runNMFinJobs
    ks = [int(k) for k in golden["c1_ks"]]
    out = runNMFinJobs(golden["A_gct"], k=ks, num_clusterings=int(golden["c1_R"]), maxniter=10000,
                       seed=int(golden["c1_seed"]), save_dir=str(tmp_path))
    for k in ks:
        assert np.array_equal(out["consensus"][str(k)], golden[f"c1_counts_argmax_k{k}"] / 20)
        assert 0.0 < out["rho"][str(k)] <= 1.0
        assert sorted(out["order"][str(k)]) == list(range(1, 41))
        assert out["membership"][str(k)].max() <= k
    assert os.path.exists(tmp_path / ".membership.gct")
    assert os.path.exists(tmp_path / ".cophenetic.txt")
    # the planted two-group structure of the bundled gct is recovered at k=2
    m2 = out["membership"]["2"]
    assert len(set(m2[:20])) == 1 and len(set(m2[20:])) == 1 and m2[0] != m2[20]


def test_runNMFinJobs_rejects_k1(golden):
    from nmfconsensus_amd.nmf import runNMFinJobs
    with pytest.raises(ValueError, match="at least two clusters"):
        runNMFinJobs(golden["A_gct"], k=[1, 2], num_clusterings=2, maxniter=10, seed=1)


def test_doNMF(golden):
    from nmfconsensus_amd import nmf
    from nmfconsensus_amd.nmf import doNMF
    r = doNMF(golden["A_gct"], 3, 10, seed=123)
    assert r["iter"] == 10
    assert relfro(r["W"], golden["fixed_k3_T10_W"]) < 1e-9
    assert relfro(r["H"], golden["fixed_k3_T10_H"]) < 1e-9
    # the engine is kept for the next call on the same matrix and rebuilt for another one
    eng = nmf._DONMF["eng"]
    r2 = doNMF(np.array(golden["A_gct"]), 3, 10, seed=123)
    assert nmf._DONMF["eng"] is eng
    assert np.array_equal(r2["W"], r["W"]) and np.array_equal(r2["H"], r["H"])
    A2 = golden["A_gct"].copy(order="F")
    A2[5, 5] += 1.0
    r3 = doNMF(A2, 3, 10, seed=123)
    assert nmf._DONMF["eng"] is not eng and not np.array_equal(r3["H"], r["H"])
    nmf.release_doNMF_engine()
    assert nmf._DONMF["eng"] is None


def test_counts_into_device_tensor(golden):
    # the multi-GPU path: counts written straight into a torch device tensor (what RCCL all-reduces)
    import torch
    from nmfconsensus_amd.distributed import run_sharded_sweep
    from nmfconsensus_amd.nmf import Engine
    ks = [int(k) for k in golden["c1_ks"]]
    with Engine(golden["A_gct"], device=0) as eng:
        parts = []
        for rank in range(3):   # three shards run one after another on one GPU, summed on the host
            t, _ = run_sharded_sweep(eng, ks, 20, rank=rank, world=3, reduce=False, maxiter=10000, seed=123)
            parts.append(t.cpu().numpy())
    total = sum(parts)
    for i, k in enumerate(ks):
        assert np.array_equal(total[i], golden[f"c1_counts_argmax_k{k}"])


def test_planted_synthetic_recovered():
    from nmfconsensus_amd.nmf import Engine
    from nmfconsensus_amd.synthetic import planted_matrix, planted_groups
    A = planted_matrix(2000, 60)
    with Engine(A) as eng:
        sw = eng.run([4], 10, maxiter=2000, seed=5)
    C = sw.consensus[0]
    g = planted_groups(60)
    same = g[:, None] == g[None, :]
    assert C[same].mean() > 0.9 and C[~same].mean() < 0.1
