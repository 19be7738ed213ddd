"""The plain-C consumer on the GPU: examples/c_sweep (built by __graft_entry__.build(), C99, no Python or torch in
the process) runs the batched sweep and the drop-in nmf_mu; its counts and iteration counts equal the Python engine's
on the same matrix bit for bit, and its nmf_mu restart matches the oracle (the C restatement of nmf_mu.c, pinned to
the reference build's golden vectors) from the same generateMatrix(ran) init: iterations exact, W/H within 1e-9."""
import os
import subprocess

import numpy as np
import pytest

from conftest import relfro

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "examples", "c_sweep")
pytestmark = pytest.mark.gpu


@pytest.mark.skipif(not os.path.exists(EXE), reason="examples/c_sweep not built (python -c 'import __graft_entry__ as g; g.build()')")
def test_c_consumer_matches_python_engine_and_reference(tmp_path, oracle):
    r = subprocess.run([EXE, str(tmp_path)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "cophenetic rho" in r.stdout and "nmf_mu k=3" in r.stdout
    m, n, ks, R = 1000, 40, [2, 3, 4, 5], 5
    A = np.fromfile(tmp_path / "A.bin", dtype=np.float64).reshape(n, m).T      # column-major on disk
    counts = np.fromfile(tmp_path / "counts.bin", dtype=np.int32).reshape(len(ks), n, n)
    iters = np.fromfile(tmp_path / "iters.bin", dtype=np.int32)
    from nmfconsensus_amd.nmf import Engine
    with Engine(np.asfortranarray(A)) as eng:
        res = eng.run(ks, R, maxiter=10000, seed=123, stop_rule=1)
    assert np.array_equal(iters, res.iters)
    assert np.array_equal(counts, np.asarray(res.counts).reshape(len(ks), n, n))
    # the drop-in restart against the oracle
    k = 3
    wh = np.fromfile(tmp_path / "nmf_mu.bin", dtype=np.float64)
    W = wh[: m * k].reshape(k, m).T
    H = wh[m * k: m * k + k * n].reshape(n, k).T
    it = int(wh[-1])
    W0, H0 = oracle.init_restart(123, m, n, k)
    Wo, Ho, ito = oracle.nmf_mu(np.asfortranarray(A), W0, H0, 10000, 1)
    assert it == ito
    assert relfro(W, Wo) < 1e-9 and relfro(H, Ho) < 1e-9
