"""The drop-in nmf_mu driven the way the reference's R driver drives it: several worker processes on one machine.

nmf.r's runExample() runs `njobs = 4` BatchJobs workers (nmf.r:13, 111: chunk(..., n.chunks = njobs)); each worker
does dyn.load("libnmf.so") and calls .C("nmf_mu", ...) per restart (nmf.r:41-45), so four processes call the library
concurrently and share the GPU (Threading).  Here four FRESH processes (spawn: none forked
from a process that touched the GPU, none re-exec'd) each load libnmf.so through ctypes and call nmf_mu back to back
on the bundled gct for their own rank -- k = 2, 3, 4 on the one-workgroup solo kernel, k = 5 on a 16-workgroup team
(compat.hip routing) -- for the reference's fixed iteration counts and its REF_COMPAT exit, three rounds each.  Every
call is checked against the reference-built golden: W / H within 1e-9 relative Frobenius error, *maxiter exact, the
return value 0.  A team that cannot assemble while the other processes hold CUs takes the library's fallback; the
results must not change.
"""
import os
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOL = 1e-9
ROUNDS = 3


def _worker(k, golden_path, start_evt, out_q):
    import sys
    sys.path.insert(0, ROOT)
    try:
        from nmfconsensus_amd import libnmf

        with np.load(golden_path, allow_pickle=False) as z:
            A = z["A_gct"]
            W0, H0 = z[f"init_k{k}_W"], z[f"init_k{k}_H"]
            want = [(T, z[f"fixed_k{k}_T{T}_W"], z[f"fixed_k{k}_T{T}_H"], T) for T in (2, 10, 200, 398)]
            want.append((10000, z[f"refc_k{k}_W"], z[f"refc_k{k}_H"], int(z[f"refc_k{k}_iter"])))
        libnmf.nmf_mu(A, W0, H0, 2)   # library load, device init and A's upload before the common start
        start_evt.wait(120)
        worst, calls, t0 = 0.0, 0, time.time()
        for _ in range(ROUNDS):
            for T, Wg, Hg, it in want:
                out = libnmf.nmf_mu(A, W0, H0, T)
                assert out["ret"] == 0, (k, T, out["ret"])
                assert out["maxiter"] == it, (k, T, out["maxiter"], it)
                err = max(np.linalg.norm(out["w0"] - Wg) / np.linalg.norm(Wg),
                          np.linalg.norm(out["h0"] - Hg) / np.linalg.norm(Hg))
                assert err < TOL, (k, T, err)
                worst = max(worst, err)
                calls += 1
        out_q.put((k, "ok", worst, calls, time.time() - t0))
    except BaseException as e:   # noqa: BLE001 -- reported to the parent, which fails the test
        out_q.put((k, "error", repr(e), 0, 0.0))
        raise


def test_four_processes_share_the_gpu_through_nmf_mu():
    import multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    start = ctx.Event()
    golden_path = os.path.join(ROOT, "tests", "golden", "golden.npz")
    procs = [ctx.Process(target=_worker, args=(k, golden_path, start, q)) for k in (2, 3, 4, 5)]
    for p in procs:
        p.start()
    time.sleep(1.0)
    start.set()
    results = []
    deadline = time.time() + 240
    while len(results) < len(procs) and time.time() < deadline:
        try:
            results.append(q.get(timeout=5))
        except Exception:   # noqa: BLE001 -- queue.Empty: keep waiting until the deadline
            if all(not p.is_alive() for p in procs) and q.empty():
                break
    for p in procs:
        p.join(timeout=30)
        if p.is_alive():
            p.kill()
            p.join()
    for r in sorted(results):
        print(f"k = {r[0]}: {r[1]}, {r[3]} calls, worst rel-Frobenius {r[2]}, {r[4]:.2f} s")
    assert len(results) == len(procs), f"{len(results)} of {len(procs)} workers reported: {results}"
    assert all(r[1] == "ok" for r in results), results
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
