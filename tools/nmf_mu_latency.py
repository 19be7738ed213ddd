#!/usr/bin/env python3
"""Per-call latency of the drop-in `nmf_mu` (nmf.r:41-45 calls it once per restart through .C) against the
reference's own nmf_mu (oracle/_ref, compiled from /root/reference sources, scipy OpenBLAS, 1 thread), at
the bundled gct's shape (1000 x 40) with the reference's init stream, maxiter 10000 (REF_COMPAT exit).
Usage (GPU box): python tools/nmf_mu_latency.py [reps]   -- prints one JSON object."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
os.environ.setdefault("OPENBLAS_NUM_THREADS", "1")


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    from nmfconsensus_amd import libnmf
    from pyoracle import RefLib

    with np.load(os.path.join(ROOT, "tests", "golden", "golden.npz"), allow_pickle=False) as z:
        A = z["A_gct"]
    m, n = A.shape
    ref = RefLib()
    out = {"shape": f"{m}x{n}", "maxiter": 10000, "reps": reps, "k": {}}
    devnull = os.open(os.devnull, os.O_WRONLY)
    saved = os.dup(1)
    os.dup2(devnull, 1)   # the warm-up calls print "Exiting nmf_mu after ..." too: stdout holds only the JSON line
    try:
        for k in (2, 5):   # first calls: HIP runtime + code objects, the solo path (k = 2) and the team engine (k = 5)
            libnmf.nmf_mu(A, *ref.generate_ran(1, m, n, k), 10)
    finally:
        os.dup2(saved, 1)
    for k in (2, 3, 4, 5):
        W0, H0 = ref.generate_ran(123, m, n, k)
        os.dup2(devnull, 1)   # both print "Exiting nmf_mu after ..." (nmf_mu.c:296)
        try:
            t = time.perf_counter()
            for _ in range(reps):
                _, _, it_ref = ref.nmf_mu(A, W0, H0, 10000)
            t_ref = (time.perf_counter() - t) / reps
            t = time.perf_counter()
            for _ in range(reps):
                r = libnmf.nmf_mu(A, W0, H0, 10000)
            t_gpu = (time.perf_counter() - t) / reps
        finally:
            os.dup2(saved, 1)
        out["k"][str(k)] = {"iterations_ref": int(it_ref), "iterations_gpu": int(r["maxiter"]),
                            "cpu_ref_ms": t_ref * 1e3, "gpu_dropin_ms": t_gpu * 1e3,
                            "cpu_us_per_iter": t_ref / it_ref * 1e6, "gpu_us_per_iter": t_gpu / r["maxiter"] * 1e6}
    os.close(saved)
    os.close(devnull)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
