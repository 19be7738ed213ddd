#!/usr/bin/env python3
"""Per-call latency of the drop-in `nmf_mu` against the reference's own nmf_mu (oracle/_ref, 1 core) on
synthetic planted matrices of real-dataset shapes (genes x samples), reference init, maxiter 10000.
Usage (GPU box): python tools/nmf_mu_latency_shapes.py [reps] -- prints one JSON object."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
os.environ.setdefault("OPENBLAS_NUM_THREADS", "1")


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    from nmfconsensus_amd import libnmf
    from nmfconsensus_amd.synthetic import planted_matrix
    from pyoracle import RefLib

    ref = RefLib()
    out = {"maxiter": 10000, "reps": reps, "shapes": {}}
    devnull = os.open(os.devnull, os.O_WRONLY)
    saved = os.dup(1)
    for m, n in ((1000, 40), (1000, 24), (600, 32), (2000, 38), (5000, 38), (8000, 60), (5000, 100)):
        A = planted_matrix(m, n)
        for k in (2, 5):   # the engine for this A (cache) and the solo path's copy, code objects
            libnmf.nmf_mu(A, *ref.generate_ran(1, m, n, k), 10)
        res = {}
        for k in (2, 3, 5):
            W0, H0 = ref.generate_ran(123, m, n, k)
            os.dup2(devnull, 1)
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
            res[str(k)] = {"iterations_ref": int(it_ref), "iterations_gpu": int(r["maxiter"]), "cpu_ref_ms": t_ref * 1e3,
                           "gpu_dropin_ms": t_gpu * 1e3, "cpu_us_per_iter": t_ref / it_ref * 1e6,
                           "gpu_us_per_iter": t_gpu / r["maxiter"] * 1e6}
        out["shapes"][f"{m}x{n}"] = res
        print(f"{m}x{n}", json.dumps(res), file=sys.stderr)
    os.close(saved)
    os.close(devnull)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
