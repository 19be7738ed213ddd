#!/usr/bin/env python3
"""Small-shape batches (C1 / C2 shapes) by kernel: the solo-kernel jobs alone, the k_small_mu blocks alone, and
both together, best of `reps` wall times per run (init, MU loops, labels, counts).  Usage: python tools/small_probe.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    from nmfconsensus_amd.nmf import Engine
    from nmfconsensus_amd.synthetic import planted_matrix
    with np.load(os.path.join(ROOT, "tests", "golden", "golden.npz"), allow_pickle=False) as z:
        gct = np.asfortranarray(z["A_gct"])
    cases = [("C1", gct, [2, 3, 4, 5], 5), ("C2", planted_matrix(1000, 40), list(range(2, 9)), 100)]
    for name, A, ks, R in cases:
        for label, kk in (("solo ranks", [k for k in ks if k <= 4]), ("block ranks", [k for k in ks if k > 4]),
                          ("all", ks)):
            for solo in ("1", "0"):
                os.environ["NMFC_SOLO"] = solo
                with Engine(A, device=0) as eng:
                    eng.run(kk, R, seed=123)
                    best, res = 1e9, None
                    for _ in range(5):
                        torch.cuda.synchronize()
                        t0 = time.perf_counter()
                        res = eng.run(kk, R, seed=123)
                        best = min(best, time.perf_counter() - t0)
                print(f"{name} {label:12s} ks={kk} NMFC_SOLO={solo}: {best * 1e3:7.2f} ms, max iters {res.iters.max()}",
                      flush=True)
    os.environ.pop("NMFC_SOLO", None)


if __name__ == "__main__":
    main()
