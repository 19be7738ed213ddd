#!/usr/bin/env python3
"""Generates tests/golden/golden_c2.npz from the REFERENCE's own nmf_mu (TEST INFRASTRUCTURE ONLY).

Run in the build container (needs /root/reference):
    make -C oracle ref && python tests/golden/make_golden_c2.py

Two sweeps, both run job by job through oracle/_ref/libnmf_ref.so (the reference's libnmf sources
compiled out-of-tree by oracle/Makefile, never copied), REF_COMPAT exit, maxiter 10000:

  c2_*   BASELINE configs[1] (C2): synthetic 1000 x 40 (nmfconsensus_amd.synthetic.planted_matrix,
         stored as c2_A), k = 2..8, R = 100, seed 123, jobs in expand.grid order (k fastest), job seed
         = seed + job_id - 1, init = the reference's generateMatrix(ran) after srand(job seed).
  c1r_*  the C1 sweep (bundled gct, k = 2..5, R = 20, seed 123) with nmf.r:37-38's R-path init:
         set.seed(job seed); W <- runif(m*k); H <- runif(k*n).  R is absent from the image, so runif
         comes from oracle/brunet_oracle.c's Mersenne-Twister restatement, itself pinned to R's
         published set.seed/runif values (tests/test_brunet_oracle.py); nmf_mu is the reference's.

Stored per sweep: job k, iterations, labels (argmax and nmf.r:128's order()[1]), int32 connectivity
counts per k, and the final H of the first two restarts of every k (W/H tolerance checks).
"""
from __future__ import annotations

import multiprocessing as mp
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden_c2.npz")


def _job(args):
    os.environ["OPENBLAS_NUM_THREADS"] = "1"
    kind, A, k, s = args
    import contextlib
    from pyoracle import Oracle, RefLib
    ref = RefLib()
    if kind == "ran":
        W0, H0 = ref.generate_ran(s, A.shape[0], A.shape[1], k)
    else:
        W0, H0 = Oracle().brunet_init(s, A.shape[0], A.shape[1], k)   # set.seed(s); runif W then H
    with open(os.devnull, "w") as dn, contextlib.redirect_stdout(dn):
        W, H, it = ref.nmf_mu(A, W0, H0, 10000)
    return it, H


def sweep(pool, tag, A, ks, R, seed, kind, out):
    jobs = []
    jid = 0
    for r in range(1, R + 1):
        for k in ks:
            jid += 1
            jobs.append((k, seed + jid - 1))
    devnull = os.open(os.devnull, os.O_WRONLY)
    saved = os.dup(1)
    os.dup2(devnull, 1)   # the reference prints "Exiting nmf_mu after ..." per call (nmf_mu.c:296)
    try:
        res = pool.map(_job, [(kind, A, k, s) for k, s in jobs])
    finally:
        os.dup2(saved, 1)
        os.close(saved)
        os.close(devnull)
    job_k = np.array([k for k, _ in jobs], dtype=np.int32)
    iters = np.array([it for it, _ in res], dtype=np.int32)
    Hs = [H for _, H in res]
    lam = np.array([np.argmax(H, axis=0) + 1 for H in Hs], dtype=np.int32)
    lro = np.array([np.argmin(H, axis=0) + 1 for H in Hs], dtype=np.int32)
    n = A.shape[1]
    out[f"{tag}_ks"] = np.array(ks, dtype=np.int32)
    out[f"{tag}_R"] = np.array(R)
    out[f"{tag}_seed"] = np.array(seed)
    out[f"{tag}_job_k"] = job_k
    out[f"{tag}_iters"] = iters
    out[f"{tag}_labels_argmax"] = lam
    out[f"{tag}_labels_rorder"] = lro
    for k in ks:
        sel = np.where(job_k == k)[0]
        for key, L in (("argmax", lam), ("rorder", lro)):
            C = np.zeros((n, n), dtype=np.int32)
            for l in L[sel]:
                C += (l[:, None] == l[None, :]).astype(np.int32)
            out[f"{tag}_counts_{key}_k{k}"] = C
        out[f"{tag}_H_k{k}"] = np.array([Hs[j] for j in sel[:2]])
        out[f"{tag}_Hjobs_k{k}"] = sel[:2].astype(np.int32)
    print(f"{tag}: {len(jobs)} jobs, iterations min {iters.min()} mean {iters.mean():.1f} max {iters.max()}",
          file=sys.stderr)


def main():
    from nmfconsensus_amd.synthetic import planted_matrix
    out = {}
    with np.load(os.path.join(os.path.dirname(OUT), "golden.npz"), allow_pickle=False) as g:
        A_gct = g["A_gct"]
    A2 = planted_matrix(1000, 40)
    out["c2_A"] = np.ascontiguousarray(A2)
    with mp.get_context("spawn").Pool(min(8, os.cpu_count() or 1)) as pool:
        sweep(pool, "c2", np.asfortranarray(A2), list(range(2, 9)), 100, 123, "ran", out)
        sweep(pool, "c1r", np.asfortranarray(A_gct), [2, 3, 4, 5], 20, 123, "runif", out)
    np.savez_compressed(OUT, **out)
    print("wrote", OUT, os.path.getsize(OUT), "bytes", file=sys.stderr)


if __name__ == "__main__":
    main()
