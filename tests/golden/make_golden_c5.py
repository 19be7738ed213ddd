#!/usr/bin/env python3
"""Generates tests/golden/golden_c5.npz from the Brunet ORACLE (TEST INFRASTRUCTURE ONLY).

    make -C oracle && python tests/golden/make_golden_c5.py [procs]

BASELINE configs[4] (C5): the BROAD nmfconsensus Brunet KL-divergence MU (NMF.div) on the synthetic
20000 x 500 matrix (nmfconsensus_amd.synthetic.planted_matrix; A is not stored, its SHA-256 is), k = 2..10,
R = 4 restarts per k (restart i runs set.seed(rseed + i), rseed = 123456789; round 6: was 1), the real stop rule
(membership every stopfreq = 10 iterations, stop after stopconv = 40 unchanged checks), maxniter 2000.
The script is not in the reference (only its call, commented out at test_nmf.r:29), so the checker is
oracle/brunet_oracle.c (parity vs the reference unpinned, see that file's header).  Each job runs on one
host core (about 10-25 min for the nine restart-1 jobs on 7 cores, ~4x that for all 36).

Stored: for restart 1 (the round-4 keys, unchanged): iterations, argmax labels (int8), each job's label margin, the
final H, the first W_ROWS rows of every final W and the whole final W of k = 10 (the full W of every job would be
8.6 MB).  For all R restarts (round 6, c5_R / c5_*_all): iterations (nk x R), argmax labels (nk x R x n, int8), label
margins and final H (c5_Hall_k{k}: R x k x n) -- the consensus counts of the R restarts follow from the labels.
"""
from __future__ import annotations

import hashlib
import multiprocessing as mp
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden_c5.npz")
M, N, KS, RSEED, MAXITER, STOPCONV, STOPFREQ = 20000, 500, list(range(2, 11)), 123456789, 2000, 40, 10
W_ROWS, W_FULL_K = 2000, 10
R = 4

_A = None


def _init_worker():
    global _A
    from nmfconsensus_amd.synthetic import planted_matrix
    _A = planted_matrix(M, N)


def _job(ki):
    k, i = ki
    from pyoracle import Oracle
    O = Oracle()
    W0, H0 = O.brunet_init(RSEED + i, M, N, k)
    t0 = time.time()
    W, H, t = O.brunet(_A, W0, H0, MAXITER, STOPCONV, STOPFREQ)
    return k, i, t, (W if i == 1 else None), H, time.time() - t0


def main():
    procs = int(sys.argv[1]) if len(sys.argv) > 1 else min(7, os.cpu_count() or 1)
    from nmfconsensus_amd.synthetic import planted_matrix
    A = planted_matrix(M, N)
    a_sha = hashlib.sha256(np.ascontiguousarray(A).tobytes(order="F")).hexdigest()
    del A
    res, allr = {}, {}
    t0 = time.time()
    # largest k first: the longest jobs start first
    jobs = [(k, i) for k in sorted(KS, reverse=True) for i in range(1, R + 1)]
    with mp.get_context("spawn").Pool(procs, initializer=_init_worker) as pool:
        for k, i, t, W, H, sec in pool.imap_unordered(_job, jobs, chunksize=1):
            allr[(k, i)] = (t, H)
            if i == 1:
                res[k] = (t, W, H)
            print(f"  k={k} restart {i}: {t} iterations, {sec:.0f} s", file=sys.stderr, flush=True)
    iters = np.array([res[k][0] for k in KS], dtype=np.int32)
    labels = np.array([np.argmax(res[k][2], axis=0) + 1 for k in KS], dtype=np.int8)
    margins = []
    for k in KS:
        S = np.sort(res[k][2], axis=0)
        margins.append(float(((S[-1] - S[-2]) / np.maximum(np.abs(S[-1]), 1e-300)).min()))
    out = dict(c5_m=np.array(M), c5_n=np.array(N), c5_ks=np.array(KS, dtype=np.int32), c5_rseed=np.array(RSEED),
               c5_maxiter=np.array(MAXITER), c5_stopconv=np.array(STOPCONV), c5_stopfreq=np.array(STOPFREQ),
               c5_A_sha256=np.array(a_sha), c5_iters=iters, c5_labels_argmax=labels,
               c5_margin_argmax=np.array(margins), c5_W_rows=np.array(W_ROWS),
               c5_W_full=res[W_FULL_K][1], c5_W_full_k=np.array(W_FULL_K))
    for k in KS:
        out[f"c5_H_k{k}"] = res[k][2]
        out[f"c5_Wtop_k{k}"] = np.ascontiguousarray(res[k][1][:W_ROWS])
    out["c5_R"] = np.array(R)
    out["c5_iters_all"] = np.array([[allr[(k, i)][0] for i in range(1, R + 1)] for k in KS], dtype=np.int32)
    out["c5_labels_all"] = np.array([[np.argmax(allr[(k, i)][1], axis=0) + 1 for i in range(1, R + 1)] for k in KS],
                                    dtype=np.int8)
    marg = []
    for k in KS:
        row = []
        for i in range(1, R + 1):
            S = np.sort(allr[(k, i)][1], axis=0)
            row.append(float(((S[-1] - S[-2]) / np.maximum(np.abs(S[-1]), 1e-300)).min()))
        marg.append(row)
    out["c5_margin_all"] = np.array(marg)
    for k in KS:
        out[f"c5_Hall_k{k}"] = np.stack([allr[(k, i)][1] for i in range(1, R + 1)])
    np.savez_compressed(OUT, **out)
    print(f"wrote {OUT} ({os.path.getsize(OUT)} bytes): iterations {iters.tolist()}, {time.time() - t0:.0f} s",
          file=sys.stderr)


if __name__ == "__main__":
    main()
