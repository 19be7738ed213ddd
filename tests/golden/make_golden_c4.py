#!/usr/bin/env python3
"""Generates tests/golden/golden_c4.npz from the REFERENCE's own nmf_mu (TEST INFRASTRUCTURE ONLY).

Run in the build container (needs /root/reference):
    make -C oracle ref && python tests/golden/make_golden_c4.py [R] [procs] [T] [S]

S (default 8) is the shard count whose uncovered shards get their first 14 jobs; 0 turns that off.

BASELINE configs[3] (C4): synthetic 60000 x 2000 (nmfconsensus_amd.synthetic.planted_matrix; A is 960 MB
and is NOT stored -- its SHA-256 is, and the GPU test refuses to compare against a different A),
k = 2..15, the first R restarts of every k (default 2: jobs 0..27 of the C4 grid, which rank 0's shard of
the 8-GPU job and the bench's per-GPU C4 shard both start with) plus the LAST T restarts of every k of the
full 1000-restart grid (default 1: jobs 13986..13999, the end of rank 7's shard), plus (round 5) the first
restart of every k inside each shard of the 8-GPU job that holds no golden job yet (`distributed.shard_range(14000,
r, 8)`, r = 1..6: jobs 1750 r .. 1750 r + 13, 84 jobs), seed 123, jobs in
expand.grid order (k fastest, nmf.r:63-68), job
seed = seed + job_id - 1, init = the reference's generateMatrix(ran) after srand(job seed), REF_COMPAT
exit (nmf_mu.c:253-282), maxiter 10000 (nmf.r:13).  Every job runs through oracle/_ref/libnmf_ref.so
(the reference's libnmf sources compiled out-of-tree by oracle/Makefile, never copied) with
single-threaded OpenBLAS, one process per core.

Stored: job k, iterations, labels under both rules (argmax, nmf.r:128's order()[1]) as int8, the
label margins (per job, the smallest relative gap between the winning and the runner-up entry of any
sample column: a divergence at a tiny margin is a near-tie, not a bug), and the final H of the first
restart of every k (and of every shard-head job of shard 3, which the rank-3 GPU test runs).  Counts and
consensus are functions of the labels (nmf.r:140-143) and are rebuilt by the test.  A partial run (after an interruption) is resumable from the checkpoint in /tmp.
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

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden_c4.npz")
CKPT = "/tmp/golden_c4_ckpt.npz"
M, N, KS, SEED, R_TOTAL = 60000, 2000, list(range(2, 16)), 123, 1000

_A = None


def _init_worker():
    os.environ["OPENBLAS_NUM_THREADS"] = "1"
    global _A
    from nmfconsensus_amd.synthetic import planted_matrix
    _A = planted_matrix(M, N)
    devnull = os.open(os.devnull, os.O_WRONLY)
    os.dup2(devnull, 1)   # the reference prints "Exiting nmf_mu after ..." per call (nmf_mu.c:296)


def _job(args):
    jid, k, s = args
    from pyoracle import RefLib
    ref = RefLib()
    W0, H0 = ref.generate_ran(s, M, N, k)
    _, H, it = ref.nmf_mu(_A, W0, H0, 10000)
    return jid, it, H


def _margin(H: np.ndarray, largest: bool) -> float:
    """min over samples of (best - runner-up) / |best| (argmax) or (runner-up - best) / |runner-up|."""
    S = np.sort(H, axis=0)
    if largest:
        gap = (S[-1] - S[-2]) / np.maximum(np.abs(S[-1]), 1e-300)
    else:
        gap = (S[1] - S[0]) / np.maximum(np.abs(S[1]), 1e-300)
    return float(gap.min())


def main():
    R = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    procs = int(sys.argv[2]) if len(sys.argv) > 2 else min(7, os.cpu_count() or 1)
    T = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    S = int(sys.argv[4]) if len(sys.argv) > 4 else 8
    from nmfconsensus_amd.synthetic import planted_matrix
    A = planted_matrix(M, N)
    a_sha = hashlib.sha256(np.ascontiguousarray(A).tobytes(order="F")).hexdigest()
    del A
    # (position in the golden, global job id, k, seed): restarts r = 1..R and r = R_TOTAL-T+1..R_TOTAL
    rs = list(range(1, R + 1)) + list(range(R_TOTAL - T + 1, R_TOTAL + 1))
    gids = [(r - 1) * len(KS) + i for r in rs for i in range(len(KS))]
    n_first, n_last = R * len(KS), T * len(KS)
    shard_heads = {}
    if S > 0:
        from nmfconsensus_amd.distributed import shard_range
        for s in range(S):
            jb, je = shard_range(R_TOTAL * len(KS), s, S)
            if not any(jb <= g < je for g in gids):
                heads = list(range(jb, min(jb + len(KS), je)))
                shard_heads[s] = list(range(len(gids), len(gids) + len(heads)))
                gids += heads
    jobs = [(p, KS[g % len(KS)], SEED + g) for p, g in enumerate(gids)]
    nj = len(jobs)
    iters = np.full(nj, -1, dtype=np.int32)
    lam = np.zeros((nj, N), dtype=np.int8)
    lro = np.zeros((nj, N), dtype=np.int8)
    mam = np.zeros(nj, dtype=np.float64)
    mro = np.zeros(nj, dtype=np.float64)
    Hkeep = {}
    if os.path.exists(CKPT):
        with np.load(CKPT, allow_pickle=False) as c:
            if str(c["a_sha"]) == a_sha:
                # positions are matched by global job id (older checkpoints hold jobs 0..n0-1 only)
                old_ids = c["gids"] if "gids" in c.files else np.arange(c["iters"].shape[0])
                pos = {int(g): q for q, g in enumerate(old_ids)}
                for p, g in enumerate(gids):
                    if g in pos:
                        q = pos[g]
                        iters[p], lam[p], lro[p], mam[p], mro[p] = (c["iters"][q], c["lam"][q], c["lro"][q],
                                                                    c["mam"][q], c["mro"][q])
                        if f"H_{q}" in c.files:
                            Hkeep[p] = c[f"H_{q}"]
    todo = [j for j in jobs if iters[j[0]] < 0]
    print(f"C4 golden: {nj} jobs, {nj - len(todo)} from checkpoint, {procs} processes", file=sys.stderr)
    keep_jobs = set()
    for k in KS:   # the final H of the first and (with T > 0) the last job of every k
        sel = [j for j, kk, _ in jobs[:n_first + n_last] if kk == k]
        keep_jobs.update([sel[0], sel[-1]])
    keep_jobs.update(shard_heads.get(3, []))
    t0 = time.time()
    done = 0

    def ckpt():
        extra = {f"H_{j}": h for j, h in Hkeep.items()}
        np.savez(CKPT, a_sha=a_sha, gids=np.array(gids), iters=iters, lam=lam, lro=lro, mam=mam, mro=mro, **extra)

    with mp.get_context("spawn").Pool(procs, initializer=_init_worker) as pool:
        for j, it, H in pool.imap_unordered(_job, todo, chunksize=1):
            iters[j] = it
            lam[j] = np.argmax(H, axis=0) + 1
            lro[j] = np.argmin(H, axis=0) + 1
            mam[j] = _margin(H, True)
            mro[j] = _margin(H, False)
            if j in keep_jobs:
                Hkeep[j] = H
            done += 1
            if done % 7 == 0:
                ckpt()
                el = time.time() - t0
                print(f"  {done}/{len(todo)} jobs, {el:.0f} s, eta {el / done * (len(todo) - done):.0f} s",
                      file=sys.stderr, flush=True)
    ckpt()
    job_k = np.array([k for _, k, _ in jobs], dtype=np.int32)
    out = dict(c4_m=np.array(M), c4_n=np.array(N), c4_ks=np.array(KS, dtype=np.int32), c4_R=np.array(R),
               c4_T=np.array(T), c4_R_total=np.array(R_TOTAL), c4_job_id=np.array(gids, dtype=np.int32),
               c4_seed=np.array(SEED), c4_A_sha256=np.array(a_sha), c4_job_k=job_k, c4_iters=iters,
               c4_labels_argmax=lam, c4_labels_rorder=lro, c4_margin_argmax=mam, c4_margin_rorder=mro)
    for k in KS:
        sel = np.array(sorted(j for j in keep_jobs if job_k[j] == k))
        out[f"c4_H_k{k}"] = np.array([Hkeep[int(j)] for j in sel])
        out[f"c4_Hjobs_k{k}"] = sel.astype(np.int32)
    np.savez_compressed(OUT, **out)
    print(f"wrote {OUT} ({os.path.getsize(OUT)} bytes): iterations min {iters.min()} mean {iters.mean():.1f} "
          f"max {iters.max()}, {time.time() - t0:.0f} s", file=sys.stderr)


if __name__ == "__main__":
    main()
