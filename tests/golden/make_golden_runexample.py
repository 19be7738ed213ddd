#!/usr/bin/env python3
"""Generates tests/golden/golden_runexample.npz from the REFERENCE's own C code (TEST INFRASTRUCTURE ONLY).

runExample() (nmf.r:6-14) -- the reference's second smoke entry -- runs
    runNMFinJobs(read.gct("20+20x1000.gct"), k = 2:5, num.clusterings = 10, maxniter = 10000, seed = 123, njobs = 4)
i.e. 40 jobs in expand.grid order (k fastest), job seed = seed + job_id - 1, each through the reference's nmf_mu
(oracle/_ref/libnmf_ref.so, compiled from /root/reference/libnmf/*.c by oracle/Makefile) from generateMatrix(ran), then
labels (nmf.r:128 under both rules), integer connectivity counts (nmf.r:140-141) and consensus = counts / 10
(nmf.r:143).  njobs only chunks the jobs over worker processes (nmf.r:111): it changes no result.

Run in the build container (needs /root/reference):  make -C oracle ref && python tests/golden/make_golden_runexample.py
Contents (data only): rx_ks, rx_R, rx_seed, rx_job_k, rx_job_seed, rx_iters, rx_labels_{argmax,rorder} (40 x 40),
rx_counts_{argmax,rorder} (4 x 40 x 40 int32), rx_consensus_{argmax,rorder} (4 x 40 x 40), gct_sha256.
"""
from __future__ import annotations

import hashlib
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, HERE)

from pyoracle import RefLib  # noqa: E402
from make_golden import counts, labels  # noqa: E402  (the nmf.r:128, :140-141 restatements of golden.npz)
from nmfconsensus_amd.gct import read_gct  # noqa: E402

GCT = "/root/reference/20+20x1000.gct"
OUT = os.path.join(HERE, "golden_runexample.npz")


def main():
    ref = RefLib()
    A = read_gct(GCT).data
    ks, R, seed = [2, 3, 4, 5], 10, 123
    job_k, job_seed, iters, L_am, L_ro = [], [], [], [], []
    jid = 0
    for _r in range(1, R + 1):
        for k in ks:
            jid += 1
            s = seed + jid - 1
            W0, H0 = ref.generate_ran(s, A.shape[0], A.shape[1], k)
            _W, H, it = ref.nmf_mu(A, W0, H0, 10000)
            job_k.append(k)
            job_seed.append(s)
            iters.append(it)
            L_am.append(labels(H, "argmax"))
            L_ro.append(labels(H, "rorder"))
    jk = np.array(job_k)
    L_am, L_ro = np.array(L_am, dtype=np.int32), np.array(L_ro, dtype=np.int32)
    out = {"rx_ks": np.array(ks, dtype=np.int32), "rx_R": np.array(R), "rx_seed": np.array(seed),
           "rx_job_k": jk.astype(np.int32), "rx_job_seed": np.array(job_seed, dtype=np.int64),
           "rx_iters": np.array(iters, dtype=np.int32), "rx_labels_argmax": L_am, "rx_labels_rorder": L_ro,
           "gct_sha256": np.frombuffer(hashlib.sha256(open(GCT, "rb").read()).digest(), dtype=np.uint8)}
    for rule, L in (("argmax", L_am), ("rorder", L_ro)):
        C = np.stack([counts(L[jk == k]) for k in ks])
        out[f"rx_counts_{rule}"] = C
        out[f"rx_consensus_{rule}"] = C / float(R)
    np.savez_compressed(OUT, **out)
    print("runExample iterations:", iters, file=sys.stderr)


if __name__ == "__main__":
    main()
