"""Bit-for-bit comparison helper for two builds of the Brunet engine (test / measurement infrastructure):
    python tools/brunet_bitcmp.py out.npz        (NMFC_LIB=<other libnmf.so> for the second build)
runs a 72-restart C5-shaped sweep (20000 x 500, k = 2..10, 8 restarts, 120 iterations) and saves iterations, counts,
H and the first 64 rows of W."""
import os, sys, numpy as np
out = sys.argv[1]
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import torch  # noqa
from nmfconsensus_amd.brunet import BrunetEngine
from nmfconsensus_amd.synthetic import planted_matrix
A = planted_matrix(20000, 500)
with BrunetEngine(A) as eng:
    r = eng.run(list(range(2, 11)), 8, maxiter=120, seed=5, stopconv=40, stopfreq=10, want_factors=True)
np.savez(out, iters=r.iters, counts=np.asarray(r.counts), **{f"H{i}": h for i, h in enumerate(r.H)}, **{f"W{i}": w[:64] for i, w in enumerate(r.W)})
print("saved", out)
