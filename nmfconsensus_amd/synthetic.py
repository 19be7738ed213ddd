"""Synthetic expression matrices for the benchmark configs, bit-identical on every host.

A = W* H* + E, non-negative fp64, m genes x n samples:
  W* ~ U(0,1) (m x 4); H* plants 4 equal sample groups (group g: H*[g, j] = 1 + U(0,1)/2, else U(0,1)/10);
  E = 0.1 |Z| with Z = sqrt(3) (U1 + U2 + U3 + U4 - 2) (Irwin-Hall: zero mean, unit variance, near-normal);
  the result is scaled to mean 2.5 (the bundled gct's scale).
Uniforms come from a counter-based splitmix64 (53-bit mantissas), so any shard can regenerate any
entry; seed 20261015.  Only IEEE +, -, * and one correctly rounded sum (math.fsum) are used: no libm
transcendentals and no BLAS, whose results depend on the host CPU's SIMD / kernel dispatch.  (Round 2's
form, Box-Muller through numpy's log1p/cos plus a BLAS W* H*, gave different bits on the build container
and on the GPU box; the C3 reference golden, tests/golden/golden_c3.npz, needs the same A on both.)
"""
from __future__ import annotations

import numpy as np

SEED = 20261015
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)
_GOLD = np.uint64(0x9E3779B97F4A7C15)

CONFIGS = {
    # name: (m, n, ks, R, description)
    "C2": (1000, 40, list(range(2, 9)), 100, "synthetic 1000x40 fp64, k=2..8, 100 restarts"),
    "C3": (20000, 500, list(range(2, 11)), 200, "synthetic 20000x500 fp64, k=2..10, 200 restarts"),
    "C4": (60000, 2000, list(range(2, 16)), 1000, "synthetic 60000x2000 fp64, k=2..15, 1000 restarts"),
    # BASELINE configs[4]: the Brunet KL-divergence MU variant (nmfc_brunet_*, nmfconsensus_amd/brunet.py)
    "C5": (20000, 500, list(range(2, 11)), 200, "Brunet KL-divergence MU, synthetic 20000x500 fp64, k=2..10, 200 restarts"),
}


def _splitmix(counter: np.ndarray) -> np.ndarray:
    z = counter * _GOLD
    z = (z ^ (z >> np.uint64(30))) * _M1
    z = (z ^ (z >> np.uint64(27))) * _M2
    return z ^ (z >> np.uint64(31))


def uniforms(stream: int, count: int, seed: int = SEED) -> np.ndarray:
    """count uniforms in [0, 1) from stream `stream` (53-bit)."""
    with np.errstate(over="ignore"):
        base = np.uint64((seed * 0x100000001B3 + stream * 0x9E3779B1) & 0xFFFFFFFFFFFFFFFF)
        ctr = base + np.arange(count, dtype=np.uint64)
        bits = _splitmix(ctr)
    return (bits >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)


def planted_matrix(m: int, n: int, kstar: int = 4, seed: int = SEED) -> np.ndarray:
    """The synthetic A (m x n, Fortran order, fp64), bit-identical on every host."""
    import math

    Wst = uniforms(1, m * kstar, seed).reshape((m, kstar), order="F")
    grp = (np.arange(n) * kstar) // n
    u = uniforms(2, kstar * n, seed).reshape((kstar, n), order="F")
    Hst = np.where(np.arange(kstar)[:, None] == grp[None, :], 1.0 + 0.5 * u, 0.1 * u)
    # W* H* as elementwise products summed in a fixed order (no BLAS, no FMA contraction)
    A = np.multiply(Wst[:, :1], Hst[:1, :], order="F")
    for q in range(1, kstar):
        A += Wst[:, q:q + 1] * Hst[q:q + 1, :]
    z = uniforms(3, m * n, seed)
    for st in (4, 5, 6):
        z += uniforms(st, m * n, seed)
    z -= 2.0
    z *= math.sqrt(3.0)
    A += (0.1 * np.abs(z)).reshape((m, n), order="F")
    del z
    A *= 2.5 / (math.fsum(A.ravel(order="K")) / (m * n))
    return np.asfortranarray(A)


def planted_groups(n: int, kstar: int = 4) -> np.ndarray:
    return (np.arange(n) * kstar) // n
