"""Per-iteration time of the one-workgroup solo kernels (nmfc_mu_solo) by rank: the difference of two fixed-count
calls (T and 2T iterations) on the bundled gct, so the upload / launch / readback cost cancels.
Usage: python tools/solo_iter_time.py [T]"""
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from nmfconsensus_amd import _lib  # noqa: E402


def main():
    T = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
    L = _lib.lib()
    A = np.asfortranarray(np.load(os.path.join(ROOT, "tests", "golden", "golden.npz"))["A_gct"])
    m, n = A.shape
    dp = ctypes.POINTER(ctypes.c_double)
    rng = np.random.default_rng(1)
    out = {}
    for k in range(2, 9):
        W0 = np.asfortranarray(rng.random((m, k)) + 0.01)
        H0 = np.asfortranarray(rng.random((k, n)) + 0.01)
        W, H = np.zeros_like(W0), np.zeros_like(H0)
        it, early = ctypes.c_int(0), ctypes.c_int(0)

        def call(t):
            t0 = time.perf_counter()
            rc = L.nmfc_mu_solo(A.ctypes.data_as(dp), m, n, k, t, 0, W0.ctypes.data_as(dp), H0.ctypes.data_as(dp),
                                W.ctypes.data_as(dp), H.ctypes.data_as(dp), ctypes.byref(it), ctypes.byref(early))
            assert rc == 0, _lib.last_error()
            return time.perf_counter() - t0
        call(10)
        a = min(call(T) for _ in range(3))
        b = min(call(2 * T) for _ in range(3))
        out[k] = (b - a) / T * 1e6
        print(f"k = {k}: {out[k]:.2f} us per iteration (T = {T}: {a * 1e3:.2f} ms, 2T: {b * 1e3:.2f} ms)", flush=True)


if __name__ == "__main__":
    main()
