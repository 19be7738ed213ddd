"""Per-k kernel timing of the Brunet engine (C5 shape, R restarts, fixed iterations).

  python tools/brunet_kbench.py [--lib path/to/libnmf.so] [--R 200] [--T 40]
Prints per k: avg ms of k_br_hnum / k_br_hupd / k_br_wupd, algorithmic TFLOP/s and the
element-restart rate (m n quotients per restart per kernel) in G/s.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=None)
    ap.add_argument("--R", type=int, default=200)
    ap.add_argument("--T", type=int, default=40)
    ap.add_argument("--ks", default="2,3,4,5,6,7,8,9,10")
    args = ap.parse_args()
    if args.lib:
        os.environ["NMFC_LIB"] = os.path.abspath(args.lib)
    import torch  # noqa: F401
    from nmfconsensus_amd import _lib
    from nmfconsensus_amd.brunet import BrunetEngine
    from nmfconsensus_amd.synthetic import planted_matrix
    m, n = 20000, 500
    A = planted_matrix(m, n)
    out = {}
    with BrunetEngine(A, 0) as eng:
        eng.run([2], 8, maxiter=4, stopconv=10 ** 6, want_counts=False)   # warm
        eng.set_timing(True)
        for k in [int(x) for x in args.ks.split(",")]:
            eng.run([k], args.R, maxiter=args.T, stopconv=10 ** 6, want_counts=False, lanes=1)
            row = {}
            for name, kid in (("hnum", _lib.BK_HNUM), ("hupd", _lib.BK_HUPD), ("wupd", _lib.BK_WUPD)):
                c, ms, fl = eng.kernel_time(kid)
                avg = ms / max(c, 1)
                row[name + "_ms"] = round(avg, 4)
                if fl:
                    row[name + "_tf"] = round(fl / (avg * 1e-3) / 1e12, 2)
                    row[name + "_gel"] = round(args.R * m * n / (avg * 1e-3) / 1e9, 1)
            out[k] = row
            print(k, json.dumps(row), flush=True)
    print(json.dumps({"lib": os.environ.get("NMFC_LIB", "default"), "R": args.R, "T": args.T, "per_k": out}))


if __name__ == "__main__":
    main()
