#!/usr/bin/env python3
"""Probe: the C3 sweep (R restarts of k = 2..10) split into L contiguous job shards run CONCURRENTLY on one
GPU, each by its own engine (own HIP stream) from its own host thread (ctypes releases the GIL), counts
summed exactly.  Measures whether concurrent kernels of independent restart groups fill the small / tail
grids better than one batched launch.  Usage: python tools/lanes_probe.py R [L ...]"""
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from nmfconsensus_amd.distributed import shard_range
    from nmfconsensus_amd.nmf import Engine
    from nmfconsensus_amd.synthetic import planted_matrix

    R = int(sys.argv[1]) if len(sys.argv) > 1 else 25
    lanes_list = [int(x) for x in sys.argv[2:]] or [1, 2, 3]
    m, n, ks = 20000, 500, list(range(2, 11))
    A = planted_matrix(m, n)
    A_dev = torch.from_numpy(A.T.copy()).cuda()
    torch.cuda.synchronize()
    ref_counts = None
    for L in lanes_list:
        engs = [Engine(a_device_ptr=A_dev.data_ptr(), shape=(m, n), device=0) for _ in range(L)]
        shards = [shard_range(len(ks) * R, i, L) for i in range(L)]

        def sweep():
            out = [None] * L

            def work(i):
                jb, je = shards[i]
                out[i] = engs[i].run(ks, R, maxiter=10000, seed=123, stop_rule=1, job_begin=jb, job_end=je)

            th = [threading.Thread(target=work, args=(i,)) for i in range(L)]
            for t in th:
                t.start()
            for t in th:
                t.join()
            return sum(o.counts.astype(np.int64) for o in out), np.concatenate([o.iters for o in out])

        sweep()   # warmup
        t0 = time.perf_counter()
        steps = 2
        for _ in range(steps):
            counts, iters = sweep()
        dt = (time.perf_counter() - t0) / steps
        if ref_counts is None:
            ref_counts = counts
        same = bool(np.array_equal(counts, ref_counts))
        print(json.dumps({"R": R, "lanes": L, "ms_per_sweep": dt * 1e3, "restarts_per_s": len(ks) * R / dt,
                          "counts_identical_to_first": same, "max_iter": int(iters.max())}), flush=True)
        for e in engs:
            e.close()


if __name__ == "__main__":
    main()
