#!/usr/bin/env python3
"""CPU baseline vs process count on this host (bench.cpu_baseline: the reference's own nmf_mu, oracle/_ref, one
single-threaded-BLAS process per core, BatchJobs njobs semantics): the per-process iteration time at 1..P
processes shows whether the host's memory bandwidth saturates inside the share the run may use.
Usage: python tools/cpu_scaling.py [--procs 1,4,8,16] [--config C3] > out.json"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--procs", default="1,4,8,16")
    ap.add_argument("--config", default="C3")
    ap.add_argument("--iters", type=int, default=40)
    a = ap.parse_args()
    import bench
    from nmfconsensus_amd.synthetic import CONFIGS
    m, n, ks, R, _ = CONFIGS[a.config]
    # mean iterations per k of the C3 sweep (BENCH_r03 / golden_c3: the reference's own exits)
    import numpy as np
    z = np.load(os.path.join(ROOT, "tests", "golden", "golden_c3.npz"))
    jk, it = z["c3_job_k"], z["c3_iters"]
    mean_it = {int(k): float(it[jk == k].mean()) for k in ks}
    rows = []
    for p in [int(x) for x in a.procs.split(",")]:
        r = bench.cpu_baseline(m, n, ks, mean_it, p, a.iters)
        rows.append({"procs": p, "restarts_per_s": r["value"], "restarts_per_s_per_proc": r["value"] / p,
                     "sec_per_iter": r["sec_per_iter"]})
        print(f"{p:3d} processes: {r['value']:.3f} restarts/s ({r['value'] / p:.4f} per process)", file=sys.stderr,
              flush=True)
    base = rows[0]["restarts_per_s_per_proc"]
    out = {"config": a.config, "host": bench.host_cpu(), "affinity_cpus": len(os.sched_getaffinity(0)),
           "iterations_per_k": a.iters, "rows": rows,
           "per_process_efficiency": {str(r["procs"]): r["restarts_per_s_per_proc"] / base for r in rows}}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
