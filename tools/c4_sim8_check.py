#!/usr/bin/env python3
"""Summarizes a `bench.py --config C4 --simulate-world 8 --dump-iters X.npy` replay (the 8 shards of the C4 8-GPU job)
and checks the iterations of the reference's golden C4 jobs (tests/golden/golden_c4.npz: the reference's own nmf_mu on
126 jobs spread over all 8 shards) against the replay's dump.  Usage: tools/c4_sim8_check.py <line.json> <iters.npy>"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
d = json.load(open(sys.argv[1]))
it = np.load(sys.argv[2])
c = d["config"]
with np.load(os.path.join(ROOT, "tests", "golden", "golden_c4.npz"), allow_pickle=False) as z:
    jid, gi, gk = z["c4_job_id"], z["c4_iters"], z["c4_job_k"]
W = d["simulated_world"]
bounds = np.cumsum([0] + c["shard_jobs"])
per_shard = [int(((jid >= bounds[r]) & (jid < bounds[r + 1])).sum()) for r in range(W)]
mism = int((it[1][jid] != gi).sum())
out = {
    "what": ("one-GPU replay of the 8 shards of the C4 8-GPU job (BASELINE configs[3]: 60000 x 2000 fp64, k = 2..15, "
             "1000 restarts = 14 000 jobs, REF_COMPAT, maxiter 10000), each shard as the N > 1 policy runs it (2 restart "
             "groups); the 8-GPU wall time is the slowest shard's (the all-reduce of 14 x 2000^2 int32 counts, 224 MB "
             "over xGMI, is not included)"),
    "shard_seconds": c["shard_seconds"], "slowest_shard_s": max(c["shard_seconds"]),
    "mean_shard_s": float(np.mean(c["shard_seconds"])),
    "projected_8gpu_restarts_per_s": d["value"], "per_gpu_restarts_per_s": c["per_gpu_restarts_per_s"],
    "shard_max_iterations": c.get("shard_max_iterations"), "mean_iterations": c["mean_iterations"],
    "counts_summed_over_shards": {"sha256": c["counts_sum_sha256"], "diag_equals_R": c["counts_diag_equals_R"],
                                  "symmetric": c["counts_symmetric"]},
    "golden_jobs_checked": int(len(jid)), "golden_jobs_per_shard": per_shard,
    "golden_iterations_equal_reference": mism == 0 and bool(np.array_equal(it[0][jid], gk)),
    "golden_iteration_mismatches": mism, "source_line": d,
}
print(json.dumps(out, indent=1))
sys.exit(0 if mism == 0 else 1)
