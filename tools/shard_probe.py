#!/usr/bin/env python3
"""One shard of the C3 strong-scaling job (distributed.shard_range rank r of W), run as bench.py's N > 1 ranks
run it, for a kernel-trace timeline of exactly that shard.
Usage: python tools/shard_probe.py --rank 2 --world 8 [--groups 1] [--repeat 1] [--dump iters.npy]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rank", type=int, default=2)
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--groups", type=int, default=1)
    ap.add_argument("--repeat", type=int, default=1)
    ap.add_argument("--config", default="C3")
    ap.add_argument("--dump", default=None)
    a = ap.parse_args()
    import numpy as np
    import torch
    from nmfconsensus_amd.distributed import RestartGroups, run_sharded_sweep, shard_range
    from nmfconsensus_amd.synthetic import CONFIGS, planted_matrix
    m, n, ks, R, _ = CONFIGS[a.config]
    dev = torch.device("cuda", 0)
    A_dev = torch.from_numpy(planted_matrix(m, n).T.copy()).to(dev)
    grp = RestartGroups(a_device_ptr=A_dev.data_ptr(), shape=(m, n), device=0, groups=a.groups)
    cnt = torch.zeros((len(ks), n, n), dtype=torch.int32, device=dev)
    for q in range(a.repeat):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        _, res = run_sharded_sweep(grp, ks, R, rank=a.rank, world=a.world, counts_tensor=cnt, reduce=False)
        torch.cuda.synchronize()
        print(f"shard {a.rank}/{a.world} groups {a.groups}: {time.perf_counter() - t0:.4f} s, max iters "
              f"{res.iters.max()}", flush=True)
    if a.dump:
        jb, je = shard_range(len(ks) * R, a.rank, a.world)
        np.save(a.dump, np.stack([np.asarray(ks)[np.arange(jb, je) % len(ks)], res.iters]))
    grp.close()


if __name__ == "__main__":
    main()
