"""Two ranks on cuda:0: the multi-GPU data path end to end in separate processes (nmf.r:111-117 fan-out).

Each rank runs exactly what `bench.py` runs at N > 1 (bench.py:236-250): `distributed.run_sharded_sweep` over its
contiguous shard of the C1 job grid on a `distributed.RestartGroups` (two engines on their own HIP streams, their
counts summed on the device) with `reduce=True` -- the library's own all-reduce of the DEVICE count tensor
(`allreduce_counts`; gloo here, since two RCCL ranks cannot share one GPU, RCCL on the 8-GPU node).  The
all-reduced device counts must equal the reference's C1 counts bit for bit, and the ranks' iterations, in rank
order, the reference's C1 iterations.
"""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, groups, A, ks, R, seed, out_path):
    import sys
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist
    from nmfconsensus_amd.distributed import RestartGroups, init_distributed, run_sharded_sweep

    os.environ["RANK"], os.environ["WORLD_SIZE"] = str(rank), str(world)
    init_distributed("gloo", timeout_s=200)
    try:
        torch.cuda.set_device(0)
        with RestartGroups(A, device=0, groups=groups) as eng:
            counts_dev, res = run_sharded_sweep(eng, ks, R, rank=rank, world=world, reduce=True, maxiter=10000,
                                                seed=seed)
            assert counts_dev.device.type == "cuda"
            torch.cuda.synchronize()
            np.save(out_path + f".counts{rank}.npy", counts_dev.cpu().numpy())
        np.save(out_path + f".iters{rank}.npy", res.iters)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("groups", [1, 2])
def test_two_ranks_run_sharded_reduce_equals_golden(golden, tmp_path, groups):
    import torch.multiprocessing as mp

    ks = [int(k) for k in golden["c1_ks"]]
    R = int(golden["c1_R"])
    out = str(tmp_path / "run")
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, 2, port, groups, golden["A_gct"], ks, R, int(golden["c1_seed"]), out))
             for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    for p in procs:
        if p.is_alive():
            p.kill()
            p.join()
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    for r in range(2):   # every rank holds the reduced counts after the all-reduce
        counts = np.load(out + f".counts{r}.npy")
        for i, k in enumerate(ks):
            assert np.array_equal(counts[i], golden[f"c1_counts_argmax_k{k}"]), (r, k)
    iters = np.concatenate([np.load(out + f".iters{r}.npy") for r in range(2)])
    assert np.array_equal(iters, golden["c1_iters"])
