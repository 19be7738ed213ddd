"""Two ranks on cuda:0: the multi-GPU data path end to end in separate processes (nmf.r:111-117 fan-out).

Each rank builds its own engine, runs its contiguous shard of the C1 job grid (distributed.run_sharded_sweep:
the engine writes the int32 counts straight into a torch device tensor), copies the counts to the host and
SUM-all-reduces them over gloo.  The reduced counts must equal the reference's C1 counts bit for bit.
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


def _rank_main(rank, world, port, A, ks, R, seed, out_path):
    import sys
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist
    from nmfconsensus_amd.distributed import run_sharded_sweep
    from nmfconsensus_amd.nmf import Engine

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        with Engine(A, device=0) as eng:
            counts_dev, res = run_sharded_sweep(eng, ks, R, rank=rank, world=world, reduce=False, maxiter=10000,
                                                seed=seed)
            assert counts_dev.device.type == "cuda"
            host = counts_dev.cpu()
        dist.all_reduce(host, op=dist.ReduceOp.SUM)
        if rank == 0:
            np.save(out_path, host.numpy())
        np.save(out_path + f".iters{rank}.npy", res.iters)
    finally:
        dist.destroy_process_group()


def test_two_ranks_allreduce_equals_golden(golden, tmp_path):
    import torch.multiprocessing as mp

    ks = [int(k) for k in golden["c1_ks"]]
    R = int(golden["c1_R"])
    out = str(tmp_path / "counts.npy")
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, 2, port, golden["A_gct"], ks, R, int(golden["c1_seed"]), out))
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
    counts = np.load(out)
    for i, k in enumerate(ks):
        assert np.array_equal(counts[i], golden[f"c1_counts_argmax_k{k}"]), k
    iters = np.concatenate([np.load(out + f".iters{r}.npy") for r in range(2)])
    assert np.array_equal(iters, golden["c1_iters"])
