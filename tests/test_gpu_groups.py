"""Restart groups and the device collective on cuda:0 (nmf.r:111-117: fan-out + reduction).

* RestartGroups (distributed.py): a shard split into 2-3 contiguous groups, each on its own engine and HIP
  stream, counts summed on the device -- must equal the reference's C1 counts, iterations and labels bit for
  bit (the N > 1 bench runs every shard this way).
* run_sharded_sweep(reduce=True) under a world-size-1 "nccl" (RCCL) process group: the int32 SUM all-reduce
  runs on the device tensor the engines wrote, ordered after the engines' streams.
"""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _c1(golden):
    return [int(k) for k in golden["c1_ks"]], int(golden["c1_R"]), int(golden["c1_seed"])


@pytest.mark.parametrize("G", [2, 3])
def test_restart_groups_device_counts_equal_golden(golden, G):
    import torch
    from nmfconsensus_amd.distributed import RestartGroups

    ks, R, seed = _c1(golden)
    counts = torch.full((len(ks), 40, 40), -7, dtype=torch.int32, device="cuda:0")   # overwritten, not accumulated
    with RestartGroups(golden["A_gct"], device=0, groups=G) as grp:
        assert grp.device == 0
        res = grp.run(ks, R, counts_tensor=counts, maxiter=10000, seed=seed)
        host = counts.cpu().numpy()
        for i, k in enumerate(ks):
            assert np.array_equal(host[i], golden[f"c1_counts_argmax_k{k}"]), k
        assert np.array_equal(res.iters, golden["c1_iters"])
        assert np.array_equal(res.labels, golden["c1_labels_argmax"])
        assert res.extras.get("groups") == G
        # a second run reuses the scratch tensors and gives the same counts
        grp.run(ks, R, counts_tensor=counts, maxiter=10000, seed=seed)
        assert np.array_equal(counts.cpu().numpy(), host)


def test_restart_groups_host_counts_and_subrange(golden):
    from nmfconsensus_amd.distributed import RestartGroups

    ks, R, seed = _c1(golden)
    with RestartGroups(golden["A_gct"], device=0, groups=2) as grp:
        full = grp.run(ks, R, maxiter=10000, seed=seed)
        for i, k in enumerate(ks):
            assert np.array_equal(full.counts[i], golden[f"c1_counts_argmax_k{k}"]), k
            assert np.array_equal(full.consensus[i], golden[f"c1_counts_argmax_k{k}"] / R)
        part = grp.run(ks, R, job_begin=13, job_end=51, maxiter=10000, seed=seed, want_factors=True)
        assert np.array_equal(part.iters, golden["c1_iters"][13:51])
        assert len(part.H) == 38


def test_counts_tensor_checks(golden):
    import torch
    from nmfconsensus_amd.distributed import run_sharded_sweep
    from nmfconsensus_amd.nmf import Engine

    ks, R, seed = _c1(golden)
    with Engine(golden["A_gct"], device=0) as eng:
        for bad in (torch.zeros((len(ks), 40, 41), dtype=torch.int32, device="cuda:0"),
                    torch.zeros((len(ks), 40, 40), dtype=torch.int64, device="cuda:0"),
                    torch.zeros((len(ks), 40, 40), dtype=torch.int32),
                    torch.zeros((len(ks), 40, 80), dtype=torch.int32, device="cuda:0")[:, :, ::2]):
            with pytest.raises(ValueError):
                run_sharded_sweep(eng, ks, R, rank=0, world=1, counts_tensor=bad, maxiter=4, seed=seed)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _nccl_main(port, A, ks, R, seed, out_path):
    import sys
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist
    from nmfconsensus_amd.distributed import RestartGroups, run_sharded_sweep

    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        assert dist.get_backend() == "nccl"
        with RestartGroups(A, device=0, groups=2) as grp:
            counts = torch.zeros((len(ks), A.shape[1], A.shape[1]), dtype=torch.int32, device="cuda:0")
            # twice: the second sweep's engines must not start writing before the first all-reduce is done
            for _ in range(2):
                counts_dev, res = run_sharded_sweep(grp, ks, R, rank=0, world=1, counts_tensor=counts, reduce=True,
                                                    maxiter=10000, seed=seed)
            assert counts_dev.data_ptr() == counts.data_ptr()
            np.save(out_path, counts_dev.cpu().numpy())
            np.save(out_path + ".iters.npy", res.iters)
    finally:
        dist.destroy_process_group()


def test_nccl_world1_allreduce_equals_golden(golden, tmp_path):
    import torch.multiprocessing as mp

    ks, R, seed = _c1(golden)
    out = str(tmp_path / "counts.npy")
    p = mp.get_context("spawn").Process(target=_nccl_main, args=(_free_port(), golden["A_gct"], ks, R, seed, out))
    p.start()
    p.join(timeout=240)
    if p.is_alive():
        p.kill()
        p.join()
    assert p.exitcode == 0, p.exitcode
    counts = np.load(out)
    for i, k in enumerate(ks):
        assert np.array_equal(counts[i], golden[f"c1_counts_argmax_k{k}"]), k
    assert np.array_equal(np.load(out + ".iters.npy"), golden["c1_iters"])
