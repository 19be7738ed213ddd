"""The N>1 path on CPU: world_size-2 gloo ranks shard the C1 job grid and SUM-all-reduce their integer
connectivity counts; the result equals the golden single-process counts bit for bit."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, ret):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import torch.distributed as dist
    from nmfconsensus_amd.distributed import run_sharded_with
    from pyoracle import Oracle

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    z = np.load(os.path.join(ROOT, "tests", "golden", "golden.npz"), allow_pickle=False)
    A = z["A_gct"]
    ks = [int(k) for k in z["c1_ks"]]
    R = int(z["c1_R"])
    O = Oracle()

    def runner(jb, je):
        counts = np.zeros((len(ks), A.shape[1], A.shape[1]), dtype=np.int32)
        for j in range(jb, je):
            k = ks[j % len(ks)]
            W0, H0 = O.init_restart(int(z["c1_seed"]) + j, A.shape[0], A.shape[1], k)
            _, H, _ = O.nmf_mu(A, W0, H0, 10000, 1)
            l = O.labels(H, 0)
            counts[j % len(ks)] += (l[:, None] == l[None, :]).astype(np.int32)
        return counts

    out = run_sharded_with(runner, ks, R, A.shape[1], rank=rank, world=world)
    if rank == 0:
        ret.put(out)
    dist.barrier()
    dist.destroy_process_group()


def test_shard_ranges_cover_jobs():
    from nmfconsensus_amd.distributed import shard_range
    for njobs in (1, 7, 80, 1800):
        for world in (1, 2, 3, 8):
            rs = [shard_range(njobs, r, world) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == njobs
            assert all(rs[i][1] == rs[i + 1][0] for i in range(world - 1))
            sizes = [e - b for b, e in rs]
            assert max(sizes) - min(sizes) <= 1


def test_weak_scaling_shards_are_the_per_gpu_workload():
    """bench.py --scaling weak: the job grid has R x N restarts per k and each of the N ranks gets one
    contiguous block that holds exactly R restarts of every k (the N = 1 workload, distinct seeds)."""
    from nmfconsensus_amd.distributed import shard_range
    ks, R = list(range(2, 11)), 200
    nk = len(ks)
    for world in (1, 2, 4, 8):
        seen = set()
        for rank in range(world):
            jb, je = shard_range(nk * R * world, rank, world)
            jobs = np.arange(jb, je)
            assert je - jb == nk * R
            per_k = np.bincount(jobs % nk, minlength=nk)        # expand.grid: k fastest
            assert (per_k == R).all()
            restarts = jobs // nk
            assert restarts.min() == rank * R and restarts.max() == (rank + 1) * R - 1
            seen.update(jobs.tolist())
        assert seen == set(range(nk * R * world))


@pytest.mark.timeout(300)
def test_gloo_world2_counts_equal_golden(golden):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = q.get(timeout=280)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    for i, k in enumerate(golden["c1_ks"]):
        assert np.array_equal(out[i], golden[f"c1_counts_argmax_k{k}"])


def _brunet_worker(rank, world, port, ret):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import torch.distributed as dist
    from nmfconsensus_amd.distributed import run_sharded_with
    from pyoracle import Oracle

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    z = np.load(os.path.join(ROOT, "tests", "golden", "golden.npz"), allow_pickle=False)
    A = np.asfortranarray(z["A_gct"][:300])
    ks, R = [2, 3], 5
    O = Oracle()

    def runner(rb, re):
        counts = np.zeros((len(ks), A.shape[1], A.shape[1]), dtype=np.int32)
        for ki, k in enumerate(ks):
            for i in range(rb, re):
                W0, H0 = O.brunet_init(123456789 + i + 1, A.shape[0], A.shape[1], k)
                _, H, _ = O.brunet(A, W0, H0, 600)
                l = O.labels(H, 0)
                counts[ki] += (l[:, None] == l[None, :]).astype(np.int32)
        return counts

    out = run_sharded_with(runner, ks, R, A.shape[1], rank=rank, world=world, unit="restart")
    if rank == 0:
        ret.put((out, runner(0, R)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_gloo_world2_brunet_restart_shards():
    """Brunet sweep sharded by restart range over 2 gloo ranks == the single-process counts."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_brunet_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    out, ref = q.get(timeout=280)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert np.array_equal(out, ref)
    assert out[0].diagonal().tolist() == [5] * out.shape[1]


class _FakeEngine:
    """Engine stand-in for the host logic of RestartGroups (no GPU): counts = one per job at [k index, 0, 0]."""

    def __init__(self, A, device, a_device_ptr=None, shape=None):
        self.m, self.n = (shape if shape else np.asarray(A).shape)
        self.device, self.h, self.calls = 0, 1, []

    def close(self):
        self.h = None

    def run(self, ks, R, job_begin=0, job_end=-1, counts_device_ptr=None, **kw):
        from nmfconsensus_amd.nmf import SweepResult
        self.calls.append((job_begin, job_end))
        nk, n = len(ks), self.n
        jobs = np.arange(job_begin, job_end)
        c = np.zeros((nk, n, n), dtype=np.int32)
        np.add.at(c[:, 0, 0], jobs % nk, 1)
        return SweepResult(ks=list(ks), R=R, n=n, counts=c, consensus=c / R, labels=np.tile(jobs[:, None], (1, n)),
                           iters=jobs.astype(np.int32), stopped_early=np.ones(len(jobs), np.int32),
                           seconds_total=1.0, job_begin=job_begin, job_end=job_end)


@pytest.mark.parametrize("G", [1, 2, 3, 8])
def test_restart_groups_split_and_merge(G):
    """RestartGroups: contiguous sub-ranges covering the shard, results merged in job order, counts summed."""
    from nmfconsensus_amd.distributed import RestartGroups
    ks, R = [2, 3, 4], 7
    grp = RestartGroups(np.zeros((10, 5)), device=0, groups=G, engine_cls=_FakeEngine)
    res = grp.run(ks, R, job_begin=4, job_end=19)
    calls = sorted(c for e in grp.engines for c in e.calls)
    assert calls[0][0] == 4 and calls[-1][1] == 19
    assert all(calls[i][1] == calls[i + 1][0] for i in range(len(calls) - 1))
    assert np.array_equal(res.iters, np.arange(4, 19))
    assert np.array_equal(res.counts[:, 0, 0], np.bincount(np.arange(4, 19) % 3, minlength=3))
    grp.close()
    with pytest.raises(ValueError):
        RestartGroups(np.zeros((10, 5)), groups=9, engine_cls=_FakeEngine)


def _failing_worker(rank, world, port, timeout_s):
    """Rank 1 dies before the counts all-reduce; rank 0 must leave the collective with an error (exit non-zero)
    within the process group's timeout instead of blocking."""
    import sys
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["RANK"], os.environ["WORLD_SIZE"] = str(rank), str(world)
    from nmfconsensus_amd.distributed import init_distributed, run_sharded_with
    init_distributed("gloo", timeout_s=timeout_s)
    if rank == 1:
        raise SystemExit(3)   # a dead rank: no all-reduce, no destroy_process_group
    run_sharded_with(lambda b, e: np.zeros((1, 4, 4), dtype=np.int32), [2], 4, 4, rank=rank, world=world)
    sys.exit(0)   # not reached: the all-reduce raises


@pytest.mark.timeout(200)
def test_gloo_dead_rank_fails_fast():
    import time
    ctx = mp.get_context("spawn")
    port = _free_port()
    timeout_s = 20.0
    ps = [ctx.Process(target=_failing_worker, args=(r, 2, port, timeout_s)) for r in range(2)]
    t0 = time.time()
    for p in ps:
        p.start()
    for p in ps:
        p.join(timeout=150)
    elapsed = time.time() - t0
    assert all(p.exitcode is not None for p in ps), "a rank is still blocked"
    for p in ps:
        if p.exitcode is None:
            p.kill()
    assert ps[1].exitcode == 3
    assert ps[0].exitcode != 0, "the surviving rank reported success without its peer"
    assert elapsed < timeout_s + 120, elapsed


def test_init_distributed_timeout_default(monkeypatch):
    import datetime
    import torch.distributed as dist
    from nmfconsensus_amd import distributed
    seen = {}
    monkeypatch.setattr(dist, "init_process_group", lambda backend, **kw: seen.update(backend=backend, **kw))
    monkeypatch.delenv("NMFC_DIST_TIMEOUT_S", raising=False)
    assert distributed.init_distributed("gloo") == distributed.DEFAULT_TIMEOUT_S
    assert seen["timeout"] == datetime.timedelta(seconds=distributed.DEFAULT_TIMEOUT_S) and "device_id" not in seen
    monkeypatch.setenv("NMFC_DIST_TIMEOUT_S", "42")
    distributed.init_distributed("nccl", device="cuda:0")
    assert seen["timeout"] == datetime.timedelta(seconds=42) and seen["device_id"] == "cuda:0"


def test_restart_groups_weights():
    """Uneven group shares (a speed knob): contiguous sub-ranges in proportion, covering the shard exactly."""
    from nmfconsensus_amd.distributed import RestartGroups
    ks, R = [2, 3, 4], 75
    grp = RestartGroups(np.zeros((10, 5)), device=0, groups=2, engine_cls=_FakeEngine, weights=[8, 1])
    res = grp.run(ks, R, job_begin=0, job_end=225)
    calls = sorted(c for e in grp.engines for c in e.calls)
    assert calls == [(0, 200), (200, 225)]
    assert np.array_equal(res.iters, np.arange(225))
    grp.close()
    with pytest.raises(ValueError):
        RestartGroups(np.zeros((10, 5)), groups=2, engine_cls=_FakeEngine, weights=[1])
