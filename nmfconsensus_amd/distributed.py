"""Multi-GPU sweep: one process per GPU, (k, restart) jobs sharded across ranks, one exchange step.

Replaces the reference's BatchJobs fan-out (nmf.r:63-68, 111-113: `chunk(getJobIds(reg),
n.chunks=njobs)` + `submitJobs`) and its file-registry reduction (nmf.r:81, 94) with:
  * a static contiguous shard of the expand.grid job list per rank (A replicated on every GPU);
  * each rank runs its shard on its own GPU with the batched engine (no data-path communication);
  * ONE collective: an integer SUM all-reduce of the (nk, n, n) connectivity-count tensor
    (torch.distributed, backend "nccl" = RCCL over xGMI on MI355X; "gloo" in the CPU tests).
Integer sums are exact, and every restart's arithmetic is independent of its placement, so the
consensus is bit-identical at 1, 2, 4 or 8 GPUs.
"""
from __future__ import annotations

import numpy as np


def shard_range(njobs: int, rank: int, world: int):
    """Contiguous near-equal split of jobs [0, njobs).  Jobs cycle through k (k fastest in the
    expand.grid order), so contiguous blocks carry near-equal sums of k, i.e. near-equal work."""
    base, rem = divmod(njobs, world)
    begin = rank * base + min(rank, rem)
    end = begin + base + (1 if rank < rem else 0)
    return begin, end


def allreduce_counts(counts, group=None):
    """SUM all-reduce of an int32 count tensor in place (torch tensor on the rank's device, or CPU for gloo)."""
    import torch.distributed as dist

    dist.all_reduce(counts, op=dist.ReduceOp.SUM, group=group)
    return counts


def _engine_device(engine):
    import torch

    dev = getattr(engine, "device", -1)
    return torch.device("cuda", dev if dev is not None and dev >= 0 else torch.cuda.current_device())


def _counts_for(engine, nk, n, counts_tensor):
    """The (nk, n, n) int32 count tensor on the engine's GPU.  The engine writes it on its own stream, so
    torch's stream is drained first: nothing torch queued on the tensor (a zero fill, the previous
    all-reduce) may still be running when the engine starts writing."""
    import torch

    if counts_tensor is None:
        counts_tensor = torch.zeros((nk, n, n), dtype=torch.int32, device=_engine_device(engine))
    if counts_tensor.is_cuda:
        torch.cuda.current_stream(counts_tensor.device).synchronize()
    return counts_tensor


def run_sharded_sweep(engine, ks, R: int, *, rank: int, world: int, counts_tensor=None, group=None, reduce: bool = True,
                      **run_kwargs):
    """Runs this rank's shard on `engine` (nmfconsensus_amd.nmf.Engine on the rank's GPU) and
    all-reduces the counts.  `counts_tensor`: a torch.int32 CUDA tensor of shape (nk, n, n) that the
    engine writes directly (device pointer) and RCCL reduces; allocated on the engine's device if None.
    The engine's run returns after its stream has finished writing the counts, so the all-reduce
    (queued on torch's stream) reads complete data.  Returns (counts_tensor_after_allreduce, local SweepResult)."""
    nk = len(ks)
    n = engine.n
    jb, je = shard_range(nk * R, rank, world)
    counts_tensor = _counts_for(engine, nk, n, counts_tensor)
    res = engine.run(ks, R, job_begin=jb, job_end=je, counts_device_ptr=counts_tensor.data_ptr(), **run_kwargs)
    if world > 1 and reduce:
        allreduce_counts(counts_tensor, group)
    return counts_tensor, res


def run_sharded_with(runner, ks, R: int, n: int, *, rank: int, world: int, group=None):
    """Host-side form used by the CPU (gloo) tests: `runner(job_begin, job_end)` returns this shard's
    (nk, n, n) int32 counts as a numpy array; the counts are SUM-all-reduced through torch.distributed."""
    import torch

    jb, je = shard_range(len(ks) * R, rank, world)
    local = np.ascontiguousarray(runner(jb, je), dtype=np.int32).reshape(len(ks), n, n)
    t = torch.from_numpy(local.copy())
    if world > 1:
        allreduce_counts(t, group)
    return t.numpy()


# ------------------------------------------------------------------------------------------------
# Brunet KL-divergence sweep (nmfc_brunet_*): jobs run k-major (for k: for restart i), so ranks take a
# contiguous range of RESTARTS for every k -- every rank gets the same mix of k, i.e. equal work.
# ------------------------------------------------------------------------------------------------
def run_sharded_brunet(engine, ks, R: int, *, rank: int, world: int, counts_tensor=None, group=None,
                       reduce: bool = True, **run_kwargs):
    """Runs this rank's restart shard on `engine` (nmfconsensus_amd.brunet.BrunetEngine) and
    all-reduces the int32 counts (RCCL on GPUs).  Returns (counts_tensor, local SweepResult)."""
    nk = len(ks)
    n = engine.n
    rb, re = shard_range(R, rank, world)
    counts_tensor = _counts_for(engine, nk, n, counts_tensor)
    res = engine.run(ks, R, restart_begin=rb, restart_end=re, counts_device_ptr=counts_tensor.data_ptr(), **run_kwargs)
    if world > 1 and reduce:
        allreduce_counts(counts_tensor, group)
    return counts_tensor, res


def run_sharded_restarts_with(runner, ks, R: int, n: int, *, rank: int, world: int, group=None):
    """Host-side form of run_sharded_brunet for the CPU (gloo) tests: `runner(restart_begin,
    restart_end)` returns this shard's (nk, n, n) int32 counts."""
    import torch

    rb, re = shard_range(R, rank, world)
    local = np.ascontiguousarray(runner(rb, re), dtype=np.int32).reshape(len(ks), n, n)
    t = torch.from_numpy(local.copy())
    if world > 1:
        allreduce_counts(t, group)
    return t.numpy()
