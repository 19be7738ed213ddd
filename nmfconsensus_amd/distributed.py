"""Multi-GPU sweep: one process per GPU, (k, restart) jobs sharded across ranks, one exchange step.

Replaces the reference's BatchJobs fan-out (nmf.r:63-68, 111-113: `chunk(getJobIds(reg),
n.chunks=njobs)` + `submitJobs`) and its file-registry reduction (nmf.r:81, 94) with:
  * a static contiguous shard of the job list per rank (A replicated on every GPU);
  * each rank runs its shard on its own GPU with the batched engine (no data-path communication),
    optionally as G restart groups: G engines on their own HIP streams, driven from G host threads,
    so the groups' launches interleave on the GPU (RestartGroups);
  * ONE collective: an integer SUM all-reduce of the (nk, n, n) connectivity-count tensor
    (torch.distributed, backend "nccl" = RCCL over xGMI on MI355X; "gloo" in the CPU tests).
Integer sums are exact, and every restart's arithmetic is independent of its placement (rank, group,
batch), so the consensus is bit-identical at 1, 2, 4 or 8 GPUs and any group count.

Sharding units: the MU engine shards the expand.grid JOB list (k fastest, nmf.r:63-68), so contiguous
blocks carry near-equal sums of k; the Brunet engine (nmfc_brunet_*) runs jobs k-major, so ranks take a
contiguous range of RESTARTS for every k.
"""
from __future__ import annotations

from concurrent.futures import ThreadPoolExecutor

import numpy as np


DEFAULT_TIMEOUT_S = 300.0


def init_distributed(backend: str = "nccl", device=None, timeout_s: float | None = None):
    """torch.distributed.init_process_group with an explicit timeout (failure containment).  A rank that dies
    (or never arrives) makes the others leave the rendezvous or the counts all-reduce with an error after
    timeout_s instead of blocking until the backend's default (10 min NCCL / 30 min gloo): they exit non-zero.
    timeout_s defaults to $NMFC_DIST_TIMEOUT_S or 300 s, far above the largest shard imbalance of a sweep
    (seconds) and the first `import torch` on a fresh box.  backend "nccl" is RCCL on ROCm; device: the rank's
    torch.device (binds the communicator to it)."""
    import datetime
    import os

    import torch.distributed as dist

    if timeout_s is None:
        timeout_s = float(os.environ.get("NMFC_DIST_TIMEOUT_S", DEFAULT_TIMEOUT_S))
    kw = {"timeout": datetime.timedelta(seconds=timeout_s)}
    if backend == "nccl" and device is not None:
        kw["device_id"] = device
    dist.init_process_group(backend, **kw)
    return timeout_s


def shard_range(njobs: int, rank: int, world: int):
    """Contiguous near-equal split of units [0, njobs)."""
    base, rem = divmod(njobs, world)
    begin = rank * base + min(rank, rem)
    end = begin + base + (1 if rank < rem else 0)
    return begin, end


def _dist_active(world: int) -> bool:
    import torch.distributed as dist

    return world > 1 or (dist.is_available() and dist.is_initialized())


def allreduce_counts(counts, group=None):
    """SUM all-reduce of an int32 count tensor in place (torch tensor on the rank's device, or CPU for gloo).
    Under gloo (the CPU tests, several ranks sharing one GPU) a device tensor is staged through host memory: the
    choice depends on the backend only, so every rank takes the same path.  RCCL ("nccl") reduces it in place."""
    import torch.distributed as dist

    if counts.is_cuda and dist.get_backend(group) == "gloo":
        host = counts.cpu()
        dist.all_reduce(host, op=dist.ReduceOp.SUM, group=group)
        counts.copy_(host)
        return counts
    dist.all_reduce(counts, op=dist.ReduceOp.SUM, group=group)
    return counts


def _check_counts(counts_tensor, nk: int, n: int, device: int):
    """The engine writes nk*n*n int32 through the raw data pointer: refuse anything else."""
    import torch

    if tuple(counts_tensor.shape) != (nk, n, n) or counts_tensor.dtype != torch.int32:
        raise ValueError(f"counts tensor must be int32 of shape {(nk, n, n)}, got {counts_tensor.dtype} "
                         f"{tuple(counts_tensor.shape)}")
    if not counts_tensor.is_contiguous():
        raise ValueError("counts tensor must be contiguous")
    if not counts_tensor.is_cuda or counts_tensor.device.index != device:
        raise ValueError(f"counts tensor must live on cuda:{device} (the engine's device), got {counts_tensor.device}")


def _counts_for(engine, nk, n, counts_tensor):
    """The (nk, n, n) int32 count tensor on the engine's GPU.  The engine writes it on its own stream, so
    torch's stream is drained first: nothing torch queued on the tensor (a zero fill, the previous
    all-reduce) may still be running when the engine starts writing."""
    import torch

    if counts_tensor is None:
        counts_tensor = torch.zeros((nk, n, n), dtype=torch.int32, device=torch.device("cuda", engine.device))
    _check_counts(counts_tensor, nk, n, engine.device)
    torch.cuda.current_stream(counts_tensor.device).synchronize()
    return counts_tensor


def merge_results(parts):
    """The SweepResults of contiguous sub-shards, in job order, as one SweepResult (counts left to the caller)."""
    from .nmf import SweepResult

    if len(parts) == 1:
        return parts[0]
    p0 = parts[0]
    cat = lambda name: np.concatenate([getattr(p, name) for p in parts])   # noqa: E731
    return SweepResult(ks=p0.ks, R=p0.R, n=p0.n, counts=None, consensus=None, labels=cat("labels"), iters=cat("iters"),
                       stopped_early=cat("stopped_early"),
                       W=sum((p.W for p in parts), []) if p0.W is not None else None,
                       H=sum((p.H for p in parts), []) if p0.H is not None else None,
                       seconds_total=max(p.seconds_total for p in parts),
                       seconds_iterate=max(p.seconds_iterate for p in parts),
                       restart_iterations=sum(p.restart_iterations for p in parts),
                       max_iter_run=max(p.max_iter_run for p in parts), job_begin=p0.job_begin,
                       job_end=parts[-1].job_end, extras={"groups": len(parts)})


class RestartGroups:
    """G restart groups on ONE GPU: G engines (each its own HIP stream, buffers and copy of A's layouts)
    over the same data matrix.  run() splits a job range into G contiguous sub-ranges, runs them from G
    host threads so the groups' launches interleave on the GPU, and sums the groups' int32 counts on the
    device.  A small shard leaves CUs idle at the all-live phase and in the tail of one group; a second
    group fills them (+1 to +2.4 % per GPU at R = 25..100 restarts per k).  Results
    are bit-identical to one group (placement never changes a bit).

    Engine-like: .m, .n, .device, .run(ks, R, job_begin=, job_end=, counts_tensor=, ...), .close()."""

    def __init__(self, A=None, device: int = -1, groups: int = 2, *, a_device_ptr: int | None = None, shape=None,
                 engine_cls=None, weights=None):
        """weights: the groups' shares of a job range (default equal; env NMFC_GROUP_WEIGHTS="w0,w1,..." when not
        given).  Placement never changes a bit, so the split is a speed choice only."""
        import os

        from .nmf import Engine

        if not 1 <= groups <= 8:
            raise ValueError("groups must be in 1..8")
        if weights is None and os.environ.get("NMFC_GROUP_WEIGHTS"):
            env = [float(x) for x in os.environ["NMFC_GROUP_WEIGHTS"].split(",")]
            weights = env if len(env) == groups else None   # the knob names a split for one group count
        if weights is not None and (len(weights) != groups or min(weights) <= 0):
            raise ValueError(f"weights must be {groups} positive numbers")
        self.weights = None if weights is None else [w / sum(weights) for w in weights]
        cls = engine_cls or Engine
        self.engines = [cls(A, device, a_device_ptr=a_device_ptr, shape=shape) for _ in range(groups)]
        e0 = self.engines[0]
        self.m, self.n, self.device = e0.m, e0.n, e0.device
        self.G = groups
        self._pool = ThreadPoolExecutor(max_workers=groups) if groups > 1 else None
        self._scratch = {}

    @property
    def h(self):   # engine-like truthiness for callers that check for a live handle
        return self.engines[0].h

    def close(self):
        for e in self.engines:
            e.close()
        if self._pool is not None:
            self._pool.shutdown()
            self._pool = None
        self._scratch = {}

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def set_timing(self, on: bool, stride: int = 1):
        for e in self.engines:
            e.set_timing(on, stride)

    def kernel_stats(self, kid: int):
        """(timed launches, ms, flop x launches, design bytes x launches, algorithmic bytes x launches) summed
        over the groups' engines for the last run."""
        c = ms = fl = b = ab = 0.0
        for e in self.engines:
            ce, mse = e.kernel_time(kid)
            be, abe = e.kernel_bytes(kid)
            c += ce
            ms += mse
            fl += e.kernel_flops(kid) * ce
            b += be * ce
            ab += abe * ce
        return int(c), ms, fl, b, ab

    def run(self, ks, R: int, *, job_begin: int = 0, job_end: int = -1, counts_tensor=None, **kw):
        """Engine.run over [job_begin, job_end) as G groups.  counts_tensor (torch int32 (nk, n, n) on this
        GPU, optional): receives the shard's counts, summed over the groups on the device; otherwise the
        result carries host counts/consensus when kw asks for them (Engine.run's want_counts)."""
        import torch

        if "counts_device_ptr" in kw:
            raise TypeError("RestartGroups.run takes counts_tensor (the groups' counts are summed into it)")
        nk = len(ks)
        jb = max(0, job_begin)
        je = nk * R if job_end < 0 else min(job_end, nk * R)
        G = min(self.G, max(1, je - jb))
        dev = torch.device("cuda", self.device)
        if counts_tensor is not None:
            _check_counts(counts_tensor, nk, self.n, self.device)
        if G == 1:
            return self.engines[0].run(ks, R, job_begin=jb, job_end=je, counts_device_ptr=None if counts_tensor is None
                                       else counts_tensor.data_ptr(), **kw)
        if self.weights is None or G != self.G:
            cuts = [jb + (je - jb) * g // G for g in range(G + 1)]
        else:
            acc = np.cumsum([0.0] + self.weights)
            cuts = [jb + int(round((je - jb) * a)) for a in acc]
            cuts[-1] = je
        sub = [(cuts[g], cuts[g + 1]) for g in range(G)]
        if any(b >= e for b, e in sub):   # a group too small for its share: equal split
            sub = [(jb + (je - jb) * g // G, jb + (je - jb) * (g + 1) // G) for g in range(G)]
        ptrs = [None] * G
        scratch = []
        if counts_tensor is not None:
            key = (nk, self.n)
            if len(self._scratch.get(key, [])) < G - 1:
                self._scratch[key] = [torch.empty((nk, self.n, self.n), dtype=torch.int32, device=dev)
                                      for _ in range(G - 1)]
            scratch = self._scratch[key][:G - 1]
            ptrs = [counts_tensor.data_ptr()] + [t.data_ptr() for t in scratch]
            torch.cuda.current_stream(dev).synchronize()   # nothing torch queued may touch them while engines write

        def one(g):
            b, e = sub[g]
            return self.engines[g].run(ks, R, job_begin=b, job_end=e, counts_device_ptr=ptrs[g], **kw)

        parts = list(self._pool.map(one, range(G)))   # each run returns after its own stream has finished
        res = merge_results(parts)
        if counts_tensor is not None:
            for t in scratch:   # the groups' counts summed on the device, in group order (exact integers)
                counts_tensor.add_(t)
            torch.cuda.current_stream(dev).synchronize()
        elif parts[0].counts is not None:
            res.counts = np.sum([p.counts for p in parts], axis=0, dtype=np.int32)
            res.consensus = res.counts / R
        return res


def run_sharded(engine, ks, R: int, *, rank: int, world: int, unit: str = "job", counts_tensor=None, group=None,
                reduce: bool = True, **run_kwargs):
    """Runs this rank's shard on `engine` (nmf.Engine, RestartGroups, or brunet.BrunetEngine with
    unit="restart") and SUM-all-reduces the counts.  `counts_tensor`: a torch.int32 CUDA tensor (nk, n, n)
    on the engine's GPU that the engine writes directly (device pointer) and RCCL reduces; allocated if
    None.  The engine's run returns after its stream has finished writing the counts, so the all-reduce
    (queued on torch's stream) reads complete data.  The all-reduce runs when reduce is set and either
    world > 1 or a process group is initialised (so a world-size-1 RCCL group exercises the collective).
    Returns (counts_tensor_after_allreduce, local SweepResult)."""
    nk = len(ks)
    counts_tensor = _counts_for(engine, nk, engine.n, counts_tensor)
    if unit == "job":
        jb, je = shard_range(nk * R, rank, world)
        if isinstance(engine, RestartGroups):
            res = engine.run(ks, R, job_begin=jb, job_end=je, counts_tensor=counts_tensor, **run_kwargs)
        else:
            res = engine.run(ks, R, job_begin=jb, job_end=je, counts_device_ptr=counts_tensor.data_ptr(), **run_kwargs)
    elif unit == "restart":
        rb, re = shard_range(R, rank, world)
        res = engine.run(ks, R, restart_begin=rb, restart_end=re, counts_device_ptr=counts_tensor.data_ptr(),
                         **run_kwargs)
    else:
        raise ValueError(f"unit must be 'job' or 'restart', got {unit!r}")
    if reduce and _dist_active(world):
        allreduce_counts(counts_tensor, group)
    return counts_tensor, res


def run_sharded_sweep(engine, ks, R: int, *, rank: int, world: int, **kw):
    """run_sharded for the MU engine (or RestartGroups): the expand.grid job list is sharded."""
    return run_sharded(engine, ks, R, rank=rank, world=world, unit="job", **kw)


def run_sharded_brunet(engine, ks, R: int, *, rank: int, world: int, **kw):
    """run_sharded for the Brunet engine: every rank runs its restart range for every k."""
    return run_sharded(engine, ks, R, rank=rank, world=world, unit="restart", **kw)


def run_sharded_with(runner, ks, R: int, n: int, *, rank: int, world: int, unit: str = "job", group=None):
    """Host-side form of run_sharded (the CPU gloo tests): `runner(begin, end)` returns this shard's
    (nk, n, n) int32 counts as a numpy array for units [begin, end) (jobs, or restarts with
    unit="restart"); the counts are SUM-all-reduced through torch.distributed."""
    import torch

    units = len(ks) * R if unit == "job" else R
    b, e = shard_range(units, rank, world)
    local = np.ascontiguousarray(runner(b, e), dtype=np.int32).reshape(len(ks), n, n)
    t = torch.from_numpy(local.copy())
    if world > 1:
        allreduce_counts(t, group)
    return t.numpy()
