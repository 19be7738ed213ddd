#!/usr/bin/env python3
"""bench.py -- NMF restarts/sec for the consensus k-sweep on MI355X (BASELINE.json metric).

A step = one full consensus sweep: every (k, restart) job of the workload runs from its libnmf
generateMatrix(ran) init through the MU iterations under the reference's stop rule (REF_COMPAT,
maxiter 10000), then labels, integer connectivity counts (RCCL SUM all-reduce when N > 1),
consensus = counts / R and the cophenetic correlation per k.  A is resident in HBM before timing.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config C3]
  N > 1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

Rank 0 prints ONE JSON line.  value = restarts completed by all ranks / max-over-ranks wall time.
Scaling: default "strong" -- the fixed job (R restarts of every k, BASELINE
north_star: "k=2..10 x 200-restart consensus ... on 8 x MI355X") is split over the N GPUs; "--scaling
weak" gives every GPU the whole per-GPU workload (the consensus is then over R x N restarts).  C4 is
always the per-GPU share of BASELINE configs[3] (1000/8 restarts of every k per GPU, weak).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

FP64_MFMA_PEAK_TFLOPS = 78.6   # MI355X dense fp64 matrix peak (spec); probe measured ~70
HBM_PEAK_GBS = 8000.0
# fp64 VALU issue: 78.6 TF = 1024 SIMDs x 2.4 GHz x 16 fp64 FMA lanes per cycle (a wave64 v_fma_f64 every 4 cycles);
# in lane-instructions per second that is 39.3 T (each FMA, add, mul or divide step counts one)
FP64_VALU_PEAK_TOPS = FP64_MFMA_PEAK_TFLOPS / 2
# Brunet: VALU lane-instructions per matrix element and iteration, per side (H update, W update), as compiled
# (csrc/brunet.hip, tools ISA listing): k FMAs of VP = W H, the divide q = a / VP (v_rcp_f64 + one Newton step
# (2 FMA) + mul + residual FMA + correction FMA = 6; 8 with the second Newton step of rounds 1-4), k FMAs
# accumulating W^T Q or Q H^T.  Round 6: N quotients share one v_rcp_f64 (batch inversion: N - 1 prefix multiplies, the
# rcp and its Newton step, 2 (N - 1) back-multiplies = 3 N instructions for N reciprocals), still 6 per quotient
BRUNET_DIV_OPS = 6
# restart groups for the whole job on one GPU (the default C3 line): the fastest measured policy (with
# the stream-K W^T A tile one group is fastest -- 500.7 vs 475.5 restarts/s for three, whose persistent launches queue behind
# each other; before it, three groups were +1.9 %)
N1_GROUPS = 1


def brunet_valu_ops_per_element(k: int) -> int:
    return 2 * (2 * k + BRUNET_DIV_OPS)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


# ------------------------------------------------------------------------------------------------
# CPU baseline: the reference's own nmf_mu (oracle/_ref, compiled from /root/reference sources) timed
# on the host cores, one single-threaded-BLAS process per core (BatchJobs njobs semantics, nmf.r:111).
# ------------------------------------------------------------------------------------------------
def _cpu_worker(args):
    os.environ["OPENBLAS_NUM_THREADS"] = "1"
    m, n, ks, T, kind = args
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np
    from nmfconsensus_amd.synthetic import planted_matrix
    import pyoracle

    A = planted_matrix(m, n)
    out = {}
    if kind == "brunet":
        O = pyoracle.Oracle()
        for k in ks:
            W0, H0 = O.brunet_init(123 + k, m, n, k)
            t0 = time.perf_counter()
            O.brunet(A, W0, H0, T, 10 ** 6, 10)
            out[k] = (time.perf_counter() - t0) / T
    elif kind == "reference":
        lib = pyoracle.RefLib()
        for k in ks:
            W0, H0 = lib.generate_ran(123 + k, m, n, k)
            t0 = time.perf_counter()
            lib.nmf_mu(A, W0, H0, T)
            out[k] = (time.perf_counter() - t0) / T
    else:
        O = pyoracle.Oracle()
        for k in ks:
            W0, H0 = O.init_restart(123 + k, m, n, k)
            t0 = time.perf_counter()
            O.nmf_mu(A, W0, H0, T, 0)
            out[k] = (time.perf_counter() - t0) / T
    return out


def host_cpu():
    """CPU model and thread counts of the host the baseline ran on (state them)."""
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"cpu_model": model, "nproc": os.cpu_count(), "affinity": len(os.sched_getaffinity(0))}


def cpu_baseline(m, n, ks, mean_iters_per_k, cores, T, brunet=False, kind="reference"):
    import multiprocessing as mp

    ref_so = os.path.join(ROOT, "oracle", "_ref", "libnmf_ref.so")
    if brunet:
        kind = "brunet"
    elif kind == "reference" and not os.path.exists(ref_so):
        raise FileNotFoundError(f"cpu_baseline kind 'reference' needs {ref_so} (built by `make -C oracle ref` where "
                                "/root/reference exists); pass --cpu-kind port to time the C restatement instead")
    ctx = mp.get_context("spawn")
    t0 = time.perf_counter()
    devnull = os.open(os.devnull, os.O_WRONLY)
    saved = os.dup(1)
    os.dup2(devnull, 1)   # the reference prints "Exiting nmf_mu after ..." per call (nmf_mu.c:296)
    try:
        with ctx.Pool(cores) as pool:
            res = pool.map(_cpu_worker, [(m, n, ks, T, kind)] * cores)
    finally:
        os.dup2(saved, 1)
        os.close(saved)
        os.close(devnull)
    wall = time.perf_counter() - t0
    t_iter = {k: sum(r[k] for r in res) / len(res) for k in ks}
    # sweep of R restarts per k on `cores` processes: CPU-seconds = R * sum_k t_iter(k) * I(k)
    per_restart_set = sum(t_iter[k] * mean_iters_per_k[k] for k in ks)
    value = len(ks) * cores / per_restart_set
    what = {"reference": "reference libnmf nmf_mu (oracle/_ref, scipy OpenBLAS, 1 thread/process)",
            "port": "oracle C restatement of nmf_mu", "brunet": "oracle C restatement of NMF.div (brunet_oracle.c)"}[kind]
    return {
        "value": value,
        "unit": "restarts/s",
        "cores": cores,
        "kind": "port" if kind == "brunet" else kind,
        "sample": (f"{what}"
                   f" x {cores} concurrent processes, {T} iterations per k={ks[0]}..{ks[-1]} on the {m}x{n} matrix; "
                   f"restarts/s extrapolated with the GPU run's mean iterations per k; sample wall {wall:.1f} s"),
        "sec_per_iter": {str(k): t_iter[k] for k in ks},
        "host": host_cpu(),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="C3", choices=["C1", "C2", "C3", "C4", "C5"])
    ap.add_argument("--maxiter", type=int, default=10000)
    ap.add_argument("--stop-rule", default="ref_compat", choices=["fixed", "ref_compat", "argmax_stable"])
    ap.add_argument("--restarts", type=int, default=None, help="override R (restarts per k)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--check-every", type=int, default=4, help="MU iterations enqueued between stop polls")
    ap.add_argument("--groups", type=int, default=0,
                    help="restart groups per GPU (engines on their own streams); 0 = auto: N1_GROUPS for the whole "
                         "job on one GPU, 2 for a strong-scaling shard (N > 1)")
    ap.add_argument("--roofline-steps", type=int, default=1,
                    help="sweeps of the separate one-group roofline pass when the timed steps use G > 1 groups")
    ap.add_argument("--overlap-host", action="store_true",
                    help="run each sweep's cophenetic step on a host thread beside the next sweep's GPU work")
    ap.add_argument("--cpu-iters", type=int, default=100, help="iterations per k in the CPU sample (~20 s wall on 16 cores)")
    ap.add_argument("--cpu-cores", type=int, default=None)
    ap.add_argument("--no-timing", action="store_true", help="disable per-launch HIP event timing")
    ap.add_argument("--timing-stride", type=int, default=5,
                    help="event-time the launches of every S-th MU iteration (S=1 times all; the default 5 is coprime "
                         "to the stop-check parity and to the poll chunk, so the sample covers odd and even "
                         "iterations and every position within a chunk)")
    ap.add_argument("--scaling", default=None, choices=["weak", "strong"],
                    help="strong (default): the fixed R restarts per k are split over the N GPUs (the north-star "
                         "job); weak: every GPU runs the full per-GPU workload (R restarts per k each, consensus "
                         "over R x N).  C4 is always weak (the per-GPU share of configs[3])")
    ap.add_argument("--simulate-world", type=int, default=0,
                    help="one-GPU replay of the N-GPU strong-scaling job: each of the N ranks' shard_range slices runs "
                         "in turn on this GPU (as restart groups, the N > 1 policy); value = restarts / max shard time. "
                         "A replay of the real shards, not a scaling curve (C3/C4 MU engine, one process)")
    ap.add_argument("--dump-iters", default=None, help="write the last step's per-job iteration counts (.npy)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="process-group backend for N > 1 (nccl = RCCL, the measured path; gloo only to rehearse "
                         "the N > 1 flow with several ranks on one GPU, together with --device)")
    ap.add_argument("--device", type=int, default=None,
                    help="HIP device of this rank (default LOCAL_RANK); rehearsal only")
    ap.add_argument("--maps-out", default=None,
                    help="write /proc/self/maps here once the library and the runtime are loaded (with Python's "
                         "faulthandler on stderr): a native crash's stack addresses can then be symbolized offline")
    ap.add_argument("--cpu-kind", default="reference", choices=["reference", "port"],
                    help="reference: the reference's own nmf_mu (oracle/_ref, fails loudly when absent); port: the "
                         "oracle's C restatement")
    args = ap.parse_args()

    import numpy as np
    import torch

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0")) if args.device is None else args.device
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        # explicit timeout: a rank that dies makes the others exit non-zero instead of blocking in the all-reduce
        from nmfconsensus_amd.distributed import init_distributed
        init_distributed(args.dist_backend, dev)

    from nmfconsensus_amd.synthetic import CONFIGS, planted_matrix
    from nmfconsensus_amd.nmf import cophenetic_batch
    from nmfconsensus_amd.distributed import RestartGroups, run_sharded_sweep, shard_range
    from nmfconsensus_amd import _lib

    if args.scaling is None:
        args.scaling = "weak" if args.config == "C4" else "strong"
    if args.config == "C5":
        return bench_brunet(args, rank, world, local, dev)
    if args.config == "C1":
        if world > 1:
            raise SystemExit("C1 is the reference's one-process case (test_nmf.r)")
        return bench_c1(args, dev)
    if args.simulate_world > 1:
        if world > 1:
            raise SystemExit("--simulate-world replays the shards in ONE process")
        return bench_simulated_world(args, dev)

    m, n, ks, R, desc = CONFIGS[args.config]
    if args.config == "C4":
        args.scaling = "weak"
        R = R // 8             # C4 is the 8-GPU job: 125 restarts of every k per GPU (at N = 8 the whole C4)
    if args.restarts:
        R = args.restarts
    if args.scaling == "weak":
        R = R * world          # whole job: R restarts per k per GPU
    nk = len(ks)
    stop_rule = {"fixed": 0, "ref_compat": 1, "argmax_stable": 2}[args.stop_rule]

    A_host = planted_matrix(m, n)
    A_dev = torch.from_numpy(A_host.T.copy()).to(dev)          # (n, m) row-major == (m, n) column-major
    torch.cuda.synchronize()
    # G restart groups per GPU (distributed.RestartGroups: G engines on their own HIP streams over the same A,
    # driven from G host threads, counts summed on the device).  Auto: the fastest measured
    # policy -- N1_GROUPS for the whole job on one GPU, 2 for a strong-scaling shard (N > 1).  Overlapping groups
    # stretch every kernel's HIP-event duration, so with G > 1 the per-kernel roofline comes from a separate
    # one-group timed pass over the same shard after the timed steps (outside the timed region).
    jb, je = shard_range(nk * R, rank, world)
    if args.groups > 0:
        G = args.groups
    elif world > 1:
        G = shard_groups(m, n, ks, jb, je, dev) if args.scaling == "strong" else 1
    else:
        G = N1_GROUPS if je - jb >= N1_GROUPS else 1
    if G > 8:
        raise SystemExit(f"--groups {G}: at most 8 restart groups per GPU")
    groups = RestartGroups(a_device_ptr=A_dev.data_ptr(), shape=(m, n), device=local, groups=G)
    dump_maps(args.maps_out)
    counts = torch.zeros((nk, n, n), dtype=torch.int32, device=dev)
    timing = not args.no_timing
    from concurrent.futures import ThreadPoolExecutor
    host = ThreadPoolExecutor(max_workers=1)

    def rho_of(cons_host):   # cophenetic correlation per k (nmf.r:165-172), the k's on parallel host threads
        r = cophenetic_batch(cons_host, symmetric=True)[0]
        return {k: float(r[i]) for i, k in enumerate(ks)}

    pending = [None]

    def step():
        # this rank's shard as G groups, counts into `counts`, RCCL SUM all-reduce when N > 1 (nmf.r:111-117)
        _, res = run_sharded_sweep(groups, ks, R, rank=rank, world=world, counts_tensor=counts, maxiter=args.maxiter,
                                   seed=123, stop_rule=stop_rule, check_every=args.check_every)
        cons = counts.to(torch.float64) / R
        rho = {}
        if rank == 0:
            cons_host = cons.cpu().numpy()
            if args.overlap_host:   # the cophenetic step of this sweep runs beside the next sweep's GPU work
                prev, pending[0] = pending[0], host.submit(rho_of, cons_host)
                rho = prev.result() if prev is not None else {}
            else:
                rho = rho_of(cons_host)
        return res, rho

    groups.set_timing(False)
    for _ in range(args.warmup):
        step()
    if pending[0] is not None:
        pending[0].result()
        pending[0] = None
    roof_pass = timing and G > 1   # per-kernel rates from a separate one-group pass (below)
    groups.set_timing(timing and not roof_pass, args.timing_stride)
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    iters_all = []
    # per kernel id: [launches, ms, flop*launches, design bytes*launches, algorithmic bytes*launches]
    acc = {kid: [0, 0.0, 0.0, 0.0, 0.0] for kid in (_lib.KID_WTA, _lib.KID_AHTW, _lib.KID_HUPD, _lib.KID_LABELS,
                                                     _lib.KID_COUNTS, _lib.KID_SMALL)}
    last = None
    for _ in range(args.steps):
        res, rho = step()
        last = (res, rho)
        iters_all.append(res.iters.copy())
        for kid, a in acc.items():
            for i, v in enumerate(groups.kernel_stats(kid)):
                a[i] += v
    if pending[0] is not None:   # the last sweep's cophenetic step is inside the timed region
        last = (last[0], pending[0].result())
        pending[0] = None
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t.item())

    if roof_pass:
        # the roofline pass: this rank's same shard on ONE restart group, HIP events as in a one-group line, after the
        # timed region (its time is not in `value`); its iterations must equal the timed sweeps' (placement never
        # changes a bit)
        one = RestartGroups(a_device_ptr=A_dev.data_ptr(), shape=(m, n), device=local, groups=1)
        scratch = torch.zeros_like(counts)
        one.set_timing(True, args.timing_stride)
        for _ in range(args.roofline_steps):
            _, r1 = run_sharded_sweep(one, ks, R, rank=rank, world=world, counts_tensor=scratch, reduce=False,
                                      maxiter=args.maxiter, seed=123, stop_rule=stop_rule, check_every=args.check_every)
            for kid, a in acc.items():
                for i, v in enumerate(one.kernel_stats(kid)):
                    a[i] += v
            if not np.array_equal(r1.iters, last[0].iters):
                raise SystemExit("roofline pass: iterations differ from the timed sweeps")
        one.close()
        torch.cuda.synchronize()

    res, rho = last
    if args.dump_iters and rank == 0:
        np.save(args.dump_iters, np.stack([np.asarray(ks)[np.arange(jb, je) % nk], res.iters]))
    total_restarts = nk * R * args.steps
    value = total_restarts / elapsed
    its = np.concatenate(iters_all)
    local_jobs = np.arange(jb, je)
    mean_iter_k = {k: float(np.mean(res.iters[(local_jobs % nk) == i])) for i, k in enumerate(ks)
                   if np.any((local_jobs % nk) == i)}
    log(f"[bench] rank {rank}: {je - jb} restarts/step, mean iters {its.mean():.1f} (max {its.max()}), "
        f"step {elapsed / args.steps:.3f} s, engine {res.seconds_total:.3f} s (iterate {res.seconds_iterate:.3f} s)")

    roof = None
    if timing and ((acc[_lib.KID_WTA][0] and acc[_lib.KID_AHTW][0]) or acc[_lib.KID_SMALL][0]):
        kernels = {}
        names = {_lib.KID_WTA: "wta", _lib.KID_AHTW: "ahtw", _lib.KID_HUPD: "hupdate", _lib.KID_LABELS: "labels",
                 _lib.KID_COUNTS: "counts", _lib.KID_SMALL: "small_mu"}
        for kid, (c, ms, fl, b, ab) in acc.items():
            if not c:
                continue
            avg_ms = ms / c
            kr = {"launches": c, "avg_ms": avg_ms, "algo_bytes_per_launch": ab / c, "design_bytes_per_launch": b / c,
                  "gbs": ab / c / (avg_ms * 1e-3) / 1e9, "design_gbs": b / c / (avg_ms * 1e-3) / 1e9}
            kr["frac_hbm"] = kr["gbs"] / HBM_PEAK_GBS
            if fl:
                kr["algo_flop_per_launch"] = fl / c
                kr["tflops"] = fl / c / (avg_ms * 1e-3) / 1e12
                kr["bound"] = "mfma"
                kr["frac"] = kr["tflops"] / FP64_MFMA_PEAK_TFLOPS
            elif kid == _lib.KID_COUNTS:
                # R n^2 label compare-adds per k group (nmf.r:140-141): integer VALU work, not HBM traffic
                ops = float(je - jb) * n * n
                kr["int_ops_per_launch"] = ops
                kr["gops"] = ops / (avg_ms * 1e-3) / 1e9
                kr["bound"] = "valu (int32 compare + add; HBM bytes reported beside)"
                kr["frac"] = None
            else:
                kr["bound"] = "hbm"
                kr["frac"] = kr["frac_hbm"]
            kernels[names[kid]] = kr
        if rank == 0:
            kernels.update(side_kernels(A_dev, m, n, max(ks)))
        dom = max([x for x in ("wta", "ahtw", "small_mu") if x in kernels],
                  key=lambda s: kernels[s]["avg_ms"] * kernels[s]["launches"])
        ach = kernels[dom]["tflops"]
        roof = {"bound": "mfma", "kernel": dom, "achieved": ach, "peak": FP64_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": ach / FP64_MFMA_PEAK_TFLOPS, "traffic": None,
                "frac_metric": "algorithmic fp64 TFLOP/s (2mnk + 2mk^2 per live restart) / 78.6 TF", "frac_metric_version": 1,
                "algo_bytes_per_launch": kernels[dom]["algo_bytes_per_launch"], "kernels": kernels,
                "note": ("achieved = algorithmic flop per launch (SURVEY 8(d): 2mnk + 2mk^2 per live restart) / "
                         "the kernel's mean HIP-event duration over the timed launches of the timed sweeps (every "
                         f"{args.timing_stride}th MU iteration's launches, plus every labels/counts "
                         "launch; 'launches' counts the timed ones); kernels[*] with bound 'hbm': algorithmic bytes "
                         "per launch / mean duration vs 8 TB/s"),
                "timing_stride": args.timing_stride}
        if roof_pass:
            roof["note"] += (f"; the timed steps ran {G} restart groups per GPU on their own streams (whose "
                             "concurrent kernels would stretch each other's HIP-event durations), so these per-kernel "
                             f"rates come from a separate one-group pass over the same shard ({args.roofline_steps} "
                             "sweep(s), after the timed region, iterations checked equal)")
            roof["source"] = f"one-group roofline pass, {args.roofline_steps} sweep(s)"
        tp = pmc_profile_for({"config": args.config, "stop_rule": args.stop_rule, "maxiter": args.maxiter,
                              "restarts": R})
        if tp:
            attach_traffic(roof, kernels, dom, *tp)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cores = args.cpu_cores or min(16, len(os.sched_getaffinity(0)))
        try:
            cpu = cpu_baseline(m, n, ks, mean_iter_k, cores, args.cpu_iters, kind=args.cpu_kind)
        except Exception as ex:  # reported loudly in the line and on stderr, never fatal for the GPU number
            log(f"[bench] CPU BASELINE FAILED: {ex!r}")
            cpu = {"value": None, "error": repr(ex), "kind": args.cpu_kind}

    if rank == 0:
        per_gpu = R / world if args.scaling == "strong" else R // world
        out = {
            "metric": metric_name(args.config, m, n, ks),
            "value": value,
            "unit": "restarts/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (planted 4-group matrix, splitmix64 seed 20261015; per-job generateMatrix(ran) init)",
            "config": {"workload": (f"{args.config}: synthetic {m}x{n} fp64, k={ks[0]}..{ks[-1]}, {R} restarts per k "
                                    f"({nk * R} jobs) in total, {per_gpu:g} restarts per k per GPU, stop rule "
                                    f"{args.stop_rule}, maxiter {args.maxiter}"),
                       "m": m, "n": n, "ks": ks, "restarts_per_k": R, "restarts_per_k_per_gpu": per_gpu,
                       "jobs": nk * R,
                       "parallelism": f"jobs sharded over {world} GPU(s) ({args.scaling} scaling), "
                                      f"{G} restart group(s) per GPU, "
                                      + ("RCCL int32 all-reduce of counts" if args.dist_backend == "nccl"
                                         else "gloo int32 all-reduce of counts (rehearsal, not a measurement)"),
                       "groups_per_gpu": G,
                       "mean_iterations": float(its.mean()), "max_iterations": int(its.max()),
                       "cophenetic_rho": {str(k): v for k, v in rho.items()}},
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    groups.close()
    if world > 1:
        torch.distributed.destroy_process_group()


def bench_c1(args, dev):
    """BASELINE configs[0], the reference's own CPU-runnable case: test_nmf.r's
    runNMFinJobs(read.gct("20+20x1000.gct"), k = 2:5, num.clusterings = 5, maxniter = 10000, seed = 123, njobs = 1)
    -- 20 restarts (jobs in expand.grid order, job seed = seed + job_id - 1) on the bundled gct (its 1000 x 40
    matrix from tests/golden/golden.npz, written there from the reference's file), REF_COMPAT stop rule.
    A step = the batched sweep (one nmfc_engine_run: init, MU loops, labels, counts, consensus) -> `value`.
    Beside it, timed once each: `dropin_flow` = the 20 restarts through the drop-in nmf_mu one call after another
    (what nmf.r does unchanged on this library), and `cpu_baseline` = the same 20 calls of the REFERENCE's own
    nmf_mu (oracle/_ref) on one core, as test_nmf.r's njobs = 1; both from the engine's init, whose W0/H0 equal
    the reference's generateMatrix(ran) bit for bit (tests/test_gpu_parity.py), and their iteration counts
    must agree with the sweep's."""
    import numpy as np
    import torch

    from nmfconsensus_amd import _lib, libnmf
    from nmfconsensus_amd.nmf import Engine

    with np.load(os.path.join(ROOT, "tests", "golden", "golden.npz"), allow_pickle=False) as z:
        A = np.asfortranarray(z["A_gct"])
    m, n = A.shape
    ks, R, seed = [2, 3, 4, 5], 5, 123
    stop_rule = {"fixed": 0, "ref_compat": 1, "argmax_stable": 2}[args.stop_rule]
    eng = Engine(A, device=dev.index)
    for _ in range(args.warmup):
        eng.run(ks, R, maxiter=args.maxiter, seed=seed, stop_rule=stop_rule)
    eng.set_timing(not args.no_timing, 1)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res = eng.run(ks, R, maxiter=args.maxiter, seed=seed, stop_rule=stop_rule)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    value = len(ks) * R * args.steps / elapsed
    roof = None
    c, ms = eng.kernel_time(_lib.KID_SMALL)
    if c:
        fl = eng.kernel_flops(_lib.KID_SMALL)
        ach = fl / (ms / c * 1e-3) / 1e12
        roof = {"bound": "mfma", "kernel": "small_mu", "achieved": ach, "peak": FP64_MFMA_PEAK_TFLOPS,
                "unit": "TFLOP/s", "frac": ach / FP64_MFMA_PEAK_TFLOPS, "traffic": None,
                "frac_metric": "algorithmic fp64 TFLOP/s / 78.6 TF", "frac_metric_version": 1,
                "note": "the small-shape phase (every restart's whole MU loop in one launch per kernel: k_solo_mu / "
                        "k_solo8_mu one workgroup per restart at m <= 1024, n <= 40, ranks 2..8; k_small_mu blocks "
                        "otherwise): algorithmic flop of all restart-iterations (4mnk + 4(m+n)k^2 each) / the phase's "
                        "HIP-event duration; latency-bound (the longest restart sets it), SURVEY 8(d): C1/C2 fit in L2"}
    init = eng.run(ks, R, maxiter=0, seed=seed, want_factors=True, want_counts=False)
    eng.close()
    its = np.asarray(res.iters)
    jobs = [(np.asfortranarray(init.W[j]), np.asfortranarray(init.H[j])) for j in range(len(ks) * R)]
    devnull = os.open(os.devnull, os.O_WRONLY)
    saved = os.dup(1)
    os.dup2(devnull, 1)   # nmf_mu prints "Exiting nmf_mu after ..." per call (nmf_mu.c:296)
    try:
        for kk in sorted({W0.shape[1] for W0, _ in jobs}):   # each path's code objects and A copy: not timed
            libnmf.nmf_mu(A, *next(j for j in jobs if j[0].shape[1] == kk), 10)
        t0 = time.perf_counter()
        dropin_its = [libnmf.nmf_mu(A, W0, H0, args.maxiter)["maxiter"] for W0, H0 in jobs]
        t_dropin = time.perf_counter() - t0
        cpu = None
        if not args.no_cpu_baseline:
            sys.path.insert(0, os.path.join(ROOT, "oracle"))
            from pyoracle import RefLib
            ref = RefLib()
            t0 = time.perf_counter()
            ref_its = [ref.nmf_mu(A, W0, H0, args.maxiter)[2] for W0, H0 in jobs]
            t_ref = time.perf_counter() - t0
    finally:
        os.dup2(saved, 1)
        os.close(saved)
        os.close(devnull)
    if not args.no_cpu_baseline:
        cpu = {"value": len(jobs) / t_ref, "unit": "restarts/s", "cores": 1, "kind": "reference",
               "sample": ("the whole C1 job: the reference's own nmf_mu (oracle/_ref, scipy OpenBLAS, 1 thread) on the "
                          f"20 restarts one after another, as test_nmf.r's njobs = 1; {t_ref * 1e3:.1f} ms"),
               "iterations_equal": bool(np.array_equal(np.asarray(ref_its), its)), "host": host_cpu()}
    out = {
        "metric": metric_name("C1", m, n, ks), "value": value, "unit": "restarts/s", "n_gpus": 1,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f64",
        "data": "the reference's bundled 20+20x1000.gct matrix (tests/golden/golden.npz); per-job generateMatrix(ran) init",
        "config": {"workload": "C1: test_nmf.r -- runNMFinJobs(gct 1000x40, k=2:5, num.clusterings=5, maxniter=10000, "
                               "seed=123), 20 restarts, stop rule " + args.stop_rule,
                   "m": m, "n": n, "ks": ks, "restarts_per_k": R, "jobs": len(jobs),
                   "mean_iterations": float(its.mean()), "max_iterations": int(its.max())},
        "dropin_flow": {"value": len(jobs) / t_dropin, "unit": "restarts/s",
                        "what": "the 20 restarts through the drop-in nmf_mu one call after another (nmf.r's .C path "
                                f"unchanged; per call k_solo_mu at k = 2..4, k_team_mu at k = 5); {t_dropin * 1e3:.1f} ms",
                        "iterations_equal": bool(np.array_equal(np.asarray(dropin_its), its))},
        "roofline": roof, "cpu_baseline": cpu,
    }
    print(json.dumps(out), flush=True)


def bench_simulated_world(args, dev):
    """--simulate-world N: the N real shards of the strong-scaling job (distributed.shard_range over the
    expand.grid job list, each as restart groups like an N > 1 rank) replayed one after another on this GPU.
    A step = all N shards; the simulated N-GPU wall time of a step is its slowest shard, value = restarts /
    that time (what N GPUs would deliver if each ran its shard at this GPU's speed; the all-reduce of 9 MB of
    counts is not included).  The counts of all shards are summed and checked against a one-GPU sweep."""
    import numpy as np
    import torch

    from nmfconsensus_amd.distributed import RestartGroups, run_sharded_sweep
    from nmfconsensus_amd.synthetic import CONFIGS, planted_matrix

    W = args.simulate_world
    m, n, ks, R, _ = CONFIGS[args.config]
    # C4 is replayed as the whole 8-GPU job of BASELINE configs[3] (R = 1000 over W shards, 1750 jobs each at W = 8),
    # not the per-GPU share the C4 line runs
    if args.restarts:
        R = args.restarts
    nk = len(ks)
    stop_rule = {"fixed": 0, "ref_compat": 1, "argmax_stable": 2}[args.stop_rule]
    A_dev = torch.from_numpy(planted_matrix(m, n).T.copy()).to(dev)
    torch.cuda.synchronize()
    G = args.groups if args.groups > 0 else max(shard_groups(m, n, ks, *shard_range_(nk * R, r, W), dev) for r in range(W))
    grp = RestartGroups(a_device_ptr=A_dev.data_ptr(), shape=(m, n), device=dev.index, groups=G)
    part = torch.zeros((nk, n, n), dtype=torch.int32, device=dev)
    total = torch.zeros_like(part)
    shard_s = np.zeros((args.steps, W))
    iters = []

    def shard(r):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        _, res = run_sharded_sweep(grp, ks, R, rank=r, world=W, counts_tensor=part, reduce=False,
                                   maxiter=args.maxiter, seed=123, stop_rule=stop_rule, check_every=args.check_every)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        log(f"[sim{W}] shard {r}: {len(res.iters)} jobs, {dt:.3f} s, mean iters {np.mean(res.iters):.1f}, "
            f"max {int(np.max(res.iters))}")
        return dt, res

    for _ in range(args.warmup):
        for r in range(W):
            shard(r)
    for s_ in range(args.steps):
        total.zero_()
        its = []
        shard_maxit = []
        for r in range(W):
            shard_s[s_, r], res = shard(r)
            total += part
            its.append(res.iters)
            shard_maxit.append(int(np.max(res.iters)))
        iters = np.concatenate(its)
    grp.close()
    worst = shard_s.max(axis=1).mean()
    value = nk * R / worst
    if args.dump_iters:
        np.save(args.dump_iters, np.stack([np.asarray(ks)[np.arange(nk * R) % nk], iters]))
    import hashlib
    counts_host = total.cpu().numpy()
    counts_sha = hashlib.sha256(counts_host.tobytes()).hexdigest()
    diag_ok = bool(all(np.all(np.diagonal(counts_host[i]) == R) for i in range(nk)))
    sym_ok = bool(np.array_equal(counts_host, np.transpose(counts_host, (0, 2, 1))))
    if nk * R <= 4000:
        # the sum of the shards' counts equals one whole sweep's (placement never changes a bit)
        ref = RestartGroups(a_device_ptr=A_dev.data_ptr(), shape=(m, n), device=dev.index, groups=1)
        whole = torch.zeros_like(part)
        _, rw = run_sharded_sweep(ref, ks, R, rank=0, world=1, counts_tensor=whole, reduce=False, maxiter=args.maxiter,
                                  seed=123, stop_rule=stop_rule, check_every=args.check_every)
        ref.close()
        same = bool(torch.equal(whole, total)) and bool(np.array_equal(rw.iters, iters))
    else:
        # the whole job on one GPU would take as long as all shards again (C4: 14 000 jobs); the shards' summed
        # counts are checked for the invariants instead (diagonal = R, symmetric) and fingerprinted, and
        # --dump-iters lets the golden jobs of every shard be compared with the reference offline
        same = None
    out = {
        "metric": metric_name(args.config, m, n, ks) + f" [one-GPU replay of the {W}-GPU strong-scaling shards]",
        "value": value, "unit": "restarts/s", "n_gpus": 1, "simulated_world": W, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": worst * 1e3, "higher_is_better": True, "scaling": "strong (simulated)",
        "vs_baseline": None, "dtype": "f64", "data": "synthetic (planted 4-group matrix, splitmix64 seed 20261015)",
        "config": {"workload": f"{args.config}: synthetic {m}x{n} fp64, k={ks[0]}..{ks[-1]}, {R} restarts per k, "
                               f"{nk * R} jobs split into {W} shard_range slices, {G} restart groups each",
                   "per_gpu_restarts_per_s": value / W, "shard_seconds": shard_s.mean(axis=0).tolist(),
                   "shard_jobs": [int(b - a) for a, b in (shard_range_(nk * R, r, W) for r in range(W))],
                   "counts_equal_whole_sweep": same, "counts_sum_sha256": counts_sha,
                   "counts_diag_equals_R": diag_ok, "counts_symmetric": sym_ok,
                   "shard_max_iterations": [int(x) for x in shard_maxit], "mean_iterations": float(iters.mean()),
                   "max_iterations": int(iters.max())},
    }
    print(json.dumps(out), flush=True)
    if same is False or not (diag_ok and sym_ok):
        raise SystemExit("simulated shards' counts differ from the whole sweep")


def shard_range_(njobs, rank, world):
    from nmfconsensus_amd.distributed import shard_range
    return shard_range(njobs, rank, world)


def shard_groups(m, n, ks, jb, je, dev):
    """Restart groups for a strong-scaling shard (jobs jb..je-1 of the expand.grid list): 2 where the shard's full-load
    W^T A grid stays below one round of the big tile on this GPU's CUs -- the engine then runs the one-item-per-workgroup
    tile and a second group fills the partial rounds (R = 25 per GPU, the 8-GPU C3 shard: +1 to +2.4 %) -- else 1: the
    stream-K tile already splits the last round over every CU, and two groups' persistent launches queue behind each
    other (R = 50: 456.1 vs 443.1 restarts/s; R = 100: 477.8 vs 479.4, tied; profiles/r06/groups_sk/).  A speed choice
    only; the packing estimate (columns = sum of k, 64 per panel, 4 panels per group) need not match the engine's exactly."""
    import math
    import torch
    if je - jb < 2:
        return 1
    cols = sum(ks[j % len(ks)] for j in range(jb, je))
    ngroups = math.ceil(math.ceil(cols / 64) / 4)
    m_pad = -(-m // 128) * 128
    items = ngroups * math.ceil(n / 128) * math.ceil(m_pad / 2048)
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    return 1 if (math.ceil(n / 128) >= 4 and items >= ncu) else 2


def dump_maps(path):
    """The process's load map (for symbolizing a native crash's return addresses against the same libraries)."""
    if path:
        import faulthandler
        faulthandler.enable()
        with open("/proc/self/maps") as src, open(path, "w") as dst:
            dst.write(src.read())


def metric_name(config, m, n, ks):
    if config in ("C3", "C5"):   # BASELINE.json metric, verbatim
        base = "NMF restarts/sec (k=2..10 sweep, 20k×500 fp64) + fp64-MFMA/HBM roofline %"
        return base if config == "C3" else base.replace("NMF restarts", "Brunet KL-divergence NMF restarts")
    return f"NMF restarts/sec (k={ks[0]}..{ks[-1]} sweep, {m}×{n} fp64) + fp64-MFMA/HBM roofline %"


def side_kernels(A_dev, m, n, k, reps=3):
    """HBM roofline of calculateNorm / calculateMaxchange (calculatenorm.c:58-66, calculatemaxchange.c:55-60)
    on the config's A (device-resident) with W, H of rank k: the libnmf convergence reductions, run beside the
    sweep (the reference's nmf_mu leaves them commented out, nmf_mu.c:220-237; the TOLX stop rule uses the
    max-change form)."""
    import ctypes
    import torch
    from nmfconsensus_amd import _lib

    L = _lib.lib()
    st = ctypes.c_void_p(torch.cuda.current_stream(A_dev.device).cuda_stream)   # the operands' producer stream
    g = torch.Generator(device=A_dev.device).manual_seed(7)
    W = torch.rand((k, m), dtype=torch.float64, device=A_dev.device, generator=g)   # (m x k) column-major
    H = torch.rand((n, k), dtype=torch.float64, device=A_dev.device, generator=g)   # (k x n) column-major
    D = torch.empty_like(A_dev)
    M0 = torch.empty_like(A_dev)
    torch.cuda.synchronize()
    out = {}
    v, ms = ctypes.c_double(0.0), ctypes.c_double(0.0)
    # one untimed call of each pass first: the first launch of a kernel loads its code object
    L.nmfc_calculate_norm_dev(A_dev.data_ptr(), W.data_ptr(), H.data_ptr(), D.data_ptr(), m, n, k, ctypes.byref(v),
                              ctypes.byref(ms), st)
    M0.copy_(A_dev)
    torch.cuda.synchronize()
    L.nmfc_calculate_maxchange_dev(D.data_ptr(), M0.data_ptr(), m, n, 2.0 ** -26.5, ctypes.byref(v), ctypes.byref(ms), st)
    t = []
    for _ in range(reps):
        rc = L.nmfc_calculate_norm_dev(A_dev.data_ptr(), W.data_ptr(), H.data_ptr(), D.data_ptr(), m, n, k,
                                       ctypes.byref(v), ctypes.byref(ms), st)
        if rc != 0:
            return {}
        t.append(ms.value)
    ab = 16.0 * m * n + 8.0 * (m + n) * k    # A read, d written, W and H read once
    avg = sum(t) / len(t)
    out["norm"] = {"launches": reps, "avg_ms": avg, "algo_bytes_per_launch": ab, "gbs": ab / (avg * 1e-3) / 1e9,
                   "bound": "hbm", "shape": f"{m}x{n}, k={k}"}
    t = []
    for _ in range(reps):
        M0.copy_(A_dev)
        torch.cuda.synchronize()
        rc = L.nmfc_calculate_maxchange_dev(D.data_ptr(), M0.data_ptr(), m, n, 2.0 ** -26.5, ctypes.byref(v),
                                            ctypes.byref(ms), st)
        if rc != 0:
            return out
        t.append(ms.value)
    ab = 24.0 * m * n                        # mat, mat0 read, mat0 written
    avg = sum(t) / len(t)
    out["maxchange"] = {"launches": reps, "avg_ms": avg, "algo_bytes_per_launch": ab,
                        "gbs": ab / (avg * 1e-3) / 1e9, "bound": "hbm", "shape": f"{m}x{n}"}
    for kr in out.values():
        kr["frac_hbm"] = kr["frac"] = kr["gbs"] / HBM_PEAK_GBS
        kr["design_bytes_per_launch"], kr["design_gbs"] = kr["algo_bytes_per_launch"], kr["gbs"]
    return out


PMC_NAMES = {"wta": ("k_wta2", "k_wta2_sk", "k_wta_narrow", "k_wta_narrow_lc"), "ahtw": ("k_ahtw4",), "hupdate": ("k_hupdate",),
             "labels": ("k_labels",), "counts": ("k_counts",)}


# the workload tools/profile_round.sh profiles (the default C3 line); profiles written before round 6 carry no
# "workload" record and were all taken on exactly this command
PMC_DEFAULT_WORKLOAD = {"config": "C3", "stop_rule": "ref_compat", "maxiter": 10000, "restarts": 200}


def pmc_profile_for(workload):
    """HBM bytes per launch of the engine kernels from the newest committed PMC passes (tools/profile_round.sh:
    FETCH_SIZE x 2 + WRITE_SIZE, averaged over every launch of one sweep like `achieved`; the variants of one
    kernel pooled by launch count) -- used only when the profile was taken on THIS kernel source (its recorded
    source hash matches) AND on this line's workload (config, stop rule, maxiter, restarts: a FIXED-1000 sweep
    launches every kernel at full load, so a REF_COMPAT sweep's per-launch average does not describe it), so the
    figures cannot go stale or be borrowed silently.  Returns ({kernel: bytes}, source) or None."""
    from nmfconsensus_amd.build import source_sha256

    import glob
    sha = source_sha256()
    for tp in sorted(glob.glob(os.path.join(ROOT, "profiles", "**", "pmc_traffic.json"), recursive=True), reverse=True):
        try:
            pm = json.load(open(tp))
        except Exception:
            continue
        if pm.get("source_sha256") != sha or pm.get("workload", PMC_DEFAULT_WORKLOAD) != workload:
            continue
        per = {}
        for k, names in PMC_NAMES.items():
            rows = [pm[nm] for nm in names if nm in pm and pm[nm].get("launches")]
            if rows:
                per[k] = sum(r["hbm_bytes_per_launch"] * r["launches"] for r in rows) / sum(r["launches"] for r in rows)
        return per, os.path.relpath(tp, ROOT)
    log(f"[bench] no committed PMC profile matches this kernel source and workload {workload}: roofline.traffic = null")
    return None


def attach_traffic(roof, kernels, dom, per, src):
    """Counter bytes per launch into the roofline object.  Counter traffic can never be below the algorithmic bytes
    (every algorithmic byte crosses HBM at least once): a profile that says so describes another workload, and
    its figure is dropped (null, with the reason) instead of reported."""
    note = (f"HBM bytes per launch (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, {src}, same kernel source and workload), "
            "averaged over every launch of one sweep like `achieved`")
    rejected = []
    for kname, b in per.items():
        if kname not in kernels:
            continue
        kr = kernels[kname]
        if b < kr.get("algo_bytes_per_launch", 0.0):
            rejected.append(kname)
            continue
        kr["traffic_bytes_per_launch"] = b
        kr["traffic_gbs"] = b / (kr["avg_ms"] * 1e-3) / 1e9
        kr["traffic_frac_hbm"] = kr["traffic_gbs"] / HBM_PEAK_GBS
    if dom in per and dom not in rejected:
        roof["traffic"], roof["traffic_unit"] = per[dom], note
    if rejected:
        roof["traffic_rejected"] = (f"{src}: counter bytes below the algorithmic bytes for {rejected} -- not this "
                                    "workload's traffic; reported as null")


def bench_brunet(args, rank, world, local, dev):
    """BASELINE configs[4]: Brunet KL-divergence MU sweep (nmfc_brunet_*).  A step = the whole
    nmfconsensus sweep (k = 2..10, R restarts each, NMF.div stop rule stopconv 40 / stopfreq 10,
    maxniter 2000) with labels, int32 counts (RCCL all-reduce when N > 1), consensus and cophenetic.
    Restarts are sharded over ranks (every rank runs its restart range for every k)."""
    import numpy as np
    import torch

    from nmfconsensus_amd.synthetic import CONFIGS, planted_matrix
    from nmfconsensus_amd.nmf import cophenetic
    from nmfconsensus_amd.brunet import BrunetEngine
    from nmfconsensus_amd.distributed import run_sharded_brunet, shard_range
    from nmfconsensus_amd import _lib

    m, n, ks, R, desc = CONFIGS["C5"]
    if args.restarts:
        R = args.restarts
    if args.scaling == "weak":
        R = R * world          # whole job: R restarts per k per GPU
    nk = len(ks)
    maxiter = min(args.maxiter, 2000)
    A_host = planted_matrix(m, n)
    A_dev = torch.from_numpy(A_host.T.copy()).to(dev)
    torch.cuda.synchronize()
    eng = BrunetEngine(a_device_ptr=A_dev.data_ptr(), shape=(m, n), device=local)
    dump_maps(args.maps_out)
    counts = torch.zeros((nk, n, n), dtype=torch.int32, device=dev)
    rb, re = shard_range(R, rank, world)
    timing = not args.no_timing

    def step():
        _, res = run_sharded_brunet(eng, ks, R, rank=rank, world=world, counts_tensor=counts, maxiter=maxiter,
                                    seed=123456789)
        cons = counts.to(torch.float64) / R
        rho = {}
        if rank == 0:
            C = cons.cpu().numpy()
            for i, k in enumerate(ks):
                rho[k] = cophenetic(C[i])[0]
        return res, rho

    eng.set_timing(False)
    for _ in range(args.warmup):
        step()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    iters_all, last = [], None
    for _ in range(args.steps):
        res, rho = step()
        last = (res, rho)
        iters_all.append(res.iters.copy())
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t.item())
    res, rho = last
    value = nk * R * args.steps / elapsed
    its = np.concatenate(iters_all)
    B = re - rb
    mean_iter_k = {k: float(np.mean(res.iters[i * B:(i + 1) * B])) for i, k in enumerate(ks)}
    log(f"[bench C5] rank {rank}: {nk * B} restarts/step, mean iters {its.mean():.1f} (max {its.max()}), "
        f"step {elapsed / args.steps:.3f} s, engine {res.seconds_total:.3f} s")
    # whole-sweep algorithmic rate: every restart-iteration does 8 m n k flop of rank-k products
    ks_job = np.repeat(np.array(ks), B)
    sweep_flop = float(np.sum(8.0 * m * n * ks_job * res.iters)) * world
    roof = None
    if timing and rank == 0:
        # Kernel roofline: the timed sweep runs several k batches concurrently on separate streams, so
        # per-launch events there overlap.  The kernels' own rates come from a serialized pass (one
        # lane) over the same matrix: every k, R restarts, 40 fixed iterations, HIP events per launch.
        eng.set_timing(True)
        # per kernel: [launches, ms, rank-k flop x launches, VALU lane-instructions x launches]
        kacc = {kid: [0, 0.0, 0.0, 0.0] for kid in (_lib.BK_HNUM, _lib.BK_HUPD, _lib.BK_WUPD)}
        for k in ks:
            eng.run([k], R, maxiter=40, stopconv=10 ** 6, want_counts=False, lanes=1)
            for kid, a in kacc.items():
                c, ms, fl = eng.kernel_time(kid)
                a[0] += c
                a[1] += ms
                a[2] += fl * c
                # rank-k flop per launch = 4 m n k per restart (one side): elements x (2k + DIV) VALU ops
                a[3] += fl * c / (4.0 * k) * (2 * k + BRUNET_DIV_OPS)
        kernels = {}
        for name, kid in (("hnum", _lib.BK_HNUM), ("hupd", _lib.BK_HUPD), ("wupd", _lib.BK_WUPD)):
            c, ms, fl, ops = kacc[kid]
            kernels[name] = {"launches": c, "avg_ms": ms / max(c, 1)}
            if fl:
                kernels[name]["algo_flop_per_launch"] = fl / c
                kernels[name]["tflops"] = fl / c / (ms / c * 1e-3) / 1e12
                kernels[name]["valu_ops_per_launch"] = ops / c
                kernels[name]["valu_tops"] = ops / c / (ms / c * 1e-3) / 1e12
                kernels[name]["frac_valu"] = kernels[name]["valu_tops"] / FP64_VALU_PEAK_TOPS
        dom = max(("hnum", "wupd"), key=lambda s: kernels[s]["avg_ms"] * kernels[s]["launches"])
        ach = kernels[dom]["valu_tops"]
        sweep_ops = float(np.sum(m * n * np.array([brunet_valu_ops_per_element(int(k)) for k in ks_job]) * res.iters)) * world
        roof = {"bound": "valu", "kernel": dom, "achieved": ach, "peak": FP64_VALU_PEAK_TOPS,
                "unit": "T fp64 VALU lane-instructions/s", "frac": ach / FP64_VALU_PEAK_TOPS, "traffic": None,
                # what `frac` measures (round 4 changed it from rank-k TFLOP/s vs 78.6 TF, which stays as
                # rank_k_frac_of_78.6TF): compare lines of the same frac_metric only
                "frac_metric": "fp64 VALU lane-instructions / 39.3 T (2k + BRUNET_DIV_OPS per quotient, pinned to "
                               "the ISA by tests/test_kernel_resources.py)",
                # version 3 (round 5): one Newton step in the divide, BRUNET_DIV_OPS 8 -> 6 per quotient
                "frac_metric_version": 3,
                "kernels": kernels,
                "rank_k_tflops": kernels[dom]["tflops"], "rank_k_frac_of_78.6TF": kernels[dom]["tflops"] / FP64_MFMA_PEAK_TFLOPS,
                "sweep_valu_tops": sweep_ops / (elapsed / args.steps) / 1e12,
                "sweep_tflops": sweep_flop / (elapsed / args.steps) / 1e12,
                "valu_ops_per_element_iteration": {str(k): brunet_valu_ops_per_element(k) for k in ks},
                "note": "fp64 VALU issue roofline: per matrix element and iteration 2 x (2k FMA + the compiled divide, "
                        f"{BRUNET_DIV_OPS} VALU instructions: the reciprocal (rcp + 1 Newton step, or its share of a batch "
                        "inversion: 3 per quotient either way) + mul + residual + correction), peak "
                        "= 1024 SIMDs x 2.4 GHz x 16 fp64 lanes per cycle = 39.3 T lane-instructions/s (the 78.6 TF "
                        "fp64 vector spec / 2); v_rcp_f64 (about 3 FMA issue slots, tools/quot_probe.hip rate mode) is "
                        "counted as one slot and address arithmetic not at all, so "
                        "the fraction is a lower bound on VALU issue use; kernel rates from a serialized 40-iteration "
                        "pass per k (R restarts); rank_k_tflops counts the 8 m n k product flops alone"}
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cores = args.cpu_cores or min(16, len(os.sched_getaffinity(0)))
        try:
            cpu = cpu_baseline(m, n, ks, mean_iter_k, cores, max(2, args.cpu_iters // 20), brunet=True)
        except Exception as ex:
            log(f"[bench] cpu baseline failed: {ex!r}")
    if rank == 0:
        out = {
            "metric": "NMF restarts/sec (Brunet KL-divergence MU, k=2..10 sweep, 20k×500 fp64) + fp64 roofline %",
            "value": value, "unit": "restarts/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": args.scaling,
            "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (planted 4-group matrix, splitmix64 seed 20261015; per-restart set.seed(rseed+i) runif init)",
            "config": {"workload": f"C5: {desc}, NMF.div stopconv 40 stopfreq 10, maxniter {maxiter}", "m": m, "n": n,
                       "ks": ks, "restarts_per_k": R, "jobs": nk * R,
                       "parallelism": f"restarts sharded over {world} GPU(s) ({args.scaling} scaling), "
                                      "RCCL int32 all-reduce of counts",
                       "mean_iterations": float(its.mean()), "max_iterations": int(its.max()),
                       "cophenetic_rho": {str(k): v for k, v in rho.items()}},
            "roofline": roof, "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    eng.close()
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
