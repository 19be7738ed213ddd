"""Cross-rank job hand-out for the N-GPU sweep, evaluated before building it.

Event simulation of N ranks running the C3 job grid with the engine's host policy (a poll every `check`
iterations, a repack when 1/`div` of the live restarts have stopped), driven by the REFERENCE's own per-job
iteration counts (tests/golden/golden_c3.npz: the reference nmf_mu on all 1800 jobs) and the per-iteration cost of
one shard measured on MI355X, f(L) = max(56, 55 + 0.72 L) us with L live columns (shard 2
trace).  Policies:
  static      every rank runs its contiguous shard (distributed.shard_range), as the product does;
  hand-out φ  each rank starts with the first φ of its shard; the rest goes to one shared FIFO queue, and a rank
              admits queued jobs into the columns its repacks free (job base iteration = the next even iteration,
              so each job runs its own full stop rule);
  lpt         static shards balanced with the iteration counts known in advance (longest-processing-time first
              on k x iterations): the ceiling of any assignment, which no run-time policy can know.
Usage: python tools/handout_sim.py [N=8]
"""
import heapq
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
z = np.load(os.path.join(ROOT, "tests", "golden", "golden_c3.npz"), allow_pickle=False)
ITERS = z["c3_iters"].astype(int)
KS = z["c3_job_k"].astype(int)
J = len(ITERS)


def f(L):
    return max(56.0, 55.0 + 0.72 * L)


def shard(r, N):
    b, rem = divmod(J, N)
    s = r * b + min(r, rem)
    return s, s + b + (1 if r < rem else 0)


def simulate(init, queue, div=20, check=4):
    N = len(init)
    queue = list(queue)[::-1]
    cap = [sum(KS[j] for j in init[r]) for r in range(N)]
    live = [{j: 0 for j in init[r]} for r in range(N)]
    it, t, nstop, at_pack = [0] * N, [0.0] * N, [0] * N, [0] * N
    heap = [(0.0, r) for r in range(N)]
    while heap:
        _, r = heapq.heappop(heap)
        for _ in range(check):
            L = sum(KS[j] for j in live[r])
            if L == 0:
                break
            t[r] += f(L)
            it[r] += 1
            for j in [j for j, b in live[r].items() if it[r] - b >= ITERS[j]]:
                del live[r][j]
                nstop[r] += 1
        nact = len(live[r])
        if nact == 0 and not queue:
            continue
        if queue and (nstop[r] - at_pack[r] >= max(1, nact // div) or nact == 0):
            used = sum(KS[j] for j in live[r])
            while queue and used + KS[queue[-1]] <= cap[r]:
                j = queue.pop()
                live[r][j] = it[r] + (it[r] % 2)
                used += KS[j]
            at_pack[r] = nstop[r]
        heapq.heappush(heap, (t[r], r))
    return t


def report(name, t, N):
    mk = max(t) / 1e6
    print(f"{name:22s} makespan {mk * 1e3:7.1f} ms  per GPU {J / N / mk:6.1f} restarts/s  "
          f"ranks {min(t) / 1e3:.0f}..{max(t) / 1e3:.0f} ms (mean {np.mean(t) / 1e3:.0f})")


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    print(f"C3 grid, {J} jobs (reference iteration counts: min {ITERS.min()}, mean {ITERS.mean():.1f}, max {ITERS.max()}), "
          f"{N} ranks, cost model f(L) = max(56, 55 + 0.72 L) us per iteration")
    report("static", simulate([list(range(*shard(r, N))) for r in range(N)], []), N)
    for phi in (0.95, 0.9, 0.85, 0.8, 0.7):
        init, q = [], []
        for r in range(N):
            s, e = shard(r, N)
            c = s + int(round(phi * (e - s)))
            init.append(list(range(s, c)))
            q += list(range(c, e))
        report(f"hand-out phi = {phi:.2f}", simulate(init, q), N)
    # LPT with known costs: the ceiling of any assignment
    load = [(0.0, r) for r in range(N)]
    lpt = [[] for _ in range(N)]
    for j in np.argsort(-(KS * ITERS), kind="stable"):
        w, r = heapq.heappop(load)
        lpt[r].append(int(j))
        heapq.heappush(load, (w + KS[j] * ITERS[j], r))
    report("lpt (costs known)", simulate(lpt, []), N)


if __name__ == "__main__":
    main()
