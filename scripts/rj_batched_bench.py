#!/usr/bin/env python3
"""Throughput of the batched reversible-jump runner (multi_gym.run_RHMC_rj_batched)
on the reference's big-sim4 geometry (32x32, K = 51 stars at the start,
P_move = [0.6, 0.2, 0.2], N_max = 120; RHMC-big-sim4.py:10-15,75-77): N chains,
each on its own seeded stream, GPU phases batched by star count.  Prints one
JSON line: wall time per MH iteration, chain-leapfrog-steps/s (move 0 runs
Nsteps steps, a jump 2 x Nsteps), and the share of the wall time spent in the
batched GPU calls (V, RHMC_steps) against the per-chain host work.

    python3 scripts/rj_batched_bench.py --chains 256 --niter 6 --nsteps 20
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hmc-stellar-toy-model_amd"))

from rhmc_amd import sampler, workloads  # noqa: E402
from rhmc_amd.photometry import mag2flux  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chains", type=int, default=256)
    ap.add_argument("--niter", type=int, default=6)
    ap.add_argument("--nsteps", type=int, default=20)
    ap.add_argument("--engine", choices=("native", "python"), default="native")
    ap.add_argument("--threads", type=int, default=0, help="native host threads (0: up to 16)")
    ap.add_argument("--pipes", type=int, default=0, help="native pipes (0: 2 from 1024 chains)")
    args = ap.parse_args()
    wl = workloads.make("B4", n_chains=args.chains)
    g = sampler.multi_gym(dt=0.05, g_xx=0.05, g_ff=4., g_ff2=4.)
    g.num_rows = g.num_cols = 32
    g.use_prior, g.alpha = True, 2.
    g.fmin, g.fmax = mag2flux(23.3) * g.flux_to_count, mag2flux(15.) * g.flux_to_count
    g.D = wl.D
    starts = []
    for c in range(args.chains):
        q = wl.q0[c].reshape(-1, 3).copy()
        q[:, 0] = np.minimum(g.flux2mag_converter(q[:, 0]), 22.5)   # above the flux wall
        starts.append(q)
    gpu = {"s": 0.0, "calls": 0}
    for name in (("V", "RHMC_steps") if args.engine == "python" else ()):  # time GPU calls
        f = getattr(g, name)

        def timed(*a, _f=f, **k):
            t0 = time.perf_counter()
            try:
                return _f(*a, **k)
            finally:
                gpu["s"] += time.perf_counter() - t0
                gpu["calls"] += 1
        setattr(g, name, timed)
    # warm-up (context, kernels) on two chains
    g.run_RHMC_rj_batched(starts[:2], [0, 1], Niter=1, Nsteps=2, dt=0.05, N_max=120,
                          P_move=[0.6, 0.2, 0.2], engine=args.engine, n_threads=args.threads)
    gpu["s"], gpu["calls"] = 0.0, 0
    t0 = time.perf_counter()
    g.run_RHMC_rj_batched(starts, list(range(args.chains)), Niter=args.niter,
                          Nsteps=args.nsteps, dt=0.05, N_max=120, P_move=[0.6, 0.2, 0.2],
                          engine=args.engine, n_threads=args.threads, n_pipes=args.pipes)
    wall = time.perf_counter() - t0
    moves = g.move_chain
    dead = getattr(g, "flag_chain", np.zeros_like(moves)) != 0
    steps = int(np.sum(np.where((moves == 0) | dead, 1, 2))) * args.nsteps
    out = {"what": "run_RHMC_rj_batched, big-sim4 geometry (32x32, K0 = 51), P_move "
                   "[0.6, 0.2, 0.2], one seeded stream per chain",
           "engine": args.engine, "pipes": args.pipes, "chains": args.chains, "iterations": args.niter + 1,
           "nsteps": args.nsteps,
           "wall_s": wall, "ms_per_iteration": wall / (args.niter + 1) * 1e3,
           "chain_leapfrog_steps_per_s": steps / wall,
           "native_call_s": getattr(g, "rj_native_s", None) if args.engine == "native" else None,
           "chain_leapfrog_steps_per_s_native_call": (steps / g.rj_native_s
                                                      if args.engine == "native" else None),
           "gpu_call_share": gpu["s"] / wall if args.engine == "python" else None,
           "gpu_calls": gpu["calls"] if args.engine == "python" else None,
           "accepted_jumps": int(np.sum(g.A_chain & (moves > 0))),
           "star_count_range_end": [int(g.N_chain[-1].min()), int(g.N_chain[-1].max())],
           "distinct_star_counts": int(len(np.unique(g.N_chain))),
           "phase_s": getattr(g, "rj_phase_s", None) if args.engine == "native" else None}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
