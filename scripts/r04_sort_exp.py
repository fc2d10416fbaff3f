#!/usr/bin/env python3
"""Experiment: does grouping chains with similar fixed-point iteration counts
into the same wave speed up the one-lane-per-chain C4 shard (131,072 chains)
or C2?  Per-chain results do not depend on wave-mates in these kernels, so a
permutation is free of parity cost.  Runs the chains in their original order
and sorted by the previous launch's p+q iteration sums, on device buffers,
and prints the kernel time of each (HIP events)."""
import json
import sys
import os

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hmc-stellar-toy-model_amd"))
from rhmc_amd import capi, workloads  # noqa: E402


def timed(ctx, P, q, p, it, st, n, K, steps, stream, reps=6):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(reps)]
    for a, b in ev:
        a.record(stream)
        ctx.leapfrog_device(P, q.data_ptr(), p.data_ptr(), n, K, steps, it.data_ptr(),
                            st.data_ptr(), stream.cuda_stream)
        b.record(stream)
    torch.cuda.synchronize()
    return [a.elapsed_time(b) for a, b in ev]


def main(wl_name, n):
    wl = workloads.make(wl_name, n_chains=n)
    dev = torch.device("cuda", 0)
    P = capi.make_params(**wl.params)
    ctx = capi.Context(wl.D, device=0)
    stream = torch.cuda.Stream(dev)
    q = torch.from_numpy(wl.q0).to(dev).contiguous()
    p = torch.from_numpy(wl.p0).to(dev).contiguous()
    it = torch.zeros((n, 2), dtype=torch.int32, device=dev)
    st = torch.zeros(n, dtype=torch.int32, device=dev)
    timed(ctx, P, q, p, it, st, n, wl.K, 500, stream, reps=2)          # warm-up, iteration counts
    base = timed(ctx, P, q, p, it, st, n, wl.K, 500, stream)
    cost = (it[:, 0] + it[:, 1]).cpu().numpy()
    order = torch.from_numpy(np.argsort(cost, kind="stable")).to(dev)
    qs, ps = q[order].contiguous(), p[order].contiguous()
    srt = timed(ctx, P, qs, ps, it, st, n, wl.K, 500, stream)
    # per-wave spread of the cost in each order (64 chains per wave)
    w = cost[: (n // 64) * 64].reshape(-1, 64)
    ws = np.sort(cost)[: (n // 64) * 64].reshape(-1, 64)
    print(json.dumps({"workload": wl_name, "chains": n, "kernel_ms_orig": base,
                      "kernel_ms_sorted": srt, "speedup": float(np.median(base) / np.median(srt)),
                      "iters_per_chain_mean": float(cost.mean()), "iters_min": int(cost.min()),
                      "iters_max": int(cost.max()),
                      "wave_max_over_mean_orig": float((w.max(1) / w.mean(1)).mean()),
                      "wave_max_over_mean_sorted": float((ws.max(1) / ws.mean(1)).mean())}))
    ctx.close()


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]))
