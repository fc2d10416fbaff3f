#!/usr/bin/env python3
"""Time one workload's leapfrog launch under each kernel family given (tools
only; the context option RHMC_OPT_KERNEL picks the family, no rebuild):
  python tools/kernel_ab.py C2 auto multiwin [--chains N] [--reps R]
Prints chain-leapfrog-steps/s and ms per 500-step launch (HIP events on the
launch stream), alternating families over the repetitions."""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "hmc-stellar-toy-model_amd"))
import torch  # noqa: E402
from rhmc_amd import capi, workloads  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("workload")
ap.add_argument("kernels", nargs="+")
ap.add_argument("--chains", type=int, default=None)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--launches", type=int, default=10)
ap.add_argument("--window-split", type=int, nargs="*", default=[0],
                help="RHMC_OPT_WINDOW_SPLIT values to alternate (multi-star kernel)")
args = ap.parse_args()
wl = workloads.make(args.workload, n_chains=args.chains)
P = capi.make_params(**wl.params)
dev = torch.device("cuda:0")
stream = torch.cuda.Stream(dev)
ctxs = {}
for k in args.kernels:
    for ws in args.window_split:
        ctx = capi.Context(wl.D, device=0, kernel=k)
        ctx.set_option(capi.OPT_WINDOW_SPLIT, ws)
        ctxs[k if len(args.window_split) == 1 else "%s/ws%d" % (k, ws)] = ctx
for r in range(args.reps):
    for k, ctx in ctxs.items():
        q = torch.from_numpy(wl.q0).to(dev)
        p = torch.from_numpy(wl.p0).to(dev)
        it = torch.zeros((wl.n_chains, 2), dtype=torch.int32, device=dev)
        st = torch.zeros(wl.n_chains, dtype=torch.int32, device=dev)
        torch.cuda.synchronize()

        def launch():
            ctx.leapfrog_device(P, q.data_ptr(), p.data_ptr(), wl.n_chains, wl.K, wl.n_steps,
                                it.data_ptr(), st.data_ptr(), stream=stream.cuda_stream)
        with torch.cuda.stream(stream):
            launch()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(args.launches):
                launch()
            e1.record(stream)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / args.launches
        bad = int((st & 1).ne(0).sum())
        print("%s %s rep %d: %.4g chain-steps/s, %.3f ms/launch, nonfinite %d"
              % (args.workload, k, r, wl.n_chains * wl.n_steps / ms * 1e3, ms, bad), flush=True)
