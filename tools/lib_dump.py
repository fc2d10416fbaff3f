#!/usr/bin/env python3
"""Run one workload's full leapfrog launch through the library named by
RHMC_LIB and save q, p, iteration counts and status (tools only; compare two
builds bit for bit with tools/lib_cmp.py):
  RHMC_LIB=build/variants/lib_x.so python tools/lib_dump.py C2 out.npz [--chains N]"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "hmc-stellar-toy-model_amd"))
import torch  # noqa: E402
from rhmc_amd import capi, workloads  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("workload")
ap.add_argument("out")
ap.add_argument("--chains", type=int, default=None)
args = ap.parse_args()
wl = workloads.make(args.workload, n_chains=args.chains)
P = capi.make_params(**wl.params)
dev = torch.device("cuda:0")
ctx = capi.Context(wl.D, device=0)
q = torch.from_numpy(wl.q0).to(dev)
p = torch.from_numpy(wl.p0).to(dev)
it = torch.zeros((wl.n_chains, 2), dtype=torch.int32, device=dev)
st = torch.zeros(wl.n_chains, dtype=torch.int32, device=dev)
ctx.leapfrog_device(P, q.data_ptr(), p.data_ptr(), wl.n_chains, wl.K, wl.n_steps,
                    it.data_ptr(), st.data_ptr(), stream=0)
torch.cuda.synchronize()
np.savez(args.out, q=q.cpu().numpy(), p=p.cpu().numpy(), it=it.cpu().numpy(),
         st=st.cpu().numpy())
print("%s: %d chains x %d steps -> %s" % (args.workload, wl.n_chains, wl.n_steps, args.out))
