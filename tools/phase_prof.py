#!/usr/bin/env python3
"""Per-phase cycle split of the single-star kernel (RHMC_KERNEL=profw16|profw32):
table build, pixel loop + reductions, fixed-point loops; cycles per step per wave."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "hmc-stellar-toy-model_amd"))
import numpy as np
import torch
from rhmc_amd import capi, workloads
n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
wl = workloads.make("C2", n_chains=n)
P = capi.make_params(**wl.params)
ctx = capi.Context(wl.D)
dev = torch.device("cuda", 0)
q = torch.from_numpy(wl.q0).to(dev).contiguous()
p = torch.from_numpy(wl.p0).to(dev).contiguous()
it = torch.zeros((n, 2), dtype=torch.int32, device=dev)
st = torch.zeros(n, dtype=torch.int32, device=dev)
s = torch.cuda.Stream(dev)
for _ in range(2):
    ctx.leapfrog_device(P, q.data_ptr(), p.data_ptr(), n, 1, 200, it.data_ptr(), st.data_ptr(), s.cuda_stream)
torch.cuda.synchronize()
a = it.cpu().numpy().astype(float)
b = st.cpu().numpy().astype(float)
if os.environ.get("RHMC_KERNEL", "").startswith(("profw", "profr")):
    print("%s n=%d cycles/step: gradient %.0f  rest %.0f  total %.0f" % (
        os.environ.get("RHMC_KERNEL"), n, a[:, 0].mean(), a[:, 1].mean(), a.sum(1).mean()))
else:
    tot = a[:, 0] + a[:, 1] + b
    print("%s n=%d cycles/step: table %.0f  pixel+reduce %.0f  loops %.0f  total %.0f" % (
        os.environ.get("RHMC_KERNEL"), n, a[:, 0].mean(), a[:, 1].mean(), b.mean(), tot.mean()))
