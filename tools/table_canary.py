#!/usr/bin/env python3
"""WinGG table-region conflicts (tools only).  Runs the
S256K100 MH loop (4,096 chains, 5 x 10 steps, three launches) through a
-DRHMC_TABLE_CANARY build and prints, per RHMC_OPT_TABLES mode, the accept
rate and the number of gradients / potentials whose table region another
launch bumped while they ran:
  RHMC_LIB=build/variants/lib_canary.so python tools/table_canary.py 0 2 5"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "hmc-stellar-toy-model_amd"))
import torch  # noqa: E402
from rhmc_amd import capi, workloads  # noqa: E402

fn = capi.lib().rhmc_debug_table_conflicts
fn.restype = ctypes.c_int
fn.argtypes = [ctypes.POINTER(ctypes.c_int64)]
wl = workloads.make("S256K100", n_chains=4096)
P = capi.make_params(**wl.params)
dev = torch.device("cuda", 0)
for mode in [int(m) for m in sys.argv[1:]]:
    ctx = capi.Context(wl.D)
    ctx.set_option(capi.OPT_TABLES, mode)
    s = torch.cuda.Stream(dev)
    q = torch.from_numpy(wl.q0).to(dev)
    acc = torch.zeros((5, wl.n_chains), dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    out = (ctypes.c_int64 * 5)()
    fn(out)   # reset
    rates = []
    for launch in range(3):
        rec = capi.MhRecord(None, None, None, None, acc.data_ptr())
        ctx.mh_device(P, q.data_ptr(), wl.n_chains, wl.K, 5, 10, f_pos=False, seed=77 + launch,
                      record=rec, stream=s.cuda_stream)
        torch.cuda.synchronize()
        rates.append(float(acc.float().mean()))
    fn(out)
    ctx.close()
    print("tables=%d accept=%s conflicts total=%d gradient=%d potential=%d bumps by "
          "gradients=%d potentials=%d q_sum=%.17g"
          % (mode, ["%.6f" % r for r in rates], out[0], out[1], out[2], out[3], out[4],
             float(q.double().sum())), flush=True)
