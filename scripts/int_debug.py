import os, sys, numpy as np
sys.path[:0] = [".", "hmc-stellar-toy-model_amd", "tests"]
from rhmc_amd import capi, workloads
import test_gpu_integrators as T
from oracle import rhmc_ref as R
wl = workloads.make("C2")
ctx = capi.Context(wl.D)
P = capi.make_params(**wl.params)
par = dict(wl.params); par["rows"], par["cols"] = wl.D.shape
m = R.RefModel(wl.D, par)
for name in T.SOLVERS:
    sid = T._sid(capi, name)
    q, p = ctx.integrate(P, sid, wl.q0, wl.p0, T.N_STEPS, f_pos=True)
    os.environ["RHMC_KERNEL"] = "windowed"
    qw, pw = ctx.integrate(P, sid, wl.q0, wl.p0, T.N_STEPS, f_pos=True)
    del os.environ["RHMC_KERNEL"]
    e = (np.abs(q - qw) / (np.abs(qw) + 1)).max(axis=1)
    bad = np.argsort(-e)[:4]
    print(name, "n>1e-9:", (e > 1e-9).sum())
    for c in bad:
        qo, po = T._oracle_run(m, name, wl.q0[c], wl.p0[c], T.N_STEPS)
        print("  chain", c, "e=%.2e" % e[c], "q0", wl.q0[c], "\n   tiledr", q[c], p[c], "\n   win   ", qw[c], pw[c], "\n   oracle", qo, po)
