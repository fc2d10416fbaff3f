"""pixk vs the default multi-star kernel and the oracle on C3 (correctness)."""
import os, sys, numpy as np
sys.path[:0] = [".", "hmc-stellar-toy-model_amd"]
from rhmc_amd import capi, workloads
from oracle import rhmc_ref as R
wl = workloads.make("C3", n_chains=1024)
ctx = capi.Context(wl.D)
P = capi.make_params(**wl.params)
q1, p1, it1, st1 = ctx.leapfrog(P, wl.q0, wl.p0, 50, return_info=True)
os.environ["RHMC_KERNEL"] = "pixk"
q2, p2, it2, st2 = ctx.leapfrog(P, wl.q0, wl.p0, 50, return_info=True)
del os.environ["RHMC_KERNEL"]
eq = np.abs(q2 - q1) / (np.abs(q1) + 1); ep = np.abs(p2 - p1) / (np.abs(p1) + 1)
print("pixk vs kr: max rel q %.2e p %.2e, iters equal %s" % (eq.max(), ep.max(), np.array_equal(it1, it2)))
par = dict(wl.params); par["rows"], par["cols"] = wl.D.shape
m = R.RefModel(wl.D, par)
for c in (0, 777):
    qo, po, NP, NQ = m.trajectory(wl.q0[c], wl.p0[c], 50, record=False)
    print("chain", c, "vs oracle: q %.2e p %.2e iters %s" % ((np.abs(q2[c]-qo)/(np.abs(qo)+1)).max(), (np.abs(p2[c]-po)/(np.abs(po)+1)).max(), (it2[c,0]==NP.sum(), it2[c,1]==NQ.sum())))
