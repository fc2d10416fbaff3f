#!/usr/bin/env python3
"""Per-phase cycle split of the register-window kernel (tools only).

Needs the phase-timing library: `make -C hmc-stellar-toy-model_amd prof`
(-DRHMC_PHASE_PROF -> build/variants/lib_prof.so), whose register-window
launches write cycles per step per wave over the chain state: the gradient,
kicks + reflection + p-loop, q-loop, flux metric + closing update, and inside
the gradient the window check, PSF factors, pixel loop and moments +
reductions (fenced s_memtime reads).
usage: RHMC_LIB=build/variants/lib_prof.so python tools/phase_prof.py [n_chains]
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "hmc-stellar-toy-model_amd"))
import torch  # noqa: E402

from rhmc_amd import capi, workloads  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
kern = "profr"
wl = workloads.make("C2", n_chains=n)
P = capi.make_params(**wl.params)
ctx = capi.Context(wl.D)
dev = torch.device("cuda", 0)
it = torch.zeros((n, 2), dtype=torch.int32, device=dev)
st = torch.zeros(n, dtype=torch.int32, device=dev)
s = torch.cuda.Stream(dev)
for _ in range(2):
    q = torch.from_numpy(wl.q0).to(dev).contiguous()
    p = torch.from_numpy(wl.p0).to(dev).contiguous()
    ctx.leapfrog_device(P, q.data_ptr(), p.data_ptr(), n, 1, 200, it.data_ptr(), st.data_ptr(),
                        s.cuda_stream)
torch.cuda.synchronize()
if kern.startswith("profr"):
    qq, pp = q.cpu().numpy(), p.cpu().numpy()
    ph = [qq[:, 0].mean(), qq[:, 1].mean(), qq[:, 2].mean(), pp[:, 0].mean()]
    print("%s n=%d cycles/step: gradient %.0f  kicks+p-loop %.0f  q-loop %.0f  flux+tail %.0f"
          "  total %.0f" % (kern, n, ph[0], ph[1], ph[2], ph[3], sum(ph)))
    itn = it.cpu().numpy().astype(float)
    g4 = [itn[:, 1].mean(), pp[:, 1].mean(), pp[:, 2].mean(), itn[:, 0].mean()]
    print("  gradient split: window check %.0f  PSF factors %.0f  pixel loop %.0f  "
          "moments + reductions %.0f" % tuple(g4))
else:
    a = it.cpu().numpy().astype(float)
    print("%s n=%d cycles/step: gradient %.0f  rest %.0f  total %.0f" % (
        kern, n, a[:, 0].mean(), a[:, 1].mean(), a.sum(1).mean()))
