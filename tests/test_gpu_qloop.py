"""GPU parity of the fixed-point loops at the pass boundaries.

The 16-lane single-star kernels evaluate the q-loop (sampler_RHMC.py:538-545)
eight iterations per pass across a chain's lanes and the p-loop (:528-535) two
per pass; the state and count kept must be those of the first iteration whose
test stops the reference's loop, and counter_max must cut the loop exactly
where the reference's `while dq > delta and counter < counter_max` does.  A
large step (dt = 1.0) with delta = 1e-10 makes the q-loop run 5-10 iterations
on C2 geometry, so the cases below cross the 8-iteration pass boundary and hit
every cap from 1 to 16.  Compared with the CPU oracle: per-chain iteration
totals exactly, the PLOOP/QLOOP cap status bits, q/p after 3 steps.
"""
import numpy as np
import pytest

from helpers import assert_state_close
from oracle.rhmc_ref import RefModel

pytestmark = pytest.mark.gpu

DT, DELTA, STEPS, CHAINS = 1.0, 1e-10, 3, 16


def _oracle(wl, cm):
    par = dict(wl.params, rows=48, cols=48, dt=DT)
    m = RefModel(wl.D, par)
    out = []
    for c in range(CHAINS):
        Q, Pm, NP, NQ = m.trajectory(wl.q0[c], wl.p0[c], STEPS, DELTA, cm, record=True)
        cap_p = cap_q = False
        for s in range(STEPS):
            if NP[s] == cm or NQ[s] == cm:
                # did the loop stop on the cap (one more iteration allowed -> more done)?
                _, _, n_p, n_q = m.step(Q[s], Pm[s], DELTA, cm + 1)
                cap_p |= bool(NP[s] == cm and n_p > cm)
                cap_q |= bool(NQ[s] == cm and n_q > cm)
        out.append((Q[-1], Pm[-1], int(NP.sum()), int(NQ.sum()), cap_p, cap_q, int(NQ.max())))
    return out


@pytest.mark.parametrize("kernel", ["auto", "regwin32", "regwin_f64"])
@pytest.mark.parametrize("cm", [1, 2, 3, 7, 8, 9, 16, 1000])
def test_fixed_point_pass_boundaries(gpu_lib, monkeypatch, kernel, cm):
    capi = gpu_lib
    from rhmc_amd import workloads
    monkeypatch.setattr(capi, "DEFAULT_KERNEL", kernel)
    wl = workloads.make("C2", n_chains=CHAINS)
    par = dict(wl.params, dt=DT, delta=DELTA, counter_max=cm)
    ctx = capi.Context(wl.D)
    q, p, it, st = ctx.leapfrog(capi.make_params(**par), wl.q0, wl.p0, STEPS, return_info=True)
    ctx.close()
    ref = _oracle(wl, cm)
    if cm == 1000:  # the uncapped loops really do cross the 8-iteration pass
        assert max(r[6] for r in ref) > 8
    for c, (qo, po, n_p, n_q, cap_p, cap_q, _) in enumerate(ref):
        assert (it[c, 0], it[c, 1]) == (n_p, n_q), (c, it[c], n_p, n_q)
        assert bool(st[c] & capi.STATUS_PLOOP_CAP) == cap_p, (c, st[c])
        assert bool(st[c] & capi.STATUS_QLOOP_CAP) == cap_q, (c, st[c])
        assert_state_close(q[c], qo, 1e-10, "q chain %d" % c)
        assert_state_close(p[c], po, 1e-9, "p chain %d" % c)
