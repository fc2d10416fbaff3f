"""Wave-mates of a NaN chain and of a far-off chain.

The register-window kernels share a wave between chains: 4 chains per wave
for one star (leapfrog_k1_tiledr), 2 for the multi-star kernels
(leapfrog_pk, leapfrog_kr).  Their PSF-factor recurrence falls back to
direct exps for the whole wave when any chain in it is NaN or farther than
rec_vmax px from its window, so a checked chain's last bits
may depend on its wave-mates.  Here each checked chain runs once beside a NaN
chain and a far chain (x = 300 / y = -250: outside the recurrence's range)
and once beside ordinary chains; the documented bound is asserted — the two
results agree to 1e-12 relative (|value| + 1) with identical fixed-point
iteration counts — and both agree with the CPU oracle to the parity bar
(1e-9 q / 1e-8 p).  Whether they were bit-identical is printed.  The NaN
chain stays NaN (status NONFINITE) and contaminates nothing else.
Reference: the step is sampler_RHMC.py:522-566 per chain; chains are
independent, so any coupling is the kernel's."""
import numpy as np
import pytest

from helpers import assert_state_close
from oracle import rhmc_ref as R
from rhmc_amd import workloads

pytestmark = pytest.mark.gpu


def _run_pair(capi, wl, kernel, q_bad, p_bad, q_ref, p_ref, checked, steps):
    ctx = capi.Context(wl.D, kernel=kernel)
    P = capi.make_params(**wl.params)
    a = ctx.leapfrog(P, q_bad, p_bad, steps, return_info=True)
    b = ctx.leapfrog(P, q_ref, p_ref, steps, return_info=True)
    ctx.close()
    qa, pa, ita, sta = a
    qb, pb, itb, stb = b
    m = R.RefModel(wl.D, dict(wl.params, rows=wl.D.shape[0], cols=wl.D.shape[1]))
    same = True
    for c in checked:
        assert np.array_equal(ita[c], itb[c]), (c, ita[c], itb[c])
        assert_state_close(qa[c], qb[c], 1e-12, "q wave-mate %d" % c)
        assert_state_close(pa[c], pb[c], 1e-12, "p wave-mate %d" % c)
        same &= np.array_equal(qa[c], qb[c]) and np.array_equal(pa[c], pb[c])
        qo, po, NP, NQ = m.trajectory(q_ref[c], p_ref[c], steps, record=False)
        assert ita[c, 0] == NP.sum() and ita[c, 1] == NQ.sum(), c
        assert_state_close(qa[c], qo, 1e-9, "q vs oracle %d" % c)
        assert_state_close(pa[c], po, 1e-8, "p vs oracle %d" % c)
    print("%s: wave-mates bit-identical: %s" % (kernel, same))
    return sta


@pytest.mark.parametrize("kernel", ["auto", "regwin32", "regwin_f64"])
def test_one_star_wave_with_nan_and_far_chain(gpu_lib, kernel):
    capi = gpu_lib
    wl = workloads.make("C2", n_chains=12)
    q_ref, p_ref = wl.q0.copy(), wl.p0.copy()
    q_bad, p_bad = q_ref.copy(), p_ref.copy()
    q_bad[4, 0] = np.nan                  # wave 1 (chains 4-7): a NaN chain ...
    q_bad[5, 1], q_bad[5, 2] = 300.0, -250.0    # ... and a far chain
    st = _run_pair(capi, wl, kernel, q_bad, p_bad, q_ref, p_ref, (0, 3, 6, 7, 8), 40)
    assert st[4] & capi.STATUS_NONFINITE
    assert not (st[[0, 3, 6, 7, 8]] & capi.STATUS_NONFINITE).any()


@pytest.mark.parametrize("kernel", ["auto", "multiwin", "multiwin_notab"])
def test_many_star_wave_with_nan_and_far_chain(gpu_lib, kernel):
    capi = gpu_lib
    wl = workloads.make("C3", n_chains=8)
    q_ref, p_ref = wl.q0.copy(), wl.p0.copy()
    q_bad, p_bad = q_ref.copy(), p_ref.copy()
    q_bad[2, 3] = np.nan                  # chains 2, 3 share a wave
    q_bad[4, 1], q_bad[4, 2] = 300.0, -250.0    # chains 4, 5 share a wave
    st = _run_pair(capi, wl, kernel, q_bad, p_bad, q_ref, p_ref, (0, 3, 5, 6), 30)
    assert st[2] & capi.STATUS_NONFINITE
    assert not (st[[0, 3, 5, 6]] & capi.STATUS_NONFINITE).any()
