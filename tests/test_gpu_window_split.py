"""Window split of the multi-star register-window kernel (leapfrog_kr, WS
waves per chain pair, RHMC_OPT_WINDOW_SPLIT): the C5 shard one GPU holds when
8192 chains are split over 8 GPUs (1024 chains, where the default picks 4
waves per pair) and a one-slot case (K = 24 on a 96-px image), run with the
split forced to 1, 2 and 4 — q, p, fixed-point counts and status words must
be bit-identical (every window's sums are the same operations in the same
order; only which wave evaluates them changes), ragged chain counts included.
The WS = 1 path is pinned to the oracle by tests/test_gpu_fullsize_multistar.py
and tests/test_gpu_parity.py; here an oracle sample also checks the default
(split) launch directly.  Reference: sampler_RHMC.py:522-566, :365-425."""
import numpy as np
import pytest

from helpers import assert_state_close
from oracle import rhmc_ref as R
from rhmc_amd import workloads
from rhmc_amd.photometry import mag2flux

pytestmark = pytest.mark.gpu


def _run(capi, D, par, q0, p0, steps, ws):
    ctx = capi.Context(D, kernel="multiwin_notab")
    ctx.set_option(capi.OPT_WINDOW_SPLIT, ws)
    assert ctx.get_option(capi.OPT_WINDOW_SPLIT) == ws
    out = ctx.leapfrog(capi.make_params(**par), q0, p0, steps, return_info=True)
    ctx.close()
    return out


def _same(a, b, what):
    for x, y, name in zip(a, b, ("q", "p", "iters", "status")):
        assert np.array_equal(x, y), "%s: %s differs" % (what, name)


def test_c5_shard_split_bit_identical(gpu_lib):
    capi = gpu_lib
    wl = workloads.make("C5", n_chains=1024)
    ref = _run(capi, wl.D, wl.params, wl.q0, wl.p0, 12, 1)
    for ws in (2, 4, 0):
        _same(_run(capi, wl.D, wl.params, wl.q0, wl.p0, 12, ws), ref, "C5 1024 chains ws=%d" % ws)
    # ragged: an odd chain count leaves a half-empty last pair and idle groups
    # (ws = 2 with an odd pair count: a workgroup's last group holds no chain
    # and mirrors the workgroup's first one)
    for n in (1, 5, 37):
        for ws in (1, 2, 4):
            out = _run(capi, wl.D, wl.params, wl.q0[:n], wl.p0[:n], 12, ws)
            _same(out, tuple(r[:n] for r in ref), "C5 %d chains ws=%d" % (n, ws))


def test_one_slot_split_bit_identical(gpu_lib):
    capi = gpu_lib
    par, ftc = workloads.base_params(dt=0.05, g_xx=0.05, g_ff=4., g_ff2=4.)
    rng = np.random.RandomState(11)
    K, n, side = 24, 70, 96
    stars = [(16. + 6 * rng.rand(), 2 + 92 * rng.rand(), 2 + 92 * rng.rand()) for _ in range(K)]
    D = workloads._image(side, stars, ftc, par["B_count"], par["fwhm_pix"], rng)
    q0 = np.empty((n, 3 * K))
    q0[:, 0::3] = [mag2flux(s[0]) * ftc for s in stars]
    q0[:, 1::3] = [s[1] for s in stars]
    q0[:, 2::3] = [s[2] for s in stars]
    q0 *= 1 + 0.01 * rng.randn(n, 3 * K)
    p0 = rng.randn(n, 3 * K) * np.sqrt(workloads.metric_diag(q0, par))
    ref = _run(capi, D, par, q0, p0, 15, 1)
    for ws in (2, 4):
        _same(_run(capi, D, par, q0, p0, 15, ws), ref, "K=24 ws=%d" % ws)
    m = R.RefModel(D, dict(par, rows=side, cols=side))
    q, p, it, st = _run(capi, D, par, q0[:3], p0[:3], 15, 4)
    for c in range(3):
        qo, po, NP, NQ = m.trajectory(q0[c], p0[c], 15, record=False)
        assert it[c, 0] == NP.sum() and it[c, 1] == NQ.sum(), (c, it[c], NP.sum(), NQ.sum())
        assert_state_close(q[c], qo, 1e-9, "q chain %d" % c)
        assert_state_close(p[c], po, 1e-8, "p chain %d" % c)


def test_window_split_option_checks(gpu_lib):
    capi = gpu_lib
    wl = workloads.make("C2", n_chains=4)
    ctx = capi.Context(wl.D)
    assert ctx.get_option(capi.OPT_WINDOW_SPLIT) == 0
    for bad in (3, 8, -1):
        with pytest.raises(capi.RhmcError):
            ctx.set_option(capi.OPT_WINDOW_SPLIT, bad)
    ctx.close()
