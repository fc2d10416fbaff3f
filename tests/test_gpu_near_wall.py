"""RHMC_STATUS_NEAR_WALL: set when a reflection of the implicit step
(sampler_RHMC.py:554-564) fires with the reflecting coordinate within 2^-40
(9.1e-13, relative to max(1, |wall|)) of its wall — f_lim for the flux, 0 and
R-1 for the positions — the chains SURVEY §8(c) reports separately because a
last-bit difference can flip such a reflection.

Constructed states: with p = 0 and dt = 1e-12 a chain barely moves in one
step, so a coordinate placed 1e-13 beyond a wall reflects near it, while one
placed 1e-6 beyond reflects without the bit.  Every kernel family that runs
the implicit step is checked, for one star and for ten."""
import numpy as np
import pytest

from rhmc_amd import workloads

pytestmark = pytest.mark.gpu


def _case(name):
    wl = workloads.make(name, n_chains=7)
    par = dict(wl.params, dt=1e-12)
    K = wl.K
    q0 = wl.q0.copy()
    p0 = np.zeros_like(q0)
    f_lim, edge = par["f_lim"], wl.D.shape[0] - 1.0
    q0[0, 0] = f_lim - 1e-13                 # flux, near
    q0[1, 0] = f_lim - 1e-6                  # flux, clear
    q0[2, 1] = -1e-13                        # x at 0, near
    q0[3, 2] = edge + 1e-13 * edge           # y at R-1, near
    q0[4, 1] = -1e-6                         # x, clear
    q0[5, 2] = edge + 1e-6                   # y, clear
    # chain 6: untouched
    return wl, par, q0, p0


@pytest.mark.parametrize("name,kernel", [
    ("C2", "auto"), ("C2", "regwin32"), ("C2", "lane1"), ("C2", "lane4"), ("C2", "generic"),
    ("C2", "windowed"), ("C3", "auto"), ("C3", "multiwin"), ("C3", "multiwin_notab"),
    ("C3", "generic"), ("C3", "windowed")])
def test_near_wall_bit(gpu_lib, name, kernel):
    capi = gpu_lib
    wl, par, q0, p0 = _case(name)
    ctx = capi.Context(wl.D, kernel=kernel)
    P = capi.make_params(**par)
    q, p, it, st = ctx.leapfrog(P, q0, p0, 1, return_info=True)
    ctx.close()
    F, XY, NEAR = capi.STATUS_REFLECT_F, capi.STATUS_REFLECT_XY, capi.STATUS_NEAR_WALL
    # (other stars of a C3 chain may start below f_lim and add REFLECT_F bits,
    # never within 2^-40 of a wall)
    want = [F | NEAR, F, XY | NEAR, XY | NEAR, XY, XY, 0]
    for c, w in enumerate(want):
        got = st[c] & (F | XY | NEAR)
        assert got & w == w, (kernel, c, got, w)
        assert bool(got & NEAR) == bool(w & NEAR), (kernel, c, got, w)
