"""Full-size parity for the multi-star bench workloads through the C-ABI, the
exact launches the bench times (mirrors tests/test_gpu_fullsize.py):

C3  48x48, K = 10, 16,384 chains (pixel-major kernel leapfrog_pk<48, 10>),
    the big-sim4 parameter set (RHMC-big-sim4.py:11-47) where the flux-wall
    reflections of sampler_RHMC.py:554-564 fire ~2-3 times per step per chain;
C5  256x256, K = 64, 8,192 chains, prior on (leapfrog_kr<float, 2, false>).

Checked: an oracle sample with exact fixed-point iteration counts (C3: 4
chains x the first 100 steps — the chaotic horizon of the reference itself at
C3 is ~100-130 steps, so the sample uses chains whose 1e-15 perturbation stays
below 1e-11 for 100 steps, measured with the oracle; C5: 4 chains x 20 steps,
through the flux wall; tests/golden/traj_c5.npz pins C5 to the reference
itself, 4 chains x 50 steps, in tests/test_gpu_parity.py);
batch invariance (ragged subsets spanning waves give bit-identical results);
determinism; launch segmentation (5 x 100 == 1 x 500 bit for bit); and the
near-wall reflection fraction SURVEY §8(c) asks to report separately.
Tolerances: 1e-9 (q) / 1e-8 (p) relative to |value| + 1."""
import numpy as np
import pytest

from helpers import assert_state_close
from oracle import rhmc_ref as R
from rhmc_amd import workloads

pytestmark = pytest.mark.gpu


def _model(wl):
    return R.RefModel(wl.D, dict(wl.params, rows=wl.D.shape[0], cols=wl.D.shape[1]))


@pytest.fixture(scope="module")
def c3(gpu_lib):
    capi = gpu_lib
    wl = workloads.make("C3")
    ctx = capi.Context(wl.D)
    P = capi.make_params(**wl.params)
    full = ctx.leapfrog(P, wl.q0, wl.p0, wl.n_steps, return_info=True)
    yield capi, wl, ctx, P, full
    ctx.close()


@pytest.fixture(scope="module")
def c5(gpu_lib):
    capi = gpu_lib
    wl = workloads.make("C5")
    ctx = capi.Context(wl.D)
    P = capi.make_params(**wl.params)
    full = ctx.leapfrog(P, wl.q0, wl.p0, wl.n_steps, return_info=True)
    yield capi, wl, ctx, P, full
    ctx.close()


def _oracle_sample(capi, wl, ctx, P, chains, steps):
    q, p, it, st = ctx.leapfrog(P, wl.q0, wl.p0, steps, return_info=True)
    m = _model(wl)
    for c in chains:
        assert not st[c] & capi.STATUS_NEAR_WALL, "sampled chain %d reflected at a wall edge" % c
        qo, po, NP, NQ = m.trajectory(wl.q0[c], wl.p0[c], steps, record=False)
        assert it[c, 0] == NP.sum() and it[c, 1] == NQ.sum(), (c, it[c], NP.sum(), NQ.sum())
        assert_state_close(q[c], qo, 1e-9, "%s q chain %d" % (wl.name, c))
        assert_state_close(p[c], po, 1e-8, "%s p chain %d" % (wl.name, c))
    return st


def test_c3_full_size_oracle_sample(c3):
    capi, wl, ctx, P, (q, p, it, st) = c3
    assert q.shape == (16384, 30)
    assert not (st & capi.STATUS_NONFINITE).any()
    assert ((st & capi.STATUS_REFLECT_F) != 0).mean() > 0.5      # the wall is exercised
    st100 = _oracle_sample(capi, wl, ctx, P, (0, 4097, 12345, 16383), 100)
    assert ((st100 & capi.STATUS_REFLECT_F) != 0).any()


def test_c3_near_wall_fraction_reported(c3):
    """chains whose reflection fired within 2^-40 of a wall are
    the ones allowed to diverge from the reference; report their share."""
    capi, wl, ctx, P, (q, p, it, st) = c3
    near = (st & capi.STATUS_NEAR_WALL) != 0
    refl = (st & (capi.STATUS_REFLECT_F | capi.STATUS_REFLECT_XY)) != 0
    print("C3 500 steps: %d of %d chains reflected, %d within 2^-40 of a wall (%.2e)"
          % (refl.sum(), len(st), near.sum(), near.mean()))
    assert not (near & ~refl).any()              # the bit implies a reflection
    assert near.mean() < 1e-2


def test_c3_batch_invariance_and_determinism(c3):
    capi, wl, ctx, P, (q, p, it, st) = c3
    idx = np.r_[0:5, 777:790, 16380:16384]        # odd offsets: wave pairs split
    qs, ps, its, sts = ctx.leapfrog(P, wl.q0[idx], wl.p0[idx], wl.n_steps, return_info=True)
    assert np.array_equal(qs, q[idx]) and np.array_equal(ps, p[idx])
    assert np.array_equal(its, it[idx]) and np.array_equal(sts, st[idx])
    q2, p2 = ctx.leapfrog(P, wl.q0, wl.p0, wl.n_steps)
    assert np.array_equal(q2, q) and np.array_equal(p2, p)


def test_c3_launch_segmentation(c3):
    capi, wl, ctx, P, (q, p, it, st) = c3
    qq, pp = wl.q0, wl.p0
    for _ in range(5):
        qq, pp = ctx.leapfrog(P, qq, pp, wl.n_steps // 5)
    assert np.array_equal(qq, q) and np.array_equal(pp, p)


def test_c5_full_size_oracle_sample(c5):
    """4 chains x 20 steps of the 8192-chain C5 launch against the oracle;
    the flux wall (sampler_RHMC.py:554-559) fires in the sample (the prior,
    :408-409, is on)."""
    capi, wl, ctx, P, (q, p, it, st) = c5
    assert q.shape == (8192, 192)
    assert not (st & capi.STATUS_NONFINITE).any()
    near = (st & capi.STATUS_NEAR_WALL) != 0
    print("C5 500 steps: %d chains within 2^-40 of a wall (%.2e)" % (near.sum(), near.mean()))
    assert near.mean() < 1e-2
    sample = (0, 2731, 5462, 8191)
    st20 = _oracle_sample(capi, wl, ctx, P, sample, 20)
    assert any(st20[c] & capi.STATUS_REFLECT_F for c in sample)


def test_c5_batch_invariance_determinism_segmentation(c5):
    capi, wl, ctx, P, (q, p, it, st) = c5
    idx = np.r_[0:3, 4095:4100, 8191:8192]
    qs, ps, its, sts = ctx.leapfrog(P, wl.q0[idx], wl.p0[idx], wl.n_steps, return_info=True)
    assert np.array_equal(qs, q[idx]) and np.array_equal(ps, p[idx])
    assert np.array_equal(its, it[idx]) and np.array_equal(sts, st[idx])
    q2, p2 = ctx.leapfrog(P, wl.q0, wl.p0, wl.n_steps)
    assert np.array_equal(q2, q) and np.array_equal(p2, p)
    qq, pp = wl.q0, wl.p0
    for _ in range(5):
        qq, pp = ctx.leapfrog(P, qq, pp, wl.n_steps // 5)
    assert np.array_equal(qq, q) and np.array_equal(pp, p)


@pytest.mark.parametrize("fused", [True, False])
def test_c5_mh_f_pos_vs_oracle(gpu_lib, fused):
    """run_RHMC's MH loop (sampler_RHMC.py:1018-1083) with the reference's
    f_pos=True on the C5 geometry (256x256, K = 64, prior): rhmc_mh with host
    draws from the C5 MH start (workloads.mh_start: every flux >= 1.5 f_lim,
    so V is finite at the start), 2 chains x 3 iterations x 5 steps, against
    the oracle's run_RHMC iterations — the four-kernel loop with its
    wave-per-chain begin / end and the windowed pixel-major V(q') (no fused
    MH kernel serves K = 64; the option must not matter).  Accepts exact,
    chains 1e-9, energies 1e-11; the draws accept and reject."""
    capi = gpu_lib
    wl = workloads.make("C5", n_chains=2)
    q0 = workloads.mh_start(wl)
    assert np.isfinite(q0).all() and (q0[:, 0::3] >= 1.5 * wl.params["f_lim"]).all()
    ctx = capi.Context(wl.D)
    ctx.set_option(capi.OPT_MH_FUSED, int(fused))
    P = capi.make_params(**wl.params)
    m = _model(wl)
    m.V_prior_const = wl.params["V_prior_const"]
    n_iter, n_steps = 3, 5
    rs = np.random.RandomState(5)
    zz = rs.randn(n_iter, 2, q0.shape[1])
    uu = rs.rand(n_iter, 2)
    out = ctx.mh(P, q0, n_iter, n_steps, f_pos=True, z=zz, u=uu, record=True)
    acc_all = []
    for c in range(2):
        q = q0[c].copy()
        for it in range(n_iter):
            Hd = m.H(q)
            p = zz[it, c] * np.sqrt(Hd)
            E0 = m.V(q, True) + m.T(p, Hd)
            assert np.isfinite(E0)
            np.testing.assert_allclose(out["E_chain"][it, c], E0, rtol=1e-11)
            assert_state_close(out["q_chain"][it, c], q, 1e-9, "q_chain %d/%d" % (it, c))
            q1, p1, _, _ = m.trajectory(q, p, n_steps, record=False)
            dE = m.V(q1, True) + m.T(p1, m.H(q1)) - E0
            a = bool((dE < 0) or (np.log(uu[it, c]) < -dE))
            assert bool(out["accept"][it, c]) == a, (it, c, dE)
            acc_all.append(a)
            if a:
                q = q1
        assert_state_close(out["q"][c], q, 1e-9, "mh q chain %d" % c)
    assert 0 < np.mean(acc_all) < 1, acc_all
    ctx.close()
