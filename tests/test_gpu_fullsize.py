"""Full-size parity for the bench workloads (BASELINE configs C2 and a C4
shard) through the C-ABI: the exact launch the bench times, checked by
size-independent properties plus a seeded sample of chains against the CPU
oracle.

* oracle sample: 6 chains of the 4096 (500 steps each) match oracle/rhmc_ref
  to 1e-9 (q) / 1e-8 (p) relative to |value| + 1, with the exact fixed-point
  iteration counts (SURVEY §8(c) tolerance);
* batch invariance: any subset of chains run on its own gives bit-identical
  results (no cross-chain coupling — wave-mates only share DPP/swizzle traffic
  inside their own 16-lane group, and window reloads only re-read data);
* determinism: the same launch twice is bit-identical;
* launch segmentation: 500 steps in one launch == 5 launches of 100 steps,
  bit for bit (the carried gradient and flux metric are recomputed from the
  same state at a launch boundary);
* reversibility: 500 steps, momentum flipped, 500 steps back returns to the
  start to within the fixed-point tolerance's drift (5e-4 relative).
"""
import numpy as np
import pytest

from oracle import rhmc_ref as R
from rhmc_amd import workloads
from rhmc_amd.shard import shard_range

pytestmark = pytest.mark.gpu


def _oracle_params(wl):
    par = dict(wl.params)
    par["rows"], par["cols"] = wl.D.shape
    return par


@pytest.fixture(scope="module")
def c2(gpu_lib):
    capi = gpu_lib
    wl = workloads.make("C2")
    ctx = capi.Context(wl.D)
    P = capi.make_params(**wl.params)
    q, p, it, st = ctx.leapfrog(P, wl.q0, wl.p0, wl.n_steps, return_info=True)
    yield capi, wl, ctx, P, (q, p, it, st)
    ctx.close()


def test_c2_full_oracle_sample(c2):
    capi, wl, ctx, P, (q, p, it, st) = c2
    assert q.shape == (4096, 3) and not (st & capi.STATUS_NONFINITE).any()
    m = R.RefModel(wl.D, _oracle_params(wl))
    for c in (0, 1, 777, 2048, 3333, 4095):
        qo, po, NP, NQ = m.trajectory(wl.q0[c], wl.p0[c], wl.n_steps, record=False)
        assert it[c, 0] == NP.sum() and it[c, 1] == NQ.sum(), c
        err_q = np.abs(q[c] - qo) / (np.abs(qo) + 1)
        err_p = np.abs(p[c] - po) / (np.abs(po) + 1)
        assert err_q.max() <= 1e-9 and err_p.max() <= 1e-8, (c, err_q, err_p)


def test_c2_batch_invariance_and_determinism(c2):
    capi, wl, ctx, P, (q, p, it, st) = c2
    idx = np.r_[0:7, 1000:1013, 4090:4096]
    qs, ps, its, sts = ctx.leapfrog(P, wl.q0[idx], wl.p0[idx], wl.n_steps, return_info=True)
    assert np.array_equal(qs, q[idx]) and np.array_equal(ps, p[idx])
    assert np.array_equal(its, it[idx]) and np.array_equal(sts, st[idx])
    q2, p2 = ctx.leapfrog(P, wl.q0, wl.p0, wl.n_steps)
    assert np.array_equal(q2, q) and np.array_equal(p2, p)


def test_c2_launch_segmentation(c2):
    capi, wl, ctx, P, (q, p, it, st) = c2
    qq, pp = wl.q0, wl.p0
    for _ in range(5):
        qq, pp = ctx.leapfrog(P, qq, pp, wl.n_steps // 5)
    assert np.array_equal(qq, q) and np.array_equal(pp, p)


def test_c2_reversibility(c2):
    capi, wl, ctx, P, (q, p, it, st) = c2
    refl = (st & (capi.STATUS_REFLECT_F | capi.STATUS_REFLECT_XY)) != 0
    qb, pb = ctx.leapfrog(P, q, -p, wl.n_steps)
    keep = ~refl           # wall reflections are reversible too, but compare the clean set
    err_q = np.abs(qb[keep] - wl.q0[keep]) / (np.abs(wl.q0[keep]) + 1)
    err_p = np.abs(-pb[keep] - wl.p0[keep]) / (np.abs(wl.p0[keep]) + 1)
    assert keep.sum() > 3000
    assert np.median(err_q) < 1e-6 and err_q.max() < 5e-4, (np.median(err_q), err_q.max())
    assert np.median(err_p) < 1e-5 and err_p.max() < 5e-3, (np.median(err_p), err_p.max())


def test_c4_shard_full_size(gpu_lib):
    """Rank 0's shard of C4 (2^20 chains over 8 GPUs = 131072 chains) in one
    launch: finite, and a seeded sample matches the oracle (100 steps)."""
    capi = gpu_lib
    wl = workloads.make("C4")
    lo, hi = shard_range(1 << 20, 8, 0)
    q0, p0 = wl.q0[lo:hi], wl.p0[lo:hi]
    assert q0.shape[0] == 131072
    ctx = capi.Context(wl.D)
    P = capi.make_params(**wl.params)
    q, p, it, st = ctx.leapfrog(P, q0, p0, 100, return_info=True)
    assert not (st & capi.STATUS_NONFINITE).any()
    m = R.RefModel(wl.D, _oracle_params(wl))
    for c in (0, 65536, 131071):
        qo, po, NP, NQ = m.trajectory(q0[c], p0[c], 100, record=False)
        assert it[c, 0] == NP.sum() and it[c, 1] == NQ.sum(), c
        assert np.abs(q[c] - qo).max() / (np.abs(qo).max() + 1) <= 1e-9
        assert np.abs(p[c] - po).max() / (np.abs(po).max() + 1) <= 1e-8
    ctx.close()
