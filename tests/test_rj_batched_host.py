"""CPU test of run_RHMC_rj_batched's orchestration (no GPU): with the two GPU
calls it makes (V and RHMC_steps) replaced by the same deterministic stand-ins
on both sides, the batched runner — per-chain streams, phases grouped by star
count, rejections restoring the old dimension — must equal one run_RHMC per
seed, record for record, and leave the global NumPy stream untouched.  The
physics is pinned on the GPU (test_gpu_sampler.py::
test_run_RHMC_rj_batched_equals_single_runs); this pins the bookkeeping."""
import numpy as np
import pytest


def _fake_gpu(g):
    def V(q, f_pos=False):
        q = np.asarray(q, dtype=np.float64)
        v = 1e-4 * np.sum(q.reshape(q.shape[0], -1) ** 2, axis=1) if q.ndim == 2 else \
            1e-4 * np.sum(q ** 2)
        return v

    def RHMC_steps(q, p, n_steps, delta=1e-6, counter_max=1000, return_info=False):
        q = np.array(q, dtype=np.float64)
        p = np.array(p, dtype=np.float64)
        for _ in range(n_steps):
            q = q + 0.01 * p
            p = 0.99 * p - 1e-4 * q
        return q, p
    g.V = V
    g.RHMC_steps = RHMC_steps
    g.V_prior_const = 1.5
    return g


def _gym():
    from rhmc_amd import sampler
    g = sampler.multi_gym(dt=0.05, g_xx=0.05, g_ff=4., g_ff2=4.)
    g.num_rows = g.num_cols = 32
    g.use_prior, g.alpha = True, 2.
    g.fmin = g.mag2flux_converter(23.3)
    g.fmax = g.mag2flux_converter(15.)
    return _fake_gpu(g)


@pytest.mark.parametrize("P_move", [[0.4, 0.3, 0.3], [0.2, 0.8, 0.0]])
def test_rj_batched_equals_per_seed_runs(P_move, capsys):
    starts = [np.array([[18., 10.2, 12.7], [19., 20.3, 18.1], [20., 15., 25.]]),
              np.array([[18.3, 10.5, 12.2], [19.4, 20.0, 18.4]]),
              np.array([[18., 10.2, 12.7], [19., 20.3, 18.1], [20., 15., 25.], [19.5, 8., 9.]]),
              np.array([[18.5, 16., 16.], [19.5, 11., 14.]])]
    seeds = [11, 12, 13, 14]
    kw = dict(f_pos=True, Niter=12, Nsteps=3, dt=0.05, N_max=10, P_move=P_move)
    singles = []
    for qm, s in zip(starts, seeds):
        h = _gym()
        np.random.seed(s)
        h.run_RHMC(qm.copy(), **kw)
        singles.append(h)
    capsys.readouterr()
    g = _gym()
    np.random.seed(5)
    before = np.random.get_state()[1].copy()
    q_end = g.run_RHMC_rj_batched([m.copy() for m in starts], seeds, engine="python", **kw)
    assert np.array_equal(np.random.get_state()[1], before)
    for c, h in enumerate(singles):
        assert np.array_equal(g.move_chain[:, c], h.move_chain)
        assert np.array_equal(g.N_chain[:, c], h.N_chain)
        assert np.array_equal(g.A_chain[:, c], h.A_chain)
        assert np.array_equal(g.q_chain[:, c], h.q_chain)
        assert np.array_equal(g.p_chain[:, c], h.p_chain)
        assert np.array_equal(g.E_chain[:, c], h.E_chain)
        assert q_end[c].size == 3 * h.Nobjs
    # the batch mixed star counts and both kinds of decision happened
    assert len(set(g.N_chain.ravel())) > 1
    assert g.A_chain.any() and not g.A_chain.all()


def test_rj_batched_python_engine_takes_list_schedules():
    """schedule_g_ff2 / schedule_beta as plain lists work on the NumPy loop as
    on the native engine (both normalise them to arrays) and give the array
    schedule's run."""
    starts = [np.array([[18., 10.2, 12.7], [19., 20.3, 18.1]]),
              np.array([[18.3, 10.5, 12.2]])]
    kw = dict(f_pos=True, Niter=6, Nsteps=2, dt=0.05, N_max=6, P_move=[0.4, 0.3, 0.3])
    a, b = _gym(), _gym()
    a.run_RHMC_rj_batched([m.copy() for m in starts], [3, 4], engine="python",
                          schedule_g_ff2=[1., 2., 4.], schedule_beta=[0.5], **kw)
    b.run_RHMC_rj_batched([m.copy() for m in starts], [3, 4], engine="python",
                          schedule_g_ff2=np.array([1., 2., 4.]), schedule_beta=np.array([0.5]),
                          **kw)
    for k in ("q_chain", "E_chain", "A_chain", "N_chain"):
        assert np.array_equal(getattr(a, k), getattr(b, k)), k
    assert a.g_ff2 == b.g_ff2 == 4.
