"""CPU tests of librhmc_rj.so (include/rhmc_rj.h), the native reversible-jump
driver, without a GPU:

* its NumPy-legacy stream replica against numpy.random.RandomState itself
  (random_sample, randn, randint, beta incl. scipy.stats.beta.rvs,
  standard_gamma, standard_exponential): bit-identical;
* its orchestration against the Python multi_gym.run_RHMC_rj_batched, both
  driven by the same deterministic stand-ins for the two engine calls
  (test_rj_batched_host._fake_gpu): identical move types, star counts and
  accept decisions, states and energies equal to within a few ulp (the
  native kinetic energy takes C libm's log where NumPy may use its own SIMD
  log: one-ulp differences, nothing else);
* dead ends (no star left, nothing to merge), host-thread invariance and
  argument errors.

The physics is pinned on the GPU (tests/test_gpu_rj_native.py)."""
import warnings

import numpy as np
import pytest

from test_rj_batched_host import _gym

STARTS = [np.array([[18., 10.2, 12.7], [19., 20.3, 18.1], [20., 15., 25.]]),
          np.array([[18.3, 10.5, 12.2], [19.4, 20.0, 18.4]]),
          np.array([[18., 10.2, 12.7], [19., 20.3, 18.1], [20., 15., 25.], [19.5, 8., 9.]]),
          np.array([[18.5, 16., 16.], [19.5, 11., 14.]])]


@pytest.fixture(scope="module")
def rj():
    from rhmc_amd import rj_native
    return rj_native


def test_exports_match_header(rj):
    import os
    import re
    from conftest import ROOT
    txt = open(os.path.join(ROOT, "include", "rhmc_rj.h")).read()
    declared = sorted(set(re.findall(r"\b(rhmc_[a-z_]+)\s*\(", txt)))
    assert sorted(rj.EXPORTS) == declared
    assert all(hasattr(rj.lib(), s) for s in declared)


@pytest.mark.parametrize("seed", [0, 1, 77, 12345, 2 ** 32 - 1])
def test_stream_replica_is_bit_identical(rj, seed):
    n = 4000
    r = np.random.RandomState(seed)
    assert np.array_equal(r.random_sample(n), rj.np_draws(seed, "random_sample", n))
    r = np.random.RandomState(seed)
    assert np.array_equal(r.randn(n), rj.np_draws(seed, "randn", n))
    for hi in (1, 2, 3, 51, 120, 1000, 2 ** 31 + 5):
        r = np.random.RandomState(seed)
        ref = [r.randint(0, hi, size=1)[0] for _ in range(200)]
        assert np.array_equal(np.array(ref, float), rj.np_draws(seed, "randint", 200, a=hi)), hi
    for a, b in ((2., 2.), (0.5, 0.7), (1., 1.), (0.3, 3.), (5., 1.5)):
        r = np.random.RandomState(seed)
        ref = [r.beta(a, b) for _ in range(300)]
        assert np.array_equal(np.array(ref), rj.np_draws(seed, "beta", 300, a=a, b=b)), (a, b)
    for s in (0.3, 1.0, 2.5):
        r = np.random.RandomState(seed)
        assert np.array_equal(r.standard_gamma(s, size=300),
                              rj.np_draws(seed, "standard_gamma", 300, a=s)), s
    r = np.random.RandomState(seed)
    assert np.array_equal(r.standard_exponential(300),
                          rj.np_draws(seed, "standard_exponential", 300))


def test_scipy_beta_rvs_is_the_replica(rj):
    """split_merge_move draws F with scipy.stats.beta.rvs on the global stream
    (sampler_RHMC.py:1302): the legacy beta of the same stream."""
    from scipy.stats import beta as BETA
    np.random.seed(3)
    np.random.randn(5)
    a = BETA.rvs(2., 2., size=1)[0]
    r = np.random.RandomState(3)
    r.randn(5)
    assert a == r.beta(2., 2.)


def _native(rj, g, starts, seeds, kw, n_threads=4, n_pipes=1, **extra):
    from rhmc_amd import capi
    qms = [g.format_q(m.copy()) for m in starts]
    P = g._params(for_energy=True)
    fake_V, fake_S = g.V, g.RHMC_steps

    def steps(q, p, ns):
        qq, pp = fake_S(q, p, ns)
        q[:] = qq
        p[:] = pp
    return rj.run(P, qms, seeds, kw["Niter"], kw["Nsteps"], kw["N_max"], kw["P_move"],
                  capi.V_FLUX_WALL if kw["f_pos"] else 0, g.num_rows, g.num_cols, g.fmin, g.fmax,
                  g.K_split, g.beta_a, g.beta_b, physics=(lambda q, fp: fake_V(q), steps),
                  n_threads=n_threads, n_pipes=n_pipes, **extra)


def _clean(g, N_max):
    """Chains whose Python run never proposed a dead end (a death / merge at
    one star, a birth / split at N_max): the reference raises there (and the
    stand-ins would carry on with zero stars), the native driver rejects."""
    mv, N = g.move_chain, g.N_chain
    dead = ((np.isin(mv, (2, 4)) & (N <= 1)) | (np.isin(mv, (1, 3)) & (N >= N_max)))
    return ~dead.any(axis=0)


@pytest.mark.parametrize("P_move", [[0.4, 0.3, 0.3], [0.2, 0.8, 0.0], [0.2, 0.0, 0.8]])
def test_native_equals_python_batched(rj, P_move):
    starts = STARTS * 10
    seeds = list(range(11, 11 + len(starts)))
    kw = dict(f_pos=True, Niter=20, Nsteps=3, dt=0.05, N_max=12, P_move=P_move)
    g = _gym()
    with warnings.catch_warnings(), np.errstate(all="ignore"):
        warnings.simplefilter("ignore")
        ok = []
        for m, s in zip(starts, seeds):      # chains whose Python run completes
            try:
                _gym().run_RHMC_rj_batched([m.copy()], [s], engine="python", **kw)
                ok.append((m, s))
            except ValueError:
                pass
        g.run_RHMC_rj_batched([m.copy() for m, _ in ok], [s for _, s in ok],
                              engine="python", **kw)
    assert len(ok) >= 5
    h = _gym()
    q_end, rec = _native(rj, h, [m for m, _ in ok], [s for _, s in ok], kw)
    clean = _clean(g, kw["N_max"])
    assert clean.sum() >= 4
    np.testing.assert_array_equal(rec["move"][:, clean], g.move_chain[:, clean])
    np.testing.assert_array_equal(rec["n_stars"][:, clean], g.N_chain[:, clean])
    np.testing.assert_array_equal(rec["accept"][:, clean].astype(bool), g.A_chain[:, clean])
    assert not rec["flags"][:, clean].any()
    for k in ("q_chain", "p_chain", "E_chain", "V_chain", "T_chain"):
        a, b = rec[k][:, clean], getattr(g, k)[:, clean]
        np.testing.assert_allclose(a, b, rtol=1e-13, atol=1e-13, err_msg=k)
    # the run really jumped
    assert (g.move_chain[:, clean] > 0).any() and len(set(g.N_chain[:, clean].ravel())) > 1


def test_dead_ends_are_rejected_and_threads_do_not_matter(rj):
    """Deaths / merges at one star: the native driver rejects them (flag
    DEAD_END, state back to the iteration's start, no accept draw) and every
    chain's record is independent of the host thread count and of the split
    into two pipes (with these stand-ins every chain's physics is its own)."""
    starts = [np.array([[18.5, 16., 16.]])] * 20 + STARTS * 5
    seeds = list(range(100, 100 + len(starts)))
    kw = dict(f_pos=True, Niter=25, Nsteps=2, dt=0.05, N_max=6, P_move=[0.2, 0.4, 0.4])
    _, r1 = _native(rj, _gym(), starts, seeds, kw, n_threads=1)
    q4, r4 = _native(rj, _gym(), starts, seeds, kw, n_threads=7)
    for pipes, t in ((2, 5), (3, 3), (4, 9)):        # that many parts on that many threads
        qp, rp = _native(rj, _gym(), starts, seeds, kw, n_threads=t, n_pipes=pipes)
        for k in r1:
            if k != "phase_s":                        # wall times
                assert np.array_equal(r1[k], r4[k]), k
                assert np.array_equal(r1[k], rp[k]), (k, pipes)
        assert all(np.array_equal(a, b) for a, b in zip(q4, qp))
    assert (r1["phase_s"] >= 0).all() and r1["phase_s"].sum() > 0
    fl = r1["flags"].astype(bool)
    assert fl.any()
    assert not r1["accept"][fl].any()
    assert (r1["n_stars"] >= 1).all() and (r1["n_stars"] <= 6).all()
    # a dead-end iteration leaves the chain where it started
    l, c = np.argwhere(fl[:-1])[0]
    assert r1["n_stars"][l + 1, c] == r1["n_stars"][l, c]
    assert np.array_equal(r1["q_chain"][l + 1, c], r1["q_chain"][l, c])
    assert all(q.size % 3 == 0 and 3 <= q.size <= 18 for q in q4)


@pytest.mark.parametrize("n_pipes", [1, 3])
def test_zero_padded_records_equal_fresh_records(rj, n_pipes):
    """records_zero_padded (include/rhmc_rj.h): a second run written into the
    first run's q_chain / p_chain, told that their rows are zero past 3
    n_stars[row], rewrites only the columns a row can have used — and its
    records equal a fresh run's bit for bit, padding included (rows whose
    star count shrank between the runs get their old columns zeroed).  A
    star-count record of zeros (no claim) makes the driver write whole rows."""
    starts = STARTS * 6
    kw = dict(f_pos=True, Niter=15, Nsteps=2, dt=0.05, N_max=10, P_move=[0.2, 0.4, 0.4])
    _, a = _native(rj, _gym(), starts, list(range(300, 324)), kw, n_pipes=n_pipes)
    seeds_b = list(range(500, 524))
    _, fresh = _native(rj, _gym(), starts, seeds_b, kw, n_pipes=n_pipes)
    assert (a["n_stars"] != fresh["n_stars"]).any()
    assert (a["n_stars"] > fresh["n_stars"]).any()      # some rows shrink between the runs
    out = {k: a[k] for k in ("q_chain", "p_chain", "n_stars")}
    _, b = _native(rj, _gym(), starts, seeds_b, kw, n_pipes=n_pipes, out=out, zero_padded=True)
    assert b["q_chain"] is a["q_chain"] and b["n_stars"] is a["n_stars"]
    for k in fresh:
        if k not in ("phase_s", "states"):
            assert np.array_equal(b[k], fresh[k]), k
    # no claim: garbage past every row's columns, star counts zero -> whole rows
    q = np.full_like(fresh["q_chain"], 7.)
    p = np.full_like(fresh["p_chain"], -7.)
    out = {"q_chain": q, "p_chain": p, "n_stars": np.zeros_like(fresh["n_stars"])}
    _, c = _native(rj, _gym(), starts, seeds_b, kw, n_pipes=n_pipes, out=out, zero_padded=True)
    assert np.array_equal(c["q_chain"], fresh["q_chain"])
    assert np.array_equal(c["p_chain"], fresh["p_chain"])
    # (a claim without the star-count record and a flag of 2 are refused:
    # tests/native/rj_asan.cpp)


def test_argument_errors(rj):
    from rhmc_amd import capi
    g = _gym()
    P = g._params(for_energy=True)
    phys = (lambda q, fp: np.zeros(len(q)), lambda q, p, ns: None)
    base = dict(n_iter=2, n_steps=1, N_max=4, P_move=[0.5, 0.25, 0.25], f_pos=1, rows=32,
                cols=32, fmin=g.fmin, fmax=g.fmax, K_split=1., beta_a=2., beta_b=2.)
    q = [g.format_q(STARTS[1].copy())]
    with pytest.raises(capi.RhmcError, match="P_move"):
        rj.run(P, q, [1], **dict(base, P_move=[0.5, 0.2, 0.2]), physics=phys)
    with pytest.raises(capi.RhmcError, match="N_max"):
        rj.run(P, q, [1], **dict(base, N_max=1025), physics=phys)
    with pytest.raises(capi.RhmcError, match="fmin"):
        rj.run(P, q, [1], **dict(base, fmin=0.), physics=phys)
    with pytest.raises(ValueError):
        rj.run(P, [g.format_q(STARTS[2].copy())], [1], **dict(base, N_max=3), physics=phys)
    with pytest.raises(ValueError, match="seeds"):
        rj.run(P, q, [-1], **base, physics=phys)
    # an engine failure surfaces as the engine's error
    with pytest.raises(RuntimeError, match="boom"):
        def bad(q, fp):
            raise RuntimeError("boom")
        rj.run(P, q, [1], **base, physics=(bad, phys[1]))


def test_states_round_trip_and_continue_a_random_state(rj):
    """rhmc_np_state rows are RandomState.get_state(): a state taken after some
    draws (a cached gaussian included) continues that stream inside the
    driver, and the states a run leaves are the streams' true positions."""
    rs = [np.random.RandomState(s) for s in (5, 6, 7)]
    rs[0].randn(3)                                  # has_gauss = 1
    rs[1].random_sample(700)                        # past a twist
    st = rj.states_from(rs)
    assert st["has_gauss"][0] == 1 and st["pos"][1] != 624
    for r, row in zip(rs, st):
        a, b = r.get_state(), rj.random_state(row).get_state()
        assert np.array_equal(a[1], b[1]) and a[2:] == b[2:]
    # the driver continuing those streams == the driver started from the
    # seeds after the same draws: compare against a fresh run of each
    starts = STARTS[:3]
    kw = dict(f_pos=True, Niter=6, Nsteps=2, dt=0.05, N_max=8, P_move=[0.4, 0.3, 0.3])
    g = _gym()
    qms = [g.format_q(m.copy()) for m in starts]
    P = g._params(for_energy=True)
    phys = (lambda q, fp: g.V(q), lambda q, p, ns: _inplace(g, q, p, ns))
    base = dict(n_iter=6, n_steps=2, N_max=8, P_move=kw["P_move"], f_pos=1, rows=g.num_rows,
                cols=g.num_cols, fmin=g.fmin, fmax=g.fmax, K_split=g.K_split, beta_a=g.beta_a,
                beta_b=g.beta_b, physics=phys)
    fresh = rj.states_from([np.random.RandomState(s) for s in (5, 6, 7)])
    _, r_seed = rj.run(P, qms, [5, 6, 7], **base)
    _, r_state = rj.run(P, qms, None, **base, states=fresh)
    for k in r_seed:
        if k != "phase_s":
            assert np.array_equal(r_seed[k], r_state[k]), k
    # the streams moved on, and a drawn-from stream starts elsewhere
    assert (r_seed["states"]["pos"] != 624).any() or \
        not np.array_equal(r_seed["states"]["key"], fresh["key"])
    _, r_used = rj.run(P, qms, None, **base, states=st)
    assert not np.array_equal(r_used["move"], r_seed["move"]) or \
        not np.array_equal(r_used["q_chain"], r_seed["q_chain"])


def _inplace(g, q, p, ns):
    qq, pp = g.RHMC_steps(q, p, ns)
    q[:] = qq
    p[:] = pp


@pytest.mark.parametrize("n_pipes", [1, 2, 4])
def test_checkpoint_resume_is_one_run(rj, n_pipes):
    """One run == a run, then a resume from its final q, K and states:
    bit-identical records (the checkpoint of the
    reference's long runs, which restart np.random from a saved state)."""
    starts = [np.array([[18.5, 16., 16.]])] * 6 + STARTS * 4
    seeds = list(range(40, 40 + len(starts)))
    kw = dict(f_pos=True, Niter=14, Nsteps=2, dt=0.05, N_max=7, P_move=[0.3, 0.35, 0.35])
    q_full, r_full = _native(rj, _gym(), starts, seeds, kw, n_threads=3, n_pipes=n_pipes)
    g = _gym()
    P = g._params(for_energy=True)
    base = dict(n_steps=2, N_max=7, P_move=kw["P_move"], f_pos=1, rows=g.num_rows,
                cols=g.num_cols, fmin=g.fmin, fmax=g.fmax, K_split=g.K_split, beta_a=g.beta_a,
                beta_b=g.beta_b, n_threads=5, n_pipes=n_pipes,
                physics=(lambda q, fp: g.V(q), lambda q, p, ns: _inplace(g, q, p, ns)))
    qms = [g.format_q(m.copy()) for m in starts]
    q_a, r_a = rj.run(P, qms, seeds, n_iter=9, **base)
    # a run of n_iter records n_iter + 1 iterations (rows 0..n_iter, as the
    # reference): 10 + 5 rows == the 15 of Niter=14
    q_b, r_b = rj.run(P, q_a, None, n_iter=4, **base, states=r_a["states"])
    assert all(np.array_equal(a, b) for a, b in zip(q_full, q_b))
    assert np.array_equal(r_full["states"], r_b["states"])
    for k in r_full:
        if k in ("phase_s", "states"):
            continue
        assert np.array_equal(r_full[k], np.concatenate([r_a[k], r_b[k]])), k
    assert r_full["flags"].any()                    # the resume crossed dead ends too


def test_state_errors(rj):
    from rhmc_amd import capi
    g = _gym()
    P = g._params(for_energy=True)
    phys = (lambda q, fp: np.zeros(len(q)), lambda q, p, ns: None)
    base = dict(n_iter=2, n_steps=1, N_max=4, P_move=[0.5, 0.25, 0.25], f_pos=1, rows=32,
                cols=32, fmin=g.fmin, fmax=g.fmax, K_split=1., beta_a=2., beta_b=2., physics=phys)
    q = [g.format_q(STARTS[1].copy())]
    with pytest.raises(ValueError, match="one state"):
        rj.run(P, q, None, **base, states=rj.states_from([np.random.RandomState(1)] * 2))
    bad = rj.states_from([np.random.RandomState(1)])
    bad["pos"] = 700
    with pytest.raises(capi.RhmcError, match="pos"):
        rj.run(P, q, None, **base, states=bad)
    with pytest.raises(ValueError, match="seed"):
        rj.run(P, q, None, **base)


def test_integration_stub_matches_the_config_layout(rj):
    """INTEGRATION.md's ctypes stub of rhmc_rj_config has the library's field
    names, offsets and size (a maintainer copies it as it is)."""
    import ctypes
    import os
    from conftest import ROOT
    s = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    i = s.index("class _RjConfig")
    ns = {"ctypes": ctypes}
    exec(s[i:s.index("\n\n", i)], ns)
    A, B = ns["_RjConfig"], rj.RjConfig
    assert [f[0] for f in A._fields_] == [f[0] for f in B._fields_]
    assert ctypes.sizeof(A) == ctypes.sizeof(B)
    assert all(getattr(A, f[0]).offset == getattr(B, f[0]).offset for f in B._fields_)


def test_pack_starts_padded_equals_full(rj):
    """rhmc_rj_pack_starts_padded: rows written into a buffer that is zero past
    3 K_prev[c] (the previous run's final rows) equal a full pack, zeros
    included, whether a row grew or shrank; without K_prev, a buffer of
    garbage is overwritten whole."""
    rs = np.random.RandomState(4)
    n, N_max = 40, 12
    old = [rs.rand(k, 3) * 5 + 15 for k in rs.randint(1, N_max + 1, n)]
    new = [rs.rand(k, 3) * 5 + 15 for k in rs.randint(1, N_max + 1, n)]
    q_old, K_old = rj.pack_starts(old, N_max, 1.5)
    fresh, K_new = rj.pack_starts(new, N_max, 1.5)
    q, K = rj.pack_starts(new, N_max, 1.5, out=q_old, K_prev=K_old)
    assert q is q_old and np.array_equal(K, K_new)
    assert np.array_equal(q, fresh)
    junk = np.full_like(fresh, 9.)
    q2, _ = rj.pack_starts(new, N_max, 1.5, out=junk)
    assert np.array_equal(q2, fresh)
    same = np.repeat(new[0][None], 30, axis=0)      # one model for every chain (the memo)
    qs, _ = rj.pack_starts(same, N_max, 1.5)
    assert np.array_equal(qs, np.repeat(fresh[:1], 30, axis=0))
