"""The native reversible-jump driver (librhmc_rj.so, include/rhmc_rj.h) on
the GPU against the NumPy loop of multi_gym.run_RHMC_rj_batched: both drive
the same engine batches (chains grouped by star count), so the move types,
star counts and accept decisions must be identical and the chains equal to
within the last-ulp differences of the host kinetic energy (C libm's log vs
NumPy's).  The reference pin is test_gpu_sampler.py::
test_run_RHMC_rj_batched_equals_single_runs[native] (chain 0 = the
reference's own rj_all run, tests/golden/rj.npz)."""
import warnings

import numpy as np
import pytest

from conftest import load_golden
from helpers import assert_state_close
from oracle import rhmc_ref as R
from test_gpu_sampler import _gym

pytestmark = pytest.mark.gpu


def _starts(qm, n, rs):
    """n starts around the golden's stars: 2-5 stars each, positions jittered."""
    out = []
    for c in range(n):
        k = 2 + c % 4
        m = np.tile(qm, (2, 1))[:k].copy()
        m[:, 0] += rs.uniform(-0.5, 0.5, k)
        m[:, 1:] += rs.uniform(-2, 2, (k, 2))
        out.append(m)
    return out


def _completing(g_factory, starts, seeds, kw):
    """(start, seed) pairs whose NumPy run completes: the reference raises on
    dead ends (no star left, nothing mergeable), where the native driver
    rejects — test_native_dead_ends_on_the_engine covers those."""
    from rhmc_amd import capi
    ok = []
    for m, s in zip(starts, seeds):
        g = g_factory()
        with warnings.catch_warnings(), np.errstate(all="ignore"):
            warnings.simplefilter("ignore")
            try:
                g.run_RHMC_rj_batched([m.copy()], [s], engine="python", **kw)
            except (ValueError, capi.RhmcError):
                continue
        ok.append((m, s))
    return ok


@pytest.mark.parametrize("sched", [False, True])
def test_native_equals_numpy_loop_many_chains(gpu_lib, sched):
    z = load_golden("rj")
    name = "rj_all"
    par = R.params_from_npz(z, name + "/par_")

    def make():
        g = _gym(par)
        g.D = z[name + "/D"]
        return g
    rs = np.random.RandomState(5)
    starts = _starts(z[name + "/q_model"], 40, rs)
    seeds = list(range(700, 740))
    kw = dict(f_pos=True, delta=1e-6, Niter=12, Nsteps=6, dt=0.05, N_max=10,
              P_move=[0.4, 0.3, 0.3])
    if sched:
        kw["schedule_g_ff2"] = np.array([1.0, 2.0, 3.0, 4.0])
    ok = _completing(make, starts, seeds, kw)
    assert len(ok) >= 20
    a, b = make(), make()
    qa = a.run_RHMC_rj_batched([m.copy() for m, _ in ok], [s for _, s in ok], engine="native",
                               **kw)
    qb = b.run_RHMC_rj_batched([m.copy() for m, _ in ok], [s for _, s in ok], engine="python",
                               **kw)
    np.testing.assert_array_equal(a.move_chain, b.move_chain)
    np.testing.assert_array_equal(a.N_chain, b.N_chain)
    np.testing.assert_array_equal(a.A_chain, b.A_chain)
    assert not a.flag_chain.any()
    assert_state_close(a.q_chain, b.q_chain, 1e-11, "q_chain")
    assert_state_close(a.p_chain, b.p_chain, 1e-11, "p_chain")
    np.testing.assert_allclose(a.E_chain, b.E_chain, rtol=1e-12)
    np.testing.assert_allclose(a.V_chain, b.V_chain, rtol=1e-12)
    for x, y in zip(qa, qb):
        assert x.size == y.size
        np.testing.assert_allclose(x, y, rtol=1e-11, atol=1e-11)
    assert a.g_ff2 == b.g_ff2
    # every move type happened and some jumps were accepted
    assert set(np.unique(a.move_chain)) >= {0, 1, 2, 3, 4}
    assert (a.move_chain[a.A_chain] > 0).any()


def test_native_dead_ends_on_the_engine(gpu_lib):
    """One-star starts with deaths and merges proposed often: the native
    driver rejects the dead ends (the reference raises) and keeps every chain
    at 1 <= K <= N_max; its chains stay finite."""
    z = load_golden("rj")
    name = "rj_all"
    par = R.params_from_npz(z, name + "/par_")
    g = _gym(par)
    g.D = z[name + "/D"]
    starts = [z[name + "/q_model"][:1].copy() for _ in range(16)]
    q = g.run_RHMC_rj_batched(starts, list(range(16)), f_pos=True, Niter=10, Nsteps=4,
                              dt=0.05, N_max=4, P_move=[0.2, 0.4, 0.4])
    assert g.flag_chain.any()
    assert not g.A_chain[g.flag_chain.astype(bool)].any()
    assert (g.N_chain >= 1).all() and (g.N_chain <= 4).all()
    assert all(np.isfinite(x).all() and 3 <= x.size <= 12 for x in q)


@pytest.mark.parametrize("pipes", [2, 3, 8])
def test_native_pipes_equal_one(gpu_lib, pipes):
    """n_pipes = 2, 3 or 8 (that many parts on as many host threads, their
    host and GPU phases overlapping, each part its own engine batches; 3 splits
    64 chains unevenly, 8 puts two parts on each of the box's four hardware
    queues) gives every chain the same moves, star counts and accepts as one
    pass, and the same states (the engine's results do not depend on the
    batch; tolerance for the kernels whose last bits follow wave-mates in rare
    non-finite / far-off cases)."""
    z = load_golden("rj")
    name = "rj_all"
    par = R.params_from_npz(z, name + "/par_")

    def make():
        g = _gym(par)
        g.D = z[name + "/D"]
        return g
    rs = np.random.RandomState(9)
    starts = _starts(z[name + "/q_model"], 64, rs)
    kw = dict(f_pos=True, delta=1e-6, Niter=8, Nsteps=6, dt=0.05, N_max=16,
              P_move=[0.4, 0.3, 0.3])
    a, b = make(), make()
    qa = a.run_RHMC_rj_batched([m.copy() for m in starts], list(range(64)), n_pipes=1, **kw)
    qb = b.run_RHMC_rj_batched([m.copy() for m in starts], list(range(64)), n_pipes=pipes, **kw)
    for k in ("move_chain", "N_chain", "A_chain", "flag_chain"):
        np.testing.assert_array_equal(getattr(a, k), getattr(b, k), err_msg=k)
    assert_state_close(a.q_chain, b.q_chain, 1e-12, "q_chain")
    np.testing.assert_allclose(a.E_chain, b.E_chain, rtol=1e-12)
    for x, y in zip(qa, qb):
        np.testing.assert_allclose(x, y, rtol=1e-12, atol=1e-12)


def test_native_across_256_stars(gpu_lib):
    """Reversible jumps around 256 stars (N_max 300, a 64x64 image of 300
    reference stars, hugek.npz): chains of 255-257 stars, so the phases mix
    the engine's 4-slot LDS-table launches with its 8-slot global-table ones
    and a birth / death / split / merge proposal moves a chain between them;
    the momentum draw and T run the one-chain-per-block kinetic kernel (rows
    of 900 doubles).  The native driver equals the NumPy loop on the same
    engine."""
    z = load_golden("hugek")
    name = "h300"
    par = R.params_from_npz(z, name + "/par_")

    def make():
        g = _gym(par)
        g.D = z[name + "/D"]
        return g
    q = z[name + "/q"][0]
    g0 = make()
    stars = np.stack([g0.flux2mag_converter(q[0::3]), q[1::3], q[2::3]], 1)
    rs = np.random.RandomState(17)
    starts = []
    for c in range(12):
        m = stars[rs.permutation(300)[:255 + c % 3]].copy()
        m[:, 1:] += rs.uniform(-0.2, 0.2, (len(m), 2))
        starts.append(m)
    seeds = list(range(900, 912))
    kw = dict(f_pos=False, delta=1e-6, Niter=5, Nsteps=3, dt=0.05, N_max=300,
              P_move=[0.2, 0.4, 0.4])
    ok = _completing(make, starts, seeds, kw)
    assert len(ok) >= 6
    a, b = make(), make()
    qa = a.run_RHMC_rj_batched([m.copy() for m, _ in ok], [s for _, s in ok], engine="native",
                               **kw)
    qb = b.run_RHMC_rj_batched([m.copy() for m, _ in ok], [s for _, s in ok], engine="python",
                               **kw)
    np.testing.assert_array_equal(a.move_chain, b.move_chain)
    np.testing.assert_array_equal(a.N_chain, b.N_chain)
    np.testing.assert_array_equal(a.A_chain, b.A_chain)
    assert_state_close(a.q_chain, b.q_chain, 1e-11, "q_chain")
    np.testing.assert_allclose(a.E_chain, b.E_chain, rtol=1e-12)
    for x, y in zip(qa, qb):
        assert x.size == y.size
        np.testing.assert_allclose(x, y, rtol=1e-11, atol=1e-11)
    assert a.N_chain[0].min() <= 256 < a.N_chain[0].max()      # both slot classes from the start
    assert (a.move_chain > 0).any()


def test_native_record_buffers_reused_only_when_unreferenced(gpu_lib):
    """With reuse_records=True (opt-in: bench.py) a second run writes its
    q_chain / p_chain records into the first run's memory only when nothing
    but the sampler holds it; the records equal a fresh sampler's either way
    (every row, padding included, is overwritten), and a caller's reference
    keeps the first run's records intact.  Without the flag a run never
    reuses them."""
    z = load_golden("rj")
    name = "rj_all"
    par = R.params_from_npz(z, name + "/par_")

    def make():
        g = _gym(par)
        g.D = z[name + "/D"]
        return g
    starts = _starts(z[name + "/q_model"], 24, np.random.RandomState(3))
    kw = dict(f_pos=True, delta=1e-6, Niter=5, Nsteps=4, dt=0.05, N_max=12,
              P_move=[0.4, 0.3, 0.3], reuse_records=True)
    g = make()
    g.run_RHMC_rj_batched(starts, list(range(24)), **kw)
    first = g.q_chain.copy()
    addr = g.q_chain.ctypes.data
    held = g.q_chain
    g.run_RHMC_rj_batched(starts, list(range(24)), **dict(kw, reuse_records=False))
    assert g.q_chain is not held and g.q_chain.ctypes.data != addr   # not opted in
    np.testing.assert_array_equal(g.q_chain, first)
    held = None
    g.run_RHMC_rj_batched(starts, list(range(24)), **kw)
    first = g.q_chain.copy()
    addr = g.q_chain.ctypes.data
    g.run_RHMC_rj_batched(starts, list(range(100, 124)), **kw)    # reuses the buffer
    assert g.q_chain.ctypes.data == addr
    fresh = make()
    fresh.run_RHMC_rj_batched(starts, list(range(100, 124)), **kw)
    np.testing.assert_array_equal(g.q_chain, fresh.q_chain)
    np.testing.assert_array_equal(g.p_chain, fresh.p_chain)
    held = g.q_chain                                                # a caller's reference
    g.run_RHMC_rj_batched(starts, list(range(24)), **kw)
    assert g.q_chain is not held
    np.testing.assert_array_equal(g.q_chain, first)
    np.testing.assert_array_equal(held, fresh.q_chain)
    view = g.p_chain[1]                                             # a view blocks it too
    before = view.copy()
    g.run_RHMC_rj_batched(starts, list(range(100, 124)), **kw)
    np.testing.assert_array_equal(view, before)
    # reused records come back read-only and are rewritten only up to each
    # row's old width (records_zero_padded); records a caller made writable
    # and wrote into are rewritten whole
    assert not g.q_chain.flags.writeable and not g.p_chain.flags.writeable
    view = before = None
    g.run_RHMC_rj_batched(starts, list(range(24)), **kw)
    np.testing.assert_array_equal(g.q_chain, first)
    g.q_chain.flags.writeable = True
    g.q_chain[...] = 5.
    g.run_RHMC_rj_batched(starts, list(range(100, 124)), **kw)
    np.testing.assert_array_equal(g.q_chain, fresh.q_chain)
    np.testing.assert_array_equal(g.p_chain, fresh.p_chain)


def test_native_recorded_V_dense_ragged(gpu_lib):
    """The same V-reuse check where the driver's phases are ragged dense
    launches (32x32, 12 - 40 stars, births and splits past the starting
    counts): every recorded V equals the engine's V of that row's q alone."""
    zb = load_golden("traj_bigk")
    par = R.params_from_npz(zb)
    g = _gym(par)
    g.D = zb["D"]
    g.K_split, g.beta_a, g.beta_b = 1., 4., 4.
    rs = np.random.RandomState(31)
    q0 = zb["Q"][0, 0].reshape(-1, 3)
    starts = []
    for c in range(40):
        m = q0[rs.permutation(100)[:12 + c % 29]].copy()
        m[:, 0] = g.flux2mag_converter(np.maximum(m[:, 0], 1.5 * par["f_lim"]))
        starts.append(m)
    kw = dict(f_pos=True, delta=1e-6, Niter=6, Nsteps=3, dt=0.05, N_max=48,
              P_move=[0.4, 0.3, 0.3])
    g.run_RHMC_rj_batched(starts, list(range(40)), **kw)
    ctx = g._context()
    P = g._params(kw["delta"], 1000, for_energy=True)
    for l in range(kw["Niter"] + 1):
        for c in range(40):
            K = int(g.N_chain[l, c])
            V, _ = ctx.energy(P, g.q_chain[l, c, :3 * K], f_pos=True)
            assert V == g.V_chain[l, c] or (np.isnan(V) and np.isnan(g.V_chain[l, c])), (l, c, K)
    assert len(np.unique(g.N_chain)) > 20 and (g.A_chain & (g.move_chain > 0)).any()


@pytest.mark.parametrize("sched", [False, True])
def test_native_recorded_V_is_the_engine_V_of_each_start(gpu_lib, sched):
    """The driver takes an iteration's V(q) from the previous iteration's end
    (V(q') when it accepted, its V(q) otherwise) while the prior parameters
    are unchanged; the reference recomputes it.  Every recorded V_chain row
    equals the engine's V of that row's q evaluated alone (one chain per
    call), bit for bit: one- to five-star chains (the one-star register-window
    energy and the per-wave kernels), with and without a g_ff2 schedule
    (which forces the recomputation on the iterations it changes)."""
    z = load_golden("rj")
    name = "rj_all"
    par = R.params_from_npz(z, name + "/par_")
    g = _gym(par)
    g.D = z[name + "/D"]
    rs = np.random.RandomState(21)
    starts = [m[:1 + c % 5] for c, m in enumerate(_starts(z[name + "/q_model"], 40, rs))]
    kw = dict(f_pos=True, delta=1e-6, Niter=10, Nsteps=6, dt=0.05, N_max=8,
              P_move=[0.4, 0.3, 0.3])
    if sched:
        kw["schedule_g_ff2"] = np.array([1., 1., 2., 2., 2., 4.])
    g.run_RHMC_rj_batched([m.copy() for m in starts], list(range(300, 340)), **kw)
    ctx = g._context()
    gff = np.ravel(kw.get("schedule_g_ff2", [g.g_ff2]))
    for l in range(kw["Niter"] + 1):
        g.g_ff2 = float(gff[min(l, gff.size - 1)])
        P = g._params(kw["delta"], 1000, for_energy=True)
        for c in range(len(starts)):
            K = int(g.N_chain[l, c])
            V, _ = ctx.energy(P, g.q_chain[l, c, :3 * K], f_pos=True)
            assert V == g.V_chain[l, c] or (np.isnan(V) and np.isnan(g.V_chain[l, c])), (l, c, K)
    assert (g.A_chain & (g.move_chain > 0)).any()
    assert set(np.unique(g.N_chain)) >= {1, 2, 3}


def test_native_checkpoint_resume_on_the_engine(gpu_lib):
    """A run of Niter = 11 (rows 0..11) == a run of Niter = 5 and a resume from
    its final q and rj_rng_states for Niter = 5 more: the same engine batches
    in the same order, so every record is bit-identical; and rng_states taken
    from fresh RandomState(seed) objects is the seeded run."""
    z = load_golden("rj")
    name = "rj_all"
    par = R.params_from_npz(z, name + "/par_")

    def make():
        g = _gym(par)
        g.D = z[name + "/D"]
        return g
    rs = np.random.RandomState(13)
    starts = _starts(z[name + "/q_model"], 48, rs)
    seeds = list(range(900, 948))
    kw = dict(f_pos=True, delta=1e-6, Nsteps=6, dt=0.05, N_max=12, P_move=[0.4, 0.3, 0.3],
              n_pipes=2)
    a, b, c = make(), make(), make()
    qa = a.run_RHMC_rj_batched([m.copy() for m in starts], seeds, Niter=11, **kw)
    qb = b.run_RHMC_rj_batched([m.copy() for m in starts], None, Niter=5, **kw,
                               rng_states=[np.random.RandomState(s) for s in seeds])
    rec_b = {k: getattr(b, k).copy() for k in ("move_chain", "N_chain", "A_chain",
                                                 "flag_chain", "q_chain", "E_chain")}
    qc = c.run_RHMC_rj_batched(qb, None, Niter=5, **kw, rng_states=b.rj_rng_states)
    for k, v in rec_b.items():
        np.testing.assert_array_equal(getattr(a, k),
                                      np.concatenate([v, getattr(c, k)]), err_msg=k)
    for x, y in zip(qa, qc):
        np.testing.assert_array_equal(x, y)
    assert np.array_equal(a.rj_rng_states, c.rj_rng_states)
    assert (a.move_chain[a.A_chain] > 0).any()


@pytest.mark.parametrize("golden,name", [("rj", "rj_bd"), ("rj", "rj_sm"), ("rj", "rj_all"),
                                         ("mh", "mh1"), ("mh", "mh3"), ("mh_sched", "g1"),
                                         ("mh_sched", "g3"), ("mh_sched", "g3vc")])
def test_native_reproduces_reference_goldens(gpu_lib, golden, name):
    """Every reference run_RHMC golden (birth/death only, split/merge only,
    all moves; within-model MH with one and three stars; g_ff2 / beta
    schedules with and without repulsion) through the native driver as chain
    0 of a batch of six (the other five: the same start on other seeds, which
    share its engine batches): moves, star counts and accepts exact, states
    and energies to the reference tolerances."""
    from test_gpu_sampler import _sched_gym
    z = load_golden(golden)
    kw = dict(f_pos=True, delta=1e-6, Niter=int(z[name + "/niter"]),
              Nsteps=int(z[name + "/nsteps"]), dt=float(z[name + "/dt"]))
    if golden == "mh_sched":
        g, sg, sb = _sched_gym(z, name)
        kw.update(schedule_g_ff2=sg, schedule_beta=sb)
    else:
        g = _gym(R.params_from_npz(z, name + "/par_"))
        g.D = z[name + "/D"]
    qm = z[name + "/q_model"]
    if golden == "rj":
        kw.update(N_max=int(z[name + "/N_max"]), P_move=list(z[name + "/P_move"]))
    else:
        kw.update(N_max=qm.shape[0], P_move=[1., 0., 0.])
    seed = int(z[name + "/seed"])
    g.run_RHMC_rj_batched([qm.copy() for _ in range(6)], [seed] + [seed + 1 + i for i in range(5)],
                          n_pipes=1, **kw)
    np.testing.assert_array_equal(g.A_chain[:, 0].astype(np.int32), z[name + "/A_chain"])
    if golden == "rj":
        np.testing.assert_array_equal(g.move_chain[:, 0], z[name + "/move_chain"])
        np.testing.assert_array_equal(g.N_chain[:, 0], z[name + "/N_chain"])
    W = z[name + "/q_chain"].shape[-1]
    assert_state_close(g.q_chain[:, 0, :W], z[name + "/q_chain"], 1e-9, "q_chain")
    assert_state_close(g.p_chain[:, 0, :W], z[name + "/p_chain"], 1e-9, "p_chain")
    np.testing.assert_allclose(g.E_chain[:, 0], z[name + "/E_chain"], rtol=1e-11)
    np.testing.assert_allclose(g.V_chain[:, 0], z[name + "/V_chain"], rtol=1e-11)
    if golden == "mh_sched":
        assert g.g_ff2 == z[name + "/g_ff2_final"] and g.beta == z[name + "/beta_final"]


@pytest.mark.parametrize("case", ["pixk_dense32", "dense_slots32", "kr_wingg64"])
def test_native_recorded_V_across_family_boundaries(gpu_lib, case):
    """The V reuse (include/rhmc_rj.h: an iteration's V(q) is the previous
    iteration's V(q') or V(q)) holds only if a chain's V does not depend on
    the launch it was evaluated in.  Births, deaths, splits and merges move
    chains across the kernel families' star-count boundaries, so each
    boundary is crossed here, and every recorded V must equal the engine's V
    of that row alone (one chain, fixed K) bit for bit:
      pixk_dense32  32x32, 8-12 stars: ragged pixel-major (2-10) <-> ragged
                    dense slot 1 (11-64) — the flagship's range;
      dense_slots32 32x32, 61-68 stars: dense slot 1 <-> dense slot 2;
      kr_wingg64    64x64, 61-68 stars: packed multi-star register-window
                    launches (<= 64) <-> ragged windowed global tables (WinGG,
                    >= 65)."""
    zb = load_golden("traj_hugek" if case == "kr_wingg64" else "traj_bigk")
    par = R.params_from_npz(zb)
    g = _gym(par)
    g.D = zb["D"]
    g.K_split, g.beta_a, g.beta_b = 1., 4., 4.
    rs = np.random.RandomState(41)
    q0 = zb["Q"][0, 0].reshape(-1, 3)
    lo, hi = (8, 12) if case == "pixk_dense32" else (61, 68)
    starts = []
    for c in range(24):
        m = q0[rs.permutation(len(q0))[:lo + c % (hi - lo + 1)]].copy()
        m[:, 0] = g.flux2mag_converter(np.maximum(m[:, 0], 1.5 * par["f_lim"]))
        starts.append(m)
    kw = dict(f_pos=True, delta=1e-6, Niter=6, Nsteps=3, dt=0.05, N_max=hi + 8,
              P_move=[0.2, 0.4, 0.4])
    g.run_RHMC_rj_batched(starts, list(range(500, 524)), **kw)
    ctx = g._context()
    P = g._params(kw["delta"], 1000, for_energy=True)
    for l in range(kw["Niter"] + 1):
        for c in range(len(starts)):
            K = int(g.N_chain[l, c])
            V, _ = ctx.energy(P, g.q_chain[l, c, :3 * K], f_pos=True)
            assert V == g.V_chain[l, c] or (np.isnan(V) and np.isnan(g.V_chain[l, c])), (l, c, K)
    edge = 10 if case == "pixk_dense32" else 64
    assert (g.N_chain <= edge).any() and (g.N_chain > edge).any()
    # a chain whose count crossed the boundary during the run
    assert ((g.N_chain.min(0) <= edge) & (g.N_chain.max(0) > edge)).any()
