"""Round-5 reference runs through every driver on the GPU.

* mh_bigk (make_goldens.py case_mh_bigk): multi_gym.run_RHMC move-0
  (P_move [1, 0, 0], f_pos, sampler_RHMC.py:1018-1083) at many stars with
  every start above the flux wall, so proposals are really accepted and
  rejected (the golden has 0 < acceptance < 1): d51 — RHMC-big-sim4.py's
  32x32 / 51-star geometry (the dense many-star kernel), w64 — the C5
  geometry, 256x256 / 64 stars (the multi-star register-window leapfrog, the
  windowed pixel-major energy of V(q') and the wave-per-chain begin / end
  kernels of the four-kernel MH loop).  Through run_RHMC (host loop),
  run_RHMC_batched (rhmc_mh with the reference's draws, fused option on and
  off) and the native driver (chain 0 of a batch).
* rj_big (case_rj_big): reversible jumps across K = 64 with
  RHMC-big-sim4.py's move parameters (beta_a = beta_b = 4) — births past 64
  stars.
* flagship (case_flagship): RHMC-big-sim4.py as written (Niter 40): every
  move type, jumps accepted, 5 -> 9 stars.

Parity bar: accept sequences, move types and star counts exact; states to
1e-9 relative (|x| + 1); energies to 1e-11 relative."""
import numpy as np
import pytest

from conftest import load_golden
from helpers import assert_state_close
from oracle import rhmc_ref as R

pytestmark = pytest.mark.gpu


def _gym(z, prefix=""):
    from test_gpu_sampler import _gym as base
    g = base(R.params_from_npz(z, prefix + "par_"))
    g.D = z[prefix + "D"]
    if prefix + "K_split" in z.files:
        g.K_split = float(z[prefix + "K_split"])
        g.beta_a, g.beta_b = float(z[prefix + "beta_a"]), float(z[prefix + "beta_b"])
    return g


def _kw(z, p):
    kw = dict(f_pos=True, delta=1e-6, Niter=int(z[p + "niter"]), Nsteps=int(z[p + "nsteps"]),
              dt=float(z[p + "dt"]))
    if p + "P_move" in z.files:
        kw.update(N_max=int(z[p + "N_max"]), P_move=[float(v) for v in z[p + "P_move"]])
    else:
        kw.update(N_max=z[p + "q_model"].shape[0], P_move=[1., 0., 0.])
    return kw


def _check_run(g, z, p, chain=None):
    """g's records (or column `chain` of a batched run's) against golden z."""
    sel = (lambda a: a) if chain is None else (lambda a: a[:, chain])
    A = z[p + "A_chain"]
    np.testing.assert_array_equal(sel(g.A_chain).astype(np.int32), A, err_msg="A_chain")
    if p + "move_chain" in z.files and hasattr(g, "move_chain") and g.move_chain is not None:
        np.testing.assert_array_equal(sel(g.move_chain), z[p + "move_chain"], err_msg="moves")
        np.testing.assert_array_equal(sel(g.N_chain), z[p + "N_chain"], err_msg="N_chain")
    W = z[p + "q_chain"].shape[-1]
    qc = sel(g.q_chain)
    assert_state_close(qc[:, :W], z[p + "q_chain"][:, :qc.shape[1]], 1e-9, "q_chain")
    if getattr(g, "p_chain", None) is not None:
        pc = sel(g.p_chain)
        assert_state_close(pc[:, :W], z[p + "p_chain"][:, :pc.shape[1]], 1e-9, "p_chain")
    np.testing.assert_allclose(sel(g.E_chain), z[p + "E_chain"], rtol=1e-11)
    np.testing.assert_allclose(sel(g.V_chain), z[p + "V_chain"], rtol=1e-11)


@pytest.mark.parametrize("name", ["d51", "w64"])
def test_mh_bigk_run_RHMC(gpu_lib, name):
    z = load_golden("mh_bigk")
    p = name + "/"
    assert 0 < z[p + "A_chain"].mean() < 1
    g = _gym(z, p)
    np.random.seed(int(z[p + "seed"]))
    g.run_RHMC(z[p + "q_model"].copy(), **_kw(z, p))
    _check_run(g, z, p)


@pytest.mark.parametrize("fused", [True, False])
@pytest.mark.parametrize("name", ["d51", "w64"])
def test_mh_bigk_run_RHMC_batched(gpu_lib, monkeypatch, name, fused):
    """rhmc_mh (the whole MH loop on the device) fed the reference's draws."""
    from rhmc_amd import capi
    monkeypatch.setattr(capi, "DEFAULT_MH_FUSED", fused)
    z = load_golden("mh_bigk")
    p = name + "/"
    g = _gym(z, p)
    np.random.seed(int(z[p + "seed"]))
    kw = _kw(z, p)
    g.run_RHMC_batched(z[p + "q_model"].copy(), f_pos=True, Niter=kw["Niter"],
                       Nsteps=kw["Nsteps"], dt=kw["dt"])
    _check_run(g, z, p, chain=0)
    np.testing.assert_allclose(g.T_chain[:, 0], z[p + "T_chain"], rtol=1e-10, atol=1e-10)


@pytest.mark.parametrize("golden,name", [("mh_bigk", "d51"), ("mh_bigk", "w64"),
                                         ("rj_big", "b64"), ("flagship", "")])
def test_native_driver_chain0(gpu_lib, golden, name):
    """librhmc_rj.so with the reference's run as chain 0 of a batch of four
    (the others: the same start on other seeds)."""
    z = load_golden(golden)
    p = name + "/" if name else ""
    g = _gym(z, p)
    kw = _kw(z, p)
    if golden == "flagship":
        st = np.random.RandomState()
        st.set_state(("MT19937", z["rng_key"], int(z["rng_pos"]), int(z["rng_gauss"][0]),
                      float(z["rng_gauss"][1])))
        states = [st] + [np.random.RandomState(s) for s in (5, 6, 7)]
        g.run_RHMC_rj_batched([z["q_model"].copy() for _ in range(4)], None, n_pipes=1,
                              rng_states=states, **kw)
    else:
        seed = int(z[p + "seed"])
        g.run_RHMC_rj_batched([z[p + "q_model"].copy() for _ in range(4)],
                              [seed, seed + 1, seed + 2, seed + 3], n_pipes=1, **kw)
    assert not g.flag_chain[:, 0].any()
    _check_run(g, z, p, chain=0)


def test_rj_big_run_RHMC_births_past_64(gpu_lib):
    """run_RHMC from 64 stars with RHMC-big-sim4.py's move parameters grows
    past 64 stars exactly as the reference does (births and splits, then
    trajectories, V and T at K = 65 ... 68)."""
    z = load_golden("rj_big")
    p = "b64/"
    g = _gym(z, p)
    np.random.seed(int(z[p + "seed"]))
    g.run_RHMC(z[p + "q_model"].copy(), **_kw(z, p))
    _check_run(g, z, p)
    assert g.N_chain.max() > 64 and 0 < g.A_chain.mean() < 1


def test_flagship_run_RHMC(gpu_lib):
    """RHMC-big-sim4.py as written (rhmc_amd.big_sim4: the script's calls in
    its order — data, noise profile — then run_RHMC with its arguments,
    Niter 40) reproduces the reference's run: every move, star count and
    accept, states and energies."""
    from rhmc_amd import big_sim4
    z = load_golden("flagship")
    saved = np.random.get_state()
    try:
        g, q_true, q_model = big_sim4.setup()
        st = np.random.get_state()
        assert np.array_equal(st[1], z["rng_key"]) and st[2] == int(z["rng_pos"])
        g.run_RHMC(q_model, Niter=int(z["niter"]), q_true=q_true, **big_sim4.RUN_KW)
    finally:
        np.random.set_state(saved)
    _check_run(g, z, "")
    assert set(np.unique(g.move_chain[g.A_chain])) == {0, 1, 2, 3, 4}
