"""Ragged chain sets (include/rhmc.h ABI 4) — the entry points the
device-resident reversible-jump driver runs on: chains of different star
counts in one launch, as rows of padded device arrays.

* rhmc_leapfrog_ragged_device / rhmc_energy_ragged_device equal fixed-K
  calls on the same chains bit for bit (the kernels are batch-invariant; a
  row list in any order, chains of 11..64 stars on the dense kernel of a
  32-px image, 65..90 on the windowed kernel of a 256-px image, 2..10 on the
  pixel-major kernel of a 32-px image, two chains of different K per wave);
* rhmc_ragged_ok names the star counts the slotted kernels serve;
* rhmc_rows_copy_device gathers / scatters rows;
* rhmc_kinetic_rows_device draws p = z sqrt(H(q)) bit for bit as the host
  (sampler_RHMC.py:1021-1022, the reference's metric, :260-292) and gives
  T(p, H(q)) (:353-363) to the last ulp of NumPy's;
* the argument checks (mixed register slots, a star count no slotted kernel
  serves)."""
import numpy as np
import pytest

from conftest import load_golden
from helpers import capi_params
from oracle import rhmc_ref as R

pytestmark = pytest.mark.gpu


def _set(par, Ks, n_pix, rs, ld):
    """Chains of the given star counts above the flux wall, zero-padded rows."""
    q = np.zeros((len(Ks), ld))
    p = np.zeros((len(Ks), ld))
    m = R.RefModel(np.zeros((n_pix, n_pix)), par)
    for c, K in enumerate(Ks):
        f = par["f_lim"] * np.exp(1 + 2 * rs.rand(K))
        x = 1 + (n_pix - 2) * rs.rand(K)
        y = 1 + (n_pix - 2) * rs.rand(K)
        row = np.stack([f, x, y], 1).reshape(-1)
        q[c, :3 * K] = row
        p[c, :3 * K] = rs.randn(3 * K) * np.sqrt(m.H(row))
    return q, p


@pytest.mark.parametrize("case", ["dense32", "win256", "pixk32"])
def test_ragged_equals_fixed_K(gpu_lib, case):
    import torch
    capi = gpu_lib
    if case == "dense32":
        z = load_golden("traj_bigk")
        D, par = z["D"], R.params_from_npz(z)
        Ks = [11, 30, 17, 64, 11, 45, 30, 23, 64, 12, 50, 11, 33]
    elif case == "pixk32":
        z = load_golden("traj_bigk")
        D, par = z["D"], R.params_from_npz(z)
        Ks = [2, 7, 10, 3, 3, 9, 5, 10, 2, 6, 8, 4, 7, 5, 9]
    else:
        z = load_golden("traj_bigk256")
        D, par = z["D"], R.params_from_npz(z)
        Ks = [65, 90, 70, 65, 88, 77, 66]
    rs = np.random.RandomState(4)
    ld = 3 * 128
    q, p = _set(par, Ks, D.shape[0], rs, ld)
    ctx = capi.Context(D)
    P = capi_params(capi, par)
    for K in set(Ks):
        assert ctx.ragged_ok(P, K)
    dev = torch.device("cuda:0")
    qd = torch.from_numpy(q.copy()).to(dev)
    pd = torch.from_numpy(p.copy()).to(dev)
    Kd = torch.tensor(Ks, dtype=torch.int32, device=dev)
    order = rs.permutation(len(Ks))[: len(Ks) - 2]      # a subset, in any order
    rows = torch.tensor(order, dtype=torch.int64, device=dev)
    lo, hi = min(Ks[i] for i in order), max(Ks[i] for i in order)
    Vd = torch.zeros(len(order), dtype=torch.float64, device=dev)
    ctx.energy_ragged_device(P, qd.data_ptr(), ld, rows.data_ptr(), Kd.data_ptr(), len(order),
                             lo, hi, capi.V_FLUX_WALL, Vd.data_ptr())
    ctx.leapfrog_ragged_device(P, qd.data_ptr(), pd.data_ptr(), ld, rows.data_ptr(),
                               Kd.data_ptr(), len(order), lo, hi, 6)
    torch.cuda.synchronize()
    qg, pg, Vg = qd.cpu().numpy(), pd.cpu().numpy(), Vd.cpu().numpy()
    for j, c in enumerate(order):
        K = Ks[c]
        V, _ = ctx.energy(P, q[c, :3 * K][None], None, f_pos=True)
        assert Vg[j] == V[0], (c, K)
        q1, p1 = ctx.leapfrog(P, q[c, :3 * K][None], p[c, :3 * K][None], 6)
        assert np.array_equal(qg[c, :3 * K], q1[0]) and np.array_equal(pg[c, :3 * K], p1[0]), c
        assert not qg[c, 3 * K:].any() and not pg[c, 3 * K:].any()
    skipped = sorted(set(range(len(Ks))) - set(order))
    assert np.array_equal(qg[skipped], q[skipped]) and np.array_equal(pg[skipped], p[skipped])
    ctx.close()


def test_ragged_ok_and_argument_checks(gpu_lib):
    import torch
    capi = gpu_lib
    z = load_golden("traj_bigk")
    par = R.params_from_npz(z)
    ctx = capi.Context(z["D"])                      # 32 px: dense from 11 stars
    P = capi_params(capi, par)
    assert [ctx.ragged_ok(P, K) for K in (1, 2, 10, 11, 64, 65, 256)] == \
        [False, True, True, True, True, True, True]   # 2-10: the pixel-major kernel
    dev = torch.device("cuda:0")
    q = torch.zeros((2, 3 * 70), dtype=torch.float64, device=dev)
    K = torch.tensor([60, 70], dtype=torch.int32, device=dev)
    with pytest.raises(capi.RhmcError) as e:          # 60 and 70 stars: one and two slots
        ctx.leapfrog_ragged_device(P, q.data_ptr(), q.data_ptr(), 210, 0, K.data_ptr(), 2, 60,
                                   70, 1)
    assert e.value.code == capi.RHMC_ERR_ARG
    with pytest.raises(capi.RhmcError) as e:          # 5 and 20 stars: two kernel families
        ctx.leapfrog_ragged_device(P, q.data_ptr(), q.data_ptr(), 210, 0, K.data_ptr(), 2, 5,
                                   20, 1)
    assert e.value.code == capi.RHMC_ERR_UNSUPPORTED
    with pytest.raises(capi.RhmcError) as e:          # 1 star: the one-star kernels
        ctx.leapfrog_ragged_device(P, q.data_ptr(), q.data_ptr(), 210, 0, K.data_ptr(), 2, 1,
                                   5, 1)
    assert e.value.code == capi.RHMC_ERR_UNSUPPORTED
    with pytest.raises(capi.RhmcError):               # ld too small for K_max
        ctx.leapfrog_ragged_device(P, q.data_ptr(), q.data_ptr(), 30, 0, K.data_ptr(), 2, 11,
                                   20, 1)
    ctx.close()
    big = load_golden("traj_bigk256")
    ctx = capi.Context(big["D"])                      # 256 px: windowed above 64 stars
    P = capi_params(capi, R.params_from_npz(big))
    assert [ctx.ragged_ok(P, K) for K in (1, 10, 64, 65, 200)] == [False] * 3 + [True] * 2
    ctx.close()


def test_rows_copy_and_kinetic(gpu_lib):
    import torch
    capi = gpu_lib
    z = load_golden("traj_bigk")
    par = R.params_from_npz(z)
    ctx = capi.Context(z["D"])
    P = capi_params(capi, par)
    rs = np.random.RandomState(8)
    Ks = [1, 3, 51, 120, 7, 64, 2]
    ld = 3 * 120
    q, _ = _set(par, Ks, 32, rs, ld)
    q[1, 0] = 0.5 * par["f_low"]                      # the H_xx clamp branch (:267-273)
    dev = torch.device("cuda:0")
    qd = torch.from_numpy(q).to(dev)
    # gather rows 5, 2, 0 (width 90) into a packed array, scatter them to rows 1, 3, 6
    src = torch.tensor([5, 2, 0], dtype=torch.int64, device=dev)
    dst = torch.tensor([1, 3, 6], dtype=torch.int64, device=dev)
    packed = torch.full((3, 90), -1.0, dtype=torch.float64, device=dev)
    ctx.rows_copy_device(qd.data_ptr(), ld, src.data_ptr(), packed.data_ptr(), 90, 0, 3, 90)
    out = torch.zeros((7, ld), dtype=torch.float64, device=dev)
    ctx.rows_copy_device(packed.data_ptr(), 90, 0, out.data_ptr(), ld, dst.data_ptr(), 3, 90)
    torch.cuda.synchronize()
    assert np.array_equal(packed.cpu().numpy(), q[[5, 2, 0], :90])
    o = out.cpu().numpy()
    assert np.array_equal(o[[1, 3, 6], :90], q[[5, 2, 0], :90]) and not o[[0, 2, 4, 5]].any()
    # momentum draw and kinetic energy
    zoff = np.concatenate([[0], np.cumsum([3 * K for K in Ks])[:-1]]).astype(np.int64)
    zz = rs.randn(sum(3 * K for K in Ks))
    pd = torch.full((7, ld), 7.0, dtype=torch.float64, device=dev)
    Td = torch.zeros(7, dtype=torch.float64, device=dev)
    Kd = torch.tensor(Ks, dtype=torch.int32, device=dev)
    zd, zoffd = torch.from_numpy(zz).to(dev), torch.from_numpy(zoff).to(dev)
    ctx.kinetic_rows_device(P, qd.data_ptr(), pd.data_ptr(), ld, Kd.data_ptr(), zd.data_ptr(),
                            zoffd.data_ptr(), 7, Td.data_ptr())
    T2 = torch.zeros(7, dtype=torch.float64, device=dev)
    ctx.kinetic_rows_device(P, qd.data_ptr(), pd.data_ptr(), ld, Kd.data_ptr(), 0, 0, 7,
                            T2.data_ptr())
    torch.cuda.synchronize()
    from rhmc_amd import sampler
    g = sampler.multi_gym(dt=par["dt"], g_xx=par["g_xx"], g_ff=par["g_ff"], g_ff2=par["g_ff2"])
    pg, Tg = pd.cpu().numpy(), Td.cpu().numpy()
    for c, K in enumerate(Ks):
        row = q[c, :3 * K]
        H = g._H_vec(row)
        pw = zz[zoff[c]:zoff[c] + 3 * K] * np.sqrt(H)
        assert np.array_equal(pg[c, :3 * K], pw), c        # the host's draw, bit for bit
        assert not pg[c, 3 * K:].any()
        np.testing.assert_allclose(Tg[c], g.T(pw, H), rtol=2e-15, atol=1e-15)
    assert np.array_equal(T2.cpu().numpy(), Tg)
    ctx.close()


def test_kinetic_rows_past_256_stars(gpu_lib):
    """Rows wider than 768 doubles take the one-chain-per-block kinetic kernel
    (up to 1024 stars, pairwise depth 5): p bit for bit as the host, T to
    NumPy's last ulp; a chain of more than 1024 stars gets T = NaN."""
    import torch
    capi = gpu_lib
    z = load_golden("traj_bigk")
    par = R.params_from_npz(z)
    ctx = capi.Context(z["D"])
    P = capi_params(capi, par)
    rs = np.random.RandomState(9)
    Ks = [300, 1024, 5, 777, 257]
    ld = 3 * 1024
    q = np.zeros((len(Ks), ld))
    for c, K in enumerate(Ks):
        q[c, 0:3 * K:3] = par["f_lim"] * np.exp(1 + 2 * rs.rand(K))
        q[c, 1:3 * K:3] = 1 + 30 * rs.rand(K)
        q[c, 2:3 * K:3] = 1 + 30 * rs.rand(K)
    dev = torch.device("cuda:0")
    qd = torch.from_numpy(q).to(dev)
    zoff = np.concatenate([[0], np.cumsum([3 * K for K in Ks])[:-1]]).astype(np.int64)
    zz = rs.randn(sum(3 * K for K in Ks))
    pd = torch.full((len(Ks), ld), 7.0, dtype=torch.float64, device=dev)
    Td = torch.zeros(len(Ks), dtype=torch.float64, device=dev)
    Kd = torch.tensor(Ks, dtype=torch.int32, device=dev)
    zd, zoffd = torch.from_numpy(zz).to(dev), torch.from_numpy(zoff).to(dev)
    ctx.kinetic_rows_device(P, qd.data_ptr(), pd.data_ptr(), ld, Kd.data_ptr(), zd.data_ptr(),
                            zoffd.data_ptr(), len(Ks), Td.data_ptr())
    torch.cuda.synchronize()
    from rhmc_amd import sampler
    g = sampler.multi_gym(dt=par["dt"], g_xx=par["g_xx"], g_ff=par["g_ff"], g_ff2=par["g_ff2"])
    pg, Tg = pd.cpu().numpy(), Td.cpu().numpy()
    for c, K in enumerate(Ks):
        H = g._H_vec(q[c, :3 * K])
        pw = zz[zoff[c]:zoff[c] + 3 * K] * np.sqrt(H)
        assert np.array_equal(pg[c, :3 * K], pw), c
        assert not pg[c, 3 * K:].any()
        np.testing.assert_allclose(Tg[c], g.T(pw, H), rtol=2e-15, atol=1e-15)
    Kbig = torch.tensor([1025], dtype=torch.int32, device=dev)
    qb = torch.zeros((1, 3 * 1025), dtype=torch.float64, device=dev)
    pb = torch.zeros_like(qb)
    Tb = torch.zeros(1, dtype=torch.float64, device=dev)
    ctx.kinetic_rows_device(P, qb.data_ptr(), pb.data_ptr(), 3 * 1025, Kbig.data_ptr(), 0, 0, 1,
                            Tb.data_ptr())
    torch.cuda.synchronize()
    assert np.isnan(Tb.cpu().numpy()[0])
    ctx.close()
