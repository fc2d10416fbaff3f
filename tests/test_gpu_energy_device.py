"""rhmc_energy_device (device buffers, caller's stream) equals the host-buffer
rhmc_energy bit for bit — V and T, with and without p, one star and many
(register-window, pixel-major, dense and windowed energy kernels), the
flux-wall bit — and launches on two streams at once give the same values."""
import numpy as np
import pytest

from rhmc_amd import capi, workloads

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("wl_name,n", [("C2", 300), ("C3", 70), ("B4", 33), ("C5", 9)])
def test_energy_device_equals_host(gpu_lib, wl_name, n):
    import torch
    wl = workloads.make(wl_name, n_chains=n)
    ctx = capi.Context(wl.D, device=0)
    P = capi.make_params(**dict(wl.params, V_prior_const=0.25))
    rng = np.random.RandomState(3)
    p = rng.randn(*wl.q0.shape)
    for f_pos in (0, capi.V_FLUX_WALL):
        V, T = ctx.energy(P, wl.q0, p, f_pos=bool(f_pos))
        dev = torch.device("cuda:0")
        q_d = torch.from_numpy(wl.q0.copy()).to(dev)
        p_d = torch.from_numpy(p.copy()).to(dev)
        V_d = torch.empty(n, dtype=torch.float64, device=dev)
        T_d = torch.empty(n, dtype=torch.float64, device=dev)
        s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
        h = n // 2
        # two halves on two streams at once
        ctx.energy_device(P, q_d.data_ptr(), p_d.data_ptr(), V_d.data_ptr(), T_d.data_ptr(), h,
                          wl.K, f_pos, s1.cuda_stream)
        ctx.energy_device(P, q_d[h:].data_ptr(), p_d[h:].data_ptr(), V_d[h:].data_ptr(),
                          T_d[h:].data_ptr(), n - h, wl.K, f_pos, s2.cuda_stream)
        torch.cuda.synchronize()
        Vh, Th = V_d.cpu().numpy(), T_d.cpu().numpy()
        # V only (no p, no T)
        V2_d = torch.empty(n, dtype=torch.float64, device=dev)
        ctx.energy_device(P, q_d.data_ptr(), 0, V2_d.data_ptr(), 0, n, wl.K, f_pos, None)
        ctx.synchronize()
        if wl_name in ("C2", "C3"):     # kernels whose last bits follow the wave-mates
            np.testing.assert_allclose(Vh, V, rtol=1e-13)
            np.testing.assert_allclose(Th, T, rtol=1e-13)
        else:
            assert np.array_equal(Vh, V) and np.array_equal(Th, T)
        assert np.array_equal(V2_d.cpu().numpy(), V)
        if f_pos:
            assert np.isinf(V).any() or (wl.q0[:, 0::3] >= wl.params["f_lim"]).all()
    ctx.close()


def test_energy_device_errors(gpu_lib):
    wl = workloads.make("C2", n_chains=4)
    ctx = capi.Context(wl.D, device=0)
    P = capi.make_params(**wl.params)
    with pytest.raises(capi.RhmcError, match="q is NULL"):
        ctx.energy_device(P, 0, 0, 0, 0, 4, 1)
    with pytest.raises(capi.RhmcError, match="K must be"):
        ctx.energy_device(P, 1, 0, 0, 0, 4, 1025)
    ctx.close()
