"""Run-to-run determinism of the windowed paths whose factor tables live in
global memory (rhmc_windowed.hpp WinGG, from 65 stars; rhmc_kernels.hip
work_tables).  The MH loop of run_RHMC (sampler_RHMC.py:697-760) over the
implicit leapfrog (:522-566) is a deterministic function of its start and seed,
so repeated launches -- on one stream, on two streams, after the table buffer
grew -- must give bit-identical chains and accept decisions.  A per-launch
stream-ordered pool allocation of these tables (hipMallocAsync/hipFreeAsync)
failed exactly this: S256K100's MH acceptance changed from run to run
(DESIGN.md section 4a).
"""
import numpy as np
import pytest
import torch

from rhmc_amd import workloads

pytestmark = pytest.mark.gpu


def _mh(capi, ctx, P, wl, q0, n, stream, n_iter=3, leap=8):
    dev = torch.device("cuda", 0)
    q = torch.from_numpy(np.ascontiguousarray(q0[:n])).to(dev)
    acc = torch.zeros((n_iter, n), dtype=torch.int32, device=dev)
    rec = capi.MhRecord(None, None, None, None, acc.data_ptr())
    ctx.mh_device(P, q.data_ptr(), n, wl.K, n_iter, leap, f_pos=False, seed=77, record=rec,
                  stream=stream.cuda_stream)
    torch.cuda.synchronize()
    return q.cpu().numpy(), acc.cpu().numpy()


def test_windowed_global_tables_deterministic(gpu_lib):
    capi = gpu_lib
    wl = workloads.make("S256K100", n_chains=2048)
    assert wl.K >= 65
    P = capi.make_params(**wl.params)
    dev = torch.device("cuda", 0)
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    ctx = capi.Context(wl.D)
    # small launch first, so the larger ones grow the stream's table buffer
    q_small, a_small = _mh(capi, ctx, P, wl, wl.q0, 256, s1)
    q_a, a_a = _mh(capi, ctx, P, wl, wl.q0, 2048, s1)
    q_b, a_b = _mh(capi, ctx, P, wl, wl.q0, 2048, s1)
    q_c, a_c = _mh(capi, ctx, P, wl, wl.q0, 2048, s2)
    ctx.close()
    ctx2 = capi.Context(wl.D)
    q_d, a_d = _mh(capi, ctx2, P, wl, wl.q0, 2048, s2)
    ctx2.close()
    assert 0.0 < a_a.mean() < 1.0
    for q, a in ((q_b, a_b), (q_c, a_c), (q_d, a_d)):
        assert np.array_equal(a, a_a)
        assert np.array_equal(q, q_a)
    # chains are independent: the first 256 match the 256-chain launch
    assert np.array_equal(a_small, a_a[:, :256])
    assert np.array_equal(q_small, q_a[:256])


def test_windowed_global_tables_two_streams_in_flight(gpu_lib):
    """Leapfrog launches queued on two streams at once (one context) read and
    write their own stream's tables: each result equals the serial one."""
    capi = gpu_lib
    wl = workloads.make("S256K100", n_chains=1024)
    P = capi.make_params(**wl.params)
    dev = torch.device("cuda", 0)
    ctx = capi.Context(wl.D)
    q0 = torch.from_numpy(wl.q0).to(dev)
    p0 = torch.from_numpy(wl.p0).to(dev)

    def run(streams):
        qs = [q0.clone() for _ in streams]
        ps = [p0.clone() for _ in streams]
        torch.cuda.synchronize()
        for _ in range(3):
            for s, q, p in zip(streams, qs, ps):
                ctx.leapfrog_device(P, q.data_ptr(), p.data_ptr(), wl.n_chains, wl.K, 4,
                                    stream=s.cuda_stream)
        torch.cuda.synchronize()
        return [(q.cpu().numpy(), p.cpu().numpy()) for q, p in zip(qs, ps)]

    (qs, ps), = run([torch.cuda.Stream(dev)])
    for q, p in run([torch.cuda.Stream(dev), torch.cuda.Stream(dev)]):
        assert np.array_equal(q, qs)
        assert np.array_equal(p, ps)
    ctx.close()


def test_windowed_global_tables_two_threads(gpu_lib):
    """rhmc_leapfrog_device from two host threads on distinct streams of one
    context (include/rhmc.h: allowed; the table buffers are per stream behind a
    mutex): each thread's chains equal a serial launch."""
    import threading
    capi = gpu_lib
    wl = workloads.make("S256K100", n_chains=1024)
    P = capi.make_params(**wl.params)
    dev = torch.device("cuda", 0)
    ctx = capi.Context(wl.D)
    q0 = torch.from_numpy(wl.q0).to(dev)
    p0 = torch.from_numpy(wl.p0).to(dev)
    serial = (q0.clone(), p0.clone())
    for _ in range(3):
        ctx.leapfrog_device(P, serial[0].data_ptr(), serial[1].data_ptr(), wl.n_chains, wl.K, 2)
    torch.cuda.synchronize()
    outs = [(q0.clone(), p0.clone()) for _ in range(2)]
    streams = [torch.cuda.Stream(dev) for _ in range(2)]
    torch.cuda.synchronize()
    errs = []

    def work(i):
        try:
            for _ in range(3):   # 2 + 2 + 2 steps
                ctx.leapfrog_device(P, outs[i][0].data_ptr(), outs[i][1].data_ptr(),
                                    wl.n_chains, wl.K, 2, stream=streams[i].cuda_stream)
        except Exception as e:  # noqa: BLE001 - reported below
            errs.append(e)

    th = [threading.Thread(target=work, args=(i,)) for i in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    torch.cuda.synchronize()
    assert not errs
    for q, p in outs:
        assert np.array_equal(q.cpu().numpy(), serial[0].cpu().numpy())
        assert np.array_equal(p.cpu().numpy(), serial[1].cpu().numpy())
    ctx.close()


def _all_paths(capi, mode, wl, n):
    """Leapfrog (status, iteration counts), energy V / T and the MH loop on the
    global-table path, on a fresh context in table mode `mode`."""
    import torch
    dev = torch.device("cuda", 0)
    P = capi.make_params(**wl.params)
    ctx = capi.Context(wl.D)
    ctx.set_option(capi.OPT_TABLES, mode)
    assert ctx.get_option(capi.OPT_TABLES) == mode
    q = torch.from_numpy(np.ascontiguousarray(wl.q0[:n])).to(dev)
    p = torch.from_numpy(np.ascontiguousarray(wl.p0[:n])).to(dev)
    it = torch.zeros((n, 2), dtype=torch.int32, device=dev)
    st = torch.zeros(n, dtype=torch.int32, device=dev)
    V = torch.zeros(n, dtype=torch.float64, device=dev)
    T = torch.zeros(n, dtype=torch.float64, device=dev)
    torch.cuda.synchronize()
    for _ in range(2):
        ctx.leapfrog_device(P, q.data_ptr(), p.data_ptr(), n, wl.K, 3, it.data_ptr(),
                            st.data_ptr())
    ctx.energy_device(P, q.data_ptr(), p.data_ptr(), V.data_ptr(), T.data_ptr(), n, wl.K)
    torch.cuda.synchronize()
    out = [x.cpu().numpy() for x in (q, p, it, st, V, T)]
    s = torch.cuda.Stream(dev)
    out += list(_mh(capi, ctx, P, wl, wl.q0, n, s, n_iter=3, leap=6))
    ctx.close()
    return out


def test_global_tables_poisoned_equal_unpoisoned(gpu_lib):
    """every table entry a launch reads, it wrote in that
    launch.  RHMC_TABLES_STREAM_POISON fills the buffer with 0xFF bytes (NaN
    doubles) before every launch: leapfrog (states, iteration counts, status),
    energy and MH must equal the default buffer bit for bit, with no chain
    non-finite.  The pool modes (round 5's per-launch stream-ordered
    allocation, which reproduces a defect outside the kernels) are refused by
    the product library."""
    capi = gpu_lib
    wl = workloads.make("S256K100", n_chains=512)
    base = _all_paths(capi, capi.TABLES_STREAM, wl, wl.n_chains)
    q, p, it, st, V, T, qm, acc = base
    assert not (st & capi.STATUS_NONFINITE).any()
    # (V is inf for a chain with a star off the image: the position support, :303-317)
    assert np.isfinite(V).mean() > 0.5 and np.isfinite(T).all() and np.isfinite(qm).all()
    assert 0.0 < acc.mean() < 1.0
    got = _all_paths(capi, capi.TABLES_STREAM_POISON, wl, wl.n_chains)
    for a, b, name in zip(got, base, ("q", "p", "iters", "status", "V", "T", "q_mh", "acc")):
        assert np.array_equal(a, b), name
    ctx = capi.Context(wl.D)
    for mode in (capi.TABLES_POOL, capi.TABLES_POOL_POISON, capi.TABLES_POOL_KEEP,
                 capi.TABLES_POOL_SYNCFREE, capi.TABLES_POOL_BARRIER):
        with pytest.raises(capi.RhmcError):
            ctx.set_option(capi.OPT_TABLES, mode)
    assert ctx.get_option(capi.OPT_TABLES) == capi.TABLES_STREAM
    ctx.close()


@pytest.mark.parametrize("Ks", [[65, 90, 70, 128, 88, 77, 66], [300, 257, 400]])
def test_global_tables_poisoned_ragged_and_hugek(gpu_lib, Ks):
    """The ragged launches (tables laid out by the launch's K_max, each chain
    reading its own K's entries) and the 8-slot kernels past 256 stars under
    the NaN fill equal the unfilled buffer bit for bit."""
    import torch
    capi = gpu_lib
    from helpers import capi_params
    from conftest import load_golden
    from oracle import rhmc_ref as R
    z = load_golden("traj_bigk256" if max(Ks) <= 128 else "traj_hugek")
    D, par = z["D"], R.params_from_npz(z)
    rs = np.random.RandomState(11)
    ld = 3 * max(Ks)
    n_pix = D.shape[0]
    m = R.RefModel(np.zeros((n_pix, n_pix)), par)
    q = np.zeros((len(Ks), ld))
    p = np.zeros((len(Ks), ld))
    for c, K in enumerate(Ks):
        row = np.stack([par["f_lim"] * np.exp(1 + 2 * rs.rand(K)), 1 + (n_pix - 2) * rs.rand(K),
                        1 + (n_pix - 2) * rs.rand(K)], 1).reshape(-1)
        q[c, :3 * K] = row
        p[c, :3 * K] = rs.randn(3 * K) * np.sqrt(m.H(row))
    dev = torch.device("cuda:0")
    res = []
    for mode in (capi.TABLES_STREAM, capi.TABLES_STREAM_POISON):
        ctx = capi.Context(D)
        ctx.set_option(capi.OPT_TABLES, mode)
        P = capi_params(capi, par)
        qd = torch.from_numpy(q.copy()).to(dev)
        pd = torch.from_numpy(p.copy()).to(dev)
        Kd = torch.tensor(Ks, dtype=torch.int32, device=dev)
        rows = torch.arange(len(Ks), dtype=torch.int64, device=dev)
        Vd = torch.zeros(len(Ks), dtype=torch.float64, device=dev)
        torch.cuda.synchronize()
        if max(Ks) <= 128:
            lo, hi = min(Ks), max(Ks)
            ctx.energy_ragged_device(P, qd.data_ptr(), ld, rows.data_ptr(), Kd.data_ptr(),
                                     len(Ks), lo, hi, capi.V_FLUX_WALL, Vd.data_ptr())
            ctx.leapfrog_ragged_device(P, qd.data_ptr(), pd.data_ptr(), ld, rows.data_ptr(),
                                       Kd.data_ptr(), len(Ks), lo, hi, 2)
            torch.cuda.synchronize()
            res.append((qd.cpu().numpy(), pd.cpu().numpy(), Vd.cpu().numpy()))
        else:   # fixed-K launches, one chain each (8 register slots)
            out = []
            for c, K in enumerate(Ks):
                V, T = ctx.energy(P, q[c, :3 * K][None], p[c, :3 * K][None], f_pos=True)
                g = ctx.gradient(P, q[c, :3 * K][None], kind=1)
                q1, p1, it, st = ctx.leapfrog(P, q[c, :3 * K][None], p[c, :3 * K][None], 1,
                                              return_info=True)
                assert not (st & capi.STATUS_NONFINITE).any()
                out.append((V, T, g, q1, p1, it))
            res.append(out)
        ctx.close()
    for r in res[1:]:
        if max(Ks) <= 128:
            for a, b in zip(r, res[0]):
                assert np.array_equal(a, b)
            assert np.isfinite(res[0][2]).all()
        else:
            for ca, cb in zip(r, res[0]):
                for a, b in zip(ca, cb):
                    assert np.array_equal(a, b)


def test_windowed_global_tables_grow_under_same_stream_threads(gpu_lib):
    """Two host threads on ONE stream, each alternating small and large
    launches (every large one may grow the stream's table buffer while the
    other thread's launch holds the old one): a launch keeps a lease on the
    buffer it was given until it is enqueued, and the old buffer is released
    only after a sync of the stream (include/rhmc.h threading contract), so
    each thread's chains equal a serial run."""
    import threading
    capi = gpu_lib
    wl = workloads.make("S256K100", n_chains=1024)
    P = capi.make_params(**wl.params)
    dev = torch.device("cuda", 0)
    q0 = torch.from_numpy(wl.q0).to(dev)
    p0 = torch.from_numpy(wl.p0).to(dev)
    sizes = (64, 1024, 128, 1024)

    def run(ctx, q, p, stream):
        for n in sizes:
            ctx.leapfrog_device(P, q.data_ptr(), p.data_ptr(), n, wl.K, 1,
                                stream=None if stream is None else stream.cuda_stream)
    ctx = capi.Context(wl.D)
    ref = (q0.clone(), p0.clone())
    torch.cuda.synchronize()
    run(ctx, ref[0], ref[1], None)
    torch.cuda.synchronize()
    ctx.close()
    for rep in range(2):
        ctx = capi.Context(wl.D)
        s = torch.cuda.Stream(dev)
        outs = [(q0.clone(), p0.clone()) for _ in range(2)]
        torch.cuda.synchronize()
        errs = []

        def work(i):
            try:
                run(ctx, outs[i][0], outs[i][1], s)
            except Exception as e:  # noqa: BLE001 - reported below
                errs.append(e)
        th = [threading.Thread(target=work, args=(i,)) for i in range(2)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        torch.cuda.synchronize()
        assert not errs
        for q, p in outs:
            assert torch.equal(q, ref[0]) and torch.equal(p, ref[1])
        ctx.close()
