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
