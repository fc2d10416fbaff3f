"""Multi-rank GPU test of the sharded kernel path: two rank
processes, both pinned to device 0 (a one-GPU box), each run their
shard_range slice of one 1,000-chain C2 set for 100 steps through
rhmc_leapfrog_device, and rank 0 gathers the states over gloo.  The gathered
q, p, fixed-point counts and status must be BIT-identical to one launch of
all 1,000 chains: chains are independent (sampler_RHMC.py:522-566 reads only
its own q, p plus the shared image) and the kernels are batch-invariant."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _sharded(tmp_path, world, n_total, steps, workload):
    out = str(tmp_path / "gathered.npy")
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RHMC_TEST_DEVICE="0")
        procs.append(subprocess.Popen(
            [sys.executable, os.path.join(ROOT, "tests", "shard_worker.py"), str(n_total),
             str(steps), out, workload], env=env, stdout=subprocess.PIPE,
            stderr=subprocess.STDOUT, text=True))
    logs = []
    for pr in procs:
        try:
            logs.append(pr.communicate(timeout=100)[0])
        except subprocess.TimeoutExpired:
            for k in procs:
                k.kill()
            raise
    assert all(pr.returncode == 0 for pr in procs), "\n".join(l[-2000:] for l in logs)
    return np.load(out)


@pytest.mark.parametrize("world,n_total,steps,workload",
                         [(2, 1000, 100, "C2"), (3, 601, 20, "C3")])
def test_sharded_ranks_bit_identical_to_one_launch(gpu_lib, tmp_path, world, n_total, steps,
                                                   workload):
    capi = gpu_lib
    from rhmc_amd import workloads
    got = _sharded(tmp_path, world, n_total, steps, workload)
    wl = workloads.make(workload, n_chains=n_total)
    ctx = capi.Context(wl.D)
    P = capi.make_params(**wl.params)
    q, p, it, st = ctx.leapfrog(P, wl.q0, wl.p0, steps, return_info=True)
    ctx.close()
    d = q.shape[1]
    np.testing.assert_array_equal(got[:, :d], q)
    np.testing.assert_array_equal(got[:, d:2 * d], p)
    np.testing.assert_array_equal(got[:, 2 * d:2 * d + 2].astype(np.int32), it)
    np.testing.assert_array_equal(got[:, 2 * d + 2].astype(np.int32), st)
    assert not (st & capi.STATUS_NONFINITE).any()
