"""Multi-process (gloo, world size 2 and 3, CPU) tests of the chain-sharding
host logic used by bench.py --gpus N and by multi-GPU callers."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import PKG_DIR, ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_total, out_path):
    import sys
    for p in (ROOT, PKG_DIR):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch.distributed as dist
    from rhmc_amd import shard, workloads
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        lo, hi = shard.shard_range(n_total, world, rank)
        wl = workloads.make("C2", n_chains=n_total)     # global set, then slice
        local = np.concatenate([wl.q0[lo:hi], wl.p0[lo:hi]], 1)
        t = shard.max_over_ranks(float(rank + 1))
        tsum = shard.sum_over_ranks(hi - lo)            # bench --mode rj: chain-steps summed
        got = shard.gather_chains(local, n_total)
        dist.barrier()
        if rank == 0:
            np.savez(out_path, gathered=got, tmax=t, tsum=tsum)
    finally:
        dist.destroy_process_group()


def test_shard_range_partitions():
    from rhmc_amd.shard import shard_range
    for n in (0, 1, 7, 4096, 1 << 20):
        for w in (1, 2, 3, 8):
            r = [shard_range(n, w, k) for k in range(w)]
            assert r[0][0] == 0 and r[-1][1] == n
            assert all(r[k][1] == r[k + 1][0] for k in range(w - 1))
            assert max(b - a for a, b in r) - min(b - a for a, b in r) <= 1
    with pytest.raises(ValueError):
        shard_range(10, 2, 2)


@pytest.mark.parametrize("world,n_total", [(2, 37), (3, 64)])
def test_gather_over_gloo(tmp_path, world, n_total):
    out = str(tmp_path / "g.npz")
    mp.spawn(_worker, args=(world, _free_port(), n_total, out), nprocs=world, join=True)
    z = np.load(out)
    from rhmc_amd import workloads
    wl = workloads.make("C2", n_chains=n_total)
    np.testing.assert_array_equal(z["gathered"], np.concatenate([wl.q0, wl.p0], 1))
    assert float(z["tmax"]) == float(world)
    assert float(z["tsum"]) == float(n_total)
