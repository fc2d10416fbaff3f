"""One rank of tests/test_gpu_shard.py (launched as a subprocess with RANK /
WORLD_SIZE / MASTER_* set): runs its contiguous shard of a C2 chain set
through rhmc_leapfrog_device on its GPU and gathers the states to rank 0
over gloo (rhmc_amd/shard.py) — the bench's multi-GPU data path."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "hmc-stellar-toy-model_amd")):
    sys.path.insert(0, p)


def main(n_total, steps, out_path, workload="C2"):
    import numpy as np
    import torch
    import torch.distributed as dist
    from rhmc_amd import capi, shard, workloads
    world, rank = int(os.environ["WORLD_SIZE"]), int(os.environ["RANK"])
    dist.init_process_group("gloo")
    gpu = int(os.environ.get("RHMC_TEST_DEVICE", rank))
    torch.cuda.set_device(gpu)
    wl = workloads.make(workload, n_chains=n_total)            # one global set
    lo, hi = shard.shard_range(n_total, world, rank)
    dev = torch.device("cuda", gpu)
    q = torch.from_numpy(wl.q0[lo:hi].copy()).to(dev)
    p = torch.from_numpy(wl.p0[lo:hi].copy()).to(dev)
    it = torch.zeros((hi - lo, 2), dtype=torch.int32, device=dev)
    st = torch.zeros(hi - lo, dtype=torch.int32, device=dev)
    ctx = capi.Context(wl.D, device=gpu)
    P = capi.make_params(**wl.params)
    stream = torch.cuda.Stream(dev)
    ctx.leapfrog_device(P, q.data_ptr(), p.data_ptr(), hi - lo, wl.K, steps, it.data_ptr(),
                        st.data_ptr(), stream.cuda_stream)
    torch.cuda.synchronize()
    local = np.concatenate([q.cpu().numpy(), p.cpu().numpy(),
                            it.cpu().numpy().astype(np.float64),
                            st.cpu().numpy().astype(np.float64)[:, None]], 1)
    got = shard.gather_chains(local, n_total)
    dist.barrier()
    if rank == 0:
        np.save(out_path, got)
    ctx.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main(int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], *sys.argv[4:])
