#!/usr/bin/env python3
"""Benchmark: chain-leapfrog-steps/s of the RHMC hot path on MI355X.

Workload (BASELINE.json configs[1]): 48x48 image, 1 star,
4096 chains per GPU, fp64.  One bench "step" = one launch of the fused
leapfrog kernel advancing every chain by `--leap` (default 500) implicit
generalized-leapfrog steps (sampler_RHMC.py:522-566); chain states stay
resident in HBM and carry over from launch to launch.

value = total chain-leapfrog-steps over all ranks / max-over-ranks wall time.

Extra objects on the JSON line:
  roofline      algorithmic HBM bytes per chain-step (SURVEY §8(d):
                2*N_pix*8 + 4*3K*8 = 36,960 B at C2) x chain-steps per launch
                / average launch time, HIP events on the launch stream;
                peak 8.0 TB/s.  `traffic` = measured HBM bytes per launch from
                profiles/*.json (rocprofv3 PMC), or null.
  cpu_baseline  the NumPy CPU port (oracle/rhmc_ref.py) on the host cores, one
                chain per process, bounded sample (rank 0, N=1 only).
  end_to_end    (leapfrog mode, N=1) the host-buffer C-ABI call rhmc_leapfrog
                on the same chains: H2D + fused launch + D2H, synchronous — the
                PCIe-inclusive rate a NumPy caller sees; never `value`.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--workload C2]
       (N>1: launched by torch.distributed.run, one rank per GPU)
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "hmc-stellar-toy-model_amd"))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
FP64_PEAK_TFLOPS = 78.6    # MI355X FP64 vector (spec)


def alg_bytes_per_step(npix, K):
    return 2 * npix * 8 + 4 * 3 * K * 8


def alg_flops_per_step(npix, K):
    return 2 * npix * (18 * K + 2)


def _cpu_worker(args):
    D, par, q0, p0, nsteps = args
    import numpy as np  # noqa: F401
    from oracle.rhmc_ref import RefModel
    m = RefModel(D, par)
    t = time.perf_counter()
    m.trajectory(q0, p0, nsteps, par["delta"], par["counter_max"], record=False)
    return time.perf_counter() - t


def cpu_baseline(wl, seconds_target=15.0):
    """Time the NumPy port, one chain per process (multiprocessing.Pool)."""
    import multiprocessing as mp
    os.environ["OMP_NUM_THREADS"] = "1"
    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:
        cores = os.cpu_count()
    cores = max(1, min(cores, 16))
    par = dict(wl.params)
    par["rows"] = par["cols"] = wl.D.shape[0]
    # calibrate one chain on this core
    t = _cpu_worker((wl.D, par, wl.q0[0], wl.p0[0], 20))
    per_step = t / 20
    nsteps = max(20, int(seconds_target / per_step / 2))
    jobs = [(wl.D, par, wl.q0[c % wl.n_chains], wl.p0[c % wl.n_chains], nsteps)
            for c in range(2 * cores)]
    ctx = mp.get_context("fork")
    t0 = time.perf_counter()
    with ctx.Pool(cores) as pool:
        pool.map(_cpu_worker, jobs)
    wall = time.perf_counter() - t0
    total = len(jobs) * nsteps
    try:
        model = [l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo")
                 if l.startswith("model name")][0]
    except Exception:
        model = "unknown"
    return {"value": total / wall, "unit": "chain-leapfrog-steps/s", "cores": cores,
            "kind": "port",
            "sample": "%d chains x %d steps of %s geometry, NumPy port of RHMC_single_step "
                      "(oracle/rhmc_ref.py), one chain per process, %s"
                      % (len(jobs), nsteps, wl.name, model)}


def load_pmc(workload):
    """rocprofv3 PMC summary of the dominant kernel (profiles/pmc_<wl>.json,
    written by scripts/pmc_summary.py): HBM bytes per launch and executed
    fp64 flops per chain-step."""
    path = os.path.join(ROOT, "profiles", "pmc_%s.json" % workload.lower())
    try:
        with open(path) as fh:
            return json.load(fh)
    except (OSError, ValueError):
        return {}


def bench_datagen(args, wl, P, ctx, dev, stream, world, rank):
    """--mode datagen: n_real Poisson realisations of the workload's true model
    image per launch (gen_noise_profile's inner loop, sampler_RHMC.py:130-133).
    Algorithmic bytes per pixel: the 8-byte write (the model is recomputed
    from the K stars in registers)."""
    import numpy as np
    import torch
    import torch.distributed as dist
    from rhmc_amd import shard
    rows, cols = wl.D.shape
    stars = np.ascontiguousarray(wl.q0[0].reshape(-1, 3))
    n_real = args.n_real
    dq = torch.from_numpy(stars).to(dev)
    out = torch.empty((n_real, rows, cols), dtype=torch.float64, device=dev)

    def launch(i):
        ctx.gen_image_device(P, dq.data_ptr(), wl.K, rows, cols, n_real, 77 + i + 1000 * rank,
                             out.data_ptr(), stream=stream.cuda_stream)
    for i in range(args.warmup):
        launch(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps)]
    t0 = time.perf_counter()
    for i, (a, b) in enumerate(ev):
        a.record(stream)
        launch(args.warmup + i)
        b.record(stream)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
        wall = shard.max_over_ranks(wall)
    launch_ms = sum(a.elapsed_time(b) for a, b in ev) / len(ev)
    draws = n_real * rows * cols
    achieved = 8.0 * draws / (launch_ms * 1e-3) / 1e9
    res = {
        "metric": "Poisson pixel draws/sec (device gen_mock_data / gen_noise_profile)",
        "value": draws * world * args.steps / wall, "unit": "pixel-draws/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": wall / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f64", "data": "synthetic (%s true stars)" % wl.name,
        "config": {"workload": "%s model image %dx%d, K=%d, %d realisations per launch"
                               % (wl.name, rows, cols, wl.K, n_real), "mode": "datagen"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                     "alg_bytes_per_pixel": 8, "kernel_ms": launch_ms},
        "cpu_baseline": None,
    }
    if rank == 0:
        print(json.dumps(res), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="C2")
    ap.add_argument("--chains", type=int, default=None, help="chains per GPU (weak scaling)")
    ap.add_argument("--global-chains", type=int, default=None,
                    help="total chains split over the ranks (strong scaling, e.g. C4 = 2^20)")
    ap.add_argument("--leap", type=int, default=None, help="leapfrog steps per launch")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-e2e", action="store_true",
                    help="skip the host-buffer (rhmc_leapfrog, PCIe-inclusive) measurement")
    ap.add_argument("--mode", choices=("leapfrog", "mh", "integrate", "hmc_random", "datagen"),
                    default="leapfrog",
                    help="mh: whole MH iterations on device (momentum draw, V+T, accept; "
                         "Philox RNG); one bench step = --mh-iter iterations of --leap steps. "
                         "integrate: --solver's explicit integrator (rhmc_integrate). "
                         "hmc_random: samplers.HMC_random trajectories of --leap steps "
                         "(rhmc_hmc_random). "
                         "datagen: --n-real Poisson realisations of the workload's model "
                         "image (rhmc_gen_image)")
    ap.add_argument("--mh-iter", type=int, default=10)
    ap.add_argument("--solver", choices=("hmc", "naive", "leap_frog"), default="leap_frog")
    ap.add_argument("--n-real", type=int, default=1000)
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))

    from rhmc_amd import shard, workloads
    if args.workload.upper() == "C4" and not args.chains and not args.global_chains:
        # C4 is one 2^20-chain set sharded over the ranks (BASELINE configs[3])
        args.global_chains = 1 << 20
    if args.global_chains:
        # one global chain set (seed 1000), this rank's contiguous shard
        wl = workloads.make(args.workload, n_chains=args.global_chains)
        lo, hi = shard.shard_range(args.global_chains, world, rank)
        wl.q0, wl.p0 = wl.q0[lo:hi].copy(), wl.p0[lo:hi].copy()
    else:
        wl = workloads.make(args.workload, n_chains=args.chains, seed_offset=rank)
    # CPU baseline first: forked workers must not inherit an initialised GPU.
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu and args.mode == "leapfrog":
        cpu = cpu_baseline(wl)

    import torch
    import torch.distributed as dist
    from rhmc_amd import capi

    if world > 1:
        dist.init_process_group("gloo")
    # RHMC_BENCH_DEVICE pins every rank to one device (rehearsing the N-rank
    # path on a one-GPU box); by default rank r of a node uses GPU r.
    gpu = int(os.environ.get("RHMC_BENCH_DEVICE", local_rank))
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)

    leap = args.leap or wl.n_steps
    P = capi.make_params(**wl.params)
    ctx = capi.Context(wl.D, device=gpu)
    q = torch.from_numpy(wl.q0).to(dev).contiguous()
    p = torch.from_numpy(wl.p0).to(dev).contiguous()
    it = torch.zeros((wl.n_chains, 2), dtype=torch.int32, device=dev)
    st = torch.zeros(wl.n_chains, dtype=torch.int32, device=dev)
    # A dedicated (non-null) torch stream: the kernel is launched on it and the
    # timing events are recorded on it.
    stream = torch.cuda.Stream(dev)

    if args.mode == "datagen":
        return bench_datagen(args, wl, P, ctx, dev, stream, world, rank)
    if args.mode == "mh":
        leap = args.leap or 10

        def launch():
            ctx.mh_device(P, q.data_ptr(), wl.n_chains, wl.K, args.mh_iter, leap, f_pos=True,
                          seed=1234 + rank, stream=stream.cuda_stream)
    elif args.mode == "integrate":
        solver = {"hmc": capi.SOLVER_HMC, "naive": capi.SOLVER_RHMC_NAIVE,
                  "leap_frog": capi.SOLVER_RHMC_LEAPFROG}[args.solver]

        def launch():
            ctx.integrate_device(P, solver, q.data_ptr(), p.data_ptr(), wl.n_chains, wl.K, leap,
                                 f_pos=True, status_ptr=st.data_ptr(), stream=stream.cuda_stream)
    elif args.mode == "hmc_random":
        # samplers.HMC_random trajectories: unit mass, per-coordinate step
        # (flux 2.0, positions 0.02), every chain `leap` steps
        dtv = torch.tensor([2.0, 0.02, 0.02] * wl.K, dtype=torch.float64, device=dev)
        nst = torch.full((wl.n_chains,), leap, dtype=torch.int32, device=dev)
        p.normal_(generator=torch.Generator(device=dev).manual_seed(7 + rank))

        def launch():
            ctx.hmc_random_device(P, dtv.data_ptr(), q.data_ptr(), p.data_ptr(), nst.data_ptr(),
                                  wl.n_chains, wl.K, status_ptr=st.data_ptr(),
                                  stream=stream.cuda_stream)
    else:
        def launch():
            ctx.leapfrog_device(P, q.data_ptr(), p.data_ptr(), wl.n_chains, wl.K, leap,
                                it.data_ptr(), st.data_ptr(), stream.cuda_stream)

    for _ in range(args.warmup):
        launch()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()

    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps)]
    t0 = time.perf_counter()
    for a, b in ev:
        a.record(stream)
        launch()
        b.record(stream)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
        wall = shard.max_over_ranks(wall)
    launch_ms = sum(a.elapsed_time(b) for a, b in ev) / len(ev)

    stat = st.cpu().numpy()
    nonfinite = int(((stat & capi.STATUS_NONFINITE) != 0).sum())
    iters = it.cpu().numpy()            # last launch: sums over its `leap` steps
    fp_stats = {"p_loop_mean": float(iters[:, 0].mean() / max(leap, 1)),
                "q_loop_mean": float(iters[:, 1].mean() / max(leap, 1)),
                "p_loop_cap_chains": int(((stat & capi.STATUS_PLOOP_CAP) != 0).sum()),
                "q_loop_cap_chains": int(((stat & capi.STATUS_QLOOP_CAP) != 0).sum()),
                "flux_wall_chains": int(((stat & capi.STATUS_REFLECT_F) != 0).sum())}

    steps_per_launch = leap * (args.mh_iter if args.mode == "mh" else 1)
    chain_steps = wl.n_chains * steps_per_launch
    total_chains = args.global_chains or wl.n_chains * world
    value = total_chains * steps_per_launch * args.steps / wall
    npix = wl.D.size
    bpu = alg_bytes_per_step(npix, wl.K)
    achieved = bpu * chain_steps / (launch_ms * 1e-3) / 1e9
    # PMC summaries describe the implicit leapfrog kernel only
    pmc = load_pmc(wl.name) if args.mode == "leapfrog" else {}
    traffic = pmc.get("hbm_bytes_per_launch")
    if traffic is not None and pmc.get("chain_steps_per_dispatch") not in (None, chain_steps):
        traffic = traffic * chain_steps / pmc["chain_steps_per_dispatch"]
    metric = "chain-leapfrog-steps/sec, 48x48 1-star 4096 chains, 1/2/4/8 MI355X"
    if wl.name != "C2" or args.chains or args.global_chains or args.mode != "leapfrog":
        # not the headline configuration: name what was run
        metric = "chain-leapfrog-steps/sec, %s %dx%d %d-star %d chains/GPU (%s)" % (
            wl.name, wl.D.shape[0], wl.D.shape[1], wl.K, wl.n_chains, args.mode)
    out = {
        "metric": metric,
        "value": value,
        "unit": "chain-leapfrog-steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": wall / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong" if args.global_chains else "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (numpy RandomState: image seed 77, chains seed 1000+rank)",
        "config": {"workload": "%s: %dx%d image, K=%d, %d chains/GPU, %d leapfrog steps per "
                               "launch" % (wl.name, wl.D.shape[0], wl.D.shape[1], wl.K,
                                           wl.n_chains, leap),
                   "chains_per_gpu": wl.n_chains, "total_chains": total_chains,
                   "image": list(wl.D.shape), "K": wl.K,
                   "leapfrog_steps_per_launch": steps_per_launch, "mode": args.mode,
                   "solver": (args.solver if args.mode == "integrate" else
                              "hmc_random" if args.mode == "hmc_random" else "implicit"),
                   "parallelism": "chain-sharded x%d" % world},
        # The contract's roofline object prices the reference's ALGORITHMIC
        # bytes (D read by both gradients + q/p in/out).  The
        # kernels keep D in LDS and the window pixels in VGPRs, so that model
        # is not a bound here (frac > 1 by construction, binding=False); the
        # measured HBM rate is traffic / kernel time (`measured_gbs`) and the
        # roof that binds is `roofline_fp64_valu` below.
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "binding": False,
                     "binding_roof": "roofline_fp64_valu",
                     "note": "achieved = algorithmic-model bytes (2*N_pix*8 + 4*3K*8 per "
                             "chain-step) / kernel time; the image is LDS/VGPR-resident, so "
                             "this model exceeds physical HBM traffic and does not bind",
                     "measured_gbs": (None if traffic is None
                                      else traffic / (launch_ms * 1e-3) / 1e9),
                     "alg_bytes_per_chain_step": bpu, "kernel_ms": launch_ms,
                     "alg_model_fp64_tflops": alg_flops_per_step(npix, wl.K) * chain_steps
                     / (launch_ms * 1e-3) / 1e12},
        "nonfinite_chains": nonfinite,
        "fixed_point_iters_per_step": fp_stats,
    }
    # The image is LDS-resident, so the algorithmic-HBM fraction above exceeds
    # 1; the physically binding roof is FP64 VALU issue: executed fp64 flops per
    # chain-step (PMC, profiles/pmc_<wl>.json) x rate / 78.6 TF/s.
    fpc = pmc.get("fp64_flops_per_chain_step")
    out["roofline_fp64_valu"] = None if fpc is None else {
        "bound": "valu-fp64", "unit": "TFLOP/s", "peak": FP64_PEAK_TFLOPS,
        "achieved": fpc * chain_steps / (launch_ms * 1e-3) / 1e12,
        "frac": fpc * chain_steps / (launch_ms * 1e-3) / 1e12 / FP64_PEAK_TFLOPS,
        "executed_fp64_flops_per_chain_step": fpc,
        "valu_active_frac": pmc.get("valu_active_frac"),
        "valu_insts_per_chain_step": pmc.get("valu_insts_per_chain_step"),
    }
    if args.mode == "leapfrog" and not args.no_e2e and world == 1:
        out["end_to_end"] = end_to_end(ctx, P, q, p, wl, leap)
    if rank == 0:
        out["cpu_baseline"] = cpu
        print(json.dumps(out), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


def end_to_end(ctx, P, q, p, wl, leap, reps=3):
    """The host-buffer boundary (rhmc_leapfrog): caller-owned
    host q/p in, H2D + the fused launch + D2H, synchronous — what the drop-in
    RHMC_single_step replacement costs a NumPy caller.  Reported beside
    `value` (never as it); after the timed region, from the current states."""
    qh, ph = q.cpu().numpy(), p.cpu().numpy()
    ctx.leapfrog(P, qh, ph, leap, K=wl.K)           # warm (allocations, copies)
    t0 = time.perf_counter()
    for _ in range(reps):
        qh, ph = ctx.leapfrog(P, qh, ph, leap, K=wl.K)
    wall = (time.perf_counter() - t0) / reps
    return {"value": wl.n_chains * leap / wall, "unit": "chain-leapfrog-steps/s",
            "ms_per_call": wall * 1e3, "calls": reps,
            "what": "rhmc_leapfrog on host arrays: H2D q/p, %d fused steps, D2H, sync "
                    "(includes the numpy copies of the Python shim)" % leap}


if __name__ == "__main__":
    main()
