#!/usr/bin/env python3
"""Benchmark: chain-leapfrog-steps/s of the RHMC hot path on MI355X.

Workload (BASELINE.json configs[1]): 48x48 image, 1 star,
4096 chains per GPU, fp64.  One bench "step" = one launch of the fused
leapfrog kernel advancing every chain by `--leap` (default 500) implicit
generalized-leapfrog steps (sampler_RHMC.py:522-566); chain states stay
resident in HBM and carry over from launch to launch.

value = total chain-leapfrog-steps over all ranks / max-over-ranks wall time.

Extra objects on the JSON line:
  roofline      the binding roof, fp64 VALU: executed fp64 FLOP per chain-step
                (rocprofv3 PMC, profiles/pmc_<wl>.json) x chain-steps per
                launch / the launch's HIP-event time on the launch stream,
                over the 78.6 TF/s fp64 vector peak; `traffic` = measured HBM
                bytes per launch (PMC), `hbm_measured_frac` its rate over
                8 TB/s; `alg_model` = SURVEY §8(d)'s algorithmic-bytes model
                (above the HBM peak by construction: D lives in LDS/VGPRs).
  cpu_baseline  the NumPy CPU port (oracle/rhmc_ref.py) on all the host CPU the
                job may use (affinity mask, capped by the cgroup CPU quota),
                one chain per worker process, ~10 s per worker (rank 0, N=1).
  end_to_end    (leapfrog mode, N=1) the host-buffer C-ABI call rhmc_leapfrog
                on the same chains: H2D + fused launch + D2H, synchronous — the
                PCIe-inclusive rate a NumPy caller sees; never `value`.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--workload C2]
  N > 1 without WORLD_SIZE in the environment: this process starts N rank
  processes of itself (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, rank r on
  GPU r) before touching a GPU, relays rank 0's JSON line and fails if any
  rank fails.  Under torch.distributed.run (WORLD_SIZE set) each process is
  one rank; --gpus must then equal WORLD_SIZE.
  --dry-run: rendezvous the ranks and print the sharding plan without
  touching a GPU (the CPU tests use it).
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import tempfile
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


def cpu_quota_cores():
    """CPUs the cgroup lets this process use (cpu.max quota / period), or None."""
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            quota, period = open(path).read().split()[:2]
            if quota != "max":
                return float(quota) / float(period)
        except (OSError, ValueError):
            pass
    try:
        quota = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        period = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        if quota > 0:
            return quota / period
    except (OSError, ValueError):
        pass
    return None


def cpu_baseline(wl, seconds_per_worker=10.0):
    """Time the NumPy port on all the host CPU this process may use: one chain
    per worker process (multiprocessing.Pool, OMP_NUM_THREADS=1), each worker
    running ~10 s.  Workers = the CPUs of the affinity mask, or the cgroup's
    CPU quota when that is smaller: the GPU box shows 256 CPUs in the mask but
    grants 16 CPUs of time, and 256 time-sliced workers measured 4.1e4
    chain-steps/s against 9.3e4 for 16 — the quota-sized pool
    is the whole host available to the job."""
    import multiprocessing as mp
    os.environ["OMP_NUM_THREADS"] = "1"
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count()
    quota = cpu_quota_cores()
    workers = max(1, min(avail, int(round(quota)) if quota else avail))
    par = dict(wl.params)
    par["rows"] = par["cols"] = wl.D.shape[0]
    # calibrate one chain on one idle core
    t = _cpu_worker((wl.D, par, wl.q0[0], wl.p0[0], 20))
    per_step = t / 20
    nsteps = max(20, int(seconds_per_worker / per_step))
    jobs = [(wl.D, par, wl.q0[c % wl.n_chains], wl.p0[c % wl.n_chains], nsteps)
            for c in range(workers)]
    ctx = mp.get_context("fork")
    t0 = time.perf_counter()
    with ctx.Pool(workers) as pool:
        worker_s = pool.map(_cpu_worker, jobs)
    wall = time.perf_counter() - t0
    total = len(jobs) * nsteps
    try:
        model = [l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo")
                 if l.startswith("model name")][0]
    except Exception:
        model = "unknown"
    return {"value": total / wall, "unit": "chain-leapfrog-steps/s", "cores": workers,
            "cores_available": avail, "cores_used": workers, "cpu_quota_cores": quota,
            "kind": "port", "worker_seconds_min": min(worker_s),
            "one_core_value": 1.0 / per_step,
            "sample": "%d chains x %d steps of %s geometry, NumPy port of RHMC_single_step "
                      "(oracle/rhmc_ref.py), one chain per worker process, %d workers = "
                      "min(affinity CPUs %d, cgroup CPU quota %s), %s"
                      % (len(jobs), nsteps, wl.name, workers, avail,
                         "none" if quota is None else "%g" % quota, model)}


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _stop(procs, live, grace=10.0):
    """SIGTERM the live ranks, then SIGKILL whatever is left after `grace` s."""
    for k in live:
        procs[k].terminate()
    end = time.monotonic() + grace
    for k in live:
        try:
            procs[k].wait(timeout=max(0.1, end - time.monotonic()))
        except subprocess.TimeoutExpired:
            procs[k].kill()
            procs[k].wait()


def spawn_ranks(n, timeout):
    """Start n rank processes of this script (one per GPU) and wait for them.

    Called before anything touches a GPU (no torch import here).  Each child
    gets RANK = LOCAL_RANK = r, WORLD_SIZE = n and a 127.0.0.1 rendezvous;
    rank 0's stdout (the JSON line) is relayed, the other ranks' stdout goes
    to stderr.  If a rank fails, the others are stopped and the exit code is
    non-zero; if the ranks are not all done `timeout` seconds after the start
    (a rank stuck in the rendezvous, a barrier or a GPU call), every rank is
    stopped (SIGTERM, SIGKILL 10 s later) and the exit code is 124."""
    port = _free_port()
    procs, outs = [], []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        out = tempfile.TemporaryFile(mode="w+")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=env, stdout=out))
        outs.append(out)
    rc = 0
    live = set(range(n))
    deadline = time.monotonic() + timeout
    while live:
        for r in sorted(live):
            code = procs[r].poll()
            if code is None:
                continue
            live.discard(r)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 1
                sys.stderr.write("bench.py: rank %d exited with %d; stopping the others\n"
                                 % (r, code))
                _stop(procs, live)
                live.clear()
        if live and time.monotonic() > deadline:
            sys.stderr.write("bench.py: ranks %s still running after --timeout %g s; "
                             "stopping every rank\n" % (sorted(live), timeout))
            _stop(procs, live)
            live.clear()
            rc = 124
        time.sleep(0.05)
    for r, out in enumerate(outs):
        out.seek(0)
        text = out.read()
        (sys.stdout if r == 0 else sys.stderr).write(text)
        out.close()
    sys.stdout.flush()
    return rc


# Sources whose bytes decide the kernels' machine code: the PMC summaries
# record their hash, and a summary taken on other sources is not used.
SOURCE_GLOBS = ("hmc-stellar-toy-model_amd/csrc/*", "hmc-stellar-toy-model_amd/Makefile",
                "include/rhmc.h")


def source_hash(root=ROOT):
    """sha256 (16 hex digits) over the kernel sources, path + bytes, in path order."""
    import glob
    import hashlib
    h = hashlib.sha256()
    files = sorted({f for g in SOURCE_GLOBS for f in glob.glob(os.path.join(root, g))
                    if os.path.isfile(f)})
    for f in files:
        h.update(os.path.relpath(f, root).replace(os.sep, "/").encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
        h.update(b"\0")
    return h.hexdigest()[:16]


def load_pmc(workload, n_chains=None, root=ROOT):
    """rocprofv3 PMC summary of the dominant kernel (profiles/pmc_<wl>.json,
    written by scripts/pmc_summary.py): HBM bytes per launch and executed
    fp64 flops per chain-step.  A launch size with its own summary
    (profiles/pmc_<wl>_<n_chains>.json: C5's 1024-chain share of 8 GPUs, whose
    window split runs other code per chain-step) takes that one.  Returns
    (summary, stale): a summary whose `src_hash` is missing or differs from
    the shipped sources' is stale — its counters describe other machine code,
    so roofline() reports no fraction."""
    path = os.path.join(root, "profiles", "pmc_%s.json" % workload.lower())
    if n_chains is not None:
        sized = os.path.join(root, "profiles", "pmc_%s_%d.json" % (workload.lower(), n_chains))
        if os.path.exists(sized):
            path = sized
    try:
        with open(path) as fh:
            pmc = json.load(fh)
    except (OSError, ValueError):
        return {}, False
    return pmc, pmc.get("src_hash") != source_hash(root)


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


def bench_rj(args, wl, gpu, world, rank):
    """--mode rj: the reversible-jump sampler (multi_gym.run_RHMC with P_move
    = [0.6, 0.2, 0.2], sampler_RHMC.py:937-1198) through the native driver
    librhmc_rj.so on this rank's chains, each on its own seeded NumPy-stream
    replica; one bench step = one run of --mh-iter iterations of --leap steps
    per trajectory.  A move-0 iteration counts --leap chain-leapfrog-steps, a
    jump 2 x --leap (its two trajectories).  Host work and GPU phases
    interleave, so there is no single dominant kernel: roofline null."""
    import numpy as np
    import torch.distributed as dist
    from rhmc_amd import sampler, shard
    from rhmc_amd.photometry import mag2flux
    n_it = args.mh_iter
    if wl is None:
        # BIGSIM4: the reference's flagship run as written (RHMC-big-sim4.py:
        # 51 true stars on 32x32, every chain from its 5 model stars, K grows by
        # births / splits, N_max 120, Nsteps 10, dt 0.05, beta_a = beta_b = 4)
        from rhmc_amd import big_sim4
        saved = np.random.get_state()
        g, _, q_model = big_sim4.setup()
        np.random.set_state(saved)
        n_chains = args.chains or 4096
        starts = [q_model.copy() for _ in range(n_chains)]
        leap = args.leap or big_sim4.RUN_KW["Nsteps"]
        kw = dict(Niter=n_it - 1, Nsteps=leap, dt=big_sim4.RUN_KW["dt"],
                  N_max=big_sim4.RUN_KW["N_max"], P_move=big_sim4.RUN_KW["P_move"])
        name, K0, D = "BIGSIM4", big_sim4.N_MODEL, g.D
    else:
        g = sampler.multi_gym(dt=0.05, g_xx=float(wl.params["g_xx"]),
                              g_ff=float(wl.params["g_ff"]), g_ff2=float(wl.params["g_ff2"]))
        g.num_rows, g.num_cols = wl.D.shape
        g.use_prior, g.alpha = True, 2.
        # the workload's own magnitude range (workloads.make) and, on the
        # big-sim geometries, the reference drivers' move parameters
        # (RHMC-big-sim4.py:39-44: K_split 1, beta_a = beta_b = 4)
        g.fmin = mag2flux({"B4": 20., "B3": 20.5}.get(wl.name, 23.3)) * g.flux_to_count
        g.fmax = mag2flux(15.) * g.flux_to_count
        if wl.name in ("B4", "B3"):
            g.K_split, g.beta_a, g.beta_b = 1., 4., 4.
        g.D = wl.D
        n_chains = wl.n_chains
        starts = []
        for c in range(n_chains):
            m = wl.q0[c].reshape(-1, 3).copy()
            m[:, 0] = np.minimum(g.flux2mag_converter(m[:, 0]), 22.5)   # above the flux wall
            starts.append(m)
        leap = args.leap or 20
        kw = dict(Niter=n_it - 1, Nsteps=leap, dt=0.05, N_max=min(256, 2 * wl.K + 20),
                  P_move=[0.6, 0.2, 0.2])
        name, K0, D = wl.name, wl.K, wl.D
    g.device = gpu
    # every chain starts with K0 stars: one [n, K0, 3] array (run_RHMC_rj_batched
    # packs it in one native pass)
    starts = np.stack(starts)
    seeds = 1000 * rank + np.arange(n_chains, dtype=np.int64)
    # successive runs write their q_chain / p_chain records into the previous
    # run's arrays (opt-in: no page faults on fresh memory inside the timing)
    kw["reuse_records"] = True
    for _ in range(args.warmup):
        g.run_RHMC_rj_batched(starts, seeds, n_pipes=args.rj_pipes, **kw)
    if world > 1:
        dist.barrier()
    steps = 0
    t0 = time.perf_counter()
    for i in range(args.steps):
        g.run_RHMC_rj_batched(starts, seeds + 7 * (i + 1),                   # (starts unchanged)
                              n_pipes=args.rj_pipes, **kw)
        # move 0: one trajectory; a jump: two, unless its proposal was a dead end
        steps += int(np.sum(np.where((g.move_chain == 0) | (g.flag_chain != 0), 1, 2))) * leap
    wall = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
        wall = shard.max_over_ranks(wall)
        steps = int(shard.sum_over_ranks(steps))
    res = {
        "metric": "chain-leapfrog-steps/sec, reversible-jump run_RHMC (%s %dx%d, K0=%d, "
                  "%d chains/GPU)" % (name, D.shape[0], D.shape[1], K0, n_chains),
        "value": steps / wall, "unit": "chain-leapfrog-steps/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": wall / args.steps * 1e3,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (%s image and starts, chain seeds 1000 rank + c)" % name,
        "config": {"workload": "%s: %dx%d image, K0=%d, %d chains/GPU, %d iterations of %d "
                               "steps per run, P_move %s, N_max %d, beta_a = beta_b = %g"
                               % (name, D.shape[0], D.shape[1], K0, n_chains, n_it, leap,
                                  kw["P_move"], kw["N_max"], g.beta_a),
                   "mode": "rj", "rj_pipes": args.rj_pipes or "auto",
                   "parallelism": "chain-sharded x%d" % world},
        "roofline": None,
        "rj": {"accept_rate_jumps": float(np.mean(g.A_chain[g.move_chain > 0]))
               if (g.move_chain > 0).any() else None,
               "accept_rate_within": float(np.mean(g.A_chain[g.move_chain == 0]))
               if (g.move_chain == 0).any() else None,
               "star_counts_end": [int(g.N_chain[-1].min()), int(g.N_chain[-1].max())],
               "dead_end_iterations": int(np.sum(g.flag_chain != 0)),
               "phase_ms_per_iteration": {k: v * 1e3 / n_it for k, v in g.rj_phase_s.items()},
               "native_call_s_last": g.rj_native_s},
        "cpu_baseline": None,
        "sources": source_hash(),
    }
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (ranks) on this node; default WORLD_SIZE or 1")
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
    ap.add_argument("--mode", choices=("leapfrog", "mh", "integrate", "hmc_random", "datagen",
                                       "rj"),
                    default="leapfrog",
                    help="mh: whole MH iterations on device (momentum draw, V+T, accept; "
                         "Philox RNG); one bench step = --mh-iter iterations of --leap steps. "
                         "integrate: --solver's explicit integrator (rhmc_integrate). "
                         "hmc_random: samplers.HMC_random trajectories of --leap steps "
                         "(rhmc_hmc_random). "
                         "datagen: --n-real Poisson realisations of the workload's model "
                         "image (rhmc_gen_image). "
                         "rj: the reversible-jump run_RHMC through librhmc_rj.so, one step "
                         "= --mh-iter iterations of --leap steps (default workload: use B4)")
    ap.add_argument("--mh-iter", type=int, default=10)
    ap.add_argument("--rj-pipes", type=int, choices=tuple(range(9)), default=0,
                    help="--mode rj: host pipes of the native driver (0: its default)")
    ap.add_argument("--f-pos", type=int, choices=(0, 1), default=1,
                    help="--mode mh: run_RHMC's f_pos (V = inf below the flux wall, "
                         "sampler_RHMC.py:303-309; the reference's default 1)")
    ap.add_argument("--mh-floor", type=float, default=1.5,
                    help="--mode mh with --f-pos 1: chain fluxes start >= this x f_lim "
                         "(workloads.mh_start)")
    ap.add_argument("--mh-unfused", action="store_true",
                    help="--mode mh: the four-kernel loop (RHMC_OPT_MH_FUSED = 0)")
    ap.add_argument("--window-split", type=int, choices=(0, 1, 2, 4), default=0,
                    help="RHMC_OPT_WINDOW_SPLIT for the multi-star register-window kernel "
                         "(0: by batch size; results bit-identical)")
    ap.add_argument("--tables", type=int, choices=(0, 1, 2, 3, 4, 5, 6), default=0,
                    help="RHMC_OPT_TABLES (diagnostic): 0 per-stream buffer, 1 the same "
                         "NaN-filled before each launch, 2 / 3 per-launch pool allocation "
                         "without / with the fill, 4 pool allocation never reused, 5 pool "
                         "allocation freed after a stream sync, 6 pool allocation behind an "
                         "event barrier")
    ap.add_argument("--solver", choices=("hmc", "naive", "leap_frog"), default="leap_frog")
    ap.add_argument("--n-real", type=int, default=1000)
    ap.add_argument("--dry-run", action="store_true",
                    help="rendezvous the ranks and print the sharding plan; no GPU work")
    ap.add_argument("--timeout", type=float, default=900.0,
                    help="seconds: --gpus N (spawned ranks) stops every rank and exits 124 "
                         "when they are not all done by then; each rank's gloo rendezvous "
                         "and barriers time out after it too")
    args = ap.parse_args()

    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None:
        n = 1 if args.gpus is None else args.gpus
        if n < 1:
            raise SystemExit("bench.py: --gpus must be >= 1")
        if n > 1:
            # one process per GPU: start the ranks before any GPU call here
            return spawn_ranks(n, args.timeout)
        world = 1
    else:
        world = int(env_world)
        if args.gpus is not None and args.gpus != world:
            raise SystemExit("bench.py: --gpus %d disagrees with WORLD_SIZE=%d"
                             % (args.gpus, world))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    _fault_injection(rank)

    from rhmc_amd import shard, workloads
    if args.workload.upper() == "BIGSIM4":
        if args.mode != "rj":
            raise SystemExit("bench.py: --workload BIGSIM4 is the reversible-jump flagship "
                             "(--mode rj)")
        if world > 1:
            init_gloo(args.timeout)
        return bench_rj(args, None, int(os.environ.get("RHMC_BENCH_DEVICE", local_rank)), world,
                        rank)
    if args.workload.upper() in ("C4", "C5") and not args.chains and not args.global_chains:
        # C4 is one 2^20-chain set, C5 one 8192-chain set, sharded over the
        # ranks (BASELINE configs[3], [4]: "... across 8x MI355X")
        args.global_chains = (1 << 20) if args.workload.upper() == "C4" else 8192
    if args.global_chains:
        # one global chain set (seed 1000), this rank's contiguous shard
        wl = workloads.make(args.workload, n_chains=args.global_chains)
        lo, hi = shard.shard_range(args.global_chains, world, rank)
        wl.q0, wl.p0 = wl.q0[lo:hi].copy(), wl.p0[lo:hi].copy()
    else:
        wl = workloads.make(args.workload, n_chains=args.chains, seed_offset=rank)
    # RHMC_BENCH_DEVICE pins every rank to one device (rehearsing the N-rank
    # path on a one-GPU box); by default rank r of a node uses GPU r.
    gpu = int(os.environ.get("RHMC_BENCH_DEVICE", local_rank))
    total_chains = args.global_chains or wl.n_chains * world
    if args.dry_run:
        return dry_run(args, wl, world, rank, gpu, total_chains)
    # CPU baseline first: forked workers must not inherit an initialised GPU.
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu and args.mode == "leapfrog":
        cpu = cpu_baseline(wl)

    import torch
    import torch.distributed as dist
    from rhmc_amd import capi

    if world > 1:
        init_gloo(args.timeout)
    if args.mode == "rj":
        return bench_rj(args, wl, int(os.environ.get("RHMC_BENCH_DEVICE", local_rank)), world,
                        rank)
    ndev = torch.cuda.device_count()
    if gpu >= ndev:
        raise SystemExit("bench.py: rank %d wants GPU %d but %d are visible"
                         % (rank, gpu, ndev))
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)

    leap = args.leap or wl.n_steps
    P = capi.make_params(**wl.params)
    ctx = capi.Context(wl.D, device=gpu)
    if args.window_split:
        ctx.set_option(capi.OPT_WINDOW_SPLIT, args.window_split)
    if args.tables:
        ctx.set_option(capi.OPT_TABLES, args.tables)
    q = torch.from_numpy(wl.q0).to(dev).contiguous()
    p = torch.from_numpy(wl.p0).to(dev).contiguous()
    it = torch.zeros((wl.n_chains, 2), dtype=torch.int32, device=dev)
    st = torch.zeros(wl.n_chains, dtype=torch.int32, device=dev)
    # A dedicated (non-null) torch stream: the kernel is launched on it and the
    # timing events are recorded on it.
    stream = torch.cuda.Stream(dev)

    if args.mode == "datagen":
        return bench_datagen(args, wl, P, ctx, dev, stream, world, rank)
    mh_acc = None
    if args.mode == "mh":
        leap = args.leap or 10
        if args.mh_unfused:
            ctx.set_option(capi.OPT_MH_FUSED, 0)
        if args.f_pos:
            # with f_pos a start below the flux wall has V = inf: every proposal
            # would be rejected before any pixel work (workloads.mh_start)
            q.copy_(torch.from_numpy(workloads.mh_start(wl, args.mh_floor)).to(dev))
        # the accept decisions of each launch (n_iter x n_chains int32 on the device)
        mh_acc = torch.zeros((args.mh_iter, wl.n_chains), dtype=torch.int32, device=dev)
        mh_rec = capi.MhRecord(None, None, None, None, mh_acc.data_ptr())

        def launch():
            ctx.mh_device(P, q.data_ptr(), wl.n_chains, wl.K, args.mh_iter, leap,
                          f_pos=bool(args.f_pos), seed=1234 + rank, record=mh_rec,
                          stream=stream.cuda_stream)
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
    launch_ms = sum(a.elapsed_time(b) for a, b in ev) / len(ev)
    steps_per_launch = leap * (args.mh_iter if args.mode == "mh" else 1)
    per_rank = None
    if world > 1:
        dist.barrier()
        mine = {"rank": rank, "gpu": gpu, "chains": int(wl.n_chains), "wall_s": wall,
                "kernel_ms": launch_ms,
                "value": wl.n_chains * steps_per_launch * args.steps / wall}
        per_rank = [None] * world
        dist.all_gather_object(per_rank, mine)
        wall = max(r["wall_s"] for r in per_rank)          # max over ranks
        vals = [r["value"] for r in per_rank]
        per_rank = {"ranks": per_rank, "min": min(vals), "max": max(vals),
                    "imbalance": max(vals) / min(vals) if min(vals) > 0 else None}

    stat = st.cpu().numpy()
    nonfinite = int(((stat & capi.STATUS_NONFINITE) != 0).sum())
    iters = it.cpu().numpy()            # last launch: sums over its `leap` steps
    fp_stats = {"p_loop_mean": float(iters[:, 0].mean() / max(leap, 1)),
                "q_loop_mean": float(iters[:, 1].mean() / max(leap, 1)),
                "p_loop_cap_chains": int(((stat & capi.STATUS_PLOOP_CAP) != 0).sum()),
                "q_loop_cap_chains": int(((stat & capi.STATUS_QLOOP_CAP) != 0).sum()),
                "flux_wall_chains": int(((stat & capi.STATUS_REFLECT_F) != 0).sum()),
                # a reflection within 1e-12 of its wall (f_lim, 0,
                # R-1; sampler_RHMC.py:554-564) can legitimately flip the other
                # way on a rounding difference — reported separately
                "near_wall_chains": int(((stat & capi.STATUS_NEAR_WALL) != 0).sum()),
                "near_wall_frac": float(((stat & capi.STATUS_NEAR_WALL) != 0).mean())}

    chain_steps = wl.n_chains * steps_per_launch
    value = total_chains * steps_per_launch * args.steps / wall
    # PMC summaries describe the implicit leapfrog kernel only
    pmc, stale = (load_pmc(wl.name, wl.n_chains) if args.mode == "leapfrog" and
                  not args.window_split else ({}, False))
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
                   "mh_fused": (None if args.mode != "mh" else not args.mh_unfused),
                   "f_pos": (None if args.mode != "mh" else args.f_pos),
                   "mh_start_flux_floor": (args.mh_floor if args.mode == "mh" and args.f_pos
                                           else None),
                   "solver": (args.solver if args.mode == "integrate" else
                              "hmc_random" if args.mode == "hmc_random" else "implicit"),
                   "parallelism": "chain-sharded x%d" % world},
        "roofline": roofline(pmc, wl, chain_steps, launch_ms, stale),
        "nonfinite_chains": nonfinite,
        "fixed_point_iters_per_step": fp_stats,
        "mh_accept_rate_last_launch": (None if mh_acc is None
                                       else float(mh_acc.float().mean().item())),
        "per_rank": per_rank,
        # the kernel sources this line ran (sha256/16 of csrc/*, Makefile, rhmc.h:
        # the same hash pmc_summary.py stores; the GPU box has no .git)
        "sources": source_hash(),
    }
    if args.mode == "leapfrog" and not args.no_e2e and world == 1:
        out["end_to_end"] = end_to_end(ctx, P, q, p, wl, leap)
    if args.tables:
        out["config"]["tables"] = args.tables
        # a -DRHMC_TABLE_CANARY diagnostic library (tools/table_canary.py) also
        # reports the table regions other work wrote into during a gradient
        fn = getattr(capi.lib(), "rhmc_debug_table_conflicts", None)
        if fn is not None:
            import ctypes
            c3 = (ctypes.c_int64 * 5)()
            fn.argtypes = [ctypes.POINTER(ctypes.c_int64)]
            fn(c3)
            out["table_conflicts"] = list(c3)
            seen = (ctypes.c_uint64 * 9)()
            capi.lib().rhmc_debug_table_seen(seen)
            import struct
            out["table_foreign_values"] = [
                {"hex": "%016x" % v, "as_f64": struct.unpack("<d", struct.pack("<Q", v))[0]}
                for v in list(seen)[1:1 + min(8, seen[0])]]
    if rank == 0:
        out["cpu_baseline"] = cpu
        print(json.dumps(out), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


def roofline(pmc, wl, chain_steps, launch_ms, stale=False):
    """The roof that binds the dominant kernel: fp64 VALU issue.

    The image is LDS-resident and each chain's window pixels sit in VGPRs, so
    HBM traffic is ~0.7 MB per launch — HBM does not bound these kernels.
    achieved = executed fp64 FLOP per chain-step (rocprofv3 PMC of the same
    kernel, profiles/pmc_<wl>.json: 64 lanes x (2 FMA + MUL + ADD) per
    instruction) x chain-steps per launch / the launch's HIP-event time;
    peak = 78.6 TF/s fp64 vector.  `traffic` = measured HBM bytes per launch
    (2*FETCH_SIZE + WRITE_SIZE, gfx950 correction), `hbm_measured_frac` its
    rate over 8 TB/s.  `alg_model` keeps SURVEY §8(d)'s algorithmic-bytes model
    (D read by both gradients + q/p in/out per chain-step), which exceeds the
    HBM peak by construction because D never leaves the chip.
    stale: the summary was taken on other kernel sources (load_pmc) — its
    counters are not used (achieved / frac / traffic null, pmc_stale true)."""
    s = launch_ms * 1e-3
    if stale:
        pmc = dict(pmc, hbm_bytes_per_launch=None, fp64_flops_per_chain_step=None,
                   valu_active_frac=None, simd_valu_issue_frac=None,
                   valu_insts_per_chain_step=None, waves_per_simd_resident=None)
    traffic = pmc.get("hbm_bytes_per_launch")
    per = pmc.get("chain_steps_per_dispatch")
    if traffic is not None and per not in (None, chain_steps):
        traffic = traffic * chain_steps / per
    fpc = pmc.get("fp64_flops_per_chain_step")
    npix = wl.D.size
    bpu = alg_bytes_per_step(npix, wl.K)
    alg_gbs = bpu * chain_steps / s / 1e9
    achieved = None if fpc is None else fpc * chain_steps / s / 1e12
    frac = None if achieved is None else achieved / FP64_PEAK_TFLOPS
    ceil = issue_ceiling(pmc.get("waves_per_simd_resident"))
    return {
        "bound": "valu-fp64", "unit": "TFLOP/s", "peak": FP64_PEAK_TFLOPS,
        "achieved": achieved,
        "frac": frac,
        # what the kernel's occupancy allows of that peak even on a stream of
        # independent fp64 FMAs: `frac` is read against this (C2: one wave per SIMD)
        "issue_ceiling": ceil,
        "frac_of_issue_ceiling": (None if frac is None or ceil is None
                                  else frac / ceil["value"]),
        "traffic": traffic,
        "kernel_ms": launch_ms,
        "chain_steps_per_launch": chain_steps,
        "executed_fp64_flops_per_chain_step": fpc,
        "valu_active_frac": pmc.get("valu_active_frac"),
        "simd_valu_issue_frac": pmc.get("simd_valu_issue_frac"),
        "valu_insts_per_chain_step": pmc.get("valu_insts_per_chain_step"),
        "pmc_source": ("profiles/pmc_%s.json (%s, revision %s, sources %s)"
                       % (wl.name.lower(), pmc.get("kernel", "?"), pmc.get("head", "?"),
                          pmc.get("src_hash", "?"))
                       if pmc else None),
        "pmc_stale": bool(stale),
        "hbm_measured_gbs": None if traffic is None else traffic / s / 1e9,
        "hbm_measured_frac": None if traffic is None else traffic / s / 1e9 / HBM_PEAK_GBS,
        "alg_model": {
            "bound": "hbm", "unit": "GB/s", "peak": HBM_PEAK_GBS,
            "bytes_per_chain_step": bpu, "achieved": alg_gbs, "frac": alg_gbs / HBM_PEAK_GBS,
            "fp64_tflops": alg_flops_per_step(npix, wl.K) * chain_steps / s / 1e12,
            "note": "SURVEY 8(d) algorithmic model (2*N_pix*8 + 4*3K*8 B per chain-step); "
                    "exceeds the HBM peak by construction: the image is read from "
                    "LDS/VGPRs, not HBM, so this is not a bound"},
    }


# cycles per independent fp64 FMA wave-instruction on one SIMD at 1 / 2 / 4
# resident waves (tools/isa_bench.hip on MI355X, DESIGN.md §4 Roofline); a
# full-rate issue is 4 cycles per wave-instruction
FMA_CYCLES_BY_WAVES = ((1.0, 9.6), (2.0, 6.4), (4.0, 5.5))


def issue_ceiling(waves):
    """The fraction of the fp64 peak that `waves` resident waves per SIMD can
    issue on a stream of independent FMAs: 4 / cycles per wave-instruction,
    interpolated linearly in the measured table (clamped at its ends)."""
    if waves is None:
        return None
    pts = FMA_CYCLES_BY_WAVES
    w = min(max(float(waves), pts[0][0]), pts[-1][0])
    for (w0, c0), (w1, c1) in zip(pts, pts[1:]):
        if w <= w1:
            cyc = c0 + (c1 - c0) * (w - w0) / (w1 - w0)
            break
    return {"value": 4.0 / cyc, "waves_per_simd": float(waves),
            "note": "4 cycles / measured cycles per independent fp64 FMA wave-instruction "
                    "at this many resident waves per SIMD (9.6 / 6.4 / 5.5 cycles at "
                    "1 / 2 / 4 waves, tools/isa_bench.hip)"}


def init_gloo(timeout):
    """The ranks' host-side process group (barriers, timing max, per-rank
    rates): gloo over 127.0.0.1, every collective bounded by `timeout` + 30 s
    (the launcher's own deadline, counted from the spawn, fires first)."""
    import datetime
    import torch.distributed as dist
    dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=timeout + 30.0))


def _fault_injection(rank):
    """RHMC_BENCH_FAULT_SLEEP=<rank>:<seconds> makes that rank sleep before
    its rendezvous (tests/test_bench_launch.py: the launcher's --timeout)."""
    spec = os.environ.get("RHMC_BENCH_FAULT_SLEEP")
    if spec:
        r, secs = spec.split(":")
        if int(r) == rank:
            time.sleep(float(secs))


def dry_run(args, wl, world, rank, gpu, total_chains):
    """The sharding plan every rank would run, gathered over gloo: no GPU
    work.  Rank 0 prints one JSON line."""
    plan = {"rank": rank, "gpu": gpu, "chains": int(wl.n_chains),
            "first_state": [float(v) for v in wl.q0[0]]}
    plans = [plan]
    if world > 1:
        import torch.distributed as dist
        init_gloo(args.timeout)
        plans = [None] * world
        dist.all_gather_object(plans, plan)
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps({"dry_run": True, "n_gpus": world, "workload": wl.name,
                          "scaling": "strong" if args.global_chains else "weak",
                          "config": {"chains_per_gpu": int(wl.n_chains),
                                     "total_chains": int(total_chains),
                                     "parallelism": "chain-sharded x%d" % world},
                          "ranks": plans}), flush=True)
    return 0


def end_to_end(ctx, P, q, p, wl, leap, reps=10):
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
    sys.exit(main() or 0)
