"""bench.py's launcher on CPU (no GPU work): `--gpus N` without WORLD_SIZE
starts N rank processes of itself before touching a GPU, the ranks
rendezvous over gloo (127.0.0.1) and rank 0 reports the plan; a --gpus that
disagrees with WORLD_SIZE fails loudly.  --dry-run stops before the first GPU
call, so this runs here.  The unit being sharded is one chain's
RHMC_single_step sequence (sampler_RHMC.py:522-566)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(args, env=None):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, "bench.py"] + args, cwd=ROOT, env=e,
                          capture_output=True, text=True, timeout=240)


def _line(out):
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout + out.stderr
    return json.loads(lines[0])


@pytest.mark.parametrize("n", [1, 2, 3, 8])
def test_gpus_flag_reaches_the_rank_count(n):
    out = _bench(["--gpus", str(n), "--dry-run"])
    assert out.returncode == 0, out.stderr[-3000:]
    d = _line(out)
    assert d["dry_run"] and d["n_gpus"] == n
    assert d["config"]["total_chains"] == 4096 * n
    assert d["config"]["parallelism"] == "chain-sharded x%d" % n
    ranks = sorted(d["ranks"], key=lambda r: r["rank"])
    assert [r["rank"] for r in ranks] == list(range(n))
    assert [r["gpu"] for r in ranks] == list(range(n))          # rank r on GPU r
    assert all(r["chains"] == 4096 for r in ranks)
    # every rank draws its own chains (seed 1000 + rank)
    firsts = {tuple(r["first_state"]) for r in ranks}
    assert len(firsts) == n


def test_gpus_flag_with_pinned_device():
    """RHMC_BENCH_DEVICE pins every rank to one device (a 1-GPU rehearsal)."""
    out = _bench(["--gpus", "2", "--dry-run"], {"RHMC_BENCH_DEVICE": "0"})
    assert out.returncode == 0, out.stderr[-3000:]
    d = _line(out)
    assert d["n_gpus"] == 2 and {r["gpu"] for r in d["ranks"]} == {0}


@pytest.mark.parametrize("wl,total,n", [("C4", 1 << 20, 2), ("C5", 8192, 2), ("C5", 8192, 8)])
def test_global_set_is_split_not_replicated(wl, total, n):
    """C4 = one 2^20-chain set, C5 one 8192-chain set, split over the ranks
    (strong scaling, BASELINE configs[3], [4])."""
    out = _bench(["--gpus", str(n), "--dry-run", "--workload", wl])
    assert out.returncode == 0, out.stderr[-3000:]
    d = _line(out)
    assert d["n_gpus"] == n
    assert d["config"]["total_chains"] == total
    assert sum(r["chains"] for r in d["ranks"]) == total
    assert sorted(r["gpu"] for r in d["ranks"]) == list(range(n))
    assert d["scaling"] == "strong"


def test_gpus_disagreeing_with_world_size_fails():
    out = _bench(["--gpus", "3", "--dry-run"],
                 {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0",
                  "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": "29512"})
    assert out.returncode != 0
    assert "disagrees with WORLD_SIZE" in out.stderr


def test_failing_rank_fails_the_launch():
    """A rank that dies makes the launcher exit non-zero (and stop the rest)."""
    out = _bench(["--gpus", "2", "--dry-run", "--workload", "nope"])
    assert out.returncode != 0


def test_stuck_rank_hits_the_timeout():
    """A rank that never reaches the rendezvous: the launcher stops every rank
    at --timeout and exits 124 instead of waiting for the driver's kill."""
    import time
    t = time.monotonic()
    out = _bench(["--gpus", "2", "--dry-run", "--timeout", "20"],
                 {"RHMC_BENCH_FAULT_SLEEP": "1:600"})
    took = time.monotonic() - t
    assert out.returncode == 124, (out.returncode, out.stderr[-2000:])
    assert "still running after --timeout" in out.stderr
    assert took < 60, took
