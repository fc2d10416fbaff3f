#!/bin/bash
# bench.py --mode rj lines: big-sim4 geometry at 4096 chains on one GPU, and
# the two-rank path rehearsed on one GPU.  Logs under gpurun_out/r04_rj/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/r04_rj
mkdir -p $O
timeout -k 10 400 python3 bench.py --mode rj --workload B4 --steps 5 --warmup 1 > $O/bench_rj_b4.json 2> $O/bench_rj_b4.err || { tail -20 $O/bench_rj_b4.err; exit 1; }
tail -1 $O/bench_rj_b4.json | cut -c1-400
RHMC_BENCH_DEVICE=0 timeout -k 10 400 python3 bench.py --mode rj --workload B4 --steps 3 --warmup 1 --gpus 2 --chains 2048 --timeout 350 > $O/bench_rj_b4_2ranks.json 2> $O/bench_rj_b4_2ranks.err || { tail -20 $O/bench_rj_b4_2ranks.err; exit 1; }
tail -1 $O/bench_rj_b4_2ranks.json | cut -c1-400
echo done
