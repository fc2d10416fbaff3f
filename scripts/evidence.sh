#!/bin/bash
# The maintained GPU evidence runs (round 6: replaces the one-off r04_* / r05_*
# scripts).  Every GPU step has its own time limit and the first failure ends
# the run.  Usage (on the GPU box, through gpurun):
#   scripts/evidence.sh OUT suite            smoke + the whole GPU suite
#   scripts/evidence.sh OUT bench [NAME...]  bench lines (default: every line
#                                            of DESIGN.md section 5's table)
#   scripts/evidence.sh OUT rj [REPEATS]     RJ lines (B4, BIGSIM4, B4 16k)
#   scripts/evidence.sh OUT pmc [WL...]      PMC passes + summaries into
#                                            profiles/pmc_<wl>.json (C2 C3 C4
#                                            C5 B3 B4 C5_1024 by default)
#   scripts/evidence.sh OUT stall WL         stall-counter passes (pmc_stall.sh)
#   scripts/evidence.sh OUT trace NAME       rocprofv3 --kernel-trace --stats of
#                                            one bench line (RJ lines add
#                                            --memory-copy-trace)
#   scripts/evidence.sh OUT det              WinGG table modes (det_tables.sh)
# OUT is a directory under gpurun_out/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:?out dir}; shift
CMD=${1:?command}; shift
mkdir -p "$O"

# name -> bench arguments
declare -A LINE=(
  [c2]=""
  [c1]="--workload C1 --no-cpu"
  [c3]="--workload C3 --no-cpu"
  [c4]="--workload C4 --no-cpu"
  [c4_shard]="--workload C4 --chains 131072 --no-cpu --no-e2e"
  [c5]="--workload C5 --no-cpu --steps 5 --warmup 1"
  [c5_shard]="--workload C5 --chains 1024 --no-cpu --no-e2e --steps 5 --warmup 1"
  [b4]="--workload B4 --no-cpu --no-e2e"
  [b3]="--workload B3 --no-cpu --no-e2e --steps 5 --warmup 1"
  [c2_mh_10x50]="--mode mh --mh-iter 10 --leap 50 --no-cpu --steps 4 --warmup 1"
  [c3_mh_5x50]="--workload C3 --mode mh --mh-iter 5 --leap 50 --no-cpu --steps 4 --warmup 1"
  [c5_mh_5x10]="--workload C5 --mode mh --mh-iter 5 --leap 10 --no-cpu --steps 2 --warmup 1 --f-pos 1"
  [c5r_mh_5x10]="--workload C5R --mode mh --mh-iter 5 --leap 10 --no-cpu --steps 2 --warmup 1 --f-pos 1"
  [c5r_mh_5x50]="--workload C5R --mode mh --mh-iter 5 --leap 50 --no-cpu --steps 2 --warmup 1 --f-pos 1"
  [rj_b4]="--workload B4 --mode rj --steps 5 --warmup 1 --no-cpu"
  [rj_bigsim4]="--workload BIGSIM4 --mode rj --steps 5 --warmup 1 --no-cpu"
  [rj_b4_16k]="--workload B4 --mode rj --chains 16384 --steps 3 --warmup 1 --no-cpu"
)
ORDER="c2 c1 c3 c4 c4_shard c5 c5_shard b4 b3 c2_mh_10x50 c3_mh_5x50 c5_mh_5x10 c5r_mh_5x10 c5r_mh_5x50 rj_b4 rj_bigsim4 rj_b4_16k"

line() {  # name: one bench line into $O/<name>.json, summary printed
  local n=$1
  timeout -k 10 400 python3 bench.py ${LINE[$n]} > "$O/$n.json" 2> "$O/$n.err" ||
    { tail -20 "$O/$n.err"; exit 1; }
  python3 - "$O/$n.json" "$n" <<'PY' | tee -a "$O/summary.txt"
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d.get("roofline") or {}
rj = d.get("rj") or {}
print(sys.argv[2], "%.4g" % d["value"], "kernel_ms", r.get("kernel_ms"), "frac", r.get("frac"),
      "of_ceiling", r.get("frac_of_issue_ceiling"), "accept", d.get("mh_accept_rate_last_launch"),
      "rj_phases_ms", rj.get("phase_ms_per_iteration"))
PY
}

case $CMD in
  suite)
    timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
      > "$O/smoke.log" 2>&1 || { tail -20 "$O/smoke.log"; exit 1; }
    tail -1 "$O/smoke.log"
    timeout -k 10 1100 python3 -u -m pytest tests -m gpu -v -rf --timeout 300 \
      --timeout-method thread > "$O/pytest_gpu.log" 2>&1
    rc=$?; tail -3 "$O/pytest_gpu.log"; exit $rc ;;
  bench)
    for n in ${*:-$ORDER}; do line "$n"; done ;;
  rj)
    for r in $(seq 1 "${1:-1}"); do for n in rj_b4 rj_bigsim4 rj_b4_16k; do line "$n"; done; done ;;
  pmc)
    for wl in ${*:-C2 C3 C4 C5 B3 B4 C5_1024}; do
      case $wl in
        C5_1024) PMC_ARGS="--chains 1024" PMC_TAG=c5_1024 bash scripts/profile_pmc.sh C5 || exit $? ;;
        *) bash scripts/profile_pmc.sh "$wl" || exit $? ;;
      esac
    done
    # chain-steps per dispatch of each workload's dominant kernel
    declare -A CS=([c2]=2048000 [c3]=8192000 [c4]=524288000 [c5]=4096000 [b3]=409600
                   [b4]=409600 [c5_1024]=512000)
    for wl in ${*:-C2 C3 C4 C5 B3 B4 C5_1024}; do
      t=$(echo "$wl" | tr 'A-Z' 'a-z')
      python3 scripts/pmc_summary.py "gpurun_out/pmc_$t" "$t" leapfrog "${CS[$t]}" \
        "${PMC_HEAD:-unknown}" > "$O/pmc_summary_$t.log" 2>&1 || { cat "$O/pmc_summary_$t.log"; exit 1; }
      cp "profiles/pmc_$t.json" "$O/"
    done ;;
  stall)
    bash scripts/pmc_stall.sh "${1:?workload}" ;;
  trace)
    n=${1:?bench line name}; extra=""
    case $n in rj_*) extra="--memory-copy-trace" ;; esac
    timeout -k 10 400 rocprofv3 --kernel-trace $extra --stats -d "$O/trace_$n" -o run \
      --output-format csv -- python3 bench.py ${LINE[$n]} > "$O/trace_$n.log" 2>&1 || exit 1
    tail -1 "$O/trace_$n.log" | cut -c1-200 ;;
  det)
    bash scripts/det_tables.sh "$O" ;;
  *) echo "unknown command $CMD"; exit 2 ;;
esac
echo "evidence $CMD done"
