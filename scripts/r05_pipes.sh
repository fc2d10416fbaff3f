#!/bin/bash
# Round 5: the native RJ driver's host pipes (device-resident driver), three
# repeats each on one box; and the host's transparent-huge-page setting.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05_pipes
mkdir -p $O
cat /sys/kernel/mm/transparent_hugepage/enabled /sys/kernel/mm/transparent_hugepage/defrag > $O/thp.txt 2>&1
for rep in 1 2 3; do
  for wl in B4 BIGSIM4; do
    for pp in 2 3 4; do
      n=${wl}_p${pp}_r$rep
      timeout -k 10 300 python3 bench.py --workload $wl --mode rj --rj-pipes $pp --steps 4 --warmup 1 > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
      python3 -c "import json; d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]); print('$n', '%.4g' % d['value'], '%.1f' % d['ms_per_step'], '%.1f' % (1e3 * d['rj']['native_call_s_last']))"
    done
  done
done
for pp in 2 3 4; do
  n=B4_16k_p$pp
  timeout -k 10 300 python3 bench.py --workload B4 --chains 16384 --mode rj --rj-pipes $pp --steps 3 --warmup 1 > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]); print('$n', '%.4g' % d['value'], '%.1f' % d['ms_per_step'], '%.1f' % (1e3 * d['rj']['native_call_s_last']))"
done
cat $O/thp.txt
echo pipes done
