cd $GRAFT_REPO_ROOT
for k in tiledw tiledw32; do for pad in 0 56000 82000; do
  RHMC_KERNEL=$k RHMC_LDS_MIN=$pad timeout -k 10 120 python3 bench.py --steps 5 --warmup 1 --no-cpu > gpurun_out/l.log 2>&1 || exit 1
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/l.log').read().strip().splitlines()[-1]); print(sys.argv[1], sys.argv[2], '%.3e' % d['value'], 'kernel_ms %.3f' % d['roofline']['kernel_ms'])" $k $pad
done; done
