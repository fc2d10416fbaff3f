#!/bin/bash
# Copy a round_final.sh run (gpurun_out/) into profiles/r03_head/ and the PMC
# summaries into profiles/, then regenerate profiles/r03_head/README.md.
#   save_head_evidence.sh REV
cd "$(dirname "$0")/.." || exit 1
REV=$1; D=profiles/r03_head
cp gpurun_out/pmc_c2.json gpurun_out/pmc_c3.json gpurun_out/pmc_c5.json profiles/ || exit 1
for w in c1 c3 c4 c5; do
  cp gpurun_out/wl_$w/bench.json $D/${w}_bench.json && cp gpurun_out/wl_$w/prof/run_kernel_stats.csv $D/${w}_kernel_stats.csv || exit 1
done
tail -1 gpurun_out/bench.log > $D/c2_bench.json
grep '^{' gpurun_out/bench_2ranks.log | tail -1 > $D/c2_bench_2ranks_one_gpu.json
cp gpurun_out/prof/run_kernel_stats.csv $D/c2_kernel_stats.csv
(tail -3 gpurun_out/pytest_gpu.log; cat gpurun_out/smoke.log) > $D/pytest_gpu_tail.txt
cp gpurun_out/kab/c5_ws.txt $D/kab_c5_window_split.txt
cp gpurun_out/kab/c4_lpc.txt $D/kab_c4_shard_lanes.txt
python3 - "$REV" <<'PY'
import csv, json, re, sys
rev, D = sys.argv[1], 'profiles/r03_head'
def trace(w):
    for row in csv.reader(open('%s/%s_kernel_stats.csv' % (D, w))):
        if 'leapfrog' in row[0]:
            return float(row[3]) / 1e6
rows = []
for w, k in (('c1', 'leapfrog_k1_tiledr<32>'), ('c2', 'leapfrog_k1_tiledr<48>'),
             ('c3', 'leapfrog_pk<48,10>'), ('c4', 'leapfrog_k1_tiledl<48,28,float,1>'),
             ('c5', 'leapfrog_kr<float,2> (WS 2)')):
    d = json.loads(open('%s/%s_bench.json' % (D, w)).read())
    rows.append('| %s | %s | %.3g | %.3f |' % (w.upper(), k, d['value'], trace(w)))
c2 = json.loads(open(D + '/c2_bench.json').read())
pm = {w: json.load(open('profiles/pmc_%s.json' % w)) for w in ('c2', 'c3', 'c5')}
npass = re.search(r'(\d+) passed', open(D + '/pytest_gpu_tail.txt').read()).group(1)
r = c2['roofline']
txt = f'''Round-3 evidence at HEAD {rev} on one MI355X (gpurun box), `scripts/round_final.sh`
(copied here by `scripts/save_head_evidence.sh`):

* `pytest_gpu_tail.txt` — smoke + the GPU suite: {npass} passed (incl. the host-ASan run of
  every C-ABI entry point, `tests/test_asan_host.py`).
* `c2_bench.json` — the default `python bench.py` line (C2): {c2['value']:.3g}
  chain-leapfrog-steps/s, kernel {r['kernel_ms']:.3f} ms per 500-step launch (HIP events on the
  launch stream), roofline valu-fp64 frac {r['frac']:.3f}, end_to_end (host buffers, {c2['end_to_end']['calls']} calls)
  {c2['end_to_end']['value']:.3g}, CPU baseline {c2['cpu_baseline']['value']:.3g} on 16 cores.
  `c2_kernel_stats.csv`: rocprofv3 `--kernel-trace --stats` of `bench.py --no-cpu`.
* `c2_bench_2ranks_one_gpu.json` — `RHMC_BENCH_DEVICE=0 bench.py --gpus 2` (both ranks on one
  card: plumbing, not scaling): n_gpus 2, total_chains 8192.
* `c1/c3/c4/c5_bench.json` + `*_kernel_stats.csv` — `scripts/profile_wl.sh C1 C3 C4 C5`
  (C4: all 2^20 chains on one GPU):

| workload | kernel | chain-leapfrog-steps/s | kernel ms / launch (trace avg) |
|---|---|---|---|
''' + '\n'.join(rows) + f'''

* `../pmc_c2.json`, `../pmc_c3.json`, `../pmc_c5.json` — PMC passes of the same revision
  (`scripts/profile_pmc.sh`, `scripts/pmc_summary.py`): SIMD VALU issue
  {pm['c2']['simd_valu_issue_frac']:.2f} / {pm['c3']['simd_valu_issue_frac']:.2f} / {pm['c5']['simd_valu_issue_frac']:.2f},
  VALU instructions per chain-step {pm['c2']['valu_insts_per_chain_step']:.0f} / {pm['c3']['valu_insts_per_chain_step']:.0f} / {pm['c5']['valu_insts_per_chain_step']:.0f}.
* `kab_c5_window_split.txt` — C5 at 8192 chains with window split 1 vs 2 (2, the default,
  `../r03_ws/`); `kab_c4_shard_lanes.txt` — C4 shard (131,072 chains) lane-group kernel with
  1 vs 4 lanes per chain (1, the default).
* Box-to-box spread of the same library is about 2 %.
'''
open(D + '/README.md', 'w').write(txt)
print(txt)
PY
