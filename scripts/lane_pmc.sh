#!/bin/bash
# PMC passes (one counter set per run) over the lane-group kernel at C4 shard
# size, plus its kernel-trace stats.  Output: gpurun_out/lane_pmc/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/lane_pmc
mkdir -p $O
N=${N:-131072}
CMD="python3 bench.py --chains $N --no-cpu --steps 2 --warmup 1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats -o run -- $CMD > $O/stats.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES -d $O/sq -o run -- $CMD > $O/sq.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 GRBM_GUI_ACTIVE -d $O/f64 -o run -- $CMD > $O/f64.log 2>&1 || exit 1
echo done
