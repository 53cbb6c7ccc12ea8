#!/bin/bash
# round 4, pass o: PMC of the default cfg5 f32-faithful GRU (16 waves per workgroup, 32-row
# tiles on overlapped slots), same counters as r3/zh for the 8-wave kernel
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4o
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAIT_ANY SQ_WAVE_CYCLES --output-format csv -d /tmp/pmc5 -o run -- python $GRAFT_REPO_ROOT/bench.py --config cfg5 --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/$O/pmc5.log 2>&1 || exit 5
python $GRAFT_REPO_ROOT/tools/pmc_summary.py /tmp/pmc5 > $GRAFT_REPO_ROOT/$O/pmc_cfg5_fp32.txt 2>&1 || exit 6
