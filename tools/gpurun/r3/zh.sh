#!/bin/bash
# round 3, pass zh: PMC of the default f32-faithful kernels (cfg4 64-row split chain with
# host-direct outputs, cfg5 32-row split GRU on overlapped slots): MFMA busy vs CU busy, L2 hits
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3zh
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAIT_ANY SQ_WAVE_CYCLES --output-format csv -d /tmp/pmc4 -o run -- python $GRAFT_REPO_ROOT/bench.py --config cfg4 --steps 40 --warmup 10 > $GRAFT_REPO_ROOT/$O/pmc4.log 2>&1 || exit 3
python $GRAFT_REPO_ROOT/tools/pmc_summary.py /tmp/pmc4 > $GRAFT_REPO_ROOT/$O/pmc_cfg4_fp32.txt 2>&1 || exit 4
timeout -s KILL 150 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAIT_ANY SQ_WAVE_CYCLES --output-format csv -d /tmp/pmc5 -o run -- python $GRAFT_REPO_ROOT/bench.py --config cfg5 --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/$O/pmc5.log 2>&1 || exit 5
python $GRAFT_REPO_ROOT/tools/pmc_summary.py /tmp/pmc5 > $GRAFT_REPO_ROOT/$O/pmc_cfg5_fp32.txt 2>&1 || exit 6
