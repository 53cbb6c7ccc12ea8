#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
rm -rf $R/gpurun_out/pmc_r1 $R/gpurun_out/pmc_r2
timeout -k 10 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU SQ_WAVES --kernel-include-regex "feature_assemble|tree_kernel" --output-format csv -d $R/gpurun_out/pmc_r1 -o run -- python $R/tools/kbench.py --rounds 1 --only h2d_slab > $R/gpurun_out/pmc_r1.log 2>&1 || exit 5
timeout -k 10 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM_RD --kernel-include-regex "feature_assemble|tree_kernel" --output-format csv -d $R/gpurun_out/pmc_r2 -o run -- python $R/tools/kbench.py --rounds 1 --only h2d_slab > $R/gpurun_out/pmc_r2.log 2>&1 || exit 6
