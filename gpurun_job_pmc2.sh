#!/bin/bash
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
rocprofv3 --list-avail > $R/gpurun_out/pmc_list.txt 2>&1
rm -rf $R/gpurun_out/pmc_c
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_IFETCH SQ_INSTS_SMEM SQ_WAVES SQ_INSTS_LDS --kernel-include-regex "feature_assemble|dedup_insert|tree_kernel" --output-format csv -d $R/gpurun_out/pmc_c -o run -- python $R/tools/kbench.py --rounds 4 --only h2d_slab,dedup_insert,feature_assemble_no_update,tree_ensemble > $R/gpurun_out/pmc_c.log 2>&1
exit 0
