#!/bin/bash
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for x in 0 1; do
rm -rf $R/gpurun_out/pmc_x$x
IGP_K1_X=$x timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM --kernel-include-regex "feature_assemble" --output-format csv -d $R/gpurun_out/pmc_x$x -o run -- python $R/tools/kbench.py --rounds 4 --only h2d_slab,feature_assemble_no_update > $R/gpurun_out/pmc_x$x.log 2>&1
rm -rf $R/gpurun_out/pmc_y$x
IGP_K1_X=$x timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC --kernel-include-regex "feature_assemble" --output-format csv -d $R/gpurun_out/pmc_y$x -o run -- python $R/tools/kbench.py --rounds 4 --only h2d_slab,feature_assemble_no_update > $R/gpurun_out/pmc_y$x.log 2>&1
done
exit 0
