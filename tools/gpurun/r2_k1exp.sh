#!/bin/bash
# Upper bound of a recent-first tx ring: K1 reading only the first 64 ring entries
# (IGP_K1_EXP=1, results differ for big rings) vs the full 256-entry read, same box
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r2k1
mkdir -p $O
for x in 0 1 0 1; do
  IGP_K1_EXP=$x timeout -k 10 300 python tools/kbench.py --rounds 30 --only feature_assemble_no_update,feature_assemble+single_update > $O/kbench_x$x.log 2>&1 || exit 1
  IGP_K1_EXP=$x timeout -k 10 300 python bench.py --steps 300 --warmup 30 > $O/bench_x$x.log 2>&1 || exit 2
done
for x in 0 1; do
  IGP_K1_EXP=$x timeout -s KILL 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum --kernel-include-regex "feature_assemble" --output-format csv -d /tmp/pmcx$x -o run -- python bench.py --steps 30 --warmup 5 > $O/pmc_x$x.log 2>&1 || exit 3
  python tools/pmc_summary.py /tmp/pmcx$x --batch 8192 > $O/pmc_k1_x$x.txt
done
