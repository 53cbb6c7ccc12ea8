#!/bin/bash
# kernel statistics of cfg5 (bonus-abuse GRU) and cfg4 (fused LTV MLP chain) at HEAD
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/prof5
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/g5 -o run -- python bench.py --config cfg5 --steps 200 --warmup 20 > $O/prof5.log 2>&1 || exit 1
python tools/rocpd_stats.py /tmp/g5/run_results.db > $O/cfg5_kernel_stats.txt
python tools/rocpd_timeline.py /tmp/g5/run_results.db --last 30 --skip-tail 3 > $O/cfg5_timeline.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/g4 -o run -- python bench.py --config cfg4 --steps 300 --warmup 30 > $O/prof4.log 2>&1 || exit 2
python tools/rocpd_stats.py /tmp/g4/run_results.db > $O/cfg4_kernel_stats.txt
timeout -k 10 300 python bench.py --scope e2e --steps 200 --warmup 20 --json-out $O/scope_e2e.json > $O/scope_e2e.log 2>&1 || exit 3
