#!/bin/bash
# cfg4 (LTV MLP 4x512) kernel breakdown
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2
timeout -k 10 200 python bench.py --config cfg4 --steps 200 --warmup 20 > gpurun_out/r2/bench_cfg4.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof4 -o run -- python bench.py --config cfg4 --steps 100 --warmup 10 > gpurun_out/r2/prof4.log 2>&1
python tools/rocpd_stats.py /tmp/prof4/run_results.db > gpurun_out/r2/cfg4_kernel_stats.txt
python tools/rocpd_timeline.py /tmp/prof4/run_results.db --last 40 --skip-tail 5 > gpurun_out/r2/cfg4_timeline.txt
