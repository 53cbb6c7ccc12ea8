#!/bin/bash
# cfg2 kernel statistics and timeline (rocprofv3 kernel trace; the last GPU step)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/cfg2prof
mkdir -p $O
timeout -k 10 200 python bench.py --config cfg2 --steps 2000 --warmup 100 --json-out $O/bench_cfg2.json > $O/bench.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/c2 -o run -- python bench.py --config cfg2 --steps 300 --warmup 30 > $O/prof.log 2>&1 || exit 2
python tools/rocpd_stats.py /tmp/c2/run_results.db > $O/cfg2_kernel_stats.txt
python tools/rocpd_timeline.py /tmp/c2/run_results.db --last 60 --skip-tail 5 > $O/cfg2_timeline.txt
