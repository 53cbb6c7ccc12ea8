#!/bin/bash
# cfg3: per-kernel standalone times + phase traces (kbench), then the overlapped timeline
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r2tl
mkdir -p $O
timeout -k 10 300 python tools/kbench.py --rounds 30 --out $O/kbench_all.json > $O/kbench_all.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/tl -o run -- python bench.py --steps 100 --warmup 10 > $O/prof.log 2>&1 || exit 2
python tools/rocpd_stats.py /tmp/tl/run_results.db > $O/kernel_stats.txt
python tools/rocpd_timeline.py /tmp/tl/run_results.db --last 60 --skip-tail 5 > $O/timeline.txt
