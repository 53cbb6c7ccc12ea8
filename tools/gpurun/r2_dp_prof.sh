#!/bin/bash
# kernel trace + roctx ranges of the driver's submit/wait (world-1 exchange bench)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2
export IGP_FORCE_EXCHANGE=1
timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace -d /tmp/prof_x -o run -- python bench.py --steps 40 --warmup 10 --accounts 65536 > gpurun_out/r2/prof_x.log 2>&1
python tools/rocpd_api_timeline.py /tmp/prof_x/run_results.db --last 300 --out gpurun_out/r2/prof_x_marker.txt
