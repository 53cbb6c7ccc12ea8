#!/bin/bash
# round 4, pass w: kernel stats of the serving bench under Zipf(1.2) after the hot-account
# apply rework (compare r4/p: update_multi_kernel 412.5 us per call, 79 % of GPU time)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=gpurun_out/r4w
mkdir -p $R/$O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/zprof -o zipf -- python $R/bench.py --steps 20 --warmup 5 --zipf 1.2 --json-out $R/$O/bench_zipf.json > $R/$O/zprof.log 2>&1 || exit 7
DB=$(ls /tmp/zprof/*/zipf_results.db /tmp/zprof/zipf_results.db 2>/dev/null | head -1)
python $R/tools/rocpd_stats.py "$DB" --top 25 > $R/$O/zipf_kernel_stats.txt 2>&1 || exit 8
