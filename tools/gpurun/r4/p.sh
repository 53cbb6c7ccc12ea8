#!/bin/bash
# round 4, pass p: PMC of the default cfg5 f32-faithful GRU (16 waves per workgroup), same
# counters as r3/zh for the 8-wave kernel; kernel stats of the serving bench under Zipf(1.2)
# traffic (where the device step is 10x the uniform one)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=gpurun_out/r4p
mkdir -p $R/$O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAIT_ANY SQ_WAVE_CYCLES --output-format csv -d /tmp/pmc5 -o run -- python $R/bench.py --config cfg5 --steps 20 --warmup 5 > $R/$O/pmc5.log 2>&1 || exit 5
python $R/tools/pmc_summary.py /tmp/pmc5 > $R/$O/pmc_cfg5_fp32.txt 2>&1 || exit 6
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/zprof -o zipf -- python $R/bench.py --steps 20 --warmup 5 --zipf 1.2 --json-out $R/$O/bench_zipf.json > $R/$O/zprof.log 2>&1 || exit 7
DB=$(ls /tmp/zprof/*/zipf_results.db /tmp/zprof/zipf_results.db 2>/dev/null | head -1)
python $R/tools/rocpd_stats.py "$DB" --top 25 > $R/$O/zipf_kernel_stats.txt 2>&1 || exit 8
python $R/tools/rocpd_timeline.py "$DB" > $R/$O/zipf_timeline.txt 2>&1 || true
