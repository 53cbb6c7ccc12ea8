#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2
timeout -k 10 300 python -u -m pytest tests/test_mlp_fused_gpu.py tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r2/t_mlp.log 2>&1 || exit 1
for i in 1 2; do
timeout -k 10 200 python bench.py --config cfg4 --steps 300 --warmup 30 > gpurun_out/r2/bench_cfg4_final$i.log 2>&1 || exit 2
done
IGP_MLP_FUSED=0 timeout -k 10 200 python bench.py --config cfg4 --steps 300 --warmup 30 > gpurun_out/r2/bench_cfg4_layers.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof4 -o run -- python bench.py --config cfg4 --steps 100 --warmup 10 > gpurun_out/r2/prof4.log 2>&1
python tools/rocpd_stats.py /tmp/prof4/run_results.db > gpurun_out/r2/cfg4_fused_kernel_stats.txt
python tools/rocpd_timeline.py /tmp/prof4/run_results.db --last 24 --skip-tail 5 > gpurun_out/r2/cfg4_fused_timeline.txt
