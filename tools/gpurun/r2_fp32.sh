#!/bin/bash
# fp32 head: numerics tests + cfg3 bench fp32 vs bf16 (same box)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r2/t_fp32.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2/smoke.log 2>&1 || exit 2
for n in fp32 bf16 fp32; do
timeout -k 10 200 python bench.py --numerics $n > gpurun_out/r2/bench_cfg3_$n.log 2>&1 || exit 3
done
