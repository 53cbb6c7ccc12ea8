#!/bin/bash
# round-end validation: GPU tests, smoke, all configs on 1 GPU, 2-rank rehearsal (gloo, shared GPU),
# rocprofv3 kernel stats of the cfg3 headline
set -o pipefail
mkdir -p gpurun_out/res
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_gpu_all.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 2
for c in cfg3 cfg2 cfg4 cfg5 heuristic; do
  timeout -k 10 300 python bench.py --config $c --json-out gpurun_out/res/bench_${c}_1gpu.json > gpurun_out/res/bench_$c.log 2>&1 || exit 3
done
export IGP_DIST_BACKEND=gloo
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 50 --warmup 5 --accounts 262144 > gpurun_out/dist_cfg3.log 2>&1 || exit 4
unset IGP_DIST_BACKEND
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/prof_final
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_final -o run -- python $R/bench.py --steps 300 --warmup 50 > $R/gpurun_out/prof_final.log 2>&1 || exit 5
