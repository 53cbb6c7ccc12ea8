#!/bin/bash
# round 3, pass m: pair-cluster MLP chain (mlp_pair.hip) parity + cfg4 A/B vs the one-workgroup
# kernel; GRU per-wave publish (ws=4) parity + A/B vs ws=3; kernel statistics of both
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3m
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_mlp_fused_gpu.py tests/test_gru_gpu.py -m gpu -v -x --timeout 120 --timeout-method thread > $O/tests.txt 2>&1
rc=$?; echo "tests rc=$rc" >> $O/status.txt
[ $rc -le 1 ] || exit 2
for pr in 1 0 1 0; do
  IGP_MLP_PAIR=$pr timeout -k 10 200 python bench.py --config cfg4 --numerics bf16 --steps 400 --warmup 40 --json-out $O/cfg4_pair$pr.json > $O/cfg4_pair$pr.log 2>&1 || exit 3
  echo "cfg4 pair=$pr $(python -c "import json;d=json.load(open('$O/cfg4_pair$pr.json'));print(round(d['value']/1e6,2),'M/s', round(d['ms_per_step']*1e3,1),'us/step p99',round(d['p99_latency_ms'],3))")" >> $O/status.txt
done
GRU_WS_ONLY=1 GRU_BATCHES=4096,2048 OUT=$O/gru_sweep.json timeout -k 10 200 python tools/gru_bench.py > $O/gru_sweep.log 2>&1 || exit 4
for w in 3 4 3 4; do
  IGP_GRU_WS_MODE=$w timeout -k 10 200 python bench.py --config cfg5 --numerics bf16 --steps 100 --warmup 10 --json-out $O/cfg5_ws$w.json > $O/cfg5_ws$w.log 2>&1 || exit 5
  echo "cfg5 ws=$w $(python -c "import json;d=json.load(open('$O/cfg5_ws$w.json'));print(round(d['value']/1e6,3),'M/s', round(d['ms_per_step']*1e3,1),'us/step p99',round(d['p99_latency_ms'],3))")" >> $O/status.txt
done
cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/p4 -o run -- python $GRAFT_REPO_ROOT/bench.py --config cfg4 --numerics bf16 --steps 200 --warmup 20 > $GRAFT_REPO_ROOT/$O/prof_cfg4.log 2>&1 || exit 6
cd $GRAFT_REPO_ROOT && python tools/rocpd_stats.py /tmp/p4/run_results.db > $O/cfg4_kernel_stats.txt
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/p5 -o run -- python $GRAFT_REPO_ROOT/bench.py --config cfg5 --numerics bf16 --steps 60 --warmup 10 > $GRAFT_REPO_ROOT/$O/prof_cfg5.log 2>&1 || exit 7
cd $GRAFT_REPO_ROOT && python tools/rocpd_stats.py /tmp/p5/run_results.db > $O/cfg5_kernel_stats.txt
