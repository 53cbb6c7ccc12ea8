#!/bin/bash
# round 3, pass w: GRU ws2 hand-off published from registers (3 barriers per step instead of 5):
# parity tests, kernel time, cfg5 bench; serving pipeline depth A/B (3 / 4 / 6 slots)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3w
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gru_gpu.py -m gpu -v -x --timeout 120 --timeout-method thread > $O/tests.txt 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 $O/tests.txt)" >> $O/status.txt
[ $rc -le 1 ] || exit 2
GRU_WS_ONLY=1 GRU_BATCHES=4096,2048 OUT=$O/gru_sweep.json timeout -k 10 200 python tools/gru_bench.py > $O/gru_sweep.log 2>&1 || exit 3
grep '"ws": [13]' $O/gru_sweep.log | cut -c1-150 >> $O/status.txt
timeout -k 10 120 python tools/gru_ws_trace.py 4096 3 > $O/gru_trace_ws3.txt 2>&1 || exit 4
for i in 1 2; do
  timeout -k 10 200 python bench.py --config cfg5 --numerics bf16 --steps 100 --warmup 10 --json-out $O/cfg5_bf16_$i.json > $O/cfg5_$i.log 2>&1 || exit 5
  echo "cfg5 bf16 $(python -c "import json;d=json.load(open('$O/cfg5_bf16_$i.json'));print(round(d['value']/1e6,3),'M/s', round(d['ms_per_step']*1e3,1),'us/step')")" >> $O/status.txt
done
for i in 1 2; do
  for d in 3 4 6; do
    timeout -k 10 300 python bench.py --steps 60 --warmup 5 --depth $d --json-out $O/serve_d${d}_$i.json > $O/serve_d${d}_$i.log 2>&1 || exit 6
    echo "serve depth $d $(python -c "import json;d=json.load(open('$O/serve_d${d}_$i.json'));print(round(d['value']/1e6,2),'M/s p50',round(d['p50_latency_ms'],2),'p99',round(d['p99_latency_ms'],2), d['host_stages_rank0'])")" >> $O/status.txt
  done
done
cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/p5 -o run -- python $GRAFT_REPO_ROOT/bench.py --config cfg5 --numerics bf16 --steps 60 --warmup 10 > $GRAFT_REPO_ROOT/$O/prof_cfg5.log 2>&1 || exit 7
cd $GRAFT_REPO_ROOT && python tools/rocpd_stats.py /tmp/p5/run_results.db > $O/cfg5_kernel_stats.txt
