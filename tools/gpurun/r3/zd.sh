#!/bin/bash
# round 3, pass zd: GRU cluster kernel with the layer-2 waves at a higher issue priority
# (s_setprio 1 / 3 vs 0): parity, standalone kernel time, cfg5 bf16 engine, phase trace
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3zd
mkdir -p $O
IGP_GRU_WS_PRIO=3 timeout -k 10 500 python -u -m pytest tests/test_gru_gpu.py -m gpu -v -x --timeout 200 --timeout-method thread -k "weight_stationary or two_clusters" > $O/tests.txt 2>&1
rc=$?; echo "tests (prio 3) rc=$rc $(tail -1 $O/tests.txt)" >> $O/status.txt
[ $rc -eq 0 ] || exit 2
for i in 1 2; do
  for p in 0 1 3; do
    IGP_GRU_WS_PRIO=$p GRU_WS_ONLY=1 GRU_BATCHES=4096 OUT=$O/gru_p${p}_$i.json timeout -k 10 200 python tools/gru_bench.py > $O/gru_p${p}_$i.log 2>&1 || exit 3
    echo "prio $p standalone $(grep '"ws": 3' $O/gru_p${p}_$i.log | cut -c1-140)" >> $O/status.txt
    IGP_GRU_WS_PRIO=$p timeout -k 10 200 python bench.py --config cfg5 --numerics bf16 --steps 100 --warmup 10 --json-out $O/cfg5_bf16_p${p}_$i.json > $O/cfg5_p${p}_$i.log 2>&1 || exit 5
    echo "prio $p cfg5 bf16 $(python -c "import json;d=json.load(open('$O/cfg5_bf16_p${p}_$i.json'));print(round(d['value']/1e6,3),'M/s', round(d['ms_per_step']*1e3,1),'us/step')")" >> $O/status.txt
  done
done
IGP_GRU_WS_PRIO=3 timeout -k 10 120 python tools/gru_ws_trace.py 4096 3 > $O/gru_trace_p3.txt 2>&1 || exit 4
