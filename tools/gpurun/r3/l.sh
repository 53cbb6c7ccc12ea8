#!/bin/bash
# round 3, pass l: GRU ws=3 start-stagger sweep, cfg4 (64-row default) / cfg5 (ws=3 default) benches
# at both numerics, serving bench ingress-thread A/B with the branch-free serializer + fast parser
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3l
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gru_gpu.py tests/test_mlp_fused_gpu.py -m gpu -v -x --timeout 120 --timeout-method thread > $O/tests.txt 2>&1
rc=$?; echo "tests rc=$rc" >> $O/status.txt
[ $rc -le 1 ] || exit 2
for st in 0 150 300 450; do
  IGP_GRU_STAGGER=$st GRU_WS_ONLY=1 GRU_BATCHES=4096 OUT=$O/gru_st$st.json timeout -k 10 200 python tools/gru_bench.py > $O/gru_st$st.log 2>&1 || exit 3
  echo "stagger=$st $(grep '"ws": 3' $O/gru_st$st.log | cut -c1-160)" >> $O/status.txt
done
for c in cfg5 cfg4; do
  for nm in bf16 fp32; do
    timeout -k 10 300 python bench.py --config $c --numerics $nm --steps 200 --warmup 20 --json-out $O/bench_${c}_$nm.json > $O/bench_${c}_$nm.log 2>&1 || exit 4
    echo "$c $nm $(python -c "import json;d=json.load(open('$O/bench_${c}_$nm.json'));print(round(d['value']/1e6,2),'M/s', round(d['ms_per_step']*1e3,1),'us/step p99',round(d['p99_latency_ms'],3))")" >> $O/status.txt
  done
done
for th in 16 24 32 16 24 32; do
  timeout -k 10 300 python bench.py --threads $th --steps 400 --warmup 40 --json-out $O/serving_t$th.json > $O/serving_t$th.log 2>&1 || exit 5
  echo "serving threads=$th $(python -c "import json;d=json.load(open('$O/serving_t$th.json'));print(round(d['value']/1e6,2),'M/s p50',round(d['p50_latency_ms'],2),'p99',round(d['p99_latency_ms'],2), d['host_stages_rank0'])")" >> $O/status.txt
done
