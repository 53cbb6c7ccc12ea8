#!/bin/bash
# round 3, pass o: k-step-major chain weights; standalone chain-kernel timings (tools/mlp_bench.py),
# MLP + GRU GPU tests, cfg4 engine A/B pair vs one-workgroup, LDS / L2 counters of both
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3o
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_mlp_fused_gpu.py tests/test_gru_gpu.py -m gpu -v -x --timeout 120 --timeout-method thread > $O/tests.txt 2>&1
rc=$?; echo "tests rc=$rc" >> $O/status.txt
[ $rc -le 1 ] || exit 2
OUT=$O/mlp_bench.json timeout -k 10 200 python tools/mlp_bench.py > $O/mlp_bench.log 2>&1 || exit 3
for pr in 1 0 1 0; do
  IGP_MLP_PAIR=$pr timeout -k 10 200 python bench.py --config cfg4 --numerics bf16 --steps 400 --warmup 40 --json-out $O/cfg4_pair$pr.json > $O/cfg4_pair$pr.log 2>&1 || exit 4
  echo "cfg4 pair=$pr $(python -c "import json;d=json.load(open('$O/cfg4_pair$pr.json'));print(round(d['value']/1e6,2),'M/s', round(d['ms_per_step']*1e3,1),'us/step p99',round(d['p99_latency_ms'],3))")" >> $O/status.txt
done
timeout -k 10 200 python bench.py --config cfg4 --numerics fp32 --steps 200 --warmup 20 --json-out $O/cfg4_fp32.json > $O/cfg4_fp32.log 2>&1 || exit 5
echo "cfg4 fp32 $(python -c "import json;d=json.load(open('$O/cfg4_fp32.json'));print(round(d['value']/1e6,2),'M/s', round(d['ms_per_step']*1e3,1),'us/step')")" >> $O/status.txt
cd /tmp && export TMPDIR=/tmp
for pr in 1 0; do
  IGP_MLP_PAIR=$pr timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS --output-format csv -d /tmp/pmc$pr -o run -- python $GRAFT_REPO_ROOT/bench.py --config cfg4 --numerics bf16 --steps 40 --warmup 10 > $GRAFT_REPO_ROOT/$O/pmc$pr.log 2>&1 || exit 6
  python $GRAFT_REPO_ROOT/tools/pmc_summary.py /tmp/pmc$pr > $GRAFT_REPO_ROOT/$O/pmc_pair$pr.txt 2>&1 || exit 7
done
