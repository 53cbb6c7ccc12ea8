#!/bin/bash
# round 3, pass zc: LTV chain also reading [n | slots] from the pinned slab (no H2D copy kernel):
# parity test, cfg4 fp32 / bf16 engine A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3zc
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_mlp_fused_gpu.py -m gpu -v -x --timeout 200 --timeout-method thread > $O/tests.txt 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 $O/tests.txt)" >> $O/status.txt
[ $rc -eq 0 ] || exit 2
for i in 1 2; do
  for h in 0 1; do
    for n in fp32 bf16; do
      IGP_LTV_HOST_IN=$h timeout -k 10 200 python bench.py --config cfg4 --numerics $n --steps 300 --warmup 20 --json-out $O/cfg4_${n}_in${h}_$i.json > $O/cfg4_${n}_in${h}_$i.log 2>&1 || exit 4
      echo "cfg4 $n host_in=$h $(python -c "import json;d=json.load(open('$O/cfg4_${n}_in${h}_$i.json'));print(round(d['value']/1e6,2),'M/s', round(d['ms_per_step']*1e3,1),'us/step p99', round(d.get('p99_latency_ms'),3))")" >> $O/status.txt
    done
  done
done
cd /tmp && export TMPDIR=/tmp && IGP_LTV_HOST_IN=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/p4 -o run -- python $GRAFT_REPO_ROOT/bench.py --config cfg4 --steps 200 --warmup 20 > $GRAFT_REPO_ROOT/$O/prof_cfg4.log 2>&1 || exit 6
cd $GRAFT_REPO_ROOT && python tools/rocpd_stats.py /tmp/p4/run_results.db > $O/cfg4_fp32_kernel_stats.txt
