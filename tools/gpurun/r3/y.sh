#!/bin/bash
# round 3, pass y: split (fp32) chain at 64 rows with the in-place barrier: parity tests, the
# diff probe, standalone times, cfg4 engine fp32 A/B (32 vs 64 rows) and the default cfg4 run
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3y
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_mlp_fused_gpu.py tests/test_kernels_gpu.py tests/test_engine_gpu.py -m gpu -v -x --timeout 120 --timeout-method thread > $O/tests.txt 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 $O/tests.txt)" >> $O/status.txt
[ $rc -eq 0 ] || exit 2
timeout -k 10 120 python tools/probe/split64_diff.py > $O/split64_diff.txt 2>&1 || exit 2
grep -v amdgpu.ids $O/split64_diff.txt >> $O/status.txt
SPLIT=1 OUT=$O/mlp_split.json timeout -k 10 200 python tools/mlp_bench.py 8192,16384 > $O/mlp_split.log 2>&1 || exit 3
grep -v amdgpu.ids $O/mlp_split.log | cut -c1-120 >> $O/status.txt
for i in 1 2; do
  for r in 32 64; do
    IGP_MLP_SPLIT_ROWS=$r timeout -k 10 200 python bench.py --config cfg4 --steps 300 --warmup 20 --json-out $O/cfg4f_r${r}_$i.json > $O/cfg4f_r${r}_$i.log 2>&1 || exit 4
    echo "cfg4 fp32 split rows=$r $(python -c "import json;d=json.load(open('$O/cfg4f_r${r}_$i.json'));print(round(d['value']/1e6,2),'M/s', round(d['ms_per_step']*1e3,1),'us/step p99', d.get('p99_latency_ms'), d['dtype'])")" >> $O/status.txt
  done
done
timeout -k 10 200 python bench.py --config cfg4 --json-out $O/cfg4_default.json > $O/cfg4_default.log 2>&1 || exit 5
echo "cfg4 default $(cat $O/cfg4_default.json | cut -c1-400)" >> $O/status.txt
cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/p4 -o run -- python $GRAFT_REPO_ROOT/bench.py --config cfg4 --steps 200 --warmup 20 > $GRAFT_REPO_ROOT/$O/prof_cfg4.log 2>&1 || exit 6
cd $GRAFT_REPO_ROOT && python tools/rocpd_stats.py /tmp/p4/run_results.db > $O/cfg4_fp32_kernel_stats.txt
