#!/bin/bash
# round 3, pass z: f32-faithful split GRU at 32 rows per workgroup: parity tests (vs 16 rows,
# vs float64 torch), cfg5 fp32 engine A/B (16 vs 32 rows), kernel statistics
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3z
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gru_gpu.py -m gpu -v -x --timeout 200 --timeout-method thread > $O/tests.txt 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 $O/tests.txt)" >> $O/status.txt
[ $rc -eq 0 ] || exit 2
for i in 1 2; do
  for r in 16 32; do
    IGP_GRU_X3_ROWS=$r timeout -k 10 250 python bench.py --config cfg5 --steps 60 --warmup 10 --json-out $O/cfg5f_r${r}_$i.json > $O/cfg5f_r${r}_$i.log 2>&1 || exit 4
    echo "cfg5 fp32 split rows=$r $(python -c "import json;d=json.load(open('$O/cfg5f_r${r}_$i.json'));print(round(d['value']/1e6,3),'M/s', round(d['ms_per_step']*1e3,1),'us/step p99', d.get('p99_latency_ms'), d['dtype'])")" >> $O/status.txt
  done
done
cd /tmp && export TMPDIR=/tmp && timeout -k 10 250 rocprofv3 --kernel-trace --stats -d /tmp/p5 -o run -- python $GRAFT_REPO_ROOT/bench.py --config cfg5 --steps 40 --warmup 10 > $GRAFT_REPO_ROOT/$O/prof_cfg5.log 2>&1 || exit 6
cd $GRAFT_REPO_ROOT && python tools/rocpd_stats.py /tmp/p5/run_results.db > $O/cfg5_fp32_kernel_stats.txt
