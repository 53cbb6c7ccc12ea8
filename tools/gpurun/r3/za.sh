#!/bin/bash
# round 3, pass za: cfg5 fp32 with one stream per pipeline slot and 32-row split GRU tiles:
# parity tests, engine A/B (overlap 32 rows / overlap 16 rows / one stream 16 rows), stats
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3za
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gru_gpu.py -m gpu -v -x --timeout 200 --timeout-method thread > $O/tests.txt 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 $O/tests.txt)" >> $O/status.txt
[ $rc -eq 0 ] || exit 2
for i in 1 2; do
  for v in "x32" "x16" "one"; do
    case $v in x32) E="";; x16) E="IGP_GRU_X3_ROWS=16";; one) E="IGP_ABUSE_STREAMS=1";; esac
    env $E timeout -k 10 250 python bench.py --config cfg5 --steps 60 --warmup 10 --json-out $O/cfg5f_${v}_$i.json > $O/cfg5f_${v}_$i.log 2>&1 || exit 4
    echo "cfg5 fp32 $v $(python -c "import json;d=json.load(open('$O/cfg5f_${v}_$i.json'));print(round(d['value']/1e6,3),'M/s', round(d['ms_per_step']*1e3,1),'us/step p99', d.get('p99_latency_ms'), d['dtype'])")" >> $O/status.txt
  done
done
cd /tmp && export TMPDIR=/tmp && timeout -k 10 250 rocprofv3 --kernel-trace --stats -d /tmp/p5 -o run -- python $GRAFT_REPO_ROOT/bench.py --config cfg5 --steps 40 --warmup 10 > $GRAFT_REPO_ROOT/$O/prof_cfg5.log 2>&1 || exit 6
cd $GRAFT_REPO_ROOT && python tools/rocpd_stats.py /tmp/p5/run_results.db > $O/cfg5_fp32_kernel_stats.txt
