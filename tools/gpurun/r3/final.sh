#!/bin/bash
# round 3, end-of-session validation at HEAD: full GPU suite, smoke, the driver's exact bench
# command (twice), every config's default run, rocprof kernel statistics of the headline
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${R3FINAL:-r3final}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests.txt 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 $O/tests.txt)" >> $O/status.txt
[ $rc -eq 0 ] || exit 2
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit 3
echo smoke ok >> $O/status.txt
for i in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --json-out $O/driver_cmd_$i.json > $O/driver_cmd_$i.log 2>&1 || exit 4
  echo "driver cmd $(python -c "import json;d=json.load(open('$O/driver_cmd_$i.json'));print(round(d['value']/1e6,2),'M/s p50',round(d['p50_latency_ms'],2),'p99',round(d['p99_latency_ms'],2),'ms/step',round(d['ms_per_step'],2))")" >> $O/status.txt
done
for c in cfg2 cfg4 cfg5; do
  timeout -k 10 300 python bench.py --config $c --json-out $O/$c.json > $O/$c.log 2>&1 || exit 5
  echo "$c $(python -c "import json;d=json.load(open('$O/$c.json'));print(round(d['value']/1e6,3),'M/s p99',round(d.get('p99_latency_ms',0),3), d['dtype'], d.get('scope'))")" >> $O/status.txt
done
timeout -k 10 300 python bench.py --scope engine_only --json-out $O/cfg3_engine.json > $O/cfg3_engine.log 2>&1 || exit 6
echo "cfg3 engine_only $(python -c "import json;d=json.load(open('$O/cfg3_engine.json'));print(round(d['value']/1e6,2),'M/s p99',round(d['p99_latency_ms'],3))")" >> $O/status.txt
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/p3 -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 40 --warmup 5 > $GRAFT_REPO_ROOT/$O/prof_serving.log 2>&1 || exit 7
cd $GRAFT_REPO_ROOT && python tools/rocpd_stats.py /tmp/p3/run_results.db > $O/serving_kernel_stats.txt
