#!/bin/bash
# round 3, pass v: re-created container, rebuilt extensions: full GPU suite, smoke, driver bench cmd
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3v
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.txt 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 $O/tests.txt)" >> $O/status.txt
[ $rc -le 1 ] || exit 2
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit 3
echo smoke ok >> $O/status.txt
for i in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --json-out $O/driver_cmd_$i.json > $O/driver_cmd_$i.log 2>&1 || exit 4
  echo "driver cmd $(python -c "import json;d=json.load(open('$O/driver_cmd_$i.json'));print(round(d['value']/1e6,2),'M/s p50',round(d['p50_latency_ms'],2),'p99',round(d['p99_latency_ms'],2),'ms/step',round(d['ms_per_step'],2))")" >> $O/status.txt
done
