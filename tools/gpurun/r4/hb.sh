#!/bin/bash
# Round 4: the driver's bench command and engine_only at HEAD
set -o pipefail
O=gpurun_out/r4hb
R=$GRAFT_REPO_ROOT
mkdir -p $R/$O
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --json-out $R/$O/bench.json > $R/$O/bench.log 2>&1
rc=$?; echo "bench rc=$rc" >> $R/$O/status.txt
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --scope engine_only --json-out $R/$O/engine.json > $R/$O/engine.log 2>&1
echo "engine rc=$?" >> $R/$O/status.txt
