#!/bin/bash
# Round 5: per-wave K1 trace (every wave: phase marks + HW_ID / XCC_ID) on cold rotating batches
set -o pipefail
O=gpurun_out/r5h
R=$GRAFT_REPO_ROOT
mkdir -p $R/$O
export TMPDIR=/tmp
KB_TRACE_OUT=$R/$O/k1trace KB_K1_MODES=- KB_ABLATE=0,255 timeout -k 10 300 python tools/kbench.py --cold --rounds 3 --only dedup_insert > $R/$O/kbench.log 2>&1
echo "kbench rc=$?" >> $R/$O/status.txt
