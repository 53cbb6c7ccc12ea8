#!/bin/bash
# Round 5: K1 phase trace with two more marks (live rows entered, level-2 loads issued)
set -o pipefail
O=gpurun_out/r5f
R=$GRAFT_REPO_ROOT
mkdir -p $R/$O
export TMPDIR=/tmp
KB_K1_MODES=- KB_ABLATE=0,255 timeout -k 10 300 python tools/kbench.py --cold --rounds 3 --only dedup_insert > $R/$O/kbench.log 2>&1
echo "kbench rc=$?" >> $R/$O/status.txt
