#!/bin/bash
# round 4: diagnostic probe for the intermittent GetFeatures mismatch after hot-account batches
set -o pipefail
R=$GRAFT_REPO_ROOT
O=gpurun_out/r4zz
mkdir -p $R/$O
export TMPDIR=/tmp
timeout -k 10 500 python -u tools/probe/hot_features_probe.py 8 > $R/$O/probe.log 2>&1
echo "probe rc=$?" >> $R/$O/status.txt
