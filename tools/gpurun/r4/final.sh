#!/bin/bash
# Round 4 last check at HEAD: the whole GPU suite and smoke()
set -o pipefail
O=gpurun_out/r4final
R=$GRAFT_REPO_ROOT
mkdir -p $R/$O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider > $R/$O/gpu_tests.log 2>&1
rc=$?; echo "gpu_tests rc=$rc" >> $R/$O/status.txt
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $R/$O/smoke.log 2>&1
echo "smoke rc=$?" >> $R/$O/status.txt
