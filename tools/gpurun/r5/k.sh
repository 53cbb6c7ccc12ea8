#!/bin/bash
# Round 5: scalar-load latency of K1 (and the other kbench kernels) with the HIP runtime's
# kernel arguments in host vs device memory (HIP_FORCE_DEV_KERNARG)
set -o pipefail
O=gpurun_out/r5k
R=$GRAFT_REPO_ROOT
mkdir -p $R/$O
export TMPDIR=/tmp
cd /tmp
for k in 0 1; do
  HIP_FORCE_DEV_KERNARG=$k KB_K1_MODES=- KB_ABLATE=255 timeout -s KILL 120 rocprofv3 --pmc SmemLatency --output-format csv -d $R/$O/pmc_k$k -o run -- \
    python $R/tools/kbench.py --cold --rounds 3 > $R/$O/pmc_k$k.log 2>&1
  rc=$?; echo "pmc k$k rc=$rc" >> $R/$O/status.txt
  case $rc in 124|134|137|139) exit $rc;; esac
  grep "ablate=" $R/$O/pmc_k$k.log >> $R/$O/status.txt
done
