#!/bin/bash
# Round 5: are K1's waits the kernel-argument loads? K1 on cold rotating batches and the
# driver's serving bench with the HIP runtime's kernarg placement switched (HIP_FORCE_DEV_KERNARG),
# plus the scalar-cache counters of K1.
set -o pipefail
O=gpurun_out/r5e
R=$GRAFT_REPO_ROOT
mkdir -p $R/$O
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $R/$O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" >> $R/$O/status.txt
  case $rc in 124|134|137|139) exit $rc;; esac
  return 0
}
for k in 0 1; do
  HIP_FORCE_DEV_KERNARG=$k KB_K1_MODES=- KB_ABLATE=0,512,255 step kbench_k$k 300 python tools/kbench.py --cold --rounds 10
done
HIP_FORCE_DEV_KERNARG=1 step bench_k1 400 python bench.py --steps 20 --warmup 5 --json-out $R/$O/bench_k1.json
HIP_FORCE_DEV_KERNARG=0 step bench_k0 400 python bench.py --steps 20 --warmup 5 --json-out $R/$O/bench_k0.json
cd /tmp
for k in 0 1; do
  HIP_FORCE_DEV_KERNARG=$k KB_K1_MODES=- KB_ABLATE=0 timeout -s KILL 120 rocprofv3 --pmc SQC_DCACHE_REQ SQC_DCACHE_MISSES SQC_TC_DATA_READ_REQ SQC_TC_STALL SQ_INSTS_SMEM SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_WAVES --output-format csv -d $R/$O/pmc_k$k -o run -- \
    python $R/tools/kbench.py --cold --rounds 1 --only dedup_insert > $R/$O/pmc_k$k.log 2>&1
  rc=$?; echo "pmc k$k rc=$rc" >> $R/$O/status.txt
  case $rc in 124|134|137|139) exit $rc;; esac
done
