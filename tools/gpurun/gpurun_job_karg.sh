#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/bench_karg0.log 2>&1 || exit 1
HIP_FORCE_DEV_KERNARG=1 timeout -k 10 300 python bench.py > gpurun_out/bench_karg1.log 2>&1 || exit 2
HIP_FORCE_DEV_KERNARG=1 timeout -k 10 300 python tools/kbench.py --rounds 10 > gpurun_out/kb_karg1.log 2>&1 || exit 3
timeout -k 10 300 python tools/kbench.py --rounds 10 > gpurun_out/kb_karg0.log 2>&1 || exit 4
