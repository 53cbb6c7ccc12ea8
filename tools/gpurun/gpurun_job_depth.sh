#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
for d in 3 4 6 8; do
timeout -k 10 300 python bench.py --depth $d > gpurun_out/bench_d$d.log 2>&1 || exit 3
done
