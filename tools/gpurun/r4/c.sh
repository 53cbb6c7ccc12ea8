#!/bin/bash
# Round 4 third pass: hot-account (Zipf) chunked apply tests + bench, uniform bench with the
# faster key encoding / THP index, the host resolve probe on the box's CPU.
set -o pipefail
O=gpurun_out/r4c
mkdir -p $O
export TMPDIR=/tmp
lscpu > $O/lscpu.txt 2>&1; cat /sys/kernel/mm/transparent_hugepage/enabled /sys/kernel/mm/transparent_hugepage/shmem_enabled >> $O/lscpu.txt 2>&1
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_dedup_gpu.py tests/test_kernels_gpu.py -v \
  --timeout 240 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
echo "tests rc=$?" >> $O/status.txt; tail -2 $O/tests.log >> $O/status.txt
timeout -k 10 300 python tools/resolve_probe.py 1048576 16 > $O/resolve_probe.log 2>&1; echo "probe rc=$?" >> $O/status.txt
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --json-out $O/bench_uniform.json > $O/bench_uniform.log 2>&1
echo "bench uniform rc=$?" >> $O/status.txt
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --zipf 1.2 --json-out $O/bench_zipf.json > $O/bench_zipf.log 2>&1
echo "bench zipf rc=$?" >> $O/status.txt
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --zipf 1.05 --json-out $O/bench_zipf105.json > $O/bench_zipf105.log 2>&1
echo "bench zipf105 rc=$?" >> $O/status.txt
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --scope engine_only --json-out $O/engine.json > $O/engine.log 2>&1
echo "engine rc=$?" >> $O/status.txt
