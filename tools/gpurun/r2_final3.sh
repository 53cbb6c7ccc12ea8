#!/bin/bash
# end-of-session validation at HEAD: GPU suite, smoke(), every BASELINE config on 1 GPU, the
# request-path scopes, and kernel traces of cfg3 / cfg2 (profilers last)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/final3
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit 2
for c in cfg3 cfg2 cfg4 cfg5 heuristic; do
  timeout -k 10 300 python bench.py --config $c --steps 2000 --warmup 100 --json-out $O/bench_$c.json >> $O/bench.log 2>&1 || exit 3
done
timeout -k 10 200 python bench.py --json-out $O/bench_default.json >> $O/bench.log 2>&1 || exit 4
timeout -k 10 300 python bench.py --scope e2e --steps 200 --warmup 20 --json-out $O/scope_e2e.json > $O/scope_e2e.log 2>&1 || exit 5
timeout -k 10 300 python bench.py --scope grpc --rpc batch --json-out $O/scope_grpc_batch.json > $O/scope_grpc_batch.log 2>&1 || exit 6
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/g3 -o run -- python bench.py --steps 300 --warmup 30 > $O/prof3.log 2>&1 || exit 7
python tools/rocpd_stats.py /tmp/g3/run_results.db > $O/cfg3_kernel_stats.txt
python tools/rocpd_timeline.py /tmp/g3/run_results.db --last 60 --skip-tail 5 > $O/cfg3_timeline.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/g2 -o run -- python bench.py --config cfg2 --steps 300 --warmup 30 > $O/prof2.log 2>&1 || exit 8
python tools/rocpd_stats.py /tmp/g2/run_results.db > $O/cfg2_kernel_stats.txt
python tools/rocpd_timeline.py /tmp/g2/run_results.db --last 60 --skip-tail 5 > $O/cfg2_timeline.txt
