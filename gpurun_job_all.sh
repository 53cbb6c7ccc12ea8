set -o pipefail
mkdir -p gpurun_out/res
for c in cfg3 cfg2 cfg4 cfg5 heuristic; do
  timeout -k 10 300 python bench.py --config $c --json-out gpurun_out/res/bench_${c}_1gpu.json > gpurun_out/res/bench_$c.log 2>&1 || exit 3
done
