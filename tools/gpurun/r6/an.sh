#!/bin/bash
# Round 6 final evidence at HEAD (depth 6, 3 tree groups): smoke, serving kernel statistics,
# SPMD world 1, world 2 / 4 rank processes on the one GPU, cfg2 serving, engine_only.
set -o pipefail
O=gpurun_out/r6an
R=$GRAFT_REPO_ROOT
mkdir -p $R/$O
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $R/$O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" >> $R/$O/status.txt
  case $rc in 0) ;; *) exit $rc;; esac
}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step srv 300 python bench.py --steps 20 --warmup 5 --json-out $R/$O/srv.json
IGP_BENCH_SPMD=1 step spmd1 300 python bench.py --steps 20 --warmup 5 --json-out $R/$O/spmd1.json
step w2 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29621 bench.py --gpus 2 --steps 10 --warmup 3 --threads 8 --json-out $R/$O/w2.json
step w4 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29622 bench.py --gpus 4 --steps 10 --warmup 3 --threads 4 --json-out $R/$O/w4.json
step cfg2 300 python bench.py --config cfg2 --steps 20 --warmup 5 --json-out $R/$O/cfg2.json
step eng 300 python bench.py --scope engine_only --steps 400 --warmup 20 --json-out $R/$O/eng.json
cd /tmp
step prof_srv 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_srv -o run -- python $R/bench.py --steps 10 --warmup 3 --json-out $R/$O/prof_srv.json
