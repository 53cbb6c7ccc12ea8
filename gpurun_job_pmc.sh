set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -q -m gpu -x > gpurun_out/t_gpu_all.log 2>&1 || exit 1
for i in 1 2 3; do timeout -k 10 300 python bench.py > gpurun_out/bench_cfg3_$i.log 2>&1 || exit 3; done
timeout -k 10 300 python tools/overlap_probe.py > gpurun_out/overlap.log 2>&1 || exit 4
cd /tmp && export TMPDIR=/tmp
rm -rf $GRAFT_REPO_ROOT/gpurun_out/pmc1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_INSTS_VALU --kernel-include-regex "tree_kernel|mlp_head|feature_assemble" --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc1 -o run -- python $GRAFT_REPO_ROOT/tools/kbench.py --rounds 5 > $GRAFT_REPO_ROOT/gpurun_out/pmc1.log 2>&1 || exit 5
