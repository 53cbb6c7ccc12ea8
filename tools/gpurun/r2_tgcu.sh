#!/bin/bash
# cfg3 same-box A/Bs: tree-group count (IGP_TREE_GROUPS) then CU split (IGP_CU_SPLIT)
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpurun/r2_tg.sh || exit 1
bash tools/gpurun/r2_cu.sh || exit 2
