#!/bin/bash
# Dev: the join phase of the north star for the in-tree library and variant builds (tools/join_abl.py).
#   bash tools/gpu_jabl.sh <tag> <variants...>   (tree = in-tree)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$1; shift; mkdir -p $OUT
for v in "$@"; do
  L=""; [ "$v" = tree ] || L=tools/abl_so/libhwbrj_$v.so
  timeout -k 10 200 env HWBRJ_LIB=$L python3 tools/join_abl.py 5 > $OUT/$v.log 2>&1 || { echo "FAIL $v"; tail -5 $OUT/$v.log; exit 1; }
  tail -1 $OUT/$v.log
done
