#!/bin/bash
# Dev session (round 4, k_join): wave-0 phase stamps of the flat and the walking join paths, then
# the GPU suite and an A/B of the two.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$1; mkdir -p $OUT
for v in jst jstn; do
  HWBRJ_LIB=tools/abl_so/libhwbrj_$v.so HWBRJ_DBG=1 timeout -k 10 200 python3 tools/run_ns.py 4 > $OUT/$v.log 2>&1 \
    || { echo "STAMP_FAIL $v"; tail -5 $OUT/$v.log; exit 1; }
  echo "== $v"; grep -E "join cyc|^[0-9]" $OUT/$v.log | tail -3
done
TESTS=${TESTS:-1} VARIANTS="tree noflat" bash tools/gpu_ab.sh $1 ${2:-3}
