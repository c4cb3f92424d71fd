#!/bin/bash
# Dev session (round 5, k_join): GPU suite, wave-0 join stamps of the round-4 and the new join,
# A/B of the tree against the round-4 build and two join variants, the two-pass S model.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$1; mkdir -p $OUT
[ "${TESTS}" = none ] || timeout -k 10 600 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo TESTS_FAIL; tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
for v in jst4 jst5; do
  [ -f tools/abl_so/libhwbrj_$v.so ] || continue
  HWBRJ_LIB=tools/abl_so/libhwbrj_$v.so HWBRJ_DBG=1 timeout -k 10 200 python3 tools/run_ns.py 4 > $OUT/$v.log 2>&1 \
    || { echo "STAMP_FAIL $v"; tail -5 $OUT/$v.log; exit 1; }
  echo "== $v"; grep -E "join cyc|^[0-9]" $OUT/$v.log | tail -3
done
bash tools/ab_libs.sh $1/ab ${2:-3} ${VARIANTS:-tree r4} || exit 1


