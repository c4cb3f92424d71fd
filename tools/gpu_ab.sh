#!/bin/bash
# Dev A/B session on one box: optional GPU test suite ($TESTS=1), alternating north-star benches of
# the in-tree library and tools/abl_so variants, optional SQ counter pass per variant on $SQK ($SQ=1).
#   VARIANTS="tree a b" bash tools/gpu_ab.sh <tag> [passes]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$1; P=${2:-2}
mkdir -p $OUT
if [ "${TESTS:-0}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1 \
    || { echo TESTS_FAIL; tail -30 $OUT/gpu_tests.log; exit 1; }
  tail -1 $OUT/gpu_tests.log
fi
bash tools/ab_libs.sh $1/ab $P $VARIANTS || exit 1
if [ "${SQ:-0}" = 1 ]; then
  for v in $VARIANTS; do
    if [ $v = tree ]; then L=""; else L=tools/abl_so/libhwbrj_$v.so; fi
    HWBRJ_LIB=$L timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
        SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VALU -T --kernel-include-regex "${SQK:-k_probe}" \
        -d $OUT/sq_$v -o run --output-format csv -- python3 tools/run_ns.py 2 > $OUT/sq_$v.log 2>&1 \
      || { echo PMC_FAIL $v; tail -5 $OUT/sq_$v.log; exit 1; }
    echo "== $v"; python3 tools/pmc_table.py $OUT/sq_$v | tee $OUT/sq_$v.txt
  done
fi
echo AB_DONE
