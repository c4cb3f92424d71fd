#!/bin/bash
# Round-4 probe split: alternating north-star benches of the in-tree library and
# the three k_probe ablations (tools/abl_so/libhwbrj_pa{1,2,3}.so, -DHWBRJ_ABL_PROBE=1/2/3), then one
# SQ counter pass per variant on k_probe.  Optional first step: the GPU test suite ($TESTS=1).
#   bash tools/gpu_r4_probe_abl.sh <tag> [passes]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$1; P=${2:-2}
mkdir -p $OUT
if [ "${TESTS:-0}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 \
    || { echo TESTS_FAIL; tail -20 $OUT/gpu_tests.log; exit 1; }
  tail -1 $OUT/gpu_tests.log
fi
bash tools/ab_libs.sh $1/ab $P tree pa1 pa2 pa3 || exit 1
for v in tree pa1 pa2 pa3; do
  if [ $v = tree ]; then L=""; else L=tools/abl_so/libhwbrj_$v.so; fi
  HWBRJ_LIB=$L timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
      SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VALU -T --kernel-include-regex 'k_probe' \
      -d $OUT/sq_$v -o run --output-format csv -- python3 tools/run_ns.py 2 > $OUT/sq_$v.log 2>&1 \
    || { echo PMC_FAIL $v; tail -5 $OUT/sq_$v.log; exit 1; }
  echo "== $v"; python3 tools/pmc_table.py $OUT/sq_$v | tee $OUT/sq_$v.txt
done
echo ABL_OK
