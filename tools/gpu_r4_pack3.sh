#!/bin/bash
# Dev session (round 4): 3-byte join keys per probe item -- GPU suite, config 3/5 sweeps of the
# in-tree library and of the -DHWBRJ_PACK3=0 build, north-star A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$1; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1 \
  || { echo TESTS_FAIL; tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 500 python3 tools/sweep.py > $OUT/sweep_tree.log 2>&1 || { echo SWEEP_FAIL; tail -5 $OUT/sweep_tree.log; exit 1; }
HWBRJ_LIB=tools/abl_so/libhwbrj_nopk.so timeout -k 10 500 python3 tools/sweep.py > $OUT/sweep_nopk.log 2>&1 || { echo SWEEP2_FAIL; exit 1; }
grep -v amdgpu $OUT/sweep_tree.log | cut -c1-150; echo ===; grep -v amdgpu $OUT/sweep_nopk.log | cut -c1-150
bash tools/ab_libs.sh $1/ab 3 tree head nopk || exit 1
