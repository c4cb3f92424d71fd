#!/bin/bash
# Round-2 GPU session: GPU tests, then the bench line (each step under its own time limit).
#   bash tools/gpu_r2.sh <tag> [pytest -k expression]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$1
mkdir -p $OUT
K=${2:-}
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$K" > $OUT/tests.log 2>&1 || { echo TESTS_FAIL; tail -30 $OUT/tests.log; exit 1; }
else
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo TESTS_FAIL; tail -30 $OUT/tests.log; exit 1; }
fi
tail -3 $OUT/tests.log
timeout -k 10 300 python bench.py > $OUT/bench.log 2>&1 || { echo BENCH_FAIL; tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
echo ALL_OK
