#!/bin/bash
# GPU session: parity tests, quick per-phase timings, bench line (no CPU baseline).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-chk}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAIL; tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python -u tools/gpu_quick.py > $O/quick.log 2>&1 || { echo QUICK_FAIL; tail -20 $O/quick.log; exit 1; }
cat $O/quick.log | grep -v amdgpu.ids
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench.log 2>&1 || { echo BENCH_FAIL; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log
echo ALL_OK
