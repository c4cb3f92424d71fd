#!/bin/bash
# GPU session: parity suite, the basic k >= 2 rows (tools/basic_kk.py), config-3 sweep, bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-kk}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAIL; grep -E "FAIL|Error|assert" $O/tests.log | head -30; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 python -u tools/basic_kk.py > $O/basic_kk.log 2>&1 || { echo KK_FAIL; tail -20 $O/basic_kk.log; exit 1; }
grep -v amdgpu.ids $O/basic_kk.log
if [ "$2" = "full" ]; then
  timeout -k 10 400 python -u tools/sweep.py 3 > $O/sweep3.log 2>&1 || { echo SWEEP_FAIL; tail -20 $O/sweep3.log; exit 1; }
  grep -v amdgpu.ids $O/sweep3.log
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench.log 2>&1 || { echo BENCH_FAIL; tail -20 $O/bench.log; exit 1; }
  tail -1 $O/bench.log | cut -c1-400
fi
