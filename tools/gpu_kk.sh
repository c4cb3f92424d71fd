#!/bin/bash
# GPU session: parity suite, then the basic k >= 2 rows (tools/basic_kk.py).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-kk}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAIL; grep -E "FAIL|Error|assert" $O/tests.log | head -30; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 python -u tools/basic_kk.py > $O/basic_kk.log 2>&1 || { echo KK_FAIL; tail -20 $O/basic_kk.log; exit 1; }
grep -v amdgpu.ids $O/basic_kk.log
