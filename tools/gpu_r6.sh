#!/bin/bash
# Dev session (round 6): a GPU test selection (TESTS, default the whole -m gpu suite; "none" skips),
# then the default bench line (BENCH=0 skips). Usage: tools/gpu_r6.sh <out subdir>
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$1; mkdir -p $OUT
if [ "${TESTS}" != none ]; then
  timeout -k 10 ${TTIME:-900} python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 240 --timeout-method thread \
    > $OUT/gpu_tests.log 2>&1 || { echo TESTS_FAIL; tail -40 $OUT/gpu_tests.log; exit 1; }
  tail -1 $OUT/gpu_tests.log
fi
if [ "${BENCH:-1}" = 1 ]; then
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 ${BENCH_ARGS} > $OUT/bench.log 2> $OUT/bench.err \
    || { echo BENCH_FAIL; tail -20 $OUT/bench.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$OUT/bench.log').read().strip().splitlines()[-1]); \
print(d['ms_per_step'], d['value'], d['roofline']['frac'], d['parity']['ok'], d['parity'].get('timed_joins_ok'), d['phase_ms'])"
fi
