#!/bin/bash
# North-star bench line plus a kernel trace of the same command, with the dispatch timeline of the
# last join (per-kernel durations, start offsets, idle gaps between dispatches).
#   bash tools/gpu_gaps.sh <tag> [extra env assignments for the A/B leg, e.g. HWBRJ_DEV_X=1]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$1
shift
mkdir -p $OUT
B="bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-e2e"
timeout -k 10 240 python3 $B > $OUT/bench.log 2>&1 || { echo BENCH_FAIL; tail -5 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('A', d['ms_per_step'], d['phase_ms'])"
if [ $# -gt 0 ]; then
  timeout -k 10 240 env "$@" python3 $B > $OUT/bench_b.log 2>&1 || { echo BENCH_B_FAIL; tail -5 $OUT/bench_b.log; exit 1; }
  tail -1 $OUT/bench_b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('B', d['ms_per_step'], d['phase_ms'])"
  timeout -k 10 240 python3 $B > $OUT/bench_a2.log 2>&1 || { echo BENCH_A2_FAIL; exit 1; }
  tail -1 $OUT/bench_a2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('A', d['ms_per_step'], d['phase_ms'])"
  timeout -k 10 240 env "$@" python3 $B > $OUT/bench_b2.log 2>&1 || { echo BENCH_B2_FAIL; exit 1; }
  tail -1 $OUT/bench_b2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('B', d['ms_per_step'], d['phase_ms'])"
fi
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/trace -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > $OUT/trace.log 2>&1 || { echo TRACE_FAIL; tail -5 $OUT/trace.log; exit 1; }
python3 tools/trace_table.py $OUT/trace > $OUT/timeline.txt && cat $OUT/timeline.txt
echo GAPS_OK
