#!/bin/bash
# Dev session (round 5, async partitioned join): its world-1 tests, the rest of the multi-GPU
# tests, bench --design partitioned (async and synchronous), and a kernel trace of the async bench
# (K joins back to back) for profiles/r05.
#   bash tools/gpu_r5m.sh gpurun_out/r5m
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$1
mkdir -p $O
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 900 $PYT tests/test_gpu_multi.py -k "async" > $O/t_async.log 2>&1 || { tail -40 $O/t_async.log; exit 1; }
tail -3 $O/t_async.log
timeout -k 10 900 $PYT tests/test_gpu_multi.py -k "not async" > $O/t_multi.log 2>&1 || { tail -40 $O/t_multi.log; exit 1; }
tail -3 $O/t_multi.log
B="python -u bench.py --design partitioned --no-cpu-baseline --no-e2e"
timeout -k 10 300 $B --steps 8 --warmup 2 > $O/bench_pj_async.json 2> $O/bench_pj_async.err || { tail -20 $O/bench_pj_async.err; exit 1; }
timeout -k 10 300 $B --steps 8 --warmup 2 --pj-sync > $O/bench_pj_sync.json 2> $O/bench_pj_sync.err || { tail -20 $O/bench_pj_sync.err; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_pja -o pja -- python -u bench.py --design partitioned \
  --no-cpu-baseline --no-e2e --steps 8 --warmup 2 > $O/prof_pja.log 2>&1 || { tail -20 $O/prof_pja.log; exit 1; }
echo done
