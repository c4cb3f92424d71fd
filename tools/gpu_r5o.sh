#!/bin/bash
# Dev session (round 5): the async partitioned join's S partitioning on a second stream
# (HWBRJ_PJ_OVL) — its async tests, then the async bench A/B against the build without it
# (tools/abl_so/libhwbrj_pjnoovl.so), interleaved three times on one box.
#   bash tools/gpu_r5o.sh gpurun_out/r5o
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$1
mkdir -p $O
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 900 $PYT tests/test_gpu_multi.py -k "async" > $O/t_async.log 2>&1 || { tail -40 $O/t_async.log; exit 1; }
tail -3 $O/t_async.log
B="python -u bench.py --design partitioned --no-cpu-baseline --no-e2e --steps 16 --warmup 3"
for i in 1 2 3; do
  timeout -k 10 300 $B > $O/ab_ovl_$i.json 2> $O/ab_ovl_$i.err || { tail -20 $O/ab_ovl_$i.err; exit 1; }
  HWBRJ_LIB=tools/abl_so/libhwbrj_pjnoovl.so timeout -k 10 300 $B > $O/ab_noovl_$i.json 2> $O/ab_noovl_$i.err \
    || { tail -20 $O/ab_noovl_$i.err; exit 1; }
  echo "ovl $(grep -o '"ms_per_step": [0-9.]*' $O/ab_ovl_$i.json) noovl $(grep -o '"ms_per_step": [0-9.]*' $O/ab_noovl_$i.json)"
done
echo done
