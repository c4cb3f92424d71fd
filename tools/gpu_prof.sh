#!/bin/bash
# Kernel trace (per-kernel average durations) + SQ counter passes on the north-star join.
#   bash tools/gpu_prof.sh <tag> [counter-set ...]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/prof_$1
mkdir -p $OUT
shift
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 tools/run_ns.py 3 > $OUT/trace.log 2>&1 || { echo "TRACE FAILED"; tail -5 $OUT/trace.log; exit 1; }
f=$(find $OUT/trace -name "*kernel_stats.csv" | head -1)
python3 tools/trace_table.py $OUT/trace
i=0
for set in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set -T --kernel-include-regex 'k_' -d $OUT/p$i -o run --output-format csv -- python3 tools/run_ns.py 2 > $OUT/p$i.log 2>&1 || { echo "PASS $i FAILED ($set)"; tail -5 $OUT/p$i.log; exit 1; }
done
if [ $i -gt 0 ]; then python3 tools/pmc_table.py $OUT > $OUT/table.txt; cat $OUT/table.txt; fi
echo PROF_OK
