#!/bin/bash
# SQ / LDS counter passes on the north-star join (each --pmc set in its own run).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/pmc_$1
mkdir -p $OUT
i=0
shift
for set in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set -T --kernel-include-regex 'k_scatter|k_probe|k_join|k_build|k_list_fill|k_surv' -d $OUT/p$i -o run --output-format csv -- python3 tools/run_ns.py 2 > $OUT/p$i.log 2>&1 || { echo "PASS $i FAILED ($set)"; tail -5 $OUT/p$i.log; exit 1; }
done
echo PMC_OK
