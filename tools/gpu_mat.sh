#!/bin/bash
# Dev: the materializing join at the north star: ablation timings, kernel trace, SQ counters.
#   bash tools/gpu_mat.sh <tag> [abl ...]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$1
shift
mkdir -p $OUT
timeout -k 10 200 python tools/mat_bench.py > $OUT/bench.log 2>&1 || { echo BENCH_FAIL; tail -5 $OUT/bench.log; exit 1; }
for v in "$@"; do
  echo "== $v" >> $OUT/bench.log
  HWBRJ_LIB=$PWD/tools/abl_so/libhwbrj_$v.so timeout -k 10 200 python tools/mat_bench.py >> $OUT/bench.log 2>&1 || { echo ABL_FAIL $v; tail -5 $OUT/bench.log; exit 1; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $OUT/trace -o run --output-format csv -- python3 tools/mat_bench.py > $OUT/trace.log 2>&1 || { echo TRACE_FAIL; tail -5 $OUT/trace.log; exit 1; }
find $OUT/trace -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VALU -T --kernel-include-regex 'k_join_mat|k_scatter_sp|k_probe' -d $OUT/pmc_sq -o run --output-format csv -- python3 tools/mat_bench.py > $OUT/pmc_sq.log 2>&1 || { echo PMC_FAIL; tail -5 $OUT/pmc_sq.log; exit 1; }
python3 tools/pmc_table.py $OUT/pmc_sq > $OUT/pmc_sq.txt
grep -v amdgpu.ids $OUT/bench.log
echo MAT_OK
