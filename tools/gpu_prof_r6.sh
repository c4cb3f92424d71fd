#!/bin/bash
# Round-6 measurement session on the north-star bench: kernel trace (+stats, and the S scatter per
# stream: the async joins' side stream vs the synchronous joins), FETCH_SIZE and WRITE_SIZE passes
# (each --pmc set in its own run), SQ/LDS counters, then the bench line on the fresh PMC file.
#   bash tools/gpu_prof_r6.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$1
mkdir -p $OUT
B="bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-e2e"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $OUT/trace -o run --output-format csv -- python3 $B > $OUT/trace.log 2>&1 || { echo TRACE_FAIL; tail -5 $OUT/trace.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -T -d $OUT/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-e2e > $OUT/pmc_fetch.log 2>&1 || { echo PMC1_FAIL; tail -5 $OUT/pmc_fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -T -d $OUT/pmc_write -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-e2e > $OUT/pmc_write.log 2>&1 || { echo PMC2_FAIL; tail -5 $OUT/pmc_write.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VALU -T --kernel-include-regex 'k_scatter|k_probe|k_join|k_build' -d $OUT/pmc_sq -o run --output-format csv -- python3 tools/run_ns.py 2 > $OUT/pmc_sq.log 2>&1 || { echo PMC3_FAIL; tail -5 $OUT/pmc_sq.log; exit 1; }
python3 tools/prof_summary.py $OUT/trace $OUT/pmc_fetch $OUT/pmc_write $OUT/pmc_traffic.json '[128000000, 1024000000, 0.01, "blocked", 1073741824, 1, 1024]' > $OUT/traffic.txt && cat $OUT/traffic.txt
python3 tools/pmc_table.py $OUT/pmc_sq > $OUT/pmc_sq.txt
find $OUT/trace -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
find $OUT/trace -name "*kernel_trace.csv" -exec python3 tools/async_kernel_ms.py {} \; > $OUT/scatter_by_stream.txt; cat $OUT/scatter_by_stream.txt
tail -1 $OUT/trace.log > $OUT/bench_traced.json
timeout -k 10 300 python bench.py --pmc-json $OUT/pmc_traffic.json > $OUT/bench.log 2>&1 || { echo BENCH_FAIL; tail -5 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
echo PROF_OK
