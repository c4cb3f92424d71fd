#!/bin/bash
# GPU session: smoke, bench (with CPU baseline), kernel-trace profile, two PMC passes.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r1/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -5 gpurun_out/r1/smoke.log; exit 1; }
tail -1 gpurun_out/r1/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/r1/bench.log 2>&1 || { echo BENCH_FAIL; tail -5 gpurun_out/r1/bench.log; exit 1; }
tail -1 gpurun_out/r1/bench.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -d gpurun_out/r1/trace -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/r1/trace.log 2>&1 || { echo TRACE_FAIL; tail -5 gpurun_out/r1/trace.log; exit 1; }
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -T -d gpurun_out/r1/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/r1/pmc_fetch.log 2>&1 || { echo PMC1_FAIL; tail -5 gpurun_out/r1/pmc_fetch.log; exit 1; }
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -T -d gpurun_out/r1/pmc_write -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/r1/pmc_write.log 2>&1 || { echo PMC2_FAIL; tail -5 gpurun_out/r1/pmc_write.log; exit 1; }
find gpurun_out/r1 -name "*.csv" | head -20
echo ALL_OK
