set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5b
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r5b/gpu_tests.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/r5b/gpu_tests.log; exit 1; }
tail -1 gpurun_out/r5b/gpu_tests.log
bash tools/ab_libs.sh r5b/ab 3 tree r4
timeout -k 10 120 tools/microbench/two_pass > gpurun_out/r5b/two_pass.txt 2>&1 || { echo TWO_PASS_FAIL; tail -5 gpurun_out/r5b/two_pass.txt; exit 1; }
cat gpurun_out/r5b/two_pass.txt
