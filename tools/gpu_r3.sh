#!/bin/bash
# Round-3 GPU steps (run through gpurun from the repo root): each step under its own time limit,
# chained so that the first failure ends the call. Usage: bash tools/gpu_r3.sh OUTDIR STEP...
#   tests:<pytest -k expr>   GPU tests matching the expression (all when empty)
#   alltests                 the whole -m gpu suite
#   bench                    bench.py (20 steps, 5 warmup)
#   pj                       tools/pj_stage.py 2 4 8
#   abl:<variants>           tools/abl_run.py over tools/abl_so variants (comma separated)
#   prof                     rocprofv3 kernel trace + stats of bench.py (5 steps)
set -e
out=$1; shift
mkdir -p "$out"
for step in "$@"; do
  case "$step" in
    tests:*) k="${step#tests:}"
      timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$k" > "$out/tests.log" 2>&1 ;;
    alltests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$out/alltests.log" 2>&1 ;;
    bench)
      timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$out/bench.log" 2>&1 ;;
    pj)
      timeout -k 10 300 python tools/pj_stage.py 2 4 8 > "$out/pj_stage.log" 2>&1 ;;
    abl:*) v="${step#abl:}"
      timeout -k 10 400 python tools/abl_run.py ${v//,/ } > "$out/abl.log" 2>&1 ;;
    prof)
      cd /tmp && export TMPDIR=/tmp
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$out/prof" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-e2e > "$GRAFT_REPO_ROOT/$out/prof.log" 2>&1
      cd "$GRAFT_REPO_ROOT" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
  echo "step $step ok" >> "$out/steps.log"
done
