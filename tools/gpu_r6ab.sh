#!/bin/bash
# Round-6 dev A/B: correctness of a variant library on a test selection (VTESTS, with HWBRJ_LIB of
# variant $2), then alternating bench passes over the variants ($3...).
#   bash tools/gpu_r6ab.sh <tag> <variant-to-test|none> <passes> <variants...>
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$1; mkdir -p $OUT
TAG=$1; V=$2; P=$3; shift 3
if [ "$V" != none ]; then
  HWBRJ_LIB=tools/abl_so/libhwbrj_$V.so timeout -k 10 600 python -u -m pytest ${VTESTS:-tests/test_gpu_async.py} -m gpu -x -q --timeout 240 --timeout-method thread \
    > $OUT/tests_$V.log 2>&1 || { echo "TESTS_FAIL $V"; tail -30 $OUT/tests_$V.log; exit 1; }
  echo "tests $V: $(tail -1 $OUT/tests_$V.log)"
fi
bash tools/ab_libs.sh $TAG/ab $P "$@"
