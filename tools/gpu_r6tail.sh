#!/bin/bash
# Round-6 dev A/B of the join's tail loop: north star, then q = 1 (long survivor runs) and PRO.
#   bash tools/gpu_r6tail.sh <tag> <variants...>
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=$1; shift
bash tools/ab_libs.sh $T/ns 3 "$@" && \
ABFLAGS="-q 1.0" bash tools/ab_libs.sh $T/q1 2 "$@" && \
ABFLAGS="-b no" bash tools/ab_libs.sh $T/pro 2 "$@"
