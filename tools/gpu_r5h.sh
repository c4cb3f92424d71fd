#!/bin/bash
# Dev session (round 5, k_join occupancy): the 2^17-bit bitmap join (32 subs per partition via
# HWBRJ_DEV_L2SUB=5, half the LDS, fewer registers) against the tree and the round-4 build.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
bash tools/ab_libs.sh $1/ab ${2:-3} tree r4 jb17w6:HWBRJ_DEV_L2SUB=5 jb17:HWBRJ_DEV_L2SUB=5 jb17w5:HWBRJ_DEV_L2SUB=5 || exit 1
