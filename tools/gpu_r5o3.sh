#!/bin/bash
# Dev session (round 5): tools/pj_stage.py at G = 1, 2, 4, 8 on the product library and on
# tools/abl_so/libhwbrj_pjnoovl.so (HWBRJ_PJ_OVL=0), for the async rank's row of DESIGN §6.
#   bash tools/gpu_r5o3.sh gpurun_out/r5o3
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$1
mkdir -p $O
timeout -k 10 400 python -u tools/pj_stage.py 1 2 4 8 > $O/pj_stage.log 2>&1 || { tail -20 $O/pj_stage.log; exit 1; }
HWBRJ_LIB=tools/abl_so/libhwbrj_pjnoovl.so timeout -k 10 400 python -u tools/pj_stage.py 1 2 4 8 > $O/pj_stage_noovl.log 2>&1 \
  || { tail -20 $O/pj_stage_noovl.log; exit 1; }
grep -h "async" $O/pj_stage.log $O/pj_stage_noovl.log
echo done
