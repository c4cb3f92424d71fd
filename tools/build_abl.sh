#!/bin/bash
# Dev-only: build variants of libhwbrj.so into tools/abl_so/ (-DHWBRJ_DEV_BUILD: ablations allowed,
# HWBRJ_DEV_* read from the environment; results invalid while ablated).
#   bash tools/build_abl.sh NAME "-DFLAG ..." [NAME "-DFLAGS" ...]
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
C=$ROOT/hwbloomradixjoin_amd/csrc
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -shared -I$C -I$ROOT/include -DHWBRJ_DEV_BUILD $flags \
    $C/hwbrj_kernels.hip -x hip $C/hwbrj_engine.cpp $C/hwbrj_api.cpp $C/hwbrj_gen.cpp $C/hwbrj_pjoin.cpp $C/hwbrj_comm.cpp \
    $C/hwbrj_pjoin_async.cpp -o $ROOT/tools/abl_so/libhwbrj_$name.so -lpthread -ldl &
done
wait
