#!/bin/bash
# Dev-only: build libhwbrj.so of a git revision (default HEAD) into tools/abl_so/libhwbrj_<name>.so,
# for A/B runs against the working tree (HWBRJ_LIB=tools/abl_so/libhwbrj_<name>.so), and export that
# revision's bench.py and Python package into tools/abl_so/<name>_py/ (ab_libs.sh runs that bench with
# that library, so a revision whose C-ABI predates the tree's bench still runs its own).
#   bash tools/build_base.sh <name> [rev]
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
name=$1; rev=${2:-HEAD}
T=$(mktemp -d)
mkdir -p $T/csrc $T/include $ROOT/tools/abl_so
for f in $(git -C $ROOT ls-tree --name-only $rev hwbloomradixjoin_amd/csrc/); do
  git -C $ROOT show $rev:$f > $T/csrc/$(basename $f)
done
git -C $ROOT show $rev:include/hwbrj.h > $T/include/hwbrj.h
sed -i 's#"../../include/hwbrj.h"#"hwbrj.h"#' $T/csrc/*.h $T/csrc/*.cpp $T/csrc/*.hip 2>/dev/null || true
C=$T/csrc
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -shared -I$C -I$T/include \
  $C/hwbrj_kernels.hip -x hip $C/hwbrj_engine.cpp $C/hwbrj_api.cpp $C/hwbrj_gen.cpp $C/hwbrj_pjoin.cpp $C/hwbrj_comm.cpp \
  $(ls $C/hwbrj_pjoin_async.cpp 2>/dev/null) \
  -o $ROOT/tools/abl_so/libhwbrj_$name.so -lpthread -ldl
P=$ROOT/tools/abl_so/${name}_py
rm -rf $P; mkdir -p $P/hwbloomradixjoin_amd
git -C $ROOT show $rev:bench.py > $P/bench.py
for f in __init__.py pjoin.py; do git -C $ROOT show $rev:hwbloomradixjoin_amd/$f > $P/hwbloomradixjoin_amd/$f; done
rm -rf $T
echo built tools/abl_so/libhwbrj_$name.so and ${name}_py from $rev
