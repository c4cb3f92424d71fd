#!/bin/bash
# Dev session (round 5): HWBRJ_PJ_OVL at W = 2 — two ranks sharing the GPU over gloo (the callback
# transport, host-synchronous exchanges), north-star shards, bench.py's partitioned_async leg, the
# product library and tools/abl_so/libhwbrj_pjnoovl.so alternated twice.
#   bash tools/gpu_r5o2.sh gpurun_out/r5o2
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$1
mkdir -p $O
run() {  # $1 = tag, $2 = port; HWBRJ_LIB from the caller
  HWBRJ_BENCH_SHARED_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port $2 bench.py --gpus 2 --steps 4 --warmup 1 --no-cpu-baseline --no-e2e \
    > $O/$1.json 2> $O/$1.err || { tail -20 $O/$1.err; return 1; }
  python3 -c "import json,sys;d=json.loads([l for l in open('$O/$1.json') if l.startswith('{')][-1]);a=d['alt_designs'];print('$1', d['ms_per_step'], {k:(v.get('ms'),v.get('sum')) for k,v in a.items() if isinstance(v,dict)})"
}
run ovl_1 29511 && HWBRJ_LIB=tools/abl_so/libhwbrj_pjnoovl.so run noovl_1 29512 && \
run ovl_2 29513 && HWBRJ_LIB=tools/abl_so/libhwbrj_pjnoovl.so run noovl_2 29514 && echo done
