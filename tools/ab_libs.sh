#!/bin/bash
# Dev-only A/B of library builds on the north-star bench: alternating passes over the variants
# (tree = the in-tree libhwbrj.so, NAME = tools/abl_so/libhwbrj_NAME.so), one bench line each.
#   bash tools/ab_libs.sh <tag> <passes> tree NAME [NAME ...]   (extra bench flags: $ABFLAGS)
#   a variant VAR=VALUE runs the in-tree library with that environment variable set, NAME:VAR=VALUE
#   the variant library NAME with it (dev builds read HWBRJ_DEV_*)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$1; P=$2; shift 2
mkdir -p $OUT
for p in $(seq $P); do
  for v in "$@"; do
    E=HWBRJ_AB_VARIANT=1
    if [ "$v" = tree ]; then L=""; elif [[ "$v" == *:*=* ]]; then L=tools/abl_so/libhwbrj_${v%%:*}.so; E=${v#*:};
    elif [[ "$v" == *=* ]]; then L=""; E=$v; else L=tools/abl_so/libhwbrj_$v.so; fi
    BP=bench.py; n=${v%%:*}; [ -f tools/abl_so/${n}_py/bench.py ] && BP=tools/abl_so/${n}_py/bench.py  # (a revision's own bench)
    timeout -k 10 240 env HWBRJ_LIB=$L $E python3 $BP --steps 20 --warmup 5 --no-cpu-baseline --no-e2e $ABFLAGS > $OUT/$v.$p.log 2>&1 || { echo "BENCH_FAIL $v"; tail -5 $OUT/$v.$p.log; exit 1; }
    tail -1 $OUT/$v.$p.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); ph=d['phase_ms']; print('$v', d['ms_per_step'], d['parity']['ok'], ' '.join(f'{k}={v:.4f}' for k,v in ph.items()))"
  done
done
echo AB_OK
