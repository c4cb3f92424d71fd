#!/bin/bash
# Dev session (round 4): XCD-aware join job order A/B (tree vs nojxcd) with the GPU suite, then the
# join's FETCH_SIZE under each (one --pmc pass per library, k_join only).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$1; mkdir -p $OUT
TESTS=${TESTS:-1} VARIANTS="tree nojxcd" bash tools/gpu_ab.sh $1 3 || exit 1
for v in tree nojxcd; do
  if [ $v = tree ]; then L=""; else L=tools/abl_so/libhwbrj_$v.so; fi
  HWBRJ_LIB=$L timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -T --kernel-include-regex "k_join$" -d $OUT/fetch_$v -o run --output-format csv -- python3 tools/run_ns.py 2 > $OUT/fetch_$v.log 2>&1 || { echo PMC_FAIL $v; tail -5 $OUT/fetch_$v.log; exit 1; }
  python3 - $OUT/fetch_$v $v <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if r["Counter_Name"] == "FETCH_SIZE"]
vals = [float(r["Counter_Value"]) for r in rows if r["Kernel_Name"].startswith("k_join")]
print(sys.argv[2], "k_join FETCH_SIZE KiB per dispatch:", [round(v) for v in vals], "-> x2 GB:", [round(2 * v * 1024 / 1e9, 3) for v in vals])
PY
done
echo JXCD_DONE
