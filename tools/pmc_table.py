"""Print per-kernel counter values (last join of the run) from rocprofv3 counter_collection CSVs."""
import csv, glob, sys
from collections import defaultdict, OrderedDict
vals = defaultdict(lambda: OrderedDict())
for d in sys.argv[1:]:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        rows = list(csv.DictReader(open(f)))
        # keep the last dispatch of each (kernel, occurrence index) of the last join
        by_kernel = defaultdict(list)
        for r in rows:
            by_kernel[(r["Kernel_Name"], r["Counter_Name"])].append(r)
        for (k, c), rs in by_kernel.items():
            rs.sort(key=lambda r: int(r["Start_Timestamp"]))
            n = 2 if k == "k_list_fill" else 1
            for j, r in enumerate(rs[-n:]):
                name = k if n == 1 else f"{k}#{'RS'[j]}"
                vals[name][c] = float(r["Counter_Value"])
                vals[name]["_ms"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
for k, cs in vals.items():
    print(k)
    for c, v in cs.items():
        print(f"   {c:26s} {v:16.0f}")
