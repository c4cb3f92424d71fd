"""Per-kernel durations of the last join in a rocprofv3 kernel trace (dispatch order)."""
import csv, glob, sys
f = glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
names = [r["Kernel_Name"].split("(")[0] for r in rows]
sc = [i for i, n in enumerate(names) if "k_scatter_r" in n]
start = sc[-1] if sc else 0
t0 = int(rows[start]["Start_Timestamp"])
for r, n in zip(rows[start:], names[start:]):
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    print(f"{n[:70]:70s} {d:8.3f} ms  (+{(int(r['Start_Timestamp']) - t0) / 1e6:7.3f})")
print(f"span {(int(rows[-1]['End_Timestamp']) - t0) / 1e6:.3f} ms")
