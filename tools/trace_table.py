"""Per-kernel durations of one join in a rocprofv3 kernel trace (dispatch order), with each
dispatch's start offset and the idle gap since the previous dispatch ended.
    python tools/trace_table.py <trace dir> [join index, default -1 = the last k_scatter_r]"""
import csv, glob, sys
f = glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
names = [r["Kernel_Name"].split("(")[0] for r in rows]
sc = [i for i, n in enumerate(names) if "k_scatter_r" in n]
start = sc[int(sys.argv[2]) if len(sys.argv) > 2 else -1] if sc else 0
# the join's zeroing memsets are enqueued just before its first kernel
while start > 0 and "fillBuffer" in names[start - 1]:
    start -= 1
t0 = int(rows[start]["Start_Timestamp"])
prev_end, busy, idle = None, 0, 0
nxt = [i for i in sc if i > start]
stop = nxt[0] if nxt else len(rows)
for r, n in zip(rows[start:stop], names[start:stop]):
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = 0 if prev_end is None else s - prev_end
    busy += e - s
    idle += max(0, gap)
    print(f"{n[:60]:60s} {(e - s) / 1e6:8.4f} ms  (+{(s - t0) / 1e6:7.4f})  gap {gap / 1e3:7.2f} us")
    prev_end = e
print(f"span {(prev_end - t0) / 1e6:.4f} ms  busy {busy / 1e6:.4f} ms  idle between dispatches {idle / 1e3:.1f} us")
