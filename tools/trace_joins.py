"""Summarise a rocprofv3 kernel trace (its SQLite results database) of joins enqueued back to back:
per-join span on the GPU (first to last dispatch of the join, found by a marker kernel that runs
once per join), the idle time between consecutive joins, and the per-kernel time of one join.

    python tools/trace_joins.py gpurun_out/r5n/prof_pja/pja_results.db --marker k_pjx_gather [--last 8]

Dev tool (reads only the trace; no GPU).
"""
import argparse
import re
import sqlite3


def short(n):
    return re.sub(r"\(.*", "", n).replace("void ", "")[:44]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--marker", default="k_pjx_gather", help="a kernel that runs once per join")
    ap.add_argument("--before", type=int, default=4, help="dispatches of a join before its marker")
    ap.add_argument("--last", type=int, default=8, help="joins to report (the timed ones)")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = list(c.execute("select name, start, end from kernels order by start"))
    marks = [i for i, r in enumerate(rows) if a.marker in r[0]]
    starts = [max(0, i - a.before) for i in marks]
    bounds = list(zip(starts, starts[1:] + [len(rows)]))[-a.last:]
    print(f"{len(rows)} dispatches, {len(marks)} joins (marker {a.marker}); the last {len(bounds)}:")
    print(f"{'join':>4} {'span ms':>8} {'busy ms':>8} {'idle before ms':>15} {'dispatches':>10}")
    print("(busy: summed dispatch time, > span where a copy on another queue overlaps a kernel)")
    prev_end = None
    for k, (i0, i1) in enumerate(bounds):
        js = rows[i0:i1]
        end = max(r[2] for r in js)  # (dispatches on other queues, e.g. host copies, overlap)
        span = (end - js[0][1]) / 1e6
        busy = sum(r[2] - r[1] for r in js) / 1e6
        idle = (js[0][1] - prev_end) / 1e6 if prev_end is not None else float("nan")
        print(f"{k:>4} {span:8.3f} {busy:8.3f} {idle:15.3f} {len(js):10d}")
        prev_end = end
    i0, i1 = bounds[-2] if len(bounds) > 1 else bounds[-1]
    agg = {}
    for r in rows[i0:i1]:
        agg[short(r[0])] = agg.get(short(r[0]), 0.0) + (r[2] - r[1]) / 1e3
    print("\nper kernel, one join (us):")
    for name, us in sorted(agg.items(), key=lambda x: -x[1]):
        print(f"  {name:46s} {us:9.1f}")
    print(f"  {'sum':46s} {sum(agg.values()):9.1f}")


if __name__ == "__main__":
    main()
