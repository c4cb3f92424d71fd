"""Dev: the bench line's dominant kernel (k_scatter_s timed in the async schedule) against a
rocprofv3 kernel trace of the same bench command (tools/gpu_prof_r6.sh: bench.py --steps K
--warmup W under --kernel-trace). Dispatch order in that command: the parity join (join stream),
W + K async joins (side stream), K synchronous phase joins (join stream), K async-timed joins
(side stream).

    python tools/dom_vs_trace.py <trace dir> <bench_traced.json> [K]
"""
import csv
import glob
import json
import statistics
import sys


def main():
    tdir, bj = sys.argv[1], sys.argv[2]
    K = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    path = glob.glob(f"{tdir}/**/*kernel_trace.csv", recursive=True)[0]
    rows = [r for r in csv.DictReader(open(path)) if "k_scatter_s" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    v = [(r["Stream_Id"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6) for r in rows]
    streams = []
    for s, _ in v:
        if s not in streams:
            streams.append(s)
    main_s, side_s = streams[0], streams[1]
    side = [m for s, m in v if s == side_s]
    sync = [m for s, m in v if s == main_s][1:]
    timed, atimed = side[-2 * K:-K], side[-K:]
    b = json.loads(open(bj).read().strip().splitlines()[-1])["roofline"]["dominant_kernel"]
    print(f"k_scatter_s dispatches in start order (stream {main_s} = the join stream, {side_s} = the async joins' side stream):")
    print("  " + "  ".join(f"s{s} {m:.4f}" for s, m in v))
    print(f"bench line ({b['schedule']}): ms {b['ms']:.4f}, mean {b.get('ms_async_mean')}, "
          f"min/max {b['ms_async_min_max']}, sync phase {b['ms_sync_phase']:.4f}")
    print(f"trace, the {K} async-timed joins: median {statistics.median(atimed):.4f}, mean {statistics.mean(atimed):.4f}, "
          f"min {min(atimed):.4f}, max {max(atimed):.4f}")
    print(f"  -> line against trace: median {100 * (b['ms'] / statistics.median(atimed) - 1):+.1f} %"
          + (f", mean {100 * (b['ms_async_mean'] / statistics.mean(atimed) - 1):+.1f} %" if b.get("ms_async_mean") else ""))
    print(f"trace, the {K} timed headline joins: median {statistics.median(timed):.4f}, mean {statistics.mean(timed):.4f}")
    print(f"trace, the synchronous phase joins: mean {statistics.mean(sync):.4f}")


if __name__ == "__main__":
    main()
