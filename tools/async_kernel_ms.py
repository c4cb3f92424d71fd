"""Per-stream dispatch times of one kernel in a rocprofv3 kernel trace (CSV) of bench.py: the
async joins run their S scatter on the Engine's side stream, the synchronous joins on the join
stream, so grouping k_scatter_s by Stream_Id separates the timed schedule's dispatches from the
one-stream phase runs. Prints, per stream, the dispatch count, mean / median / min / max ms.

    python tools/async_kernel_ms.py gpurun_out/r6b/trace/run_kernel_trace.csv [--kernel k_scatter_s]

Dev tool (reads only the trace; no GPU).
"""
import argparse
import csv
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--kernel", default="k_scatter_s")
    a = ap.parse_args()
    by = {}
    for r in csv.DictReader(open(a.csv)):
        if a.kernel + "(" not in r["Kernel_Name"] and not r["Kernel_Name"].endswith(a.kernel):
            continue
        ms = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        by.setdefault((r["Stream_Id"], r["Queue_Id"]), []).append(ms)
    print(f"{a.kernel}: dispatches per (stream, queue), ms")
    for (st, q), v in sorted(by.items()):
        print(f"  stream {st:>3} queue {q:>3}: n {len(v):3d}  mean {statistics.mean(v):.4f}  "
              f"median {statistics.median(v):.4f}  min {min(v):.4f}  max {max(v):.4f}")


if __name__ == "__main__":
    main()
