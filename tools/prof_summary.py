"""Summarise rocprofv3 outputs of bench.py into per-phase numbers (committed under profiles/).

    python tools/prof_summary.py <trace_dir> <pmc_fetch_dir> <pmc_write_dir> <out.json> [config...]

Kernel-trace: per-dispatch durations of the last synchronous (one-queue) join of the run. PMC
(bytes, the same in either schedule): the last join, index kernels labelled by their queue's last
scatter. PMC: FETCH_SIZE and WRITE_SIZE
(KiB per dispatch; printed below as KiB x 1024 / 1e9 = GB) from two separate --pmc passes; on gfx950 FETCH_SIZE reports half the bytes of
wide coalesced reads (MI355X_MICROARCH.md, HBM), so hbm_bytes = (2*FETCH_SIZE + WRITE_SIZE)*1024.
Infinity-Cache hits are included in these counters.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

# kernel -> phase (hwbrj_engine.cpp Engine::enqueue)
PHASE_OF = {"k_build_global": "build", "k_build": "build", "k_probe_global": "probe",
            "k_probe": "probe", "k_join_split": "join", "k_join": "join", "k_plan": "index",
            "k_list_fill": "index", "k_mat_build": "materialize", "k_mat_probe": "materialize"}


def one(path_glob):
    f = glob.glob(path_glob, recursive=True)
    if not f:
        raise SystemExit(f"missing {path_glob}")
    return f[0]


def last_join(names):
    """Indices of the dispatches of the last join: after the previous join's last kernel (k_join,
    which also reduces the counts) up to its own, so kernels the bench runs after the joins (its
    copy-rate measurement) are not counted. The S pass may come first (Engine::enqueue) or the R
    side."""
    ends = [i for i, n in enumerate(names) if n == "k_join"]
    if not ends:
        return list(range(len(names)))
    b = ends[-2] + 1 if len(ends) > 1 else 0
    return list(range(b, ends[-1] + 1))


def joins(names):
    """Dispatch index ranges of every join (each ends with its k_join)."""
    ends = [i for i, n in enumerate(names) if n == "k_join"]
    return [list(range(b, e + 1)) for b, e in zip([0] + [x + 1 for x in ends[:-1]], ends)]


def last_one_queue_join(names, queues):
    """The last join whose dispatches all ran on one queue (a synchronous join: its kernel times
    are its own; in an async join the R side's kernels wait behind the S scatter's, and their
    durations include that wait). Falls back to the last join."""
    for idx in reversed(joins(names)):
        if len({queues[i] for i in idx if not names[i].startswith("__amd")}) == 1:  # (runtime blits: own queue)
            return idx
    return last_join(names)


def label(names, idx, queues=None):
    """Phase of each dispatch: plan / list-fill kernels belong to the side of the last scatter on
    their own queue (async joins run the S pass on a second stream, so the R side's plan can start
    after the S scatter; one-stream joins have one queue, where this is the last scatter)."""
    out, side = [], {}
    q = queues or [0] * len(names)
    for i in idx:
        n = names[i]
        if n in ("k_scatter_r", "k_scatter_s"):
            side[q[i]] = n[-1]
            out.append(n[-1] + "_scatter")
        elif n in ("k_plan", "k_list_fill"):
            out.append(side.get(q[i], "r") + "_index")
        else:
            out.append(PHASE_OF.get(n, "other"))
    return out


def main():
    tdir, fdir, wdir, out = sys.argv[1:5]
    tr = list(csv.DictReader(open(one(f"{tdir}/**/*kernel_trace.csv"))))
    tr.sort(key=lambda r: int(r["Start_Timestamp"]))
    names = [r["Kernel_Name"] for r in tr]
    tq = [r["Queue_Id"] for r in tr]
    idx = last_one_queue_join(names, tq)  # kernel times: the last synchronous join's
    labs = label(names, idx, tq)
    phases = defaultdict(lambda: {"ms": 0.0, "kernels": []})
    for i, lab in zip(idx, labs):
        r = tr[i]
        ms = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        phases[lab]["ms"] += ms
        phases[lab]["kernels"].append({"name": names[i], "ms": round(ms, 4)})

    def counters(d, cname):
        rows = list(csv.DictReader(open(one(f"{d}/**/*counter_collection.csv"))))
        rows = [r for r in rows if r["Counter_Name"] == cname]
        rows.sort(key=lambda r: int(r["Start_Timestamp"]))
        nm = [r["Kernel_Name"] for r in rows]
        ix = last_join(nm)
        return list(zip(label(nm, ix, [r["Queue_Id"] for r in rows]), (float(rows[i]["Counter_Value"]) for i in ix)))

    fetch, write = defaultdict(float), defaultdict(float)
    for lab, v in counters(fdir, "FETCH_SIZE"):
        fetch[lab] += v
    for lab, v in counters(wdir, "WRITE_SIZE"):
        write[lab] += v
    res = {"config_key": None, "library": None, "phases": {}}
    if len(sys.argv) > 5:
        res["config_key"] = json.loads(sys.argv[5])
    # the library that was profiled (bench.py uses this traffic only for the same stamp)
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import hwbloomradixjoin_amd as hw
    res["library"] = hw.version()
    for lab, p in phases.items():
        res["phases"][lab] = {
            "ms": round(p["ms"], 4), "kernels": p["kernels"],
            "fetch_kib": round(fetch.get(lab, 0.0), 1), "write_kib": round(write.get(lab, 0.0), 1),
            "hbm_bytes": round((2 * fetch.get(lab, 0.0) + write.get(lab, 0.0)) * 1024),
        }
    json.dump(res, open(out, "w"), indent=1)
    for lab, p in res["phases"].items():
        gbs = p["hbm_bytes"] / (p["ms"] * 1e-3) / 1e9 if p["ms"] else 0
        print(f"{lab:10s} {p['ms']:8.4f} ms  fetch(raw, x2 in total) {p['fetch_kib']*1024/1e9:7.3f} GB  write "
              f"{p['write_kib']*1024/1e9:7.3f} GB  -> {p['hbm_bytes']/1e9:7.3f} GB  {gbs:8.1f} GB/s")


if __name__ == "__main__":
    main()
