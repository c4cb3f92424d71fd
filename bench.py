#!/usr/bin/env python3
"""bench.py -- headline benchmark of the MI355X bloom radix join (BASELINE.json metric).

One step = one full BPRO join (filter build + probe + both partition passes + join + count) over
HBM-resident synthetic relations with the reference generator's key multiset
(src/generator.c:304-415): |R| = 128M, |S| = 1024M, q = 0.01, -b blocked, m = 2^30, k = 1,
B = 1024 (the reference default, src/main.c:393). value = probe tuples (|S|) per second over the
whole job. The K timed joins are enqueued back to back (hwbrj_join_device_async) and waited for
once, as a pipeline of joins runs; the phase breakdown comes from K synchronous joins afterwards.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N   (N > 1)

N > 1: one rank per GPU (RCCL backend). Strong scaling by default (BASELINE config 4): one
|S| = 1024M range-sharded over the ranks (the reference's per-thread chunking of S,
src/parallel_radix_join_bloom.c:1646-1672), R replicated, every rank builds the filter from its
copy of R, so the data path has no collective; value = |S| / the slowest rank's time, and the
per-rank counts summed over the ranks must equal the golden. --scaling weak (every rank its own
full |S|) is an A/B option, never the default. Counts are reduced after the timed region.

Prints ONE JSON line (rank 0) with roofline (dominant kernel, HIP-event timed) and cpu_baseline
(the oracle's multithreaded restatement of the reference, "port", on a bounded sample).
"""
from __future__ import annotations

import argparse
import json
import statistics
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "probe-tuples/sec, |R|=128M |S|=1024M q=0.01, 1/2/4/8 MI355X; %HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
# golden counts of the reference binary at this exact config
GOLDEN = {(128000000, 1024000000, 0.01, "blocked", 1 << 30, 1, 1024): (124236515, 10240000)}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("-r", "--r-size", type=int, default=128000000)
    ap.add_argument("-s", "--s-size", type=int, default=1024000000)
    ap.add_argument("-q", "--s-sel", type=float, default=0.01)
    ap.add_argument("-b", "--bloom-filter", default="blocked")
    ap.add_argument("-m", "--bloom-size", type=int, default=1 << 30)
    ap.add_argument("-k", "--bloom-hashes", type=int, default=1)
    ap.add_argument("-B", "--bloom-block-size", type=int, default=1024)
    ap.add_argument("-n", "--nthreads", type=int, default=2, help="generator threads (multiset)")
    ap.add_argument("--scaling", choices=("strong", "weak"), default="strong",
                    help="strong (default, BASELINE config 4): one |S| range-sharded over the ranks; "
                         "weak (A/B only): every rank joins its own full |S|")
    ap.add_argument("--design", choices=("replicated", "partitioned"), default="replicated",
                    help="N > 1: R replicated on every rank (no exchange), or R and the join "
                         "partitioned over the ranks (R and survivor all-to-alls, slice all-gather)")
    ap.add_argument("--transport", choices=("native", "torch"), default="native",
                    help="--design partitioned: the library's own RCCL communicator (collectives on "
                         "the join stream), or torch.distributed callbacks (the only choice when "
                         "ranks share a GPU)")
    ap.add_argument("--pj-sync", action="store_true",
                    help="--design partitioned, native: the synchronous join (host waits on its two "
                         "counts messages) instead of the async one (padded exchanges, joins back to back)")
    ap.add_argument("--filter-bcast", action="store_true",
                    help="replicated design: rank 0 builds the filter, ncclBroadcast sends it to "
                         "every rank (the north_star's bitmap broadcast) instead of a rebuild per rank")
    ap.add_argument("--no-alt-designs", action="store_true",
                    help="N > 1 (or any process group): skip the extra legs that time the other "
                         "multi-GPU designs on the same ranks after the headline (alt_designs)")
    ap.add_argument("--alt-steps", type=int, default=5, help="timed joins per alt_designs leg")
    ap.add_argument("--alt-timeout", type=float, default=150.0,
                    help="seconds the alt_designs legs may take before the headline is printed without "
                         "the rest and every rank exits (a collective that never completes)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the PCIe-inclusive end-to-end time")
    ap.add_argument("--cpu-sample", type=int, default=0,
                    help="S tuples in the CPU baseline run (0: the full |S|, the same workload)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="port threads (0: every allowed CPU, capped by OMP_NUM_THREADS)")
    ap.add_argument("--pmc-json", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    return ap.parse_args()


JOIN_KEY_NAMES = {0: "32-bit codes", 1: "packed keys", 2: "mixed (packed, unstaged items 32-bit)"}


def join_key_bytes(st) -> float:
    """Bytes per join key between build/probe and k_join, as the join ran them (hwbrj_stats_t
    join_keys, join_key_bits): join_key_bits / 8 for packed keys (the mixed format's unstaged runs
    are a small share; 18 bits at the north star), else 4."""
    return st.join_key_bits / 8.0 if st.join_keys in (1, 2) else 4.0


def modeled_bytes(nR: int, nS: int, filtered: int, m: int, word_bytes: float, key_bytes: float = 4.0) -> dict:
    """Implementation bytes beyond the algorithmic 8-byte tuple reads (reported,
    never in the headline): partition words written and read back, survivor keys, the filter."""
    return {
        "partition_words_R": 2.0 * 4.0 * nR,          # k_scatter_r writes, k_build reads
        "partition_words_S": 2.0 * word_bytes * nS,   # k_scatter_s writes, k_probe reads
        "join_codes_R": 2.0 * key_bytes * nR,         # k_build writes, k_join reads
        "survivors": 2.0 * key_bytes * filtered,      # k_probe writes, k_join reads
        "filter_slices": 2.0 * m / 8.0,               # k_build writes, k_probe loads
    }


def e2e_time(hw, torch, dR, dS, args, nS, reps=3):
    """SURVEY.md s8(d)'s t_e2e: H2D of R and S from pinned host memory, the join, and the counts'
    D2H (hwbrj_join_device returns them on the host), median of `reps`. Reported beside the
    headline, never as `value` (which has the inputs resident in HBM)."""
    hR = torch.empty(dR.shape, dtype=torch.int32, pin_memory=True)
    hS = torch.empty(dS.shape, dtype=torch.int32, pin_memory=True)
    hR.copy_(dR)
    hS.copy_(dS)
    torch.cuda.synchronize()
    tot, h2d = [], []
    for _ in range(reps):
        t0 = time.perf_counter()
        dR.copy_(hR, non_blocking=True)
        dS.copy_(hS, non_blocking=True)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        hw.join_device(dR, dS, args)
        t2 = time.perf_counter()
        tot.append(t2 - t0)
        h2d.append(t1 - t0)
    del hR, hS
    ms = sorted(tot)[len(tot) // 2] * 1e3
    hm = sorted(h2d)[len(h2d) // 2] * 1e3
    nbytes = 8 * (dR.shape[0] + dS.shape[0])
    return {"ms": round(ms, 3), "value": round(nS / (ms * 1e-3), 1), "unit": "probe-tuples/s",
            "h2d_ms": round(hm, 3), "h2d_GBps": round(nbytes / (hm * 1e-3) / 1e9, 1),
            "what": "H2D of R and S (pinned host memory) + join + counts D2H, median of 3; not value"}


def main():
    a = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    import torch
    import hwbloomradixjoin_amd as hw

    # HWBRJ_BENCH_SHARED_GPU=1 (rehearsal only): ranks share the visible GPUs round-robin, with
    # gloo for the few host-side collectives, so the N > 1 path runs on a one-GPU box
    shared = os.environ.get("HWBRJ_BENCH_SHARED_GPU") == "1"
    if shared:
        local = local % torch.cuda.device_count()
    torch.cuda.set_device(local)
    hw.lib().hwbrj_set_device(local)
    dist = None
    # HWBRJ_BENCH_DIST=1: the process group (RCCL) even at world 1, so a one-GPU box runs the
    # N > 1 code path's init, barriers and reductions over RCCL
    if world > 1 or os.environ.get("HWBRJ_BENCH_DIST") == "1":
        import torch.distributed as dist
        if shared:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    nR, nS_total = a.r_size, a.s_size
    if a.design == "partitioned":
        a.scaling = "strong"  # (R and one S are sharded over the ranks)
    if a.scaling == "strong":
        lo, hi = hw.shard_range(nS_total, rank, world)
        total_units = nS_total
    else:
        lo, hi = 0, nS_total
        total_units = nS_total * world
    nS = hi - lo
    if a.design == "partitioned":
        rlo, rhi = hw.shard_range(nR, rank, world)  # this rank's R rows
    else:
        rlo, rhi = 0, nR
    dR = torch.empty((rhi - rlo, 2), dtype=torch.int32, device="cuda")
    dS = torch.empty((nS, 2), dtype=torch.int32, device="cuda")
    hw.generate_device_range(dR, nR, rlo, a.nthreads, nR, nR, 1.0, 12345)  # src/main.c:410-431 (-x 12345)
    hw.generate_device_range(dS, nS_total, lo, a.nthreads, 2**31 - 1, nR, a.s_sel,
                             54321 + (rank if a.scaling == "weak" else 0))  # :443-466 (-y 54321)
    torch.cuda.synchronize()
    args = hw.BloomFilterArgs.from_flag(a.bloom_filter, a.bloom_size, a.bloom_hashes,
                                        a.bloom_block_size)

    if a.design == "partitioned":
        return run_partitioned(a, hw, torch, dist, rank, world, local, dR, dS, args, shared)
    if a.filter_bcast:
        if shared:
            raise SystemExit("--filter-bcast needs one GPU per rank (RCCL)")
        from hwbloomradixjoin_amd import pjoin
        pjoin.comm_init()
        pjoin.set_filter_broadcast(True)

    # one untimed parity run (counts reduced over ranks)
    st = hw.join_device(dR, dS, args)
    cdev = "cpu" if shared else "cuda"  # where the count / time reductions live
    counts = torch.tensor([st.filtered, st.matches], dtype=torch.int64, device=cdev)
    lo_c, hi_c = counts.clone(), counts.clone()
    per_rank = [[int(x) for x in counts.tolist()]]
    if dist:  # every rank's own (filtered, matches), before the sum
        gathered = [torch.empty_like(counts) for _ in range(world)]
        dist.all_gather(gathered, counts.clone())
        per_rank = [[int(x) for x in t.tolist()] for t in gathered]
        dist.all_reduce(counts)
        dist.all_reduce(lo_c, op=dist.ReduceOp.MIN)
        dist.all_reduce(hi_c, op=dist.ReduceOp.MAX)
    filtered, matches = (int(x) for x in counts.tolist())  # summed over the ranks
    ranks_agree = bool(torch.equal(lo_c, hi_c))
    if a.scaling == "weak":  # every rank joined the whole workload: its own counts are the join's
        filtered, matches = (int(x) for x in hi_c.tolist())
    # warmup on the stream the timed joins use (its first launches set up its hardware queue)
    stream = torch.cuda.Stream()
    for _ in range(a.warmup):
        hw.join_device_async(dR, dS, args, stream=stream)
    warm = hw.join_wait_all(capacity=a.warmup) if a.warmup else []

    # Timed region: K full joins enqueued back to back on one stream (hwbrj_join_device_async: no
    # host round trip between them), bracketed by barrier + synchronize; HIP events on that same
    # stream give the device time of the K joins (the roofline's launch duration).
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(a.steps):
        hw.join_device_async(dR, dS, args, stream=stream)
    ev1.record(stream)
    timed = hw.join_wait_all(capacity=max(a.steps, 1))  # every timed join's own counts
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    dev_ms = ev0.elapsed_time(ev1) / max(a.steps, 1)  # device ms per join on this rank
    # every join is checked, not only the last (the reference sums every thread's count of every
    # run, src/parallel_radix_join_bloom.c:1696-1707): the warmup and each timed join must give the
    # parity run's counts
    ref = (st.filtered, st.matches)
    bad = [i for i, s in enumerate(timed) if (s.filtered, s.matches) != ref]
    wbad = [i for i, s in enumerate(warm) if (s.filtered, s.matches) != ref]
    if len(timed) != a.steps or bad or wbad or len(warm) != a.warmup:
        raise SystemExit(f"timed joins: {len(timed)} collected for {a.steps} enqueued; joins {bad} (warmup "
                         f"{wbad}) differ from the parity run {ref}")
    timed_ok = torch.tensor([len(timed) - len(bad), len(timed)], dtype=torch.int64,
                            device="cpu" if shared else "cuda")
    if dist:
        dist.all_reduce(timed_ok)
    timed_ok = [int(x) for x in timed_ok.tolist()]
    last = timed[-1] if timed else hw.join_wait()

    # per-phase device times (HIP events, one synchronous join each, after the timed region)
    sums = {}
    for _ in range(a.steps):
        st = hw.join_device(dR, dS, args)
        for f in ("ms_total", "ms_r_scatter", "ms_r_index", "ms_build", "ms_s_scatter",
                  "ms_s_index", "ms_probe", "ms_surv", "ms_join"):
            sums[f] = sums.get(f, 0.0) + getattr(st, f)
    # the dominant kernel (k_scatter_s) as the timed joins run it: K more back-to-back async joins,
    # each timing its S scatter with events on the side stream that runs it beside the R side
    # (hwbrj_set_async_timing); the synchronous joins above give the one-stream phase split
    hw.set_async_timing(True)
    try:
        for _ in range(a.steps):
            hw.join_device_async(dR, dS, args, stream=stream)
        tj = hw.join_wait_all(capacity=max(a.steps, 1))
    finally:
        hw.set_async_timing(False)
    if any((s.filtered, s.matches) != ref for s in tj):
        raise SystemExit("the async-timed joins differ from the parity run")
    async_sc = [s.ms_s_scatter for s in tj if s.ms_s_scatter > 0]
    if dist:
        t = torch.tensor([elapsed, dev_ms], dtype=torch.float64, device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, dev_ms = (float(x) for x in t.tolist())
    out = headline_line(a, hw, torch, dist, rank, world, dR, dS, args, st, last, sums, elapsed, dev_ms,
                        total_units, filtered, matches, ranks_agree, per_rank, shared, async_sc) if rank == 0 else None
    if out is not None:
        out["parity"]["timed_joins_ok"] = f"{timed_ok[0]}/{timed_ok[1]}"
        out["parity"]["timed_joins_what"] = ("every timed join's own (filtered, matches) equal to the parity "
                                             "run's (hwbrj_join_wait_all), summed over the ranks")
    # the other multi-GPU designs on the same ranks, after the headline (never its value); every
    # leg runs under its own watchdog: a leg that has not finished in --alt-timeout seconds (a
    # collective that never completes) makes rank 0 print the headline with the legs reported so far
    # and the stalled leg named, and every rank exit with status 124 (a timeout is not a clean run)
    alt = None
    if dist and not a.no_alt_designs and not a.filter_bcast:
        alt = {}
        alt_designs(a, hw, torch, dist, rank, world, local, dR, dS, args, shared, alt, out)
    if rank == 0:
        out["alt_designs"] = alt
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


def headline_line(a, hw, torch, dist, rank, world, dR, dS, args, st, last, sums, elapsed, dev_ms, total_units,
                  filtered, matches, ranks_agree, per_rank, shared, async_sc=()):
    """Rank 0's bench line of the replicated design (its alt_designs are filled in by the caller)."""
    nR, nS_total = a.r_size, a.s_size
    nS = dS.shape[0]
    K = max(a.steps, 1)
    mean = {k: v / K for k, v in sums.items()}
    # Roofline: ALG_BYTES = sizeof(tuple_t) * (|R| + |S|), every input tuple read
    # once; achieved = ALG_BYTES / t / (G * 8 TB/s) with t = the slowest rank's device time per join
    # (HIP events over the timed region). Everything else the pipeline moves is modeled_bytes.
    alg_bytes = 8.0 * (nR + nS_total) if a.scaling == "strong" else 8.0 * (nR + nS) * world
    achieved = alg_bytes / (dev_ms * 1e-3) / 1e9
    peak = HBM_PEAK_GBS * world
    pm, pmc_note = load_pmc(a.pmc_json, [nR, nS, a.s_sel, a.bloom_filter, a.bloom_size, a.bloom_hashes,
                                         a.bloom_block_size], hw.version()) if world == 1 else (None, "N > 1")
    traffic = sum(p.get("hbm_bytes", 0) for p in pm["phases"].values()) if pm else None
    # the dominant kernel against its own s8(d) bytes: k_scatter_s reads every S tuple once (8 B)
    dom = max(("r_scatter", "build", "s_scatter", "probe", "join"), key=lambda p: mean["ms_" + p])
    dom_alg = {"r_scatter": 8.0 * nR, "s_scatter": 8.0 * nS}.get(dom)
    dom_ms_sync = mean["ms_" + dom]
    # its ms in the timed joins' own schedule (S scatter on the side stream beside the R side; the
    # frac below uses it), the one-stream synchronous joins' phase time beside it
    use_async = dom == "s_scatter" and len(async_sc) > 0
    dom_ms = statistics.median(async_sc) if use_async else dom_ms_sync  # (median: one slow join of K moves a mean)
    word_bytes = 4.0  # S partition words (4 bytes in every format)
    roofline = {"bound": "hbm", "achieved": round(achieved, 1), "peak": peak, "unit": "GB/s",
                "frac": round(achieved / peak, 4), "traffic": traffic,
                "algorithmic_bytes": alg_bytes, "launch": "one full join (every kernel of BPRO)",
                "launch_ms": round(dev_ms, 4),
                "modeled_bytes": modeled_bytes(nR, nS, st.filtered, a.bloom_size if args else 0,
                                               word_bytes, join_key_bytes(last)),
                "join_keys": {"format": JOIN_KEY_NAMES.get(last.join_keys), "bits": last.join_key_bits,
                              "unstaged_items": last.unstaged_items,
                              "what": "the key format the timed joins handed to k_join (the last one's "
                                      "hwbrj_stats_t.join_keys)"},
                "pmc_source": os.path.relpath(a.pmc_json, ROOT) if pm else None,
                "pmc_library": pm.get("library") if pm else None,
                "traffic_note": pmc_note,
                "dominant_kernel": {
                    "name": {"s_scatter": "k_scatter_s", "r_scatter": "k_scatter_r",
                             "probe": "k_probe", "build": "k_build", "join": "k_join"}[dom],
                    "ms": round(dom_ms, 4), "algorithmic_bytes": dom_alg,
                    "schedule": ("async two-stream joins (the timed schedule): S scatter events on its side "
                                 f"stream, median of {len(async_sc)} back-to-back joins" if use_async else
                                 "synchronous one-stream joins (phase events)"),
                    "ms_async_min_max": [round(min(async_sc), 4), round(max(async_sc), 4)] if use_async else None,
                    "ms_async_mean": round(statistics.mean(async_sc), 4) if use_async else None,
                    "ms_sync_phase": round(dom_ms_sync, 4),
                    "achieved": round(dom_alg / (dom_ms * 1e-3) / 1e9, 1) if dom_alg else None,
                    "frac": round(dom_alg / (dom_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if dom_alg else None,
                    "traffic": pm["phases"].get(dom, {}).get("hbm_bytes") if pm else None}}

    if world == 1:  # the measured copy rate beside the spec peak (not the frac's denominator)
        cbw = round(hw.copy_bandwidth(4 << 30, 5), 1)
        roofline["copy_measured"] = {"GBps": cbw, "frac_of_copy": round(achieved / cbw, 4),
                                     "what": "hwbrj_copy_bandwidth: streaming 16-byte nt copy of 4 GiB, "
                                             "(read + write) bytes / median time of 5; the spec peak "
                                             "stays the denominator"}
    cpu = None
    if world == 1 and not a.no_cpu_baseline:
        cpu = cpu_baseline(a, hw)
    e2e = None
    if world == 1 and not a.no_e2e:
        e2e = e2e_time(hw, torch, dR, dS, args, nS)

    key = (nR, nS_total, a.s_sel, a.bloom_filter, a.bloom_size, a.bloom_hashes, a.bloom_block_size)
    gold = GOLDEN.get(key)
    value = total_units * a.steps / elapsed
    out = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "probe-tuples/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(elapsed / K * 1e3, 4),
        "higher_is_better": True,
        "scaling": a.scaling,
        "vs_baseline": None,
        "dtype": "int32",
        "data": "synthetic: reference generator key multiset, seeded permutation, in HBM",
        "config": {"workload": f"PRO + -b {a.bloom_filter}, |R|={nR} |S|={nS_total} q={a.s_sel}, "
                               f"m={a.bloom_size} k={a.bloom_hashes} B={a.bloom_block_size}",
                   "r_size": nR, "s_size": nS_total, "selectivity": a.s_sel,
                   "bloom": a.bloom_filter, "m": a.bloom_size, "k": a.bloom_hashes,
                   "B": a.bloom_block_size,
                   "parallelism": (f"dp{world}: every rank the whole |S| (own order), R replicated"
                                   if a.scaling == "weak" else f"S range-sharded x{world}, R replicated"),
                   "filter": ("built on rank 0, ncclBroadcast to every rank" if a.filter_bcast
                              else "rebuilt from R on every rank")},
        "roofline": roofline,
        "cpu_baseline": cpu,
        "e2e": e2e,
        "parity": {"filtered": filtered, "matches": matches,
                   "per": "rank (weak scaling: every rank joined the whole workload)"
                          if a.scaling == "weak" else "sum over the ranks",
                   "ranks_agree": ranks_agree if a.scaling == "weak" else None,
                   "golden": list(gold) if gold else None,
                   "ok": (gold == (filtered, matches) and (ranks_agree or a.scaling != "weak"))
                         if gold else None,
                   "per_rank": per_rank},
        "dist": {"world_size_seen": dist.get_world_size() if dist else 1,
                 "backend": dist.get_backend() if dist else None,
                 "shared_gpu_rehearsal": shared},
        "phase_ms": {k[3:]: round(v, 4) for k, v in mean.items()},
        "alt_designs": None,
        "published_ref": {"value": 3.98e8, "config": "blocked B=512 k=1 m=2^30, 2x Xeon Gold 6226 "
                          "48 threads (thesis data, BASELINE.md)"},
    }
    return out


def pj_async_steps(pjoin, dR, dS, nR, args, K, depth=8, x=None):
    """K async partitioned joins (hwbrj_join_partitioned_rccl_async; with x, a pjoin.TorchExchange:
    hwbrj_join_partitioned_async over its callbacks) back to back, at most `depth` in flight: no
    host wait but the collection of the oldest. Their stats, in order."""
    out, inflight = [], 0
    for _ in range(K):
        if inflight == depth:
            out.append(pjoin.join_partitioned_wait())
            inflight -= 1
        if x is None:
            pjoin.join_partitioned_rccl_async(dR, dS, nR, args)
        else:
            pjoin.join_partitioned_async(dR, dS, nR, args, x)
        inflight += 1
    for _ in range(inflight):
        out.append(pjoin.join_partitioned_wait())
    return out


ALT_LEGS = ("partitioned_async", "bcast", "partitioned")  # by what one node run decides


def alt_designs(a, hw, torch, dist, rank, world, local, dR, dS, args, shared, out, line=None):
    """The designs the headline does not run, timed on the same ranks and shards right after it, so
    one multi-GPU run decides between them:
      bcast        the replicated design with the north_star's bitmap broadcast: rank 0 builds the
                   filter slices, ncclBroadcast sends them (hwbrj_set_filter_broadcast); K joins
                   enqueued back to back, HIP events, max over ranks (one GPU per rank: RCCL);
      partitioned  R range-sharded too, partitions owned by ranks: the R chunk and survivor
                   all-to-alls and the slice all-gather (hwbrj_join_partitioned_rccl; the torch
                   callback transport when ranks share a GPU); host-synchronous, so timed by wall
                   clock between barriers, max over ranks;
      partitioned_async  the same join with padded exchanges and no host wait
                   (hwbrj_join_partitioned_rccl_async; when ranks share a GPU, the same async join
                   over the torch callbacks, host-synchronous): K joins back to back, wall clock
                   between barriers, max over ranks.
    Each leg reports its ms per join, the probe-tuples/s that gives, and every rank's own
    (filtered, matches), whose sums must be the headline's counts. A failing leg is reported, and
    never stops the headline line. The legs run in ALT_LEGS order, the async partitioned join first
    (the design a node run has to decide) and the host-synchronous one last, each under its own
    --alt-timeout watchdog: when one expires, rank 0 prints `line` (the headline) with the legs
    done so far, the stalled leg under "timed_out_leg" and the legs not run, and every rank exits
    with status 124 (a hung collective cannot be abandoned and the next leg started).
    HWBRJ_BENCH_HOOK_STALL_LEG=<leg> (tests only) makes that leg sleep past its watchdog."""
    from hwbloomradixjoin_amd import pjoin
    nR, nS_total = a.r_size, a.s_size
    K = max(1, min(a.steps, a.alt_steps))
    cdev = "cpu" if shared else "cuda"
    out.update({"steps": K, "what": "the other multi-GPU designs on the same ranks and shards after the "
                                    "headline's timed region (DESIGN.md s6); value = |S| / the slowest rank"})

    def gather_counts(st):
        c = torch.tensor([st.filtered, st.matches], dtype=torch.int64, device=cdev)
        g = [torch.empty_like(c) for _ in range(world)]
        dist.all_gather(g, c)
        per = [[int(x) for x in t.tolist()] for t in g]
        return per, [sum(col) for col in zip(*per)]

    def slowest(x):
        t = torch.tensor([x], dtype=torch.float64, device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    stall = os.environ.get("HWBRJ_BENCH_HOOK_STALL_LEG")

    def expire(name):
        if line is not None:
            later = list(ALT_LEGS[ALT_LEGS.index(name) + 1:])
            line["alt_designs"] = dict(out, timed_out_leg=name, timeout_s=a.alt_timeout, not_run=later)
            print(json.dumps(line), flush=True)
        os._exit(124)

    def leg(name, run):
        dog = threading.Timer(a.alt_timeout, expire, args=(name,))
        dog.daemon = True
        dog.start()
        try:
            if stall == name:  # (test hook: a leg that never completes)
                time.sleep(a.alt_timeout * 20 + 5)
            ms, per, tot = run()
            out[name] = {"ms": round(ms, 4), "value": round(nS_total / (ms * 1e-3), 1),
                         "per_rank": per, "sum": tot}
        except Exception as e:  # (reported; the headline stands)
            out[name] = {"failed": str(e)[:300]}
        finally:
            dog.cancel()

    native = not shared
    if native:
        pjoin.comm_init()
    slice_filter = args is not None and not (args.variant == hw.BASIC and args.k > 1)

    def bcast():
        pjoin.set_filter_broadcast(True)
        try:
            per, tot = gather_counts(hw.join_device(dR, dS, args))
            stream = torch.cuda.Stream()
            hw.join_device_async(dR, dS, args, stream=stream)
            hw.join_wait()
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            dist.barrier()
            torch.cuda.synchronize()
            ev0.record(stream)
            for _ in range(K):
                hw.join_device_async(dR, dS, args, stream=stream)
            ev1.record(stream)
            sts = hw.join_wait_all(capacity=K)
            torch.cuda.synchronize()
            dist.barrier()
            if len(sts) != K or any((s.filtered, s.matches) != tuple(per[rank]) for s in sts):
                raise RuntimeError("broadcast joins disagree with its first join")
            return slowest(ev0.elapsed_time(ev1) / K), per, tot
        finally:
            pjoin.set_filter_broadcast(False)

    def partitioned():
        rlo, rhi = hw.shard_range(nR, rank, world)
        dRs = dR[rlo:rhi]
        if native:
            def join():
                return pjoin.join_partitioned_rccl(dRs, dS, nR, args)
        else:
            x = pjoin.TorchExchange(torch.device("cuda", local))

            def join():
                return pjoin.join_partitioned(dRs, dS, nR, args, x)
        per, tot = gather_counts(join())
        join()
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(K):
            join()
        torch.cuda.synchronize()
        dist.barrier()
        return slowest((time.perf_counter() - t0) / K * 1e3), per, tot

    def partitioned_async():
        rlo, rhi = hw.shard_range(nR, rank, world)
        dRs = dR[rlo:rhi]
        x = None if native else pjoin.TorchExchange(torch.device("cuda", local))
        sts = pj_async_steps(pjoin, dRs, dS, nR, args, 2, x=x)  # (the plan join, then one async)
        per, tot = gather_counts(sts[-1])
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        sts = pj_async_steps(pjoin, dRs, dS, nR, args, K, x=x)
        torch.cuda.synchronize()
        dist.barrier()
        if any((s.filtered, s.matches) != (sts[0].filtered, sts[0].matches) for s in sts):
            raise RuntimeError("async partitioned joins disagree")
        return slowest((time.perf_counter() - t0) / K * 1e3), per, tot

    for name in ALT_LEGS:
        if name == "bcast" and not (native and slice_filter):
            out[name] = {"skipped": "needs one GPU per rank (RCCL) and a slice filter"}
        elif name != "bcast" and not (args is None or slice_filter):
            out[name] = {"skipped": "basic k > 1 has no partition slices"}
        else:
            leg(name, {"bcast": bcast, "partitioned": partitioned, "partitioned_async": partitioned_async}[name])
    if native:
        pjoin.comm_destroy()
    return out


def run_partitioned(a, hw, torch, dist, rank, world, local, dR, dS, args, shared):
    """--design partitioned: every step is one hwbrj_join_partitioned on every rank (R and S range
    shards; R chunks and survivors exchanged, slices all-gathered; the exchanges are synchronous,
    so a step is timed by wall clock between barriers + synchronize)."""
    from hwbloomradixjoin_amd import pjoin
    nR, nS_total = a.r_size, a.s_size
    native = a.transport == "native" and not shared
    use_async = native and not a.pj_sync
    if native:  # the library's own RCCL communicator, collectives on the join stream
        pjoin.comm_init()

        def join():
            return pjoin.join_partitioned_rccl(dR, dS, nR, args)
    else:  # torch.distributed callbacks (HWBRJ_PJ_FORCE_COLL=1: collectives even at world 1)
        x = pjoin.TorchExchange(torch.device("cuda", local),
                                force_collectives=os.environ.get("HWBRJ_PJ_FORCE_COLL") == "1")

        def join():
            return pjoin.join_partitioned(dR, dS, nR, args, x)
    cdev = "cpu" if shared else "cuda"
    if use_async:  # (the first async join runs synchronously and makes the exchange plan)
        st = pj_async_steps(pjoin, dR, dS, nR, args, 1)[0]
    else:
        st = join()
    counts = torch.tensor([st.filtered, st.matches], dtype=torch.int64, device=cdev)
    if dist:
        dist.all_reduce(counts)
    filtered, matches = (int(v) for v in counts.tolist())
    if use_async:
        pj_async_steps(pjoin, dR, dS, nR, args, a.warmup)
    else:
        for _ in range(a.warmup):
            join()
    info0 = pjoin.pj_async_info() if use_async else None
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    sums = {}
    if use_async:  # K joins enqueued back to back (<= 8 in flight), no host wait between them
        sts = pj_async_steps(pjoin, dR, dS, nR, args, a.steps)
        sums["ms_total"] = sum(s.ms_total for s in sts)
        same = all((s.filtered, s.matches) == (st.filtered, st.matches) for s in sts)
    else:
        for _ in range(a.steps):
            st = join()
            for f in ("ms_total", "ms_r_scatter", "ms_r_index", "ms_build", "ms_s_scatter", "ms_surv",
                      "ms_join"):
                sums[f] = sums.get(f, 0.0) + getattr(st, f)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if use_async:
        info1 = pjoin.pj_async_info()
        async_rep = {"plan_blocks": {"BR_chunks": info1["BR"], "BI_items": info1["BI"], "BW_words": info1["BW"]},
                     "reruns_in_timed": info1["overflow_reruns"] - info0["overflow_reruns"],
                     "async_in_timed": info1["async_joins"] - info0["async_joins"],
                     "events_ms_per_join_rank0": round(sums["ms_total"] / max(a.steps, 1), 4),
                     "rank0_counts_all_equal": bool(same),
                     "timing": "wall clock over K joins enqueued back to back; events: each join's "
                               "first to last operation on the join stream (HIP events)"}
    else:
        async_rep = None
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    if rank != 0:
        if native:
            pjoin.comm_destroy()
        if dist:
            dist.destroy_process_group()
        return
    K = max(a.steps, 1)
    ms = elapsed / K * 1e3
    alg_bytes = 8.0 * (nR + nS_total)
    achieved = alg_bytes / (ms * 1e-3) / 1e9
    key = (nR, nS_total, a.s_sel, a.bloom_filter, a.bloom_size, a.bloom_hashes, a.bloom_block_size)
    gold = GOLDEN.get(key)
    out = {
        "metric": METRIC, "value": round(nS_total * a.steps / elapsed, 1), "unit": "probe-tuples/s",
        "n_gpus": world, "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(ms, 4),
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "int32",
        "data": "synthetic: reference generator key multiset, seeded permutation, in HBM",
        "config": {"workload": f"PRO + -b {a.bloom_filter}, |R|={nR} |S|={nS_total} q={a.s_sel}, "
                               f"m={a.bloom_size} k={a.bloom_hashes} B={a.bloom_block_size}",
                   "r_size": nR, "s_size": nS_total, "selectivity": a.s_sel,
                   "bloom": a.bloom_filter, "m": a.bloom_size, "k": a.bloom_hashes,
                   "B": a.bloom_block_size,
                   "parallelism": f"R and S range-sharded x{world}, partitions owned by ranks "
                                  "(R + survivor all-to-all, slice all-gather)",
                   "transport": ("native RCCL (join stream), async: padded exchanges" if use_async else
                                 "native RCCL (join stream), synchronous" if native else
                                 "torch.distributed callbacks")},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS * world,
                     "unit": "GB/s", "frac": round(achieved / (HBM_PEAK_GBS * world), 4),
                     "traffic": None, "algorithmic_bytes": alg_bytes,
                     "launch": "one partitioned join (kernels and exchanges, wall clock)",
                     "launch_ms": round(ms, 4)},
        "cpu_baseline": None,
        "parity": {"filtered": filtered, "matches": matches, "golden": list(gold) if gold else None,
                   "ok": (gold == (filtered, matches)) if gold else None},
        "dist": {"world_size_seen": dist.get_world_size() if dist else 1,
                 "backend": dist.get_backend() if dist else None, "shared_gpu_rehearsal": shared},
        "stage_ms_rank0": {k[3:]: round(v / K, 4) for k, v in sums.items()},
        "pj_async": async_rep,
    }
    print(json.dumps(out), flush=True)
    if native:
        pjoin.comm_destroy()
    if dist:
        dist.destroy_process_group()


def load_pmc(path: str, key: list, library: str):
    """Per-phase HBM bytes of one join (tools/prof_summary.py output) when they were collected on
    this exact configuration AND on a library with this run's stamp (hwbrj_version(): the hash of
    the product sources and every non-default knob), else None. Returns (pmc or None, note)."""
    try:
        pm = json.load(open(path))
    except (OSError, ValueError):
        return None, f"{os.path.relpath(path, ROOT)} missing"
    if pm.get("config_key") != key:
        return None, "no PMC traffic profiled for this configuration"
    if pm.get("library") != library:
        return None, (f"PMC traffic was profiled on '{pm.get('library')}', this run's library is "
                      f"'{library}': not used")
    return pm, "PMC traffic of this library (FETCH_SIZE x2 + WRITE_SIZE, one join)"


def host_cpu() -> dict:
    """The host's CPU model, logical CPU count and the CPUs this process may run on."""
    model = "unknown"
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                model = ln.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    allowed = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    return {"model": model, "nproc": os.cpu_count(), "allowed_cpus": allowed}


# Calibration (BASELINE.md "Calibration of the CPU port"): on the same 8-core host the reference
# binary needs 6.0 s where this port needs 13.0-13.6 s (C2, -n 8, re-measured in round 3), i.e. the
# port runs at 0.45x it.
def filter_calibration(orc, R, S, variant, m, k, B, threads, nprobe=64_000_000):
    """The reference's OWN filter code (oracle/_ref/libbloomref.so: its src/hash.c and
    src/bloom_filter.c compiled unmodified) against the port's (oracle/oracle.c) on this host, at
    `threads` threads over the same keys: the add loop over R and the contains loop over the first
    `nprobe` S keys, ns per key per thread. These loops are where the reference spends ~90 % of its
    time, so their ratio is the port's calibration, measured where it runs."""
    import ctypes
    import threading

    import numpy as np
    if not orc.have_ref():
        return None
    rk = np.ascontiguousarray(R[:, 0])
    sk = np.ascontiguousarray(S[: min(nprobe, S.shape[0]), 0])

    def par(fn, keys):
        per = keys.shape[0] // threads
        ts = [threading.Thread(target=fn, args=(keys.ctypes.data + 4 * t * per,
                                                per if t < threads - 1 else keys.shape[0] - per * t))
              for t in range(threads)]
        t0 = time.perf_counter()
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        return (time.perf_counter() - t0) * 1e9 * threads / max(1, keys.shape[0])

    ra = orc._RefArgs(variant, m, k, B)
    st = orc.ref().bloom_filter_create(ctypes.byref(ra), 42)
    ref_add = par(lambda p, n: orc.ref().ref_add_all(st, p, n), rk)
    ref_has = par(lambda p, n: orc.ref().ref_count(st, p, n), sk)
    orc.ref().bloom_filter_destroy(st)
    f = orc._Bloom()
    L = orc.lib()
    if L.orc_bloom_init(ctypes.byref(f), variant, m, k, B, 42):
        return None
    port_add = par(lambda p, n: L.orc_bloom_add_all_atomic(ctypes.byref(f), p, n), rk)
    port_has = par(lambda p, n: L.orc_count_filtered(ctypes.byref(f), p, n), sk)
    L.orc_bloom_free(ctypes.byref(f))
    return {"threads": threads, "keys_add": int(rk.shape[0]), "keys_contains": int(sk.shape[0]),
            "ns_per_key_thread": {"reference_add": round(ref_add, 1), "port_add": round(port_add, 1),
                                  "reference_contains": round(ref_has, 1), "port_contains": round(port_has, 1)},
            "port_vs_reference_contains": round(ref_has / port_has, 3),
            "what": "the reference's own bloom_filter.c (libbloomref.so, built from its sources) vs the "
                    "port's filter code, same keys, same threads, this host; >1 = the port is faster"}


def cpu_baseline(a, hw):
    """The oracle's pthreads restatement of BPRO (oracle/oracle.c, "port") on the GPU host's CPU:
    full |R| and filter, the first --cpu-sample tuples of S (default: all of it), timed over the
    reference's TOTAL-TIME region, once on every CPU this process may use (capped by
    OMP_NUM_THREADS, the box's CPU share) and once at 8 threads (the reference's measured -n 8).
    Beside it, the calibration: the reference's own filter loops against the port's, measured on
    this host (filter_calibration)."""
    info = host_cpu()
    try:
        from oracle import pyoracle as orc
        sample = min(a.cpu_sample, a.s_size) if a.cpu_sample > 0 else a.s_size
        cap = int(os.environ.get("OMP_NUM_THREADS") or info["allowed_cpus"])
        threads = a.cpu_threads if a.cpu_threads > 0 else max(1, min(info["allowed_cpus"], cap))
        R = hw.generate_host(a.r_size, a.nthreads, a.r_size, a.r_size, 1.0, 12345, threads)
        # a |S|=sample relation of the same generator (same q, same key ranges)
        S = hw.generate_host(sample, a.nthreads, 2**31 - 1, a.r_size, a.s_sel, 54321, threads)
        variant = {"basic": 0, "blocked": 1, "sectorized": 2}.get(a.bloom_filter, 0)
        use = a.bloom_filter != "no"
        runs = {}
        for t in sorted({threads, 8}):
            res, filt, tm = orc.bpro(R, S, t, variant, a.bloom_size, a.bloom_hashes,
                                     a.bloom_block_size, use)
            runs[t] = (sample / (tm["total"] / 1e6), tm["total"] / 1e6, filt, res,
                       [round(x / 1e6, 3) for x in tm["phases"]])
        v, secs, filt, res, phases = runs[threads]
        cal = None
        if use and variant != 2:  # (the reference has no sectorized filter)
            try:
                cal = filter_calibration(orc, R, S, variant, a.bloom_size, a.bloom_hashes,
                                         a.bloom_block_size, threads)
            except Exception as e:  # noqa: BLE001 (reported, never required)
                cal = {"failed": str(e)}
        return {"value": round(v, 1), "unit": "probe-tuples/s", "cores": threads, "kind": "port",
                "host": info, "value_n8": round(runs[8][0], 1),
                "cores_cap": (f"OMP_NUM_THREADS={cap}: the GPU pool's CPU share for one GPU's job "
                              "(BASELINE.md)"),
                "phases_s": dict(zip(("r_loop1_add", "r_scatter", "s_loop1_contains", "s_scatter",
                                      "pass2", "join"), phases)),
                "calibration": cal,
                "sample": (f"|R|={a.r_size}, |S|={sample} tuples of the same generator "
                           f"(q={a.s_sel}), m={a.bloom_size}"
                           + (" (the full workload)" if sample == a.s_size else " (S sample)")
                           + f"; oracle orc_bpro TOTAL-TIME {secs:.3f} s on {threads} threads "
                           f"({runs[8][1]:.3f} s on 8), filtered={filt} matches={res}. "
                           "calibration: the reference's own filter code timed beside the port's "
                           "on this host (BASELINE.md)")}
    except Exception as e:  # the baseline is reported, never required for the GPU line
        return {"value": None, "unit": "probe-tuples/s", "cores": None, "kind": "port",
                "host": info, "sample": f"failed: {e}"}


if __name__ == "__main__":
    main()
