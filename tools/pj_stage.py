"""Dev: one rank's work at G-way scaling on one GPU (north-star shapes): the replicated design
(full R, S/G) against the partitioned one (R/G and S/G shards; with world = 1 its exchanges are
local copies, so the stage times are the rank's compute plus those copies).
    python tools/pj_stage.py [G ...]"""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import hwbloomradixjoin_amd as hw
from hwbloomradixjoin_amd import pjoin
nR, nS = 128000000, 1024000000
args = hw.BloomFilterArgs(hw.BLOCKED, 1 << 30, 1, 1024)
for G in [int(x) for x in sys.argv[1:]] or [1, 8]:
    dR = torch.empty((nR, 2), dtype=torch.int32, device="cuda")
    hw.generate_device(dR, 2, nR, nR, 1.0, 12345)
    dS = torch.empty((nS // G, 2), dtype=torch.int32, device="cuda")
    hw.generate_device_range(dS, nS, 0, 2, 2**31 - 1, nR, 0.01, 54321)
    best = None
    for i in range(4):
        st = hw.join_device(dR, dS, args)
        best = st if best is None or st.ms_total < best.ms_total else best
    print(f"G={G} replicated rank: total {best.ms_total:.3f} ms (r_sc {best.ms_r_scatter:.3f} build {best.ms_build:.3f} "
          f"s_sc {best.ms_s_scatter:.3f} probe {best.ms_probe:.3f} join {best.ms_join:.3f}) counts {best.filtered} {best.matches}", flush=True)
    dRs = dR[: nR // G].contiguous()
    del dR
    torch.cuda.empty_cache()
    x = pjoin.TorchExchange(torch.device("cuda", 0))
    best = None
    for i in range(4):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        st = pjoin.join_partitioned(dRs, dS, nR, args, x)
        wall = (time.perf_counter() - t0) * 1e3
        if best is None or wall < best[0]:
            best = (wall, st)
    w, st = best
    print(f"G={G} partitioned rank (world 1, torch callbacks): wall {w:.3f} ms: R pass {st.ms_r_scatter:.3f} R xchg {st.ms_r_index:.3f} "
          f"build {st.ms_build:.3f} S pass {st.ms_s_scatter:.3f} xchg(slices+surv) {st.ms_surv:.3f} join {st.ms_join:.3f} "
          f"counts {st.filtered} {st.matches}", flush=True)
    # the same rank over the library's own RCCL communicator (world 1: send/recv to self)
    pjoin.comm_init()
    best = None
    for i in range(4):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        st = pjoin.join_partitioned_rccl(dRs, dS, nR, args)
        wall = (time.perf_counter() - t0) * 1e3
        if best is None or wall < best[0]:
            best = (wall, st)
    # the async form: 8 joins enqueued back to back after the plan join, each join's device time
    # from its HIP events, and the wall time of the 8
    pjoin.join_partitioned_rccl_async(dRs, dS, nR, args)
    pjoin.join_partitioned_wait()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(8):
        pjoin.join_partitioned_rccl_async(dRs, dS, nR, args)
    sts = [pjoin.join_partitioned_wait() for i in range(8)]
    wall8 = (time.perf_counter() - t0) * 1e3 / 8
    info = pjoin.pj_async_info()
    pjoin.comm_destroy()
    ev = sorted(x.ms_total for x in sts)
    print(f"G={G} partitioned rank (world 1, native RCCL, async): wall {wall8:.3f} ms per join over 8, events "
          f"median {ev[4]:.3f} min {ev[0]:.3f} ms; reruns {info['overflow_reruns']}, plan BR {info['BR']} BI {info['BI']} "
          f"BW {info['BW']}; counts {sts[-1].filtered} {sts[-1].matches}", flush=True)
    w, st = best
    print(f"G={G} partitioned rank (world 1, native RCCL): wall {w:.3f} ms: R pass {st.ms_r_scatter:.3f} R xchg {st.ms_r_index:.3f} "
          f"build {st.ms_build:.3f} S pass {st.ms_s_scatter:.3f} xchg(slices+surv) {st.ms_surv:.3f} join {st.ms_join:.3f} "
          f"counts {st.filtered} {st.matches}", flush=True)
    del dRs, dS, x
    torch.cuda.empty_cache()
