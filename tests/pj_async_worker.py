"""torch.distributed.run worker of tests/test_gpu_multi.py (not a test module): the async
partitioned join (hwbrj_join_partitioned_async over pjoin.TorchExchange, gloo) of the F3 relations,
R and S range-sharded over the ranks, which share the one GPU. Scenario argv[1]:
  steady   the plan join, then 3 async joins back to back (no rerun)
  overflow a plan made too small (HWBRJ_HOOK_PJ_PLAN_DIV): the next join overflows on some rank,
           every rank reruns it synchronously
  shape    after a plan, rank 1's S shard changes size alone (the failed mode on that rank): every
           rank reruns the join
  fail1    rank 1 runs the async join in the failed mode (HWBRJ_HOOK_PJ_ASYNC_FAIL)
argv[5] (optional): the filter, "blocked" (k = 1, B = 1024; the default), "sect" or "pro".
Rank 0 prints "sum: ok filtered matches" per join (each summed over the ranks) and the async-info
deltas as "info: async reruns"; exit 3 with the library's error on stderr."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import hwbloomradixjoin_amd as hw  # noqa: E402
from hwbloomradixjoin_amd import pjoin  # noqa: E402


def main():
    scen = sys.argv[1]
    r, s, m = (int(x) for x in sys.argv[2:5])
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    hw.lib().hwbrj_set_device(0)
    dist.init_process_group("gloo")
    rlo, rhi = hw.shard_range(r, rank, world)
    lo, hi = hw.shard_range(s, rank, world)
    dR = torch.empty((rhi - rlo, 2), dtype=torch.int32, device="cuda")
    dS = torch.empty((hi - lo, 2), dtype=torch.int32, device="cuda")
    hw.generate_device_range(dR, r, rlo, 2, r, r, 1.0, 12345)
    hw.generate_device_range(dS, s, lo, 2, 2**31 - 1, r, 0.01, 54321)
    # (argv[5], optional: "pro" = no filter, "sect" = sectorized k = 2 B = 512; default blocked k = 1)
    flt = sys.argv[5] if len(sys.argv) > 5 else "blocked"
    args = {"blocked": hw.BloomFilterArgs(hw.BLOCKED, m, 1, 1024), "pro": None,
            "sect": hw.BloomFilterArgs.from_flag("sectorized", m, 2, 512)}[flt]
    x = pjoin.TorchExchange(torch.device("cuda", 0))

    def report(sts):
        for st in sts:
            t = torch.tensor([st.filtered, st.matches], dtype=torch.int64)
            dist.all_reduce(t)
            if rank == 0:
                print(f"sum: ok {int(t[0])} {int(t[1])}", flush=True)

    try:
        i0 = pjoin.pj_async_info()
        if scen == "overflow":
            hw.set_test_hook(hw.HOOK_PJ_PLAN_DIV, 8)
        pjoin.join_partitioned_async(dR, dS, r, args, x)  # (synchronous: the plan)
        report([pjoin.join_partitioned_wait()])
        i1 = pjoin.pj_async_info()
        if scen == "shape" and rank == 1:
            dS = dS[: dS.shape[0] - 1000]  # (the F3 counts then change: the sum is checked by count)
        if scen == "fail1" and rank == 1:
            hw.set_test_hook(hw.HOOK_PJ_ASYNC_FAIL, 1)
        n = 3 if scen == "steady" else 1
        for _ in range(n):
            pjoin.join_partitioned_async(dR, dS, r, args, x)
        report([pjoin.join_partitioned_wait() for _ in range(n)])
        i2 = pjoin.pj_async_info()
        if scen == "shape":  # the synchronous join of the same (changed) shards, for reference
            st = pjoin.join_partitioned(dR, dS, r, args, x)
            t = torch.tensor([st.filtered, st.matches], dtype=torch.int64)
            dist.all_reduce(t)
            if rank == 0:
                print(f"sync: {int(t[0])} {int(t[1])}", flush=True)
        if rank == 0:
            print(f"info: {i2['async_joins'] - i1['async_joins']} {i2['overflow_reruns'] - i1['overflow_reruns']} "
                  f"{i2['last_rerun_flag']} {i1['sync_plan_joins'] - i0['sync_plan_joins']}", flush=True)
    except RuntimeError as e:
        print(f"rank {rank}: {e}", file=sys.stderr, flush=True)
        sys.exit(3)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
