"""torch.distributed.run worker of tests/test_gpu_multi.py (not a test module): the partitioned
join of the F3 relations, R and S range-sharded over the ranks, with rank argv[1] made to fail its
shard check (hwbrj_set_test_hook HWBRJ_HOOK_PJ_FAIL_RANK, -1 = none). The ranks share the one GPU
and exchange through torch.distributed over gloo (pjoin.TorchExchange). Exit 0 with rank 0 printing
"sum: ok filtered matches" (summed over the ranks), or 3 with the library's error on stderr."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import hwbloomradixjoin_amd as hw  # noqa: E402
from hwbloomradixjoin_amd import pjoin  # noqa: E402


def main():
    fail, r, s, m = (int(x) for x in sys.argv[1:5])
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    hw.lib().hwbrj_set_device(0)
    dist.init_process_group("gloo")
    hw.set_test_hook(hw.HOOK_PJ_FAIL_RANK, fail)
    rlo, rhi = hw.shard_range(r, rank, world)
    lo, hi = hw.shard_range(s, rank, world)
    dR = torch.empty((rhi - rlo, 2), dtype=torch.int32, device="cuda")
    dS = torch.empty((hi - lo, 2), dtype=torch.int32, device="cuda")
    hw.generate_device_range(dR, r, rlo, 2, r, r, 1.0, 12345)
    hw.generate_device_range(dS, s, lo, 2, 2**31 - 1, r, 0.01, 54321)
    try:
        st = pjoin.join_partitioned(dR, dS, r, hw.BloomFilterArgs(hw.BLOCKED, m, 1, 1024))
    except RuntimeError as e:
        print(f"rank {rank}: {e}", file=sys.stderr, flush=True)
        sys.exit(3)
    t = torch.tensor([st.filtered, st.matches], dtype=torch.int64)
    dist.all_reduce(t)  # (gloo: host tensors)
    if rank == 0:
        print(f"sum: ok {int(t[0])} {int(t[1])}", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
