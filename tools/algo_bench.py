"""Dev: the per-partition join functions (PRO / PRH / PRHO, hwbrj_join_device_algo) at the north
star, and basic k = 1 (whose jobs take the hash path): best-of-4 device times per phase."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import hwbloomradixjoin_amd as hw
nR, nS = 128000000, 1024000000
dR = torch.empty((nR, 2), dtype=torch.int32, device="cuda")
dS = torch.empty((nS, 2), dtype=torch.int32, device="cuda")
hw.generate_device(dR, 2, nR, nR, 1.0, 12345)
hw.generate_device(dS, 2, 2**31 - 1, nR, 0.01, 54321)
args = hw.BloomFilterArgs(hw.BLOCKED, 1 << 30, 1, 1024)
basic = hw.BloomFilterArgs(hw.BASIC, 1 << 30, 1, 1024)
for name, algo, a in (("BPRO", hw.ALGO_PRO, args), ("BPRH", hw.ALGO_PRH, args), ("BPRHO", hw.ALGO_PRHO, args),
                      ("basic1", hw.ALGO_PRO, basic)):
    best = None
    for _ in range(4):
        st = hw.join_device(dR, dS, a, algorithm=algo)
        best = st if best is None or st.ms_total < best.ms_total else best
    print(f"{name:6s} total {best.ms_total:.3f} ms join {best.ms_join:.3f} ms "
          f"(filtered {best.filtered}, matches {best.matches})", flush=True)
