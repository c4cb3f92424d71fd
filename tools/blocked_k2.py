"""Dev: BASELINE config-3 rows with k >= 2 on the LDS-slice path (blocked B=1024/512, sectorized),
|R| = 128M, |S| = 1024M, q = 0.01, m = 2^30: best-of-3 device times."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import hwbloomradixjoin_amd as hw
nR, nS = 128000000, 1024000000
dR = torch.empty((nR, 2), dtype=torch.int32, device="cuda")
dS = torch.empty((nS, 2), dtype=torch.int32, device="cuda")
hw.generate_device(dR, 2, nR, nR, 1.0, 12345)
hw.generate_device(dS, 2, 2**31 - 1, nR, 0.01, 54321)
for name, a in (("blocked B=1024 k=2", hw.BloomFilterArgs(hw.BLOCKED, 1 << 30, 2, 1024)),
                ("blocked B=512 k=2", hw.BloomFilterArgs(hw.BLOCKED, 1 << 30, 2, 512)),
                ("sectorized k=2", hw.BloomFilterArgs(hw.SECTORIZED, 1 << 30, 2, 1024)),
                ("blocked B=512 k=3", hw.BloomFilterArgs(hw.BLOCKED, 1 << 30, 3, 512))):
    best = None
    for _ in range(3):
        st = hw.join_device(dR, dS, a)
        best = st if best is None or st.ms_total < best.ms_total else best
    print(f"{os.environ.get('TAG', 'CUR'):6s} {name:20s} total {best.ms_total:.3f} probe {best.ms_probe:.3f} "
          f"join {best.ms_join:.3f} filtered {best.filtered} matches {best.matches}", flush=True)
