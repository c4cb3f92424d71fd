"""Basic filter, k = 1..4, at the north-star sizes (|R| = 128M, |S| = 1024M, q = 0.01, m = 2^30):
per-phase device times and counts against the goldens (KIND_BASIC_KK for k >= 2).
    python tools/basic_kk.py
"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import hwbloomradixjoin_amd as hw

nR, nS, INT_MAX = 128000000, 1024000000, 2**31 - 1
gold = {1: 124152740, 2: 55852594, 3: 37788150}
dR = torch.empty((nR, 2), dtype=torch.int32, device="cuda")
dS = torch.empty((nS, 2), dtype=torch.int32, device="cuda")
hw.generate_device(dR, 2, nR, nR, 1.0, 12345)
hw.generate_device(dS, 2, INT_MAX, nR, 0.01, 54321)
torch.cuda.synchronize()
for k in [int(a) for a in sys.argv[1:]] or (1, 2, 3, 4):
    best = None
    for _ in range(3):
        st = hw.join_device(dR, dS, hw.BloomFilterArgs(hw.BASIC, 1 << 30, k, 1024))
        best = st if best is None or st.ms_total < best.ms_total else best
    ok = "" if k not in gold else (" OK" if (best.filtered, best.matches) == (gold[k], 10240000) else " MISMATCH")
    print(f"basic k={k}: {best.ms_total:7.3f} ms | r_sc {best.ms_r_scatter:.3f} build {best.ms_build:.3f} "
          f"s_sc {best.ms_s_scatter:.3f} probe {best.ms_probe:.3f} surv {best.ms_surv:.3f} join {best.ms_join:.3f} | "
          f"filtered {best.filtered} matches {best.matches}{ok}", flush=True)
