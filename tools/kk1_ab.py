"""A/B of the basic k = 1 pipelines at the north-star sizes (|R| = 128M, |S| = 1024M, q = 0.01,
m = 2^30): A = the slice path (bmix words, the join's hash tables), B = the
bit-pass path of k >= 2 (HWBRJ_DEV_KK1: survivors re-partitioned by code, R partitioned by code,
bitmap join). Alternating runs, best of 5 each; counts against the published row 124,152,740.
    python tools/kk1_ab.py
"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import hwbloomradixjoin_amd as hw

nR, nS, INT_MAX = 128000000, 1024000000, 2**31 - 1
dR = torch.empty((nR, 2), dtype=torch.int32, device="cuda")
dS = torch.empty((nS, 2), dtype=torch.int32, device="cuda")
hw.generate_device(dR, 2, nR, nR, 1.0, 12345)
hw.generate_device(dS, 2, INT_MAX, nR, 0.01, 54321)
torch.cuda.synchronize()
a = hw.BloomFilterArgs(hw.BASIC, 1 << 30, 1, 1024)
best = {}
for rep in range(6):
    for name in ("A slice", "B bitpass"):
        if name.startswith("B"):
            os.environ["HWBRJ_DEV_KK1"] = "1"
        else:
            os.environ.pop("HWBRJ_DEV_KK1", None)
        st = hw.join_device(dR, dS, a)
        assert (st.filtered, st.matches) == (124152740, 10240000), (name, st.filtered, st.matches)
        if rep and (name not in best or st.ms_total < best[name].ms_total):
            best[name] = st
for name, st in best.items():
    print(f"basic k=1 {name:10s}: {st.ms_total:7.3f} ms | r_sc {st.ms_r_scatter:.3f} r_ix {st.ms_r_index:.3f} "
          f"build {st.ms_build:.3f} s_sc {st.ms_s_scatter:.3f} s_ix {st.ms_s_index:.3f} probe {st.ms_probe:.3f} "
          f"surv {st.ms_surv:.3f} join {st.ms_join:.3f} | filtered {st.filtered} matches {st.matches}", flush=True)
