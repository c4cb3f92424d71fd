"""Dev: time the materializing join at the north-star shape (one pass of the partitioned pipeline
with payloads: k_scatter_*p, k_build, k_probe with survivor positions, k_join_mat)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import hwbloomradixjoin_amd as hw
nR, nS = 128000000, 1024000000
q = float(sys.argv[1]) if len(sys.argv) > 1 else 0.01
dR = torch.empty((nR, 2), dtype=torch.int32, device="cuda")
dS = torch.empty((nS, 2), dtype=torch.int32, device="cuda")
hw.generate_device(dR, 2, nR, nR, 1.0, 12345)
hw.generate_device(dS, 2, 2**31 - 1, nR, q, 54321)
args = hw.BloomFilterArgs(hw.BLOCKED, 1 << 30, 1, 1024)
cap = int(q * nS) + 1
for i in range(4):
    st, pairs, ms = hw.join_materialize_device(dR, dS, args, capacity=cap)
    chk = bool((dR[pairs[:, 0].long(), 0] == dS[pairs[:, 1].long(), 0]).all().item())
    print(f"q={q} materializing join {ms:.3f} ms: r_sc {st.ms_r_scatter:.3f} r_ix {st.ms_r_index:.3f} "
          f"build {st.ms_build:.3f} s_sc {st.ms_s_scatter:.3f} s_ix {st.ms_s_index:.3f} probe {st.ms_probe:.3f} "
          f"join {st.ms_join:.3f}; filtered {st.filtered} pairs {pairs.shape[0]} (keys equal: {chk})", flush=True)
    del pairs
