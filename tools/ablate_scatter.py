"""Time k_scatter on S with ablations (dev-only; results are invalid while ablated)."""
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
for rep in range(2):
    for ab in [0, 1, 2, 3, 4, 7, 8, 12]:
        for sce in ["4", "8"]:
            os.environ["HWBRJ_SC_ABLATE"] = str(ab)
            os.environ["HWBRJ_SCE"] = sce
            try:
                st = hw.join_device(dR, dS, args)
                print(f"ablate={ab:2d} sce={sce} s_scatter={st.ms_s_scatter:.3f} r_scatter={st.ms_r_scatter:.3f}", flush=True)
            except Exception as e:
                print(f"ablate={ab} sce={sce} error {e}", flush=True)
os.environ["HWBRJ_SC_ABLATE"] = "0"
st = hw.join_device(dR, dS, args)
print("final", st.filtered, st.matches)
