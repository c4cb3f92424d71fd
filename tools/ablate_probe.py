"""Time k_probe with ablations (dev-only; results are invalid while ablated)."""
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
knob = sys.argv[1] if len(sys.argv) > 1 else "HWBRJ_PR_ABLATE"
vals = sys.argv[2].split(",") if len(sys.argv) > 2 else ["0", "1", "2", "3"]
for rep in range(2):
    for ab in vals:
        os.environ[knob] = ab
        st = hw.join_device(dR, dS, args)
        print(f"{knob}={ab:3s} total={st.ms_total:.3f} s_scatter={st.ms_s_scatter:.3f} s_index={st.ms_s_index:.3f} probe={st.ms_probe:.3f} join={st.ms_join:.3f} build={st.ms_build:.3f} filtered={st.filtered} matches={st.matches}", flush=True)
os.environ[knob] = "0"
