"""Dev: mean join-phase ms of N synchronous north-star joins (HWBRJ_LIB selects the library;
ablation builds give invalid counts, which are printed, not checked)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import hwbloomradixjoin_amd as hw
steps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
nR, nS = 128000000, 1024000000
dR = torch.empty((nR, 2), dtype=torch.int32, device="cuda")
dS = torch.empty((nS, 2), dtype=torch.int32, device="cuda")
hw.generate_device(dR, 2, nR, nR, 1.0, 12345)
hw.generate_device(dS, 2, 2**31 - 1, nR, 0.01, 54321)
args = hw.BloomFilterArgs(hw.BLOCKED, 1 << 30, 1, 1024)
hw.join_device(dR, dS, args)
js, ts = [], []
for i in range(steps):
    st = hw.join_device(dR, dS, args)
    js.append(st.ms_join)
    ts.append(st.ms_total)
print(os.environ.get("HWBRJ_LIB", "tree"), "join", round(sum(js) / steps, 4), "total", round(sum(ts) / steps, 4),
      "counts", st.filtered, st.matches, flush=True)
