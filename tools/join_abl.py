"""Dev: mean phase ms (every phase of hwbrj_stats_t) of N synchronous north-star joins (HWBRJ_LIB selects the library;
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
PH = ("r_scatter", "r_index", "build", "s_scatter", "s_index", "probe", "join", "total")
acc = {k: 0.0 for k in PH}
for i in range(steps):
    st = hw.join_device(dR, dS, args)
    for k in PH:
        acc[k] += getattr(st, "ms_" + k)
print(os.environ.get("HWBRJ_LIB", "tree"), " ".join("%s %.4f" % (k, acc[k] / steps) for k in PH),
      "counts", st.filtered, st.matches, flush=True)
