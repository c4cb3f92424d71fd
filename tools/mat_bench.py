"""Dev: time the materializing join (count pipeline + pairs pass) at the north-star shape."""
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
for i in range(3):
    st, pairs, ms = hw.join_materialize_device(dR, dS, args)
    ok = pairs.shape[0] == st.matches
    # every pair joins equal keys: R payload = R row, S payload = S row (generator layout)
    chk = bool((dR[pairs[:, 0].long(), 0] == dS[pairs[:, 1].long(), 0]).all().item())
    print(f"q={q} count-join {st.ms_total:.3f} ms + pairs pass {ms:.3f} ms, pairs {pairs.shape[0]} "
          f"(= matches: {ok}, keys equal: {chk})", flush=True)
    del pairs
# the R table build alone (one S tuple)
st, pairs, ms = hw.join_materialize_device(dR, dS[:1], args)
print(f"R table build + 1-tuple probe: {ms:.3f} ms", flush=True)
