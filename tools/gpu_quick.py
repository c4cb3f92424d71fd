"""First-contact GPU check: small joins vs the oracle, then the north-star shape."""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import hwbloomradixjoin_amd as hw
from oracle import pyoracle as orc

def run(nR, nS, q, variant, m, k, B, nthr=2, check=True):
    R = orc.relation(nR, nthr, nR, nR, 1.0, 1)
    S = orc.relation(nS, nthr, 2**31 - 1, nR, q, 2)
    dR = torch.from_numpy(R).cuda(); dS = torch.from_numpy(S).cuda()
    args = None if variant is None else hw.BloomFilterArgs(variant, m, k, B)
    st = hw.join_device(dR, dS, args)
    line = f"nR={nR} nS={nS} q={q} var={variant} m={m} k={k} B={B}: filtered={st.filtered} matches={st.matches} mode={st.mode} fmt={st.format} F={st.partitions} NSUB={st.subparts} ms={st.ms_total:.3f}"
    if check:
        res, filt, _ = orc.bpro(R, S, 8, variant if variant is not None else 0, m, k, B, variant is not None)
        ok = (res == st.matches) and (filt == st.filtered)
        line += f" | oracle filtered={filt} matches={res} {'OK' if ok else 'MISMATCH'}"
    print(line, flush=True)

run(1000, 16000, 0.01, 1, 2**16, 1, 1024)
run(100000, 1000000, 0.01, 1, 2**22, 1, 1024)
run(1000000, 16000000, 0.01, 1, 2**24, 1, 1024)
run(1000000, 16000000, 0.01, 1, 2**24, 1, 512)
run(1000000, 16000000, 0.01, 0, 2**24, 1, 1024)
run(1000000, 16000000, 0.01, 1, 2**24, 3, 1024)
run(1000000, 16000000, 0.01, 0, 2**24, 4, 1024)
run(1000000, 16000000, 1.0, None, 0, 0, 0)
run(1000000, 16000000, 0.01, 2, 2**24, 3, 1024)
# north star via device generator
nR, nS = 128000000, 1024000000
dR = torch.empty((nR, 2), dtype=torch.int32, device="cuda")
dS = torch.empty((nS, 2), dtype=torch.int32, device="cuda")
hw.generate_device(dR, 2, nR, nR, 1.0, 12345)
hw.generate_device(dS, 2, 2**31 - 1, nR, 0.01, 54321)
args = hw.BloomFilterArgs(hw.BLOCKED, 2**30, 1, 1024)
for i in range(6):
    os.environ["HWBRJ_SCE"] = "8" if i % 2 else "4"
    st = hw.join_device(dR, dS, args)
    print("SCE", os.environ["HWBRJ_SCE"], end=" ")
    print(f"NS run {i}: filtered={st.filtered} (want 124236515) matches={st.matches} (want 10240000) total={st.ms_total:.3f} ms | r_sc {st.ms_r_scatter:.3f} r_ix {st.ms_r_index:.3f} build {st.ms_build:.3f} s_sc {st.ms_s_scatter:.3f} s_ix {st.ms_s_index:.3f} probe {st.ms_probe:.3f} surv {st.ms_surv:.3f} join {st.ms_join:.3f}", flush=True)
