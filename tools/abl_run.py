"""Dev-only: phase times of the north-star join for the variant libraries under tools/abl_so/
(built with -DHWBRJ_ABL_* ablations; their results are invalid). One process per variant:
    python tools/abl_run.py BASE NOCRC ...
"""
import os, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import os, sys
sys.path.insert(0, sys.argv[1])
import torch
import hwbloomradixjoin_amd as hw
nR, nS = 128000000, int(os.environ.get("ABL_NS", "1024000000"))
dR = torch.empty((nR, 2), dtype=torch.int32, device="cuda")
dS = torch.empty((nS, 2), dtype=torch.int32, device="cuda")
hw.generate_device(dR, 2, nR, nR, 1.0, 12345)
hw.generate_device(dS, 2, 2**31 - 1, nR, float(os.environ.get("ABL_Q", "0.01")), 54321)
args = None if os.environ.get("ABL_PRO") else hw.BloomFilterArgs(hw.BLOCKED, 1 << 30, 1, 1024)
best = None
for i in range(4):
    st = hw.join_device(dR, dS, args)
    if i and (best is None or st.ms_total < best.ms_total):
        best = st
print(f"{sys.argv[2]:40s} total {best.ms_total:.3f} r_sc {best.ms_r_scatter:.3f} build {best.ms_build:.3f} "
      f"s_sc {best.ms_s_scatter:.3f} s_ix {best.ms_s_index:.3f} probe {best.ms_probe:.3f} join {best.ms_join:.3f} "
      f"counts {best.filtered} {best.matches} {'OK' if nS != 1024000000 or os.environ.get('ABL_Q') or os.environ.get('ABL_PRO') or (best.filtered, best.matches) == (124236515, 10240000) else 'BAD'}", flush=True)
'''
for spec in sys.argv[1:]:
    # NAME[@VAR=VAL,VAR=VAL]: a tools/abl_so variant (CUR: the in-tree library) under extra env vars
    v, _, extra = spec.partition("@")
    env = dict(os.environ, HWBRJ_LIB=os.path.join(ROOT, "tools", "abl_so", f"libhwbrj_{v}.so"))
    if v == "CUR":  # the in-tree library
        env.pop("HWBRJ_LIB")
    for kv in filter(None, extra.split(",")):
        k, _, val = kv.partition("=")
        env[k] = val
    v = spec
    r = subprocess.run([sys.executable, "-c", CHILD, ROOT, v], env=env, timeout=120)
    if r.returncode != 0:
        print(f"{v}: exit {r.returncode}")
        sys.exit(1)
