"""BASELINE.json configs 3 and 5 at full size on one MI355X (|R| = 128M, |S| = 1024M):
  config 3: filter variants (basic / blocked B=1024,512,64 / sectorized) at m = 2^30, k = 1 and 2;
  config 5: selectivity sweep q in {0.001, 0.01, 0.1, 1.0}, uniform S (reference generator) and
            Zipf theta = 0.75 S (the reference's gen_zipf stream; q < 1 is this build's extension).
Best-of-3 device time per row; counts checked against the goldens / exact expectations.
    python tools/sweep.py [3] [5]
"""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import hwbloomradixjoin_amd as hw

nR, nS = 128000000, 1024000000
INT_MAX = 2**31 - 1
which = set(sys.argv[1:]) or {"3", "5"}
dR = torch.empty((nR, 2), dtype=torch.int32, device="cuda")
dS = torch.empty((nS, 2), dtype=torch.int32, device="cuda")
hw.generate_device(dR, 2, nR, nR, 1.0, 12345)


def run(label, args, want=None, reps=3):
    best = None
    for _ in range(reps):
        st = hw.join_device(dR, dS, args)
        if best is None or st.ms_total < best.ms_total:
            best = st
    ok = "" if want is None else (" OK" if (best.filtered, best.matches) == want else f" MISMATCH want {want}")
    print(f"{label:44s} {best.ms_total:7.3f} ms {nS / best.ms_total / 1e6:7.1f} G probe-tuples/s | "
          f"s_sc {best.ms_s_scatter:.3f} probe {best.ms_probe:.3f} build {best.ms_build:.3f} join {best.ms_join:.3f} | "
          f"filtered {best.filtered} matches {best.matches}{ok}", flush=True)
    return best


if "3" in which:
    hw.generate_device(dS, 2, INT_MAX, nR, 0.01, 54321)
    torch.cuda.synchronize()
    print("# config 3: filter variants, q = 0.01, m = 2^30")
    gold = {("blocked", 1024, 1): (124236515, 10240000), ("blocked", 1024, 2): (55849475, 10240000),
            ("blocked", 512, 1): (124271673, 10240000), ("blocked", 512, 2): (55845538, 10240000),
            ("basic", 0, 1): (124152740, 10240000), ("basic", 0, 2): (55852594, 10240000)}
    for k in (1, 2):
        for v, B in (("basic", 0), ("blocked", 1024), ("blocked", 512), ("blocked", 64), ("sectorized", 1024)):
            run(f"-b {v}{' -B ' + str(B) if B else ''} -k {k}", hw.BloomFilterArgs.from_flag(v, 1 << 30, k, B or 1024),
                gold.get((v, B, k)))
    run("-b no (PRO)", None, (nS, 10240000))

if "5" in which:
    print("# config 5: selectivity sweep, blocked m = 2^30 k = 1 (B = 1024)")
    a = hw.BloomFilterArgs(hw.BLOCKED, 1 << 30, 1, 1024)
    gold = {0.01: (124236515, 10240000)}
    for q in (0.001, 0.01, 0.1, 1.0):
        hw.generate_device(dS, 2, INT_MAX, nR, q, 54321)
        torch.cuda.synchronize()
        st = run(f"uniform S, q = {q}", a, gold.get(q))
        assert st.matches == round(nS * q) or q not in (0.001, 0.01, 0.1, 1.0)
    for q in (0.001, 0.01, 0.1, 1.0):
        t0 = time.time()
        hw.create_relation_zipf_device(dS, nR, 0.75, 54321, q, 16)
        torch.cuda.synchronize()
        gen_s = time.time() - t0
        st = run(f"zipf 0.75 S, q = {q} (gen {gen_s:.0f} s)", a)
        n_above = int(nS * (1 - q))
        assert st.matches == nS - n_above and st.filtered >= st.matches, (st.matches, nS - n_above)
