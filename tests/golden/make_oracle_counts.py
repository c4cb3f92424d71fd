"""Pin the full-size counts no reference fixture holds with the oracle (oracle/oracle.c, the CPU
restatement of BPRO that tests/test_oracle.py checks against the reference's own hash.c /
bloom_filter.c and against every count the reference binary and the thesis data published).

Writes tests/golden/oracle_counts.json: filtered ("S-tuples after filter") and Results of
|R| = 128M, |S| = 1024M joins of the reference generator's key multiset (hw.generate_host, the
multiset the device generator and bench.py produce) for the rows of BASELINE.json configs 3 and 5
that neither SURVEY.md s8c nor the thesis pins: the sectorized variant (this build's extension),
the register-blocked B = 64 row and the selectivity sweep q in {0.001, 0.1, 1.0}.

    python tests/golden/make_oracle_counts.py [threads]     (~20 GB of RAM, a few minutes)
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import hwbloomradixjoin_amd as hw  # noqa: E402  (host generator only: no GPU is used)
from oracle import pyoracle as orc  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
INT_MAX = 2**31 - 1
NR, NS = 128000000, 1024000000
# (q, variant, m, k, B)
ROWS = [
    (0.01, "sectorized", 1 << 30, 2, 1024),
    (0.01, "sectorized", 1 << 30, 1, 1024),
    (0.01, "blocked", 1 << 30, 1, 64),
    (0.001, "blocked", 1 << 30, 1, 1024),
    (0.1, "blocked", 1 << 30, 1, 1024),
    (1.0, "blocked", 1 << 30, 1, 1024),
]
VAR = {"basic": 0, "blocked": 1, "sectorized": 2}


def main():
    threads = int(sys.argv[1]) if len(sys.argv) > 1 else (os.cpu_count() or 8)
    R = hw.generate_host(NR, 2, NR, NR, 1.0, 12345, threads)
    out, S, s_q = [], None, None
    for (q, v, m, k, B) in ROWS:
        if q != s_q:
            S = None
            S = hw.generate_host(NS, 2, INT_MAX, NR, q, 54321, threads)
            s_q = q
        t0 = time.time()
        res, filt, _ = orc.bpro(R, S, threads, VAR[v], m, k, B, True)
        row = {"r": NR, "s": NS, "q": q, "variant": v, "m": m, "k": k, "B": B,
               "filtered": int(filt), "results": int(res)}
        out.append(row)
        print(row, f"{time.time() - t0:.1f} s", flush=True)
    json.dump({"_source": "oracle/oracle.c orc_bpro on hw.generate_host relations "
                          "(tests/golden/make_oracle_counts.py)", "rows": out},
              open(os.path.join(HERE, "oracle_counts.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
