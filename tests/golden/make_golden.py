"""Regenerate the reference-derived fixtures in tests/golden/ (run in the container that has
/root/reference; the GPU box only reads the JSON).

  ref_kats.json     hash_crc / hash_crapwow of the reference's own src/hash.c (oracle/_ref) on
                    edge and pseudo-random keys
  ref_filters.json  the reference's own src/bloom_filter.c (oracle/_ref, seed 42): popcount and
                    sha256 of the filter after inserting R, and the filtered count of S, for small
                    relations of the reference generator multiset (oracle.gen_keys, the
                    generation order is irrelevant to both numbers)

    python tests/golden/make_golden.py
"""
import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import pyoracle as orc  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
INT_MAX = 2**31 - 1

FILTER_CASES = [
    # (variant, m, k, B)
    (1, 1 << 20, 1, 1024), (1, 1 << 20, 1, 512), (1, 1 << 20, 2, 512), (1, 1 << 20, 3, 64),
    (1, 1 << 20, 1, 32), (1, 1 << 20, 4, 8), (1, 1 << 18, 1, 1024), (1, 1 << 22, 5, 256),
    (1, 1 << 20, 2, 4), (1, 1 << 16, 1, 2048),
    (0, 1 << 20, 1, 0), (0, 1 << 20, 2, 0), (0, 1 << 22, 3, 0), (0, 1 << 16, 1, 0),
    (0, 1 << 20, 8, 0),
]


def main():
    if not orc.have_ref():
        orc.build()
    ref = orc.ref()
    keys = [0, 1, 2, 42, -1, -42, 12345, 128000000, 128000001, INT_MAX, -INT_MAX - 1]
    rng = np.random.default_rng(20260101)
    keys += [int(x) for x in rng.integers(-2**31, 2**31, size=500)]
    kats = [{"key": k, "crc32c": ref.hash_crc(42, k), "crapwow": ref.hash_crapwow(42, k),
             "crc32c_seed7": ref.hash_crc(7, k), "crapwow_seed7": ref.hash_crapwow(7, k)}
            for k in keys]
    json.dump({"_source": "reference src/hash.c via oracle/_ref (tests/golden/make_golden.py)",
               "kats": kats}, open(os.path.join(HERE, "ref_kats.json"), "w"), indent=0)

    nR, nS, q = 50000, 400000, 0.01
    R = orc.gen_keys(nR, 2, nR, nR, 1.0)
    S = orc.gen_keys(nS, 2, INT_MAX, nR, q)
    out = []
    for (v, m, k, B) in FILTER_CASES:
        bm, filt = orc.ref_bloom(R, S, v, m, k, B if v else 1024)
        out.append({"variant": v, "m": m, "k": k, "B": B if v else 1024,
                    "popcount": int(np.unpackbits(bm).sum()),
                    "sha256": hashlib.sha256(bm.tobytes()).hexdigest(), "filtered": filt})
        print(out[-1], flush=True)
    json.dump({"_source": "reference src/bloom_filter.c via oracle/_ref (make_golden.py)",
               "r": nR, "s": nS, "q": q, "nthreads": 2, "cases": out},
              open(os.path.join(HERE, "ref_filters.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
