"""CPU tests of the rand()-driven generators (--non-unique, --full-range, -z): the library's
restated glibc rand() against libc's own rand(), the library's relations against the oracle's
(which calls libc srand/rand exactly as src/generator.c does), and the reference binary's counts
on those relations (tests/golden/survey_counts.json "F3_generators")."""
import ctypes
import json
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = json.load(open(os.path.join(HERE, "golden", "survey_counts.json")))["F3_generators"]


@pytest.mark.parametrize("seed", [0, 1, 12345, 54321, 2**31 - 1, 2**31, 2**32 - 1])
def test_rand_restatement_is_glibc_rand(hw, seed):
    libc = ctypes.CDLL("libc.so.6")
    libc.srand(ctypes.c_uint(seed))
    want = np.array([libc.rand() for _ in range(5000)], dtype=np.int32)
    assert np.array_equal(hw.rand_stream(seed, 5000), want)


@pytest.mark.parametrize("mode,q", [("nonunique", 0.01), ("nonunique", 0.5), ("nonunique", 1.0),
                                    ("fullrange", 0.01), ("fullrange", 1.0)])
def test_rand_relations_equal_oracle(hw, orc, mode, q):
    for nR, nS in [(1000, 20000), (77777, 123457)]:
        R, S = hw.reference_relations(nR, nS, q, non_unique=mode == "nonunique",
                                      full_range=mode == "fullrange", r_seed=7, s_seed=8)
        R2, S2 = orc.reference_relations(nR, nS, q, mode, r_seed=7, s_seed=8)
        assert np.array_equal(R, R2) and np.array_equal(S, S2)


@pytest.mark.parametrize("theta,alpha,n", [(0.75, 1000, 50000), (0.5, 100000, 200000),
                                           (1.2, 1, 100), (0.0, 5000, 30000)])
def test_zipf_equals_oracle(hw, orc, theta, alpha, n):
    S = hw.create_relation_zipf(n, alpha, theta, 54321, 4)
    _, S2 = orc.reference_relations(alpha, n, 1.0, "zipf", theta, s_seed=54321)
    assert np.array_equal(S, S2)
    assert S[:, 0].min() >= 1 and S[:, 0].max() <= alpha


def test_nonunique_golden_counts(hw, orc):
    """--non-unique -q 0.01 -b blocked -k 1, 1e6/16e6, m = 2^24: the reference binary's counts."""
    g, row = GOLD, GOLD["nonunique"]
    R, S = hw.reference_relations(g["r"], g["s"], row["q"], non_unique=True,
                                  r_seed=g["r_seed"], s_seed=g["s_seed"])
    res, filt, _ = orc.bpro(R, S, 8, 1, g["m"], row["k"], g["B"])
    assert (filt, res) == (row["filtered"], row["results"])


def test_zipf_golden_counts(hw, orc):
    """-z 0.75: every S key lies in [1, |R|], so filtered = Results = |S|."""
    g, row = GOLD, GOLD["zipf"]
    R, S = hw.reference_relations(g["r"], g["s"] // 8, skew=row["z"], r_seed=g["r_seed"],
                                  s_seed=g["s_seed"], host_threads=8)
    res, filt, _ = orc.bpro(R, S, 8, 1, g["m"], row["k"], g["B"])
    assert filt == res == g["s"] // 8


def test_cli_parses_generator_flags(hw):
    import subprocess
    out = subprocess.run([hw.CLI_PATH, "-h"], capture_output=True, text=True, timeout=60)
    for flag in ("--skew", "--non-unique", "--full-range"):
        assert flag in out.stdout
