"""The materializing pipeline (JOIN_RESULT_MATERIALIZE, src/parallel_radix_join_bloom.c:307-312):
payloads carried through the partition passes (k_scatter_*p, k_build, k_probe with survivor
positions, k_join_mat). Pair multisets against the oracle (orc_join_pairs) for every filter mode
and word format, the scatter's skew path, slice segments, the global-mode fallback, the capacity
contract, and the north star at full size."""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
INT_MAX = 2**31 - 1


def to_dev(cuda, a):
    return cuda.from_numpy(np.ascontiguousarray(a, dtype=np.int32)).cuda()


@pytest.fixture(scope="module")
def gen3(hw):
    """The rand()-driven relations of SURVEY.md s8c F3 (bit-exact reference generators, host)."""
    g = json.load(open(os.path.join(HERE, "golden", "survey_counts.json")))["F3_generators"]
    kw = dict(r_seed=g["r_seed"], s_seed=g["s_seed"], host_threads=8)
    return {"nonunique": hw.reference_relations(g["r"], g["s"], g["nonunique"]["q"], non_unique=True, **kw),
            "zipf": hw.reference_relations(g["r"], g["s"], skew=g["zipf"]["z"], **kw)}


def _sorted_pairs(p):
    p = np.asarray(p).reshape(-1, 2)
    return p[np.lexsort((p[:, 1], p[:, 0]))]


def _args(hw):
    return {
        "blocked_packed": hw.BloomFilterArgs(hw.BLOCKED, 1 << 24, 1, 1024),
        "blocked_code": hw.BloomFilterArgs(hw.BLOCKED, 1 << 24, 1, 2048),   # B > F: code words
        "blocked_k3": hw.BloomFilterArgs(hw.BLOCKED, 1 << 24, 3, 512),
        "sectorized_k2": hw.BloomFilterArgs(hw.SECTORIZED, 1 << 24, 2, 1024),
        "basic_k1": hw.BloomFilterArgs(hw.BASIC, 1 << 24, 1),
        "basic_k3": hw.BloomFilterArgs(hw.BASIC, 1 << 22, 3),
        "two_segments": hw.BloomFilterArgs(hw.BLOCKED, 1 << 31, 1, 1024),  # 2 slice segments
        "global_b4": hw.BloomFilterArgs(hw.BLOCKED, 1 << 20, 1, 4),         # side-pass fallback
        "nobloom": None,
    }


def _check(hw, cuda, orc, R, S, args):
    st, pairs, _ = hw.join_materialize_device(to_dev(cuda, R), to_dev(cuda, S), args)
    want = orc.join_pairs(R, S)
    assert st.matches == want.shape[0] == pairs.shape[0]
    assert np.array_equal(_sorted_pairs(pairs.cpu().numpy()), _sorted_pairs(want))
    return st


@pytest.mark.parametrize("name", ["blocked_packed", "blocked_code", "blocked_k3", "sectorized_k2",
                                  "basic_k1", "basic_k3", "two_segments", "global_b4", "nobloom"])
def test_pairs_every_mode(hw, cuda, orc, name):
    """PK/FK relations with random payloads: pairs equal the oracle's; filtered equals the
    counting join's."""
    rng = np.random.default_rng(5)
    R = orc.relation(400000, 2, 400000, 400000, 1.0, 1)
    S = orc.relation(3000000, 2, INT_MAX, 400000, 0.2, 2)
    R[:, 1] = rng.integers(-2**31, 2**31, size=R.shape[0])
    S[:, 1] = rng.integers(-2**31, 2**31, size=S.shape[0])
    args = _args(hw)[name]
    st = _check(hw, cuda, orc, R, S, args)
    cnt = hw.join_device(to_dev(cuda, R), to_dev(cuda, S), args)
    assert (st.filtered, st.matches) == (cnt.filtered, cnt.matches)


@pytest.mark.parametrize("name", ["blocked_packed", "basic_k1", "nobloom"])
def test_pairs_skewed_partitions(hw, cuda, orc, name):
    """Hot keys that overfill one partition in every scatter round (the skew path's direct
    halves): key 77 in a third of R, key 88 in a tenth of S; plus duplicates and extreme keys."""
    rng = np.random.default_rng(9)
    Rk = np.concatenate([np.full(20000, 77), np.full(100, 88), rng.integers(-5000, 5000, size=40000),
                         [INT_MAX, -INT_MAX - 1]])
    Sk = np.concatenate([np.full(500, 77), np.full(100000, 88), rng.integers(-6000, 6000, size=900000),
                         [INT_MAX, -INT_MAX - 1, 77]])
    rng.shuffle(Rk)
    rng.shuffle(Sk)
    R = np.stack([Rk, rng.integers(-2**31, 2**31, size=Rk.size)], 1).astype(np.int32)
    S = np.stack([Sk, rng.integers(-2**31, 2**31, size=Sk.size)], 1).astype(np.int32)
    _check(hw, cuda, orc, R, S, _args(hw)[name])


@pytest.mark.parametrize("name", ["blocked_packed", "blocked_k3", "basic_k3", "two_segments", "nobloom"])
def test_pairs_edge_sizes(hw, cuda, orc, name):
    """Empty and ragged relations (no pairs, one pair, sizes off every chunk / workgroup multiple)."""
    rng = np.random.default_rng(13)
    for nR, nS in [(0, 1000), (1000, 0), (1, 1), (1, 5000), (7, 33), (4097, 4099), (100003, 400009)]:
        Rk = rng.permutation(nR).astype(np.int64) + 1
        Sk = rng.integers(0, 2 * max(nR, 1) + 2, size=nS)
        R = np.stack([Rk, rng.integers(-2**31, 2**31, size=nR)], 1).astype(np.int32).reshape(-1, 2)
        S = np.stack([Sk, rng.integers(-2**31, 2**31, size=nS)], 1).astype(np.int32).reshape(-1, 2)
        _check(hw, cuda, orc, R, S, _args(hw)[name])


def test_pairs_zipf_and_nonunique(hw, cuda, orc, gen3):
    for mode in ("zipf", "nonunique"):
        R, S = gen3[mode]
        _check(hw, cuda, orc, R, S[:4000000], _args(hw)["blocked_packed"])


def test_capacity_contract(hw, cuda, orc):
    """Too small a capacity: return code 7 with the match count; the wrapper re-runs at size."""
    R = orc.relation(100000, 2, 100000, 100000, 1.0, 3)
    S = orc.relation(1000000, 2, INT_MAX, 100000, 0.5, 4)
    st, pairs, _ = hw.join_materialize_device(to_dev(cuda, R), to_dev(cuda, S),
                                              _args(hw)["blocked_packed"], capacity=1000)
    want = orc.join_pairs(R, S)
    assert st.matches == want.shape[0] == pairs.shape[0] == 500000
    assert np.array_equal(_sorted_pairs(pairs.cpu().numpy()), _sorted_pairs(want))


def test_northstar_materialized(hw, cuda):
    """|R| = 128M, |S| = 1024M, q = 0.01 (BASELINE configs[1]): 10.24M pairs; every pair joins
    equal keys (the generator's payload is the row index) and no S row appears twice (R is a
    primary key)."""
    import torch
    nR, nS = 128000000, 1024000000
    dR = torch.empty((nR, 2), dtype=torch.int32, device="cuda")
    dS = torch.empty((nS, 2), dtype=torch.int32, device="cuda")
    hw.generate_device(dR, 2, nR, nR, 1.0, 12345)
    hw.generate_device(dS, 2, INT_MAX, nR, 0.01, 54321)
    st, pairs, ms = hw.join_materialize_device(dR, dS, hw.BloomFilterArgs(hw.BLOCKED, 1 << 30, 1, 1024),
                                               capacity=10240000)
    assert (st.filtered, st.matches, pairs.shape[0]) == (124236515, 10240000, 10240000)
    assert bool((dR[pairs[:, 0].long(), 0] == dS[pairs[:, 1].long(), 0]).all().item())
    assert torch.unique(pairs[:, 1]).numel() == 10240000
    print(f"north-star materializing join: {ms:.3f} ms")
