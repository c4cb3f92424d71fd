"""Seeded randomized parity sweep: the HIP path against the oracle over random configurations.

Every case draws, from its own seed, a filter configuration the reference accepts (variant, m, k,
B: src/bloom_filter.c:25-34), a per-partition join (PRO / PRH / PRHO,
src/parallel_radix_join_bloom.c:259-555), relation sizes with ragged tails and a key distribution
(dense unique keys, duplicates in a narrow range, the full int32 range with negatives, Zipf-skewed
probes, one hot key). The bar is the other parity tests' bar: `filtered` and `Results` equal the
oracle's `orc.bpro` on the same tuples; every fourth case also materializes the result and its pair
multiset equals `orc.join_pairs`, and every third runs the partitioned multi-GPU join on one rank
(hwbrj_join_partitioned, every exchange a local copy) where its geometry allows. The same cases also
go through the schedule bench.py times: groups of 8 enqueued back to back with
hwbrj_join_device_async (empty R, one-tuple S, global-bitmap and basic k >= 2 launches mixed in a
group), every join's counts collected with hwbrj_join_wait_all and compared with its own oracle
result. The cases are fixed by their seeds, so a failure names a reproducible configuration (see
`case()`).
"""
import numpy as np
import pytest

INT_MIN, INT_MAX = -2**31, 2**31 - 1
NCASES = 192


def case(seed: int):
    """(variant name, m, k, B, algorithm, Rk, Sk) of fuzz case `seed`."""
    rng = np.random.default_rng(1000 + seed)
    variant = ["no", "basic", "blocked", "sectorized"][rng.integers(0, 4)]
    log2m = int(rng.integers(6, 33))
    m = 1 << log2m
    k = int(rng.choice([1, 1, 1, 2, 3, 4, 7])) if variant != "basic" else int(rng.choice([1, 1, 2, 3, 5]))
    B = 1 << int(rng.integers(1, min(log2m, 11) + 1))  # 2 .. min(m, 2048), a divisor of m
    algorithm = int(rng.integers(0, 3))
    nR = int(rng.choice([0, 1, 63, 1025] + [int(rng.integers(1, 200000))] * 3))
    nS = int(rng.choice([1, 7, 4097] + [int(rng.integers(1, 600000))] * 2 + [int(rng.integers(1, 2000000))]))
    dist = ["unique", "dups", "wide", "zipf", "hot"][rng.integers(0, 5)]
    if dist == "unique":
        Rk = rng.permutation(nR).astype(np.int64) + 1
        Sk = rng.integers(0, 2 * max(nR, 1) + 2, size=nS)
    elif dist == "dups":
        span = max(nR // 4, 1)
        Rk = rng.integers(-span, span + 1, size=nR)
        Sk = rng.integers(-2 * span, 2 * span + 1, size=nS)
    elif dist == "wide":
        Rk = rng.integers(INT_MIN, INT_MAX, size=nR, endpoint=True)
        Sk = np.concatenate([rng.choice(Rk, size=nS // 2) if nR else rng.integers(0, 9, size=nS // 2),
                             rng.integers(INT_MIN, INT_MAX, size=nS - nS // 2, endpoint=True)])
    elif dist == "zipf":
        Rk = rng.permutation(nR).astype(np.int64) + 1
        z = rng.zipf(1.2 + rng.random(), size=nS)
        Sk = np.where(z <= nR, z, rng.integers(nR + 1, 4 * nR + 9, size=nS))
    else:
        Rk = rng.permutation(nR).astype(np.int64) + 1
        hot = int(Rk[0]) if nR else 5
        Sk = np.where(rng.random(nS) < 0.9, hot, rng.integers(0, nR + 9, size=nS))
    return variant, m, k, B, algorithm, Rk.astype(np.int32), np.asarray(Sk).astype(np.int32)


_ORC = {}  # seed -> the oracle's (filtered, results), shared by the synchronous and async tests


def _inputs(hw, seed):
    variant, m, k, B, algorithm, Rk, Sk = case(seed)
    rng = np.random.default_rng(seed)
    R, S = _rel(Rk, rng), _rel(Sk, rng)
    return R, S, hw.BloomFilterArgs.from_flag(variant, m, k, B), algorithm


def _oracle(orc, seed, R, S, args):
    if seed not in _ORC:
        if args is None:
            res, filt, _ = orc.bpro(R, S, 4, 0, 0, 0, 0, use_bloom=False)
        else:
            res, filt, _ = orc.bpro(R, S, 4, args.variant, args.m, args.k, args.B)
        _ORC[seed] = (filt, res)
    return _ORC[seed]


def _rel(keys, rng):
    return np.stack([keys, rng.integers(INT_MIN, INT_MAX, size=keys.size, endpoint=True).astype(np.int32)], 1)


def _sorted_pairs(p):
    p = np.asarray(p).reshape(-1, 2)
    return p[np.lexsort((p[:, 1], p[:, 0]))]


def test_fuzz_cases_are_reference_configurations(hw):
    """The sweep only draws configurations the reference accepts (CPU-side check of the sampler)."""
    for s in range(NCASES):
        variant, m, k, B, _, Rk, Sk = case(s)
        args = hw.BloomFilterArgs.from_flag(variant, m, k, B)
        assert args is None or hw.assert_args(args), (s, variant, m, k, B)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(NCASES))
def test_fuzz_counts_vs_oracle(hw, cuda, orc, seed):
    R, S, args, algorithm = _inputs(hw, seed)
    dR = cuda.from_numpy(R).cuda()
    dS = cuda.from_numpy(S).cuda()
    st = hw.join_device(dR, dS, args, algorithm=algorithm)
    filt, res = _oracle(orc, seed, R, S, args)
    assert (st.filtered, st.matches) == (filt, res), (seed, case(seed)[:5], st)
    if seed % 3 == 1:
        from hwbloomradixjoin_amd import pjoin
        try:
            st3 = pjoin.join_partitioned(dR, dS, R.shape[0], args)
        except RuntimeError as e:  # global-bitmap mode (B < 8) and basic k >= 2 have no slices
            assert "partition slices" in str(e), e
        else:
            assert (st3.filtered, st3.matches) == (filt, res), (seed, "partitioned", st3)
    if seed % 4 == 0:
        st2, pairs, _ = hw.join_materialize_device(dR, dS, args)
        want = orc.join_pairs(R, S)
        assert st2.matches == want.shape[0] == pairs.shape[0] == res
        assert np.array_equal(_sorted_pairs(pairs.cpu().numpy()), _sorted_pairs(want))


GROUP = 8


@pytest.mark.gpu
@pytest.mark.parametrize("group", range(NCASES // GROUP))
def test_fuzz_async_back_to_back(hw, cuda, orc, group):
    """Cases 8g .. 8g + 7 enqueued back to back through hwbrj_join_device_async on one stream (no
    host wait between them: consecutive joins differ in filter, mode and sizes), then one
    hwbrj_join_wait_all: every join's (filtered, matches) against its own oracle result."""
    seeds = range(group * GROUP, (group + 1) * GROUP)
    ins = [_inputs(hw, s) for s in seeds]
    dev = [(cuda.from_numpy(R).cuda(), cuda.from_numpy(S).cuda()) for R, S, _, _ in ins]
    want = [_oracle(orc, s, R, S, a) for s, (R, S, a, _) in zip(seeds, ins)]
    stream = cuda.cuda.Stream()
    for (dR, dS), (_, _, a, _) in zip(dev, ins):
        hw.join_device_async(dR, dS, a, stream=stream)
    sts = hw.join_wait_all()
    assert len(sts) == GROUP
    got = [(st.filtered, st.matches) for st in sts]
    assert got == want, [(s, case(s)[:4], g, w) for s, g, w in zip(seeds, got, want) if g != w]
