"""Async joins (hwbrj_join_device_async, the schedule bench.py times): EVERY join checked.

Async joins run their S pass on a second stream beside the R side (HWBRJ_OVL_ASYNC, DESIGN.md §7
round 5) and keep their counts in a per-join device ring (hwbrj_join_wait_all), so each join of a
back-to-back run is compared with the oracle on its own inputs, not only the last one. Consecutive
joins alternate filter configurations and S relations, so a join that read a buffer of the join
before it (a cross-stream race between the side stream's S pass and the R side's zeroing, or a
stale count slot) gives a wrong count somewhere in the sequence. The reference checks every run's
count (src/parallel_radix_join_bloom.c:1696-1707 sums every thread's count).
"""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = json.load(open(os.path.join(HERE, "golden", "survey_counts.json")))
ORC_FULL = json.load(open(os.path.join(HERE, "golden", "oracle_counts.json")))["rows"]
INT_MAX = 2**31 - 1

# (variant, m, k, B) or None (PRO): blocked k = 1 / 2, sectorized k = 2, PRO, basic k = 1 and k = 2,
# m = 2^31 (two slice segments, nseg = 2)
CONFIGS = [("blocked", 1 << 24, 1, 1024), ("blocked", 1 << 24, 2, 512), ("sectorized", 1 << 24, 2, 1024),
           None, ("basic", 1 << 24, 1, 1024), ("blocked", 1 << 31, 1, 1024), ("basic", 1 << 22, 2, 1024)]


def mk(hw, a):
    return None if a is None else hw.BloomFilterArgs.from_flag(a[0], a[1], a[2], a[3])


@pytest.fixture(scope="module")
def rels(hw, cuda):
    """|R| = 1M and three S relations of the reference generator (different seeds and q), on the
    host (for the oracle) and on the device."""
    nR = 1000000
    R = hw.generate_host(nR, 2, nR, nR, 1.0, 31, 8)
    Ss = [hw.generate_host(n, 2, INT_MAX, nR, q, seed, 8)
          for n, q, seed in [(4000000, 0.05, 41), (3000001, 0.5, 42), (5000000, 0.01, 43)]]
    dev = lambda a: cuda.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    return R, dev(R), Ss, [dev(S) for S in Ss]


@pytest.fixture(scope="module")
def expected(orc, rels):
    """The oracle's (filtered, matches) for every (config, S) pair, computed once."""
    R, _, Ss, _ = rels
    out = {}
    for ci, a in enumerate(CONFIGS):
        for si, S in enumerate(Ss):
            if a is None:
                res, filt, _ = orc.bpro(R, S, 8, 0, 0, 0, 0, use_bloom=False)
            else:
                v = {"basic": 0, "blocked": 1, "sectorized": 2}[a[0]]
                res, filt, _ = orc.bpro(R, S, 8, v, a[1], a[2], a[3])
            out[ci, si] = (filt, res)
    return out


def _seq(n):
    """n (config, S) pairs: every consecutive pair differs in both."""
    return [(i % len(CONFIGS), (i * 2 + i // len(CONFIGS)) % 3) for i in range(n)]


def test_wait_all_checks_every_back_to_back_join(hw, cuda, rels, expected):
    """14 async joins back to back with no host wait between them (two passes over the seven
    configurations, S relations rotating), then one hwbrj_join_wait_all: 14 stats, oldest first,
    each equal to the oracle on its own (config, S)."""
    _, dR, _, dSs = rels
    seq = _seq(14)
    stream = cuda.cuda.Stream()
    for ci, si in seq:
        hw.join_device_async(dR, dSs[si], mk(hw, CONFIGS[ci]), stream=stream)
    sts = hw.join_wait_all()
    assert len(sts) == len(seq)
    for j, ((ci, si), st) in enumerate(zip(seq, sts)):
        assert (st.filtered, st.matches) == expected[ci, si], (j, CONFIGS[ci], si, st)
        assert st.ms_total == 0  # (async: counts only)
    assert hw.join_wait_all() == []  # (collected)


def test_wait_after_every_async_join(hw, cuda, rels, expected):
    """Every join through the async (two-stream) schedule, each waited before the next is
    enqueued: the same sequence, hwbrj_join_wait after each."""
    _, dR, _, dSs = rels
    for j, (ci, si) in enumerate(_seq(10)):
        hw.join_device_async(dR, dSs[si], mk(hw, CONFIGS[ci]))
        st = hw.join_wait()
        assert (st.filtered, st.matches) == expected[ci, si], (j, CONFIGS[ci], si, st)


@pytest.mark.parametrize("ci", range(len(CONFIGS)), ids=lambda i: str(CONFIGS[i]))
def test_three_back_to_back_per_config(hw, cuda, rels, expected, ci):
    """Three back-to-back joins of one configuration over the three S relations: each asserted."""
    _, dR, _, dSs = rels
    a = mk(hw, CONFIGS[ci])
    for si in range(3):
        hw.join_device_async(dR, dSs[si], a)
    sts = hw.join_wait_all()
    assert [(s.filtered, s.matches) for s in sts] == [expected[ci, si] for si in range(3)]


def test_ring_wraps_beyond_its_slots(hw, cuda, rels, expected):
    """More joins than the ring's 64 result slots without a wait: the 65th enqueue collects the
    first 64 on the host, and wait_all still returns all 70, in order, each right."""
    _, dR, _, dSs = rels
    small = [dSs[0][:200000], dSs[1][:150001]]
    a = mk(hw, CONFIGS[0])
    want = []
    for si in range(2):
        hw.join_device_async(dR, small[si], a)
        want.append(hw.join_wait())
    for j in range(70):
        hw.join_device_async(dR, small[j % 2], a)
    sts = hw.join_wait_all(capacity=100)
    assert len(sts) == 70
    for j, st in enumerate(sts):
        assert (st.filtered, st.matches) == (want[j % 2].filtered, want[j % 2].matches), j


def test_wait_all_capacity_and_last(hw, cuda, rels, expected):
    """A capacity below the pending joins raises (code 7, the oldest written); join_wait after it
    still returns the last join; a synchronous join starts a new collection."""
    _, dR, _, dSs = rels
    a = mk(hw, CONFIGS[1])
    for si in range(3):
        hw.join_device_async(dR, dSs[si], a)
    with pytest.raises(RuntimeError, match="hwbrj_join_wait_all"):
        hw.join_wait_all(capacity=2)
    st = hw.join_wait()
    assert (st.filtered, st.matches) == expected[1, 2]
    hw.join_device_async(dR, dSs[0], a)
    st = hw.join_device(dR, dSs[1], a)
    assert (st.filtered, st.matches) == expected[1, 1] and st.ms_total > 0
    assert hw.join_wait_all() == []  # (the synchronous join collected both)


def test_two_streams_every_join(hw, cuda, rels, expected):
    """Async joins alternating between two caller streams (each orders after the other's pending
    join): every join's counts."""
    _, dR, _, dSs = rels
    s1, s2 = cuda.cuda.Stream(), cuda.cuda.Stream()
    seq = _seq(6)
    for j, (ci, si) in enumerate(seq):
        hw.join_device_async(dR, dSs[si], mk(hw, CONFIGS[ci]), stream=s1 if j % 2 == 0 else s2)
    sts = hw.join_wait_all()
    assert [(s.filtered, s.matches) for s in sts] == [expected[c] for c in seq]


def test_northstar_async_every_join(hw, cuda):
    """The north star through the timed schedule: blocked k = 1, sectorized k = 2, blocked k = 2,
    PRO and blocked k = 1 again, back to back on one stream, each against F4 (the reference binary)
    or the oracle's full-size counts (tests/golden/oracle_counts.json)."""
    g = GOLD["F4_northstar"]
    nR, nS = g["r"], g["s"]
    R = cuda.empty((nR, 2), dtype=cuda.int32, device="cuda")
    S = cuda.empty((nS, 2), dtype=cuda.int32, device="cuda")
    hw.generate_device(R, 2, nR, nR, 1.0, 12345)
    hw.generate_device(S, 2, INT_MAX, nR, g["q"], 54321)
    sec2 = [r for r in ORC_FULL if r["variant"] == "sectorized" and r["k"] == 2 and r["q"] == g["q"]
            and r["m"] == g["m"] and r["B"] == 1024][0]
    runs = [(hw.BloomFilterArgs(hw.BLOCKED, g["m"], 1, g["B"]), (g["k1_filtered"], g["results"])),
            (hw.BloomFilterArgs(hw.SECTORIZED, g["m"], 2, 1024), (sec2["filtered"], sec2["results"])),
            (hw.BloomFilterArgs(hw.BLOCKED, g["m"], 2, g["B"]), (g["k2_filtered"], g["results"])),
            (None, (nS, g["results"])),
            (hw.BloomFilterArgs(hw.BLOCKED, g["m"], 1, g["B"]), (g["k1_filtered"], g["results"]))]
    stream = cuda.cuda.Stream()
    for a, _ in runs:
        hw.join_device_async(R, S, a, stream=stream)
    sts = hw.join_wait_all()
    assert [(s.filtered, s.matches) for s in sts] == [w for _, w in runs]
    for _ in range(3):  # and the headline's exact loop
        hw.join_device_async(R, S, runs[0][0], stream=stream)
    assert [(s.filtered, s.matches) for s in hw.join_wait_all()] == [runs[0][1]] * 3
    del R, S
    cuda.cuda.empty_cache()


def test_async_timing_of_the_s_scatter(hw, cuda, rels, expected):
    """hwbrj_set_async_timing: every async join of a back-to-back run reports the device time of
    its S scatter as it ran on the side stream (ms_s_scatter > 0, the other phases 0), counts
    unchanged; off again, async joins report no phase time."""
    _, dR, _, dSs = rels
    a = mk(hw, CONFIGS[0])
    hw.set_async_timing(True)
    try:
        for si in range(3):
            hw.join_device_async(dR, dSs[si], a)
        sts = hw.join_wait_all()
    finally:
        hw.set_async_timing(False)
    assert [(s.filtered, s.matches) for s in sts] == [expected[0, si] for si in range(3)]
    assert all(s.ms_s_scatter > 0 and s.ms_probe == 0 and s.ms_total == 0 for s in sts), sts
    hw.join_device_async(dR, dSs[0], a)
    assert hw.join_wait().ms_s_scatter == 0
