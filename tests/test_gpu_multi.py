"""GPU tests of the multi-GPU machinery on one MI355X: the library's native RCCL transport
(hwbrj_comm.cpp) at world 1, the north_star's filter broadcast in the replicated design, bench.py's
N > 1 paths over the RCCL process group at world 1, and the partitioned join's status agreement
(a rank that fails alone makes every rank return instead of hanging in a collective).

RCCL refuses two ranks on one GPU, so runs with several ranks share the GPU over gloo
(HWBRJ_BENCH_SHARED_GPU=1) and the torch.distributed callback transport; the native transport and
the broadcast run at world 1, where their RCCL calls (grouped send/recv to self, in-place
all-gather, broadcast from rank 0) execute for real on the join stream.

Bar: bit-exact counts against the goldens or the oracle on the same inputs.
"""
import json
import os
import signal
import socket
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
GOLD = json.load(open(os.path.join(HERE, "golden", "survey_counts.json")))
INT_MAX = 2**31 - 1


def to_dev(cuda, a):
    return cuda.from_numpy(np.ascontiguousarray(a, dtype=np.int32)).cuda()


def rel(keys):
    keys = np.asarray(keys, dtype=np.int64).astype(np.int32)
    return np.stack([keys, np.arange(keys.size, dtype=np.int32)], 1)


def torchrun(world, args, env_extra, timeout=300, script=None):
    """bench.py (or `script` with `args`) under torch.distributed.run in its own process group,
    killed as a group on timeout (no rank outlives the test). Returns (returncode, stdout, stderr);
    returncode None = timeout."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, **env_extra)
    for k in ("HWBRJ_BENCH_SHARED_GPU", "HWBRJ_BENCH_DIST", "HWBRJ_PJ_FORCE_COLL", "HWBRJ_RCCL_SELF"):
        if k not in env_extra:
            env.pop(k, None)
    if script is None:
        target = [os.path.join(ROOT, "bench.py"), "--gpus", str(world), "--steps", "2", "--warmup", "1",
                  "--no-cpu-baseline", "--no-e2e"]
    else:
        target = [os.path.join(HERE, script)]
    p = subprocess.Popen(["python", "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
                          "--master-addr", "127.0.0.1", "--master-port", str(port)]
                         + target + [str(x) for x in args],
                         stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env, cwd=ROOT,
                         start_new_session=True)
    try:
        out, err = p.communicate(timeout=timeout)
        return p.returncode, out, err
    except subprocess.TimeoutExpired:
        os.killpg(p.pid, signal.SIGKILL)
        out, err = p.communicate()
        return None, out, err


def last_json(out):
    return json.loads([x for x in out.splitlines() if x.startswith("{")][-1])


# ------------------------------------------------------------ the native transport at world 1
@pytest.fixture
def rccl1(hw):
    from hwbloomradixjoin_amd import pjoin
    assert pjoin.comm_init() == (1, 0)  # no process group: a world-1 communicator
    yield pjoin
    pjoin.set_filter_broadcast(False)
    pjoin.comm_destroy()


PJ_ARGS = [None, ("blocked", 1 << 24, 1, 1024), ("blocked", 1 << 22, 3, 512), ("basic", 1 << 20, 1, 0),
           ("sectorized", 1 << 22, 4, 512), ("blocked", 1 << 31, 2, 512)]


@pytest.mark.parametrize("self_rccl", [False, True], ids=["self-copy", "self-rccl"])
@pytest.mark.parametrize("a", PJ_ARGS, ids=str)
def test_partitioned_rccl_world1_vs_oracle(hw, cuda, orc, rccl1, a, self_rccl, monkeypatch):
    """hwbrj_join_partitioned_rccl: the R-chunk and survivor all-to-alls as grouped
    ncclSend/ncclRecv and the slice all-gather as ncclAllGather on the join stream (no host drain
    before them); counts equal the oracle's, empty and odd-sized shards included. A rank's own
    block is a device copy; HWBRJ_RCCL_SELF=1 sends it through ncclSend/ncclRecv instead, so the
    RCCL calls run at world 1."""
    if self_rccl:
        monkeypatch.setenv("HWBRJ_RCCL_SELF", "1")
    args = None if a is None else hw.BloomFilterArgs.from_flag(a[0], a[1], a[2], a[3] or 1024)
    rng = np.random.default_rng(41)
    for nR, nS in [(0, 1000), (1000, 0), (7, 33), (100003, 400009), (1000000, 4000000)]:
        Rk = rng.permutation(nR).astype(np.int64) + 1
        Sk = rng.integers(0, 2 * max(nR, 1) + 2, size=nS)
        R, S = rel(Rk), rel(Sk)
        st = rccl1.join_partitioned_rccl(to_dev(cuda, R), to_dev(cuda, S), nR, args)
        if args is None:
            res, filt, _ = orc.bpro(R, S, 8, 0, 0, 0, 0, use_bloom=False)
        else:
            res, filt, _ = orc.bpro(R, S, 8, args.variant, args.m, args.k, args.B)
        assert (st.filtered, st.matches) == (filt, res), (a, nR, nS, st)


def test_partitioned_rccl_northstar(hw, cuda, rccl1):
    """The north-star golden through the native partitioned join."""
    g = GOLD["F4_northstar"]
    R = cuda.empty((g["r"], 2), dtype=cuda.int32, device="cuda")
    S = cuda.empty((g["s"], 2), dtype=cuda.int32, device="cuda")
    hw.generate_device(R, 2, g["r"], g["r"], 1.0, 12345)
    hw.generate_device(S, 2, INT_MAX, g["r"], g["q"], 54321)
    st = rccl1.join_partitioned_rccl(R, S, g["r"], hw.BloomFilterArgs(hw.BLOCKED, g["m"], 1, g["B"]))
    del R, S
    assert (st.filtered, st.matches) == (g["k1_filtered"], g["results"])


@pytest.mark.parametrize("a", [("blocked", 1 << 24, 1, 1024), ("blocked", 1 << 24, 4, 512),
                               ("sectorized", 1 << 24, 2, 1024), ("basic", 1 << 24, 1, 1024),
                               ("blocked", 1 << 31, 2, 512)], ids=str)
def test_filter_broadcast_world1(hw, cuda, orc, rccl1, a):
    """hwbrj_set_filter_broadcast: the replicated join with the slices built on rank 0 and sent by
    ncclBroadcast on the join stream (the north_star's bitmap broadcast). Counts equal the F3
    goldens / the oracle, and the exported filter is the reference layout's, bit for bit, as
    without the broadcast."""
    g = GOLD["F3_grid"]
    R = hw.generate_host(g["r"], 2, g["r"], g["r"], 1.0, 1)
    S = hw.generate_host(g["s"], 2, INT_MAX, g["r"], g["q"], 2)
    args = hw.BloomFilterArgs.from_flag(*a)
    dR, dS = to_dev(cuda, R), to_dev(cuda, S)
    plain = hw.join_device(dR, dS, args)
    want = hw.export_filter(a[1]).copy()
    rccl1.set_filter_broadcast(True)
    st = hw.join_device(dR, dS, args)
    assert (st.filtered, st.matches) == (plain.filtered, plain.matches)
    assert np.array_equal(hw.export_filter(a[1]), want)
    res, filt, _ = orc.bpro(R, S, 8, args.variant, args.m, args.k, args.B)
    assert (st.filtered, st.matches) == (filt, res)


# ------------------------------------------------- bench.py over the RCCL process group, world 1
@pytest.mark.parametrize("case", ["partitioned-native", "partitioned-native-sync", "partitioned-torch-nccl",
                                  "replicated-bcast"])
def test_bench_rccl_world1(hw, case):
    """bench.py's multi-GPU designs under torch.distributed.run with the RCCL ("nccl") group at
    world 1 (HWBRJ_BENCH_DIST=1): the native partitioned transport (the async join, K joins back to
    back with no overflow rerun in the timed region; and the synchronous one), the torch callback
    transport with its collectives forced (HWBRJ_PJ_FORCE_COLL=1: all_to_all_single /
    all_gather_into_tensor on device uint8 over RCCL), and the replicated design with the filter
    broadcast."""
    g = GOLD["F3_grid"]
    base = ["-r", g["r"], "-s", g["s"], "-m", g["m"]]
    env = {"HWBRJ_BENCH_DIST": "1"}
    if case.startswith("partitioned-native"):  # (the rank's own blocks through ncclSend / ncclRecv too)
        args = base + ["--design", "partitioned", "--transport", "native"]
        if case.endswith("sync"):
            args.append("--pj-sync")
        env["HWBRJ_RCCL_SELF"] = "1"
    elif case == "partitioned-torch-nccl":
        args = base + ["--design", "partitioned", "--transport", "torch"]
        env["HWBRJ_PJ_FORCE_COLL"] = "1"
    else:
        args = base + ["--filter-bcast"]
    rc, out, err = torchrun(1, args, env)
    assert rc == 0, out[-2000:] + err[-3000:]
    line = last_json(out)
    assert (line["parity"]["filtered"], line["parity"]["matches"]) == (g["rows"]["1024"][0], g["results"])
    assert line["dist"]["backend"] == "nccl" and line["dist"]["world_size_seen"] == 1
    assert line["scaling"] == "strong"
    if case == "partitioned-native":
        pa = line["pj_async"]
        assert pa["reruns_in_timed"] == 0 and pa["async_in_timed"] == line["steps"], pa
        assert pa["rank0_counts_all_equal"] and pa["events_ms_per_join_rank0"] > 0, pa
    elif case == "partitioned-native-sync":
        assert line["pj_async"] is None


# ------------------------------------------------- status agreement (no hang on one rank's error)
@pytest.mark.parametrize("fail_rank", [0, 1])
def test_partitioned_rank_failure_does_not_hang(hw, fail_rank):
    """One rank of two fails the capacity check alone (HWBRJ_HOOK_PJ_FAIL_RANK, as an oversized
    shard would): the ranks agree on their statuses before the first collective, so both return an
    error promptly (torch.distributed.run exits nonzero) instead of the other rank waiting in the
    R all-to-all forever. Without the hook the same run succeeds and its counts sum to the golden."""
    g = GOLD["F3_grid"]
    args = [g["r"], g["s"], g["m"]]
    rc, out, err = torchrun(2, [fail_rank] + args, {}, timeout=240, script="pj_rank_worker.py")
    assert rc is not None, "ranks hung: " + err[-3000:]
    assert rc != 0
    assert "shard too large" in err
    assert f"rank {fail_rank} failed" in err
    if fail_rank == 1:
        rc, out, err = torchrun(2, [-1] + args, {}, timeout=240, script="pj_rank_worker.py")
        assert rc == 0, err[-3000:]
        ok = [line.split()[-2:] for line in out.splitlines() if line.startswith("sum: ok ")]
        assert len(ok) == 1, out[-2000:]
        assert (int(ok[0][0]), int(ok[0][1])) == (g["rows"]["1024"][0], g["results"])


def test_partitioned_rccl_failure_world1(hw, cuda, orc, rccl1, hook):
    """The native transport's status agreement with a failing rank: at world 1
    the rank fails its shard check (HWBRJ_HOOK_PJ_FAIL_RANK = 0), hwbrj_join_partitioned_rccl
    returns the error instead of entering a collective, and the next join on the same Engine and
    communicator is correct."""
    g = GOLD["F3_grid"]
    R = hw.generate_host(g["r"], 2, g["r"], g["r"], 1.0, 1)
    S = hw.generate_host(g["s"], 2, INT_MAX, g["r"], g["q"], 2)
    dR, dS = to_dev(cuda, R), to_dev(cuda, S)
    args = hw.BloomFilterArgs(hw.BLOCKED, g["m"], 1, 1024)
    hook(hw.HOOK_PJ_FAIL_RANK, 0)
    with pytest.raises(RuntimeError, match="shard too large"):
        rccl1.join_partitioned_rccl(dR, dS, g["r"], args)
    hw.set_test_hook(hw.HOOK_PJ_FAIL_RANK, -1)
    st = rccl1.join_partitioned_rccl(dR, dS, g["r"], args)
    assert (st.filtered, st.matches) == (g["rows"]["1024"][0], g["results"])


def test_partitioned_rccl_understated_r_total(hw, cuda, orc, rccl1):
    """the receive bounds of the native transport come from the caller's nR_total. Every
    rank's |R| shard travels with the R counts, so shards that sum to more than nR_total fail on every
    rank alike before the R all-to-all (code 2), and the next join is correct."""
    g = GOLD["F3_grid"]
    R = hw.generate_host(g["r"], 2, g["r"], g["r"], 1.0, 1)
    S = hw.generate_host(g["s"], 2, INT_MAX, g["r"], g["q"], 2)
    dR, dS = to_dev(cuda, R), to_dev(cuda, S)
    args = hw.BloomFilterArgs(hw.BLOCKED, g["m"], 1, 1024)
    with pytest.raises(RuntimeError, match="R shards hold"):
        rccl1.join_partitioned_rccl(dR, dS, g["r"] // 2, args)
    st = rccl1.join_partitioned_rccl(dR, dS, g["r"], args)
    assert (st.filtered, st.matches) == (g["rows"]["1024"][0], g["results"])


@pytest.mark.parametrize("a", [("blocked", 1 << 24, 1, 1024), ("sectorized", 1 << 24, 2, 1024),
                               ("basic", 1 << 24, 1, 1024), ("blocked", 1 << 31, 2, 512)], ids=str)
def test_filter_broadcast_nonroot_world1(hw, cuda, orc, rccl1, hook, a):
    """The broadcast join's non-root side (BuildParams::no_slices: k_build sub-partitions R for the
    join and writes no filter slice; the slices arrive by ncclBroadcast), which a world-1 run never
    takes by itself. HWBRJ_HOOK_BCAST_NONROOT = 1: the slices the root join
    left in place are received unchanged (a broadcast from rank 0 at world 1), and the counts equal
    the oracle's, so the non-root R runs are right. = 2: the slices are zeroed first; the filter
    then rejects every S tuple, so the non-root k_build wrote no slice."""
    g = GOLD["F3_grid"]
    R = hw.generate_host(g["r"], 2, g["r"], g["r"], 1.0, 1)
    S = hw.generate_host(g["s"], 2, INT_MAX, g["r"], g["q"], 2)
    args = hw.BloomFilterArgs.from_flag(*a)
    dR, dS = to_dev(cuda, R), to_dev(cuda, S)
    res, filt, _ = orc.bpro(R, S, 8, args.variant, args.m, args.k, args.B)
    rccl1.set_filter_broadcast(True)
    st = hw.join_device(dR, dS, args)  # as the root: builds the slices
    assert (st.filtered, st.matches) == (filt, res)
    hook(hw.HOOK_BCAST_NONROOT, 1)
    st = hw.join_device(dR, dS, args)
    assert (st.filtered, st.matches) == (filt, res)
    hook(hw.HOOK_BCAST_NONROOT, 2)
    st = hw.join_device(dR, dS, args)
    assert (st.filtered, st.matches) == (0, 0)
    hook(hw.HOOK_BCAST_NONROOT, 0)
    st = hw.join_device(dR, dS, args)  # the root again rebuilds them
    assert (st.filtered, st.matches) == (filt, res)


# ------------------------------------------------- the async partitioned join
def _ref_counts(orc, R, S, args):
    if args is None:
        res, filt, _ = orc.bpro(R, S, 8, 0, 0, 0, 0, use_bloom=False)
    else:
        res, filt, _ = orc.bpro(R, S, 8, args.variant, args.m, args.k, args.B)
    return filt, res


@pytest.mark.parametrize("self_rccl", [False, True], ids=["self-copy", "self-rccl"])
@pytest.mark.parametrize("a", PJ_ARGS, ids=str)
def test_partitioned_async_world1_vs_oracle(hw, cuda, orc, rccl1, a, self_rccl, monkeypatch):
    """hwbrj_join_partitioned_rccl_async: the first join of a shape runs synchronously and makes the
    plan; the next ones (3 enqueued back to back, no host wait between them) use padded exchanges
    and device-built owner tables, with no rerun. Every join's counts equal the oracle's; a new
    shape's first join finds the old plan (the failed mode: it is rerun synchronously, same counts,
    and makes the new plan). HWBRJ_RCCL_SELF=1 puts the padded blocks and the flag's all-reduce through RCCL."""
    if self_rccl:
        monkeypatch.setenv("HWBRJ_RCCL_SELF", "1")
    args = None if a is None else hw.BloomFilterArgs.from_flag(a[0], a[1], a[2], a[3] or 1024)
    rng = np.random.default_rng(43)
    for nR, nS in [(0, 1000), (7, 33), (100003, 400009), (1000000, 4000000)]:
        Rk = rng.permutation(nR).astype(np.int64) + 1
        Sk = rng.integers(0, 2 * max(nR, 1) + 2, size=nS)
        R, S = rel(Rk), rel(Sk)
        want = _ref_counts(orc, R, S, args)
        dR, dS = to_dev(cuda, R), to_dev(cuda, S)
        # a new shape: the plan join (synchronous, or the failed mode rerun), then 3 back to back
        rccl1.join_partitioned_rccl_async(dR, dS, nR, args)
        st = rccl1.join_partitioned_wait()
        assert (st.filtered, st.matches) == want, (a, nR, nS, st)
        i0 = rccl1.pj_async_info()
        assert i0["plan_valid"] == 1 and i0["last_rerun_flag"] in (0, 2), i0
        for _ in range(3):
            rccl1.join_partitioned_rccl_async(dR, dS, nR, args)
        assert rccl1.pj_async_info()["in_flight"] == 3
        for k in range(3):
            st = rccl1.join_partitioned_wait()
            assert (st.filtered, st.matches) == want, (a, nR, nS, k, st)
        i1 = rccl1.pj_async_info()
        assert i1["in_flight"] == 0 and i1["async_joins"] - i0["async_joins"] == 3, (i0, i1)
        assert i1["overflow_reruns"] == i0["overflow_reruns"], (i0, i1)
        del dR, dS


def test_partitioned_async_northstar_back_to_back(hw, cuda, rccl1):
    """The north-star golden through the async join: the plan join, then 3 joins
    enqueued back to back; each join's device time is reported from its HIP events."""
    g = GOLD["F4_northstar"]
    R = cuda.empty((g["r"], 2), dtype=cuda.int32, device="cuda")
    S = cuda.empty((g["s"], 2), dtype=cuda.int32, device="cuda")
    hw.generate_device(R, 2, g["r"], g["r"], 1.0, 12345)
    hw.generate_device(S, 2, INT_MAX, g["r"], g["q"], 54321)
    args = hw.BloomFilterArgs(hw.BLOCKED, g["m"], 1, g["B"])
    i0 = rccl1.pj_async_info()  # (the counters are the Engine's, over every communicator)
    for _ in range(4):
        rccl1.join_partitioned_rccl_async(R, S, g["r"], args)
    sts = [rccl1.join_partitioned_wait() for _ in range(4)]
    info = rccl1.pj_async_info()
    del R, S
    for st in sts:
        assert (st.filtered, st.matches) == (g["k1_filtered"], g["results"])
    assert info["overflow_reruns"] == i0["overflow_reruns"], (i0, info)
    assert info["async_joins"] - i0["async_joins"] == 3 and info["sync_plan_joins"] - i0["sync_plan_joins"] == 1
    assert all(st.ms_total > 0 for st in sts[1:])
    assert info["BR"] >= info["last_r_block"] and info["BW"] >= info["last_word_block"], info


def test_partitioned_async_overflow_rerun_world1(hw, cuda, orc, rccl1, hook):
    """A plan too small for the join (HWBRJ_HOOK_PJ_PLAN_DIV divides its block bounds): the padded
    blocks overflow, the device flag is set, and the wait reruns the join synchronously -- counts
    unchanged -- and makes a new plan; once the hook is off, the plan it makes holds and the joins
    run async without reruns."""
    g = GOLD["F3_grid"]
    R = hw.generate_host(g["r"], 2, g["r"], g["r"], 1.0, 1)
    S = hw.generate_host(g["s"], 2, INT_MAX, g["r"], g["q"], 2)
    dR, dS = to_dev(cuda, R), to_dev(cuda, S)
    args = hw.BloomFilterArgs(hw.BLOCKED, g["m"], 1, 1024)
    want = (g["rows"]["1024"][0], g["results"])
    i0 = rccl1.pj_async_info()  # (the counters are the Engine's, over every communicator)
    hook(hw.HOOK_PJ_PLAN_DIV, 8)
    rccl1.join_partitioned_rccl_async(dR, dS, g["r"], args)  # (synchronous: makes the small plan)
    rccl1.join_partitioned_rccl_async(dR, dS, g["r"], args)  # (overflows)
    for _ in range(2):
        st = rccl1.join_partitioned_wait()
        assert (st.filtered, st.matches) == want
    i = rccl1.pj_async_info()
    assert i["overflow_reruns"] - i0["overflow_reruns"] == 1 and i["last_rerun_flag"] == 1, (i0, i)
    assert i["plan_valid"] == 1
    hw.set_test_hook(hw.HOOK_PJ_PLAN_DIV, 0)
    # the plan the rerun made under the hook is still too small: one more overflow, whose rerun
    # (hook off) makes a plan that holds
    rccl1.join_partitioned_rccl_async(dR, dS, g["r"], args)
    st = rccl1.join_partitioned_wait()
    assert (st.filtered, st.matches) == want
    i2 = rccl1.pj_async_info()
    assert i2["overflow_reruns"] - i0["overflow_reruns"] == 2, (i0, i2)
    for _ in range(3):
        rccl1.join_partitioned_rccl_async(dR, dS, g["r"], args)
    for _ in range(3):
        st = rccl1.join_partitioned_wait()
        assert (st.filtered, st.matches) == want
    i3 = rccl1.pj_async_info()
    assert i3["overflow_reruns"] == i2["overflow_reruns"] and i3["async_joins"] - i2["async_joins"] == 3, (i2, i3)


def test_partitioned_async_failed_mode_world1(hw, cuda, orc, rccl1, hook):
    """The failed mode (HWBRJ_HOOK_PJ_ASYNC_FAIL: this rank sends empty counts messages with a failed
    status, as after a shape change, and still takes part in every collective): the flag is set on
    every rank, the wait reruns the join synchronously and the counts are right. A join of another
    shape than the plan's takes the same path by itself. Also: more than 8 joins in flight is
    refused, and a wait with none in flight is an error."""
    g = GOLD["F3_grid"]
    R = hw.generate_host(g["r"], 2, g["r"], g["r"], 1.0, 1)
    S = hw.generate_host(g["s"], 2, INT_MAX, g["r"], g["q"], 2)
    dR, dS = to_dev(cuda, R), to_dev(cuda, S)
    args = hw.BloomFilterArgs(hw.BLOCKED, g["m"], 1, 1024)
    want = (g["rows"]["1024"][0], g["results"])
    with pytest.raises(RuntimeError, match="no partitioned join"):
        rccl1.join_partitioned_wait()
    i0 = rccl1.pj_async_info()  # (the counters are the Engine's, over every communicator)
    rccl1.join_partitioned_rccl_async(dR, dS, g["r"], args)
    assert (lambda s: (s.filtered, s.matches))(rccl1.join_partitioned_wait()) == want
    hook(hw.HOOK_PJ_ASYNC_FAIL, 1)
    rccl1.join_partitioned_rccl_async(dR, dS, g["r"], args)
    st = rccl1.join_partitioned_wait()
    assert (st.filtered, st.matches) == want
    i = rccl1.pj_async_info()
    assert i["overflow_reruns"] - i0["overflow_reruns"] == 1 and i["last_rerun_flag"] == 2, (i0, i)
    hw.set_test_hook(hw.HOOK_PJ_ASYNC_FAIL, 0)
    # another shape: half of S
    half = S[: S.shape[0] // 2]
    res, filt, _ = orc.bpro(R, half, 8, args.variant, args.m, args.k, args.B)
    dH = to_dev(cuda, half)
    rccl1.join_partitioned_rccl_async(dR, dH, g["r"], args)
    st = rccl1.join_partitioned_wait()
    assert (st.filtered, st.matches) == (filt, res)
    assert rccl1.pj_async_info()["overflow_reruns"] - i0["overflow_reruns"] == 2
    for _ in range(8):
        rccl1.join_partitioned_rccl_async(dR, dH, g["r"], args)
    with pytest.raises(RuntimeError, match="too many"):
        rccl1.join_partitioned_rccl_async(dR, dH, g["r"], args)
    for _ in range(8):
        st = rccl1.join_partitioned_wait()
        assert (st.filtered, st.matches) == (filt, res)
    # a single-GPU join after async ones on the same Engine is ordered after them and correct
    st = hw.join_device(dR, dS, args)
    assert (st.filtered, st.matches) == want
    # arguments the partitioned join refuses (basic k = 2: no partition slices), after a plan: the
    # join runs in the failed mode, its wait reruns it synchronously, which returns the error; the
    # plan is dropped and the next join (synchronous, a new plan) is right
    rccl1.join_partitioned_rccl_async(dR, dS, g["r"], hw.BloomFilterArgs(hw.BASIC, 1 << 24, 2, 1024))
    with pytest.raises(RuntimeError, match="partition slices"):
        rccl1.join_partitioned_wait()
    assert rccl1.pj_async_info()["plan_valid"] == 0
    rccl1.join_partitioned_rccl_async(dR, dS, g["r"], args)
    st = rccl1.join_partitioned_wait()
    assert (st.filtered, st.matches) == want


def test_bench_alt_watchdog_world1(hw):
    """bench.py's alt_designs legs each run under their own watchdog (a collective that never
    completes on a node must not cost the headline, nor the legs before it): the bcast leg is made
    to stall (HWBRJ_BENCH_HOOK_STALL_LEG). Rank 0 still prints the headline line, its parity ok, with
    partitioned_async (the first leg) reported with the F3 counts, bcast named as the timed-out leg,
    partitioned as not run, and the run exits non-zero (status 124 on the rank)."""
    g = GOLD["F3_grid"]
    rc, out, err = torchrun(1, ["-r", g["r"], "-s", g["s"], "-m", g["m"], "--alt-timeout", "30"],
                            {"HWBRJ_BENCH_DIST": "1", "HWBRJ_BENCH_HOOK_STALL_LEG": "bcast"})
    assert rc not in (0, None), out[-2000:] + err[-3000:]
    line = last_json(out)
    want = [g["rows"]["1024"][0], g["results"]]
    assert [line["parity"]["filtered"], line["parity"]["matches"]] == want
    alt = line["alt_designs"]
    assert alt["timed_out_leg"] == "bcast" and alt["timeout_s"] == 30 and alt["not_run"] == ["partitioned"], alt
    assert alt["partitioned_async"]["sum"] == want, alt
    assert "bcast" not in alt and "partitioned" not in alt, alt


def test_partitioned_async_after_release_world1(hw, cuda, orc, rccl1):
    """hwbrj_release between async joins frees the plan's buffers: the next async join runs in the
    failed mode (every collective with empty messages, flag 2), its wait reruns it synchronously
    with the right counts and makes a new plan, and the join after that is async again. PRO (no
    filter) and a sectorized filter, the two other slice paths."""
    rng = np.random.default_rng(47)
    nR, nS = 300007, 1200011
    Rk = rng.permutation(nR).astype(np.int64) + 1
    Sk = rng.integers(0, 2 * nR, size=nS)
    R, S = rel(Rk), rel(Sk)
    dR, dS = to_dev(cuda, R), to_dev(cuda, S)
    for args in (None, hw.BloomFilterArgs.from_flag("sectorized", 1 << 24, 2, 512)):
        want = _ref_counts(orc, R, S, args)
        for _ in range(2):  # the plan join, then an async one
            rccl1.join_partitioned_rccl_async(dR, dS, nR, args)
        for _ in range(2):
            st = rccl1.join_partitioned_wait()
            assert (st.filtered, st.matches) == want, (args, st)
        hw.lib().hwbrj_release()
        i0 = rccl1.pj_async_info()
        for _ in range(2):  # failed mode (rerun: a new plan), then async on the new plan
            rccl1.join_partitioned_rccl_async(dR, dS, nR, args)
            st = rccl1.join_partitioned_wait()
            assert (st.filtered, st.matches) == want, (args, st)
        i1 = rccl1.pj_async_info()
        assert i1["overflow_reruns"] - i0["overflow_reruns"] == 1 and i1["last_rerun_flag"] == 2, (i0, i1)
        assert i1["async_joins"] - i0["async_joins"] == 2 and i1["plan_valid"] == 1, (i0, i1)


@pytest.mark.parametrize("scen,world,flt", [("steady", 2, "blocked"), ("overflow", 2, "blocked"), ("shape", 2, "blocked"),
                                            ("fail1", 2, "blocked"), ("steady", 4, "blocked"), ("overflow", 4, "blocked"),
                                            ("steady", 2, "pro"), ("steady", 4, "sect")])
def test_partitioned_async_ranks_shared_gpu(hw, orc, scen, world, flt):
    """The async partitioned join with two and four ranks (hwbrj_join_partitioned_async over
    torch.distributed gloo callbacks, every rank on the one GPU): the W > 1 parts of the padded layout -- destination
    blocks found among the block starts, two sources per owner table, survivor blocks per source --
    the plan max-reduced over the ranks, and the collective reruns: a plan too small (the flag set
    on a rank reruns the join on both), a shard that changes size on one rank only (the failed mode
    there), a rank forced into the failed mode. Counts summed over the ranks equal F3 (or, for the
    changed shard, the oracle on the same shards). PRO and sectorized k = 2 are checked against the
    oracle on the same relations (hwbrj.generate_host, the generator the ranks' shards come from)."""
    g = GOLD["F3_grid"]
    rc, out, err = torchrun(world, [scen, g["r"], g["s"], g["m"], flt], {}, timeout=300, script="pj_async_worker.py")
    assert rc == 0, out[-2000:] + err[-3000:]
    sums = [tuple(int(v) for v in l.split()[-2:]) for l in out.splitlines() if l.startswith("sum: ok ")]
    info = [[int(v) for v in l.split()[1:]] for l in out.splitlines() if l.startswith("info: ")]
    assert len(info) == 1, out[-2000:]
    n_async, reruns, flag, plan_joins = info[0]
    assert plan_joins == 1
    want = (g["rows"]["1024"][0], g["results"])
    R = S = None
    if flt != "blocked" or scen == "shape":  # the oracle on the same relations (F3 holds blocked k = 1)
        R = hw.generate_host(g["r"], 2, g["r"], g["r"], 1.0, 12345, 8)
        S = hw.generate_host(g["s"], 2, INT_MAX, g["r"], 0.01, 54321, 8)
    if flt != "blocked":
        want = _ref_counts(orc, R, S, None if flt == "pro" else
                           hw.BloomFilterArgs.from_flag("sectorized", g["m"], 2, 512))
    if scen == "steady":
        assert sums == [want] * 4 and (n_async, reruns) == (3, 0), out[-2000:]
    elif scen == "overflow":
        assert sums == [want] * 2 and (n_async, reruns, flag) == (1, 1, 1), out[-2000:]
    elif scen == "fail1":
        assert sums == [want] * 2 and (n_async, reruns, flag) == (1, 1, 2), out[-2000:]
    else:
        # rank 1's S shard lost its last 1000 rows (pj_async_worker.py "shape"): the oracle on them
        lo, hi = hw.shard_range(g["s"], 1, world)
        shaped = np.concatenate([S[:hi - 1000], S[hi:]])
        got = _ref_counts(orc, R, shaped, hw.BloomFilterArgs(hw.BLOCKED, g["m"], 1, 1024))
        sync = [tuple(int(v) for v in l.split()[-2:]) for l in out.splitlines() if l.startswith("sync: ")]
        assert sums[0] == want and sums[1] == got == sync[0] and sums[1] != want, out[-2000:]
        assert (n_async, reruns, flag) == (1, 1, 2), out[-2000:]
