"""GPU tests of the operator surface beyond single-device counts: the multi-GPU sharding behind
BPRO / the CLI (--gpus), the print_timing contract, stream ordering of back-to-back joins, the
.tbl loader, the device Zipf generator, and edge cases the round-1 suite left out (basic filters
on structured keys, m = 2^32, basic k >= 2 on the materialization and skew-split paths).

Bar: bit-exact counts against the goldens or the oracle on the same inputs.
"""
import json
import os
import re
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = json.load(open(os.path.join(HERE, "golden", "survey_counts.json")))
ORC = json.load(open(os.path.join(HERE, "golden", "oracle_counts.json")))
INT_MAX = 2**31 - 1


def to_dev(cuda, a):
    return cuda.from_numpy(np.ascontiguousarray(a, dtype=np.int32)).cuda()


def rel(keys):
    keys = np.asarray(keys, dtype=np.int64).astype(np.int32)
    return np.stack([keys, np.arange(keys.size, dtype=np.int32)], 1)


def cli(hw, *args, timeout=600):
    out = subprocess.run([hw.CLI_PATH, *map(str, args)], capture_output=True, text=True,
                         timeout=timeout)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
    return out.stdout


def counts(stdout):
    f = re.search(r"S-tuples after filter: (\d+)", stdout)
    r = re.search(r"\[INFO \] Results = (\d+)\. DONE\.", stdout)
    return (int(f.group(1)) if f else None), int(r.group(1))


@pytest.mark.parametrize("gpus", [2, 8])
def test_cli_gpus_shards_golden(hw, gpus):
    """--gpus=G: S range-sharded into G shards (here all on the one visible device, one after the
    other; on a node shard g runs on device g mod #devices), R replicated, counts summed. The sums
    are the single-device golden."""
    g = GOLD["F3_grid"]
    out = cli(hw, "-a", "PRO", "-r", g["r"], "-s", g["s"], "-q", "0.01", "-b", "blocked",
              "-m", g["m"], "-k", 1, "-n", 2, f"--gpus={gpus}")
    assert counts(out) == (g["rows"]["1024"][0], g["results"])


def test_bpro_set_gpus(hw):
    g = GOLD["F3_grid"]
    R = hw.Relation(hw.generate_host(g["r"], 2, g["r"], g["r"], 1.0, 1))
    S = hw.Relation(hw.generate_host(g["s"], 2, INT_MAX, g["r"], g["q"], 2))
    hw.set_gpus(8)
    try:
        for k, want in zip(g["k"], g["rows"]["512"]):
            res = hw.BPRO(R, S, 4, hw.BloomFilterArgs(hw.BLOCKED, g["m"], k, 512))
            assert res.totalresults == g["results"]
        assert hw.PRO(R, S, 2).totalresults == g["results"]
    finally:
        hw.set_gpus(0)


def test_print_timing_contract(hw, capfd):
    """print_timing (src/parallel_radix_join_bloom.c:1509-1547): PROBE-TIME-USECS is the probe
    share of the join, so 0 < probe <= join; PARTITION + JOIN = TOTAL. BRJ prints no
    'S-tuples after filter' line (src/parallel_radix_join_bloom.c:1807-1975)."""
    g = GOLD["F3_grid"]
    R = hw.Relation(hw.generate_host(g["r"], 2, g["r"], g["r"], 1.0, 1))
    S = hw.Relation(hw.generate_host(g["s"], 2, INT_MAX, g["r"], g["q"], 2))
    a = hw.BloomFilterArgs(hw.BLOCKED, g["m"], 1, 1024)
    capfd.readouterr()
    hw.BPRO(R, S, 2, a)
    out = capfd.readouterr().out
    lines = out.splitlines()
    tot = float(lines[lines.index("TOTAL-TIME-USECS, TOTAL-TUPLES, NSEC-PER-TUPLE: ") + 1].split()[0])
    part, probe, join = (float(x) for x in
                         lines[lines.index("PARTITION-TIME-USECS, PROBE-TIME-USECS, JOIN-TIME-USECS: ") + 1].split())
    assert 0 < probe <= join and abs(part + join - tot) < 1e-3 * tot + 1
    cyc = [int(x) for x in lines[lines.index("RUNTIME TOTAL, BUILD, PART (cycles): ") + 1].split()]
    assert cyc[0] > cyc[2] > 0 and 0 <= cyc[1] < cyc[0]
    assert "S-tuples after filter" in out
    hw.BRJ(R, S, 2, a)
    out = capfd.readouterr().out
    assert "S-tuples after filter" not in out and "TOTAL-TIME-USECS" in out


def test_timing_cycles_cover_the_device_join(hw, capfd):
    """RUNTIME TOTAL (cycles) and TOTAL-TIME-USECS time the same region, as in the reference
    (src/parallel_radix_join_bloom.c:1107-1131, :1477-1484): the H2D copies and allocations are
    staged before the cycle counter starts, so cycles / TSC rate is the device join plus the launch
    and completion latency (5 % + 0.25 ms), not the ~PCIe copy of S."""
    nR, nS = 32000000, 256000000
    R = hw.Relation(hw.generate_host(nR, 2, nR, nR, 1.0, 1))
    S = hw.Relation(hw.generate_host(nS, 2, INT_MAX, nR, 0.01, 2))
    a = hw.BloomFilterArgs(hw.BLOCKED, 1 << 28, 1, 1024)
    hz = hw.lib().hwbrj_tsc_hz()
    assert hz > 1e8
    for _ in range(2):  # (the first call also loads the kernels)
        capfd.readouterr()
        hw.BPRO(R, S, 2, a)
        lines = capfd.readouterr().out.splitlines()
    tot = float(lines[lines.index("TOTAL-TIME-USECS, TOTAL-TUPLES, NSEC-PER-TUPLE: ") + 1].split()[0])
    cyc = int(lines[lines.index("RUNTIME TOTAL, BUILD, PART (cycles): ") + 1].split()[0])
    host_us = cyc / hz * 1e6
    assert tot > 300 and abs(host_us - tot) <= 0.05 * tot + 250, (host_us, tot)


def test_joins_on_two_streams_are_ordered(hw, cuda):
    """A join enqueued on one stream and the next on another share the device's scratch: the second
    waits for the first (hwbrj_engine.cpp enqueue). Both end with the golden counts."""
    g = GOLD["F3_grid"]
    R = cuda.empty((g["r"], 2), dtype=cuda.int32, device="cuda")
    S = cuda.empty((g["s"], 2), dtype=cuda.int32, device="cuda")
    hw.generate_device(R, 2, g["r"], g["r"], 1.0, 11)
    hw.generate_device(S, 2, INT_MAX, g["r"], g["q"], 22)
    s1, s2 = cuda.cuda.Stream(), cuda.cuda.Stream()
    a1 = hw.BloomFilterArgs(hw.BLOCKED, g["m"], 1, 1024)
    a2 = hw.BloomFilterArgs(hw.BASIC, g["m"], 2, 1024)
    for _ in range(3):
        hw.join_device_async(R, S, a1, stream=s1)
        st = hw.join_device(R, S, a2)  # the library's own stream
        assert (st.filtered, st.matches) == (g["rows"]["basic"][1], g["results"])
        hw.join_device_async(R, S, a2, stream=s1)
        hw.join_device_async(R, S, a1, stream=s2)
        sts = hw.join_wait_all()
        assert [(st.filtered, st.matches) for st in sts] == [(g["rows"]["basic"][1], g["results"]),
                                                             (g["rows"]["1024"][0], g["results"])]


def test_back_to_back_joins_of_mixed_configs_on_one_stream(hw, cuda):
    """Async joins of different filter configurations back to back on one stream: no wait packet
    between them (stream order), the counts zeroed by each join's own first kernel (the R scatter's
    workgroup 0; the basic k >= 2 pipeline zeroes by memset), the job table cleared when its layout
    changes. Every join's counts (hwbrj_join_wait_all) are its golden's."""
    g = GOLD["F3_grid"]
    R = cuda.empty((g["r"], 2), dtype=cuda.int32, device="cuda")
    S = cuda.empty((g["s"], 2), dtype=cuda.int32, device="cuda")
    hw.generate_device(R, 2, g["r"], g["r"], 1.0, 11)
    hw.generate_device(S, 2, INT_MAX, g["r"], g["q"], 22)
    s1 = cuda.cuda.Stream()
    blocked = hw.BloomFilterArgs(hw.BLOCKED, g["m"], 1, 1024)
    basic2 = hw.BloomFilterArgs(hw.BASIC, g["m"], 2, 1024)
    basic1 = hw.BloomFilterArgs(hw.BASIC, g["m"], 1, 1024)
    want = {id(blocked): g["rows"]["1024"][0], id(basic2): g["rows"]["basic"][1], id(basic1): g["rows"]["basic"][0]}
    for seq in ((basic2, blocked, basic1), (blocked, basic1, basic2), (basic1, basic2, blocked), (blocked, blocked)):
        for a in seq:
            hw.join_device_async(R, S, a, stream=s1)
        sts = hw.join_wait_all()
        assert [(st.filtered, st.matches) for st in sts] == [(want[id(a)], g["results"]) for a in seq], seq
    st = hw.join_device(R, S, basic1)
    assert (st.filtered, st.matches) == (want[id(basic1)], g["results"])


def test_tbl_loader(hw, orc, tmp_path):
    """-R / -S files (src/generator.c:685-741 read_relation): header line skipped, 'key payload',
    'key,payload' and bare-key formats, a [WARN ] line for the first negative key. Counts equal the
    oracle's on the parsed relations."""
    rng = np.random.default_rng(8)
    Rk = rng.permutation(200000).astype(np.int64) - 5  # includes negative keys
    Sk = rng.integers(-10, 400000, size=900000)
    Rp = rng.integers(0, 2**31 - 1, size=Rk.size)
    fr, fs, fb = tmp_path / "R.tbl", tmp_path / "S.tbl", tmp_path / "Sb.tbl"
    fr.write_text("key payload\n" + "".join(f"{k} {p}\n" for k, p in zip(Rk, Rp)))
    fs.write_text("key,payload\n" + "".join(f"{k},{i}\n" for i, k in enumerate(Sk)))
    fb.write_text("key\n" + "".join(f"{k}\n" for k in Sk))
    R = np.stack([Rk, Rp], 1).astype(np.int32)
    S = rel(Sk)
    res, filt, _ = orc.bpro(R, S, 8, 1, 1 << 22, 2, 512, True)
    for sfile in (fs, fb):
        out = cli(hw, "-a", "PRO", "-r", Rk.size, "-s", Sk.size, "-R", fr, "-S", sfile,
                  "-b", "blocked", "-m", 1 << 22, "-k", 2, "-B", 512)
        assert "[INFO ] Loading relation R with size" in out
        assert "[INFO ] Loading relation S with size" in out
        assert re.search(r"\[WARN \] key=-\d+, payload=\d+", out)
        assert counts(out) == (filt, res)


def test_cli_persist_round_trip(hw, orc, tmp_path):
    """--persist (a -DPERSIST_RELATIONS reference build, src/generator.c:408-412 and
    src/main.c:482-485): the CLI writes R.tbl and S.tbl as it generates them and, materializing,
    the pairs to Out.tbl (src/tuple_buffer.h:155-236). Out.tbl is the oracle's pair multiset on the
    written relations, and -R R.tbl -S S.tbl reproduces the counts."""
    def run(*args):
        out = subprocess.run([hw.CLI_PATH, *map(str, args)], capture_output=True, text=True, timeout=600,
                             cwd=tmp_path, env=dict(os.environ, HWBRJ_MATERIALIZE="1"))
        assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
        return out.stdout
    flags = ["-a", "PRO", "-r", 200000, "-s", 1000000, "-q", 0.05, "-b", "blocked", "-m", 1 << 22, "-k", 2]
    out = run(*flags, "--persist")
    assert '[INFO ] Persisting the join result to "Out.tbl" ...' in out
    load = lambda f: np.loadtxt(tmp_path / f, dtype=np.int64, comments="#", ndmin=2).astype(np.int32)  # noqa: E731
    R, S, pairs = load("R.tbl"), load("S.tbl"), load("Out.tbl")
    assert (tmp_path / "R.tbl").read_text().startswith("#KEY, VAL\n") and R.shape == (200000, 2)
    res, filt, _ = orc.bpro(R, S, 8, hw.BLOCKED, 1 << 22, 2, 1024)
    assert counts(out) == (filt, res) == (filt, 50000)
    want = orc.join_pairs(R, S)
    key = lambda x: x[np.lexsort((x[:, 1], x[:, 0]))]  # noqa: E731
    assert np.array_equal(key(pairs), key(want))
    out2 = run(*flags, "-R", tmp_path / "R.tbl", "-S", tmp_path / "S.tbl")
    assert counts(out2) == (filt, res)


def test_device_zipf_equals_host_zipf(hw, cuda):
    """hwbrj_create_relation_zipf_device at q = 1 is the -z relation (src/genzipf.c:98-158) of
    hwbrj_create_relation_zipf, key for key and row for row."""
    for (n, alpha, theta, seed) in [(2000000, 1000000, 0.75, 54321), (300001, 5000, 1.1, 7)]:
        h = hw.create_relation_zipf(n, alpha, theta, seed, 8)
        d = cuda.empty((n, 2), dtype=cuda.int32, device="cuda")
        hw.create_relation_zipf_device(d, alpha, theta, seed, 1.0, 8)
        assert np.array_equal(d.cpu().numpy(), h)


@pytest.fixture(scope="module")
def full_R(hw, cuda):
    nR = 128000000
    R = cuda.empty((nR, 2), dtype=cuda.int32, device="cuda")
    hw.generate_device(R, 2, nR, nR, 1.0, 12345)
    return R


@pytest.mark.parametrize("row", ORC["rows"], ids=lambda r: f"{r['variant']}-q{r['q']}-k{r['k']}-B{r['B']}")
def test_full_size_rows_vs_oracle(hw, cuda, full_R, row):
    """BASELINE configs 3 and 5 at full size (|R| = 128M, |S| = 1024M): the sectorized rows, the
    register-blocked B = 64 row and the selectivity sweep, against the oracle's counts on the same
    multiset (tests/golden/make_oracle_counts.py)."""
    S = cuda.empty((row["s"], 2), dtype=cuda.int32, device="cuda")
    hw.generate_device(S, 2, INT_MAX, row["r"], row["q"], 54321)
    st = hw.join_device(full_R, S, hw.BloomFilterArgs.from_flag(row["variant"], row["m"], row["k"], row["B"]))
    del S
    assert (st.filtered, st.matches) == (row["filtered"], row["results"])


# BASELINE config 5: Zipf theta = 0.75 S x q. The matching rows draw keys from the alphabet
# 1..|R| (src/genzipf.c:98-158); this build's q < 1 extension gives floor(|S| (1 - q)) rows the
# unique keys |R| + 1 .. |R| + floor(|S| (1 - q)), the same non-matching keys as the uniform
# generator at that q (src/generator.c:341-351). Every alphabet key passes the filter (no false
# negatives), so `filtered` is the oracle-pinned uniform count at the same q (q = 1: the reference's
# own -z relation, filtered = Results = |S|).
ZIPF_Q = [(0.001, 116057774), (0.01, 124236515), (0.1, 206036818), (1.0, 1024000000)]


@pytest.mark.parametrize("q,filtered", ZIPF_Q, ids=lambda v: str(v))
def test_zipf_q_rows_full_size(hw, cuda, full_R, q, filtered):
    nS = 1024000000
    S = cuda.empty((nS, 2), dtype=cuda.int32, device="cuda")
    hw.create_relation_zipf_device(S, 128000000, 0.75, 54321, q, 16)
    st = hw.join_device(full_R, S, hw.BloomFilterArgs(hw.BLOCKED, 1 << 30, 1, 1024))
    del S
    assert st.matches == nS - int(nS * (1 - q))
    assert st.filtered == filtered


@pytest.mark.parametrize("q", [0.001, 0.01, 0.1, 1.0])
def test_zipf_q_small_vs_oracle(hw, cuda, orc, q):
    """The Zipf + q relation at |R| = 1M, |S| = 16M, generated on the GPU: its non-matching keys
    are exactly |R| + 1 .. |R| + floor(|S| (1 - q)), and the join of the same tuples equals the
    oracle's (blocked k = 1 and 3, basic k = 2)."""
    nR, nS = 1000000, 16000000
    R = hw.generate_host(nR, 2, nR, nR, 1.0, 12345)
    dS = cuda.empty((nS, 2), dtype=cuda.int32, device="cuda")
    hw.create_relation_zipf_device(dS, nR, 0.75, 54321, q, 8)
    S = dS.cpu().numpy()
    n_above = int(nS * (1 - q))
    above = np.sort(S[S[:, 0] > nR, 0])
    assert np.array_equal(above, np.arange(nR + 1, nR + 1 + n_above))
    assert S[:, 0].min() >= 1 and np.array_equal(np.sort(S[:, 1]), np.arange(nS))
    for a in [(hw.BLOCKED, 1 << 24, 1, 1024), (hw.BLOCKED, 1 << 24, 3, 512), (hw.BASIC, 1 << 24, 2, 1024)]:
        st = hw.join_device(to_dev(cuda, R), dS, hw.BloomFilterArgs(*a))
        res, filt, _ = orc.bpro(R, S, 8, *a)
        assert (st.filtered, st.matches) == (filt, res) and res == nS - n_above, (a, st)


def oracle_check(hw, cuda, orc, R, S, args):
    st = hw.join_device(to_dev(cuda, R), to_dev(cuda, S), args)
    if args is None:
        res, filt, _ = orc.bpro(R, S, 8, 0, 0, 0, 0, use_bloom=False)
    else:
        res, filt, _ = orc.bpro(R, S, 8, args.variant, args.m, args.k, args.B)
    assert (st.filtered, st.matches) == (filt, res), (st, filt, res)
    return st


@pytest.mark.parametrize("args", [(0, 1 << 22, 1, 1024), (0, 1 << 22, 3, 1024), (1, 1 << 22, 1, 1024), None],
                         ids=str)
def test_structured_keys(hw, cuda, orc, args):
    """Keys that share their low bits (multiples of 64 and of 2^16): the basic filter's join
    sub-partition comes from bmix(key), not from the key's low bits."""
    a = None if args is None else hw.BloomFilterArgs(*args)
    for mult in (64, 1 << 16):
        Rk = np.arange(1, 150001, dtype=np.int64) * mult
        Sk = np.concatenate([Rk[::3], np.arange(150001, 450001, dtype=np.int64) * mult])
        oracle_check(hw, cuda, orc, rel(Rk), rel(Sk), a)


@pytest.mark.parametrize("variant", [0, 1])
def test_m_2_32(hw, cuda, orc, variant):
    """m = 2^32 bits, where the reference's uint32 size arithmetic wraps (mod_m widens, so
    (uint32)m == 0 means no masking, src/bloom_filter.c:59-63)."""
    rng = np.random.default_rng(12)
    Rk = rng.integers(-2**31, 2**31, size=300000)
    Sk = np.concatenate([Rk[:50000], rng.integers(-2**31, 2**31, size=700000)])
    for k in (1, 3):
        oracle_check(hw, cuda, orc, rel(Rk), rel(Sk), hw.BloomFilterArgs(variant, 1 << 32, k, 1024))


def test_basic_kk_materialize_and_skew(hw, cuda, orc, hook):
    """Basic k = 3 on the materialization path and with the join's skew split forced."""
    rng = np.random.default_rng(13)
    nR = 200000
    Rk = rng.permutation(nR) + 1
    ranks = rng.zipf(1.3, size=2000000)
    Sk = np.where(ranks <= nR, ranks, rng.integers(nR + 1, 10 * nR, size=ranks.size))
    R, S = rel(Rk), rel(Sk)
    a = hw.BloomFilterArgs(hw.BASIC, 1 << 20, 3, 1024)
    oracle_check(hw, cuda, orc, R, S, a)
    st, pairs, _ = hw.join_materialize_device(to_dev(cuda, R), to_dev(cuda, S), a)
    want = orc.join_pairs(R, S)
    p = pairs.cpu().numpy()
    assert st.matches == want.shape[0] == p.shape[0]
    key = lambda x: x[np.lexsort((x[:, 1], x[:, 0]))]  # noqa: E731
    assert np.array_equal(key(p), key(want))
    hook(hw.HOOK_JOIN_SPLIT, "700")
    oracle_check(hw, cuda, orc, R, S, a)


# ------------------------------------------------------- partitioned multi-GPU join (s8f row 3)
PJ_ARGS = [None, ("blocked", 1 << 24, 1, 1024), ("blocked", 1 << 22, 3, 512), ("basic", 1 << 20, 1, 0),
           ("sectorized", 1 << 22, 4, 512), ("blocked", 1 << 31, 2, 512)]


@pytest.mark.parametrize("a", PJ_ARGS, ids=str)
def test_partitioned_world1_vs_oracle(hw, cuda, orc, a):
    """hwbrj_join_partitioned on one rank (every exchange a local copy): the R chunks go through
    the gather/relist path, the survivors through the pack/item-table path and k_join's item_base
    descriptors; counts equal the oracle's."""
    from hwbloomradixjoin_amd import pjoin
    args = None if a is None else hw.BloomFilterArgs.from_flag(a[0], a[1], a[2], a[3] or 1024)
    rng = np.random.default_rng(21)
    for nR, nS in [(0, 1000), (1000, 0), (7, 33), (100003, 400009), (1000000, 4000000)]:
        Rk = rng.permutation(nR).astype(np.int64) + 1
        Sk = rng.integers(0, 2 * max(nR, 1) + 2, size=nS)
        R, S = rel(Rk), rel(Sk)
        st = pjoin.join_partitioned(to_dev(cuda, R), to_dev(cuda, S), nR, args)
        if args is None:
            res, filt, _ = orc.bpro(R, S, 8, 0, 0, 0, 0, use_bloom=False)
        else:
            res, filt, _ = orc.bpro(R, S, 8, args.variant, args.m, args.k, args.B)
        assert (st.filtered, st.matches) == (filt, res), (a, nR, nS, st)


def test_partitioned_world1_skew_and_dups(hw, cuda, orc, gen3, hook):
    """Duplicate R keys (hash-path join jobs) and a Zipf S with the skew split forced."""
    from hwbloomradixjoin_amd import pjoin
    hook(hw.HOOK_JOIN_SPLIT, "700")
    for mode in ("nonunique", "zipf"):
        R, S = gen3[1][mode]
        S = S[:4000000]
        args = hw.BloomFilterArgs(hw.BLOCKED, 1 << 24, 1, 1024)
        st = pjoin.join_partitioned(to_dev(cuda, R), to_dev(cuda, S), R.shape[0], args)
        res, filt, _ = orc.bpro(R, S, 8, 1, 1 << 24, 1, 1024, True)
        assert (st.filtered, st.matches) == (filt, res)


@pytest.fixture(scope="module")
def gen3(hw):
    g = GOLD["F3_generators"]
    kw = dict(r_seed=g["r_seed"], s_seed=g["s_seed"], host_threads=8)
    return g, {"nonunique": hw.reference_relations(g["r"], g["s"], g["nonunique"]["q"], non_unique=True, **kw),
               "zipf": hw.reference_relations(g["r"], g["s"], skew=g["zipf"]["z"], **kw)}


@pytest.mark.parametrize("world,flags", [(2, []), (4, []), (2, ["-b", "sectorized", "-k", "2"]),
                                         (4, ["-b", "basic"]), (2, ["-b", "no"])], ids=str)
def test_bench_partitioned_ranks(hw, orc, world, flags):
    """bench.py --design partitioned end to end under torch.distributed.run: R and S range shards,
    R chunk and survivor all-to-alls, slice all-gather, rehearsed with `world` ranks on one GPU
    (HWBRJ_BENCH_SHARED_GPU=1: gloo through host memory). The reduced counts are the golden."""
    import socket
    g = GOLD["F3_grid"]
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    root = os.path.dirname(HERE)
    env = dict(os.environ, HWBRJ_BENCH_SHARED_GPU="1", HWBRJ_PJ_CHECK="1")
    out = subprocess.run(["python", "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
                          "--master-addr", "127.0.0.1", "--master-port", str(port),
                          os.path.join(root, "bench.py"), "--gpus", str(world), "--steps", "2", "--warmup", "1",
                          "--design", "partitioned", "-r", str(g["r"]), "-s", str(g["s"]), "-m", str(g["m"])]
                         + flags, capture_output=True, text=True, timeout=300, env=env, cwd=root)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
    line = json.loads([x for x in out.stdout.splitlines() if x.startswith("{")][-1])
    assert line["n_gpus"] == world
    want = {(): g["rows"]["1024"][0], ("-b", "sectorized", "-k", "2"): None, ("-b", "basic"): g["rows"]["basic"][0],
            ("-b", "no"): g["s"]}[tuple(flags)]
    if want is None:  # sectorized (no reference count): the oracle on bench.py's relations
        R = hw.generate_host(g["r"], 2, g["r"], g["r"], 1.0, 12345)
        S = hw.generate_host(g["s"], 2, INT_MAX, g["r"], 0.01, 54321)
        want = orc.bpro(R, S, 8, hw.SECTORIZED, g["m"], 2, 1024)[1]
    assert (line["parity"]["filtered"], line["parity"]["matches"]) == (want, g["results"])


# ------------------------------------- BPRH / BPRHO: the histogram per-partition joins (s8f row 2)
@pytest.mark.parametrize("algo", [1, 2], ids=["PRH", "PRHO"])
@pytest.mark.parametrize("a", [None, ("blocked", 1 << 20, 1, 1024), ("basic", 1 << 20, 3, 0),
                               ("blocked", 1 << 16, 2, 4), ("blocked", 1 << 31, 2, 512)], ids=str)
def test_histogram_joins_vs_oracle(hw, cuda, orc, algo, a):
    """histogram_join / histogram_optimized_join (src/parallel_radix_join_bloom.c:350-555) as
    k_join variants: unique and duplicate R keys, negative and extreme keys, hot S keys."""
    args = None if a is None else hw.BloomFilterArgs.from_flag(a[0], a[1], a[2], a[3] or 1024)
    rng = np.random.default_rng(31)
    cases = [(rng.permutation(100003) + 1, rng.integers(0, 200010, size=400009)),
             (np.concatenate([rng.integers(-3000, 3000, size=60000), [INT_MAX, -INT_MAX - 1, 0, -1] * 3]),
              np.concatenate([rng.integers(-4000, 4000, size=500000), [INT_MAX, -INT_MAX - 1, 0, -1] * 5])),
             (np.concatenate([np.full(20000, 5), np.arange(100, 50000)]),
              np.concatenate([np.full(3000, 5), np.arange(0, 60000)])),
             (np.arange(1, 8), np.arange(0, 40))]
    for Rk, Sk in cases:
        R, S = rel(Rk), rel(Sk)
        st = hw.join_device(to_dev(cuda, R), to_dev(cuda, S), args, algorithm=algo)
        if args is None:
            res, filt, _ = orc.bpro(R, S, 8, 0, 0, 0, 0, use_bloom=False)
        else:
            res, filt, _ = orc.bpro(R, S, 8, args.variant, args.m, args.k, args.B)
        assert (st.filtered, st.matches) == (filt, res), (algo, a, st)


@pytest.mark.parametrize("algo", [1, 2], ids=["PRH", "PRHO"])
def test_histogram_joins_northstar(hw, full_R, cuda, algo):
    """The north-star golden through the histogram joins."""
    g = GOLD["F4_northstar"]
    S = cuda.empty((1024000000, 2), dtype=cuda.int32, device="cuda")
    hw.generate_device(S, 2, INT_MAX, 128000000, g["q"], 54321)
    st = hw.join_device(full_R, S, hw.BloomFilterArgs(hw.BLOCKED, g["m"], 1, g["B"]), algorithm=algo)
    del S
    assert (st.filtered, st.matches) == (g["k1_filtered"], g["results"])


def test_weak_scaling_ranks_reach_the_golden(hw, cuda):
    """bench.py --scaling weak (an A/B option): rank r joins the whole |S| generated with seed
    54321 + r. The seed orders the tuples only (the key multiset is the reference generator's), so
    every rank's counts are the north-star golden."""
    import torch
    g = json.load(open(os.path.join(HERE, "golden", "survey_counts.json")))["F4_northstar"]
    nR, nS = 128000000, 1024000000
    dR = torch.empty((nR, 2), dtype=torch.int32, device="cuda")
    dS = torch.empty((nS, 2), dtype=torch.int32, device="cuda")
    hw.generate_device(dR, 2, nR, nR, 1.0, 12345)
    for rank in (1, 7):
        hw.generate_device(dS, 2, INT_MAX, nR, g["q"], 54321 + rank)
        st = hw.join_device(dR, dS, hw.BloomFilterArgs(hw.BLOCKED, g["m"], 1, g["B"]))
        assert (st.filtered, st.matches) == (g["k1_filtered"], g["results"])


def test_copy_bandwidth_is_plausible(hw, cuda):
    """hwbrj_copy_bandwidth (the roofline's measured copy rate): a streaming copy on one MI355X runs
    between 1 TB/s and the 8 TB/s spec peak (read + write bytes per second)."""
    g = hw.copy_bandwidth(1 << 30, 3)
    assert 1000.0 < g < 8000.0, g
    with pytest.raises(RuntimeError):
        hw.copy_bandwidth(15, 1)
