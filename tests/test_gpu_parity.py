"""GPU parity tests: the HIP path (through the C-ABI) against the reference's counts and the oracle.

Bar: bit-exact. `filtered` ("S-tuples after filter", src/parallel_radix_join_bloom.c:1253) and
`Results` (src/main.c:480) must equal the golden counts / the oracle on the same inputs, and the
exported filter must be byte-identical to the reference's bloom_filter.c bitmap.
"""
import hashlib
import json
import os
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = json.load(open(os.path.join(HERE, "golden", "survey_counts.json")))
FILT = json.load(open(os.path.join(HERE, "golden", "ref_filters.json")))
INT_MAX = 2**31 - 1
VAR = {"basic": 0, "blocked": 1}


def dev_rel(hw, cuda, n, maxid, thr, q, seed, nthr=2):
    t = cuda.empty((n, 2), dtype=cuda.int32, device="cuda")
    if n:
        hw.generate_device(t, nthr, maxid, thr, q, seed)
    return t


def to_dev(cuda, a):
    return cuda.from_numpy(np.ascontiguousarray(a, dtype=np.int32)).cuda()


@pytest.fixture(scope="module")
def f3(hw, cuda):
    g = GOLD["F3_grid"]
    return (dev_rel(hw, cuda, g["r"], g["r"], g["r"], 1.0, 11),
            dev_rel(hw, cuda, g["s"], INT_MAX, g["r"], g["q"], 22))


@pytest.mark.parametrize("Bname", ["32", "64", "128", "256", "512", "1024", "basic"])
def test_f3_grid(hw, f3, Bname):
    g = GOLD["F3_grid"]
    R, S = f3
    for k, want in zip(g["k"], g["rows"][Bname]):
        v, B = (hw.BASIC, 1024) if Bname == "basic" else (hw.BLOCKED, int(Bname))
        st = hw.join_device(R, S, hw.BloomFilterArgs(v, g["m"], k, B))
        assert (st.filtered, st.matches) == (want, g["results"]), (Bname, k, st)


def test_basic_multi_hash_takes_slice_path(hw, f3):
    """Basic k >= 2 runs on the partition slices (MODE_SLICE_BASIC = 2, KIND_BASIC_KK), not the
    global-bitmap fallback (mode 3)."""
    g = GOLD["F3_grid"]
    R, S = f3
    for k in (2, 5):
        assert hw.join_device(R, S, hw.BloomFilterArgs(hw.BASIC, g["m"], k, 1024)).mode == 2


def test_f3_extra_and_pro(hw, cuda, f3):
    g = GOLD["F3_grid"]
    R, S = f3
    for row in g["extra"]:
        st = hw.join_device(R, S, hw.BloomFilterArgs(VAR[row["variant"]], g["m"], row["k"], row["B"]))
        assert (st.filtered, st.matches) == (row["filtered"], g["results"])
    S1 = dev_rel(hw, cuda, g["s"], INT_MAX, g["r"], 1.0, 5)  # BASELINE config 1 (-b no, q=1.0)
    st = hw.join_device(R, S1, None)
    assert st.matches == st.filtered == g["nobloom_q1_results"]


@pytest.mark.parametrize("row", GOLD["F1_fast"] + GOLD["F1_mid"],
                         ids=lambda r: f"{r['variant']}-r{r['r']}-m{r['m']}-k{r['k']}-s{r['s']}")
def test_f1_rows(hw, cuda, row):
    R = dev_rel(hw, cuda, row["r"], row["r"], row["r"], 1.0, 3)
    S = dev_rel(hw, cuda, row["s"], INT_MAX, row["r"], row["q"], 4)
    st = hw.join_device(R, S, hw.BloomFilterArgs(VAR[row["variant"]], row["m"], row["k"], row["B"]))
    assert (st.filtered, st.matches) == (row["filtered"], row["results"])


@pytest.fixture(scope="module")
def full_scale(hw, cuda):
    """The north-star relations: |R| = 128M, |S| = 1024M (S regenerated per q)."""
    nR = 128000000
    R = dev_rel(hw, cuda, nR, nR, nR, 1.0, 12345)
    cache = {}

    def S_for(q):
        if q not in cache:
            cache.clear()
            cuda.cuda.empty_cache()
            cache[q] = dev_rel(hw, cuda, 1024000000, INT_MAX, nR, q, 54321)
        return cache[q]
    return R, S_for


def test_northstar_golden(hw, full_scale):
    g = GOLD["F4_northstar"]
    R, S_for = full_scale
    S = S_for(g["q"])
    st = hw.join_device(R, S, hw.BloomFilterArgs(hw.BLOCKED, g["m"], 1, g["B"]))
    assert (st.filtered, st.matches) == (g["k1_filtered"], g["results"])
    st = hw.join_device(R, S, hw.BloomFilterArgs(hw.BLOCKED, g["m"], 2, g["B"]))
    assert (st.filtered, st.matches) == (g["k2_filtered"], g["results"])
    # the full-size filter popcount (F2) through the export path
    for row in [r for r in GOLD["F2_popcount"] if r["r"] == 128000000]:
        hw.join_device(R, S, hw.BloomFilterArgs(VAR[row["variant"]], row["m"], row["k"], row["B"]))
        bm = hw.export_filter(row["m"])
        assert int(np.unpackbits(bm).sum()) == row["popcount"]


@pytest.mark.parametrize("world", [2, 8])
def test_northstar_rank_shards_sum_to_golden(hw, full_scale, cuda, world):
    """What every rank of `bench.py --gpus N --scaling strong` computes: the replicated R and the
    rank's S range regenerated on the device (generate_device_range, shard_range); the per-rank
    counts summed over ranks (the all_reduce) must be the single-GPU golden."""
    g = GOLD["F4_northstar"]
    R, _ = full_scale
    nS = 1024000000
    tot = [0, 0]
    for rank in range(world):
        lo, hi = hw.shard_range(nS, rank, world)
        S = cuda.empty((hi - lo, 2), dtype=cuda.int32, device="cuda")
        hw.generate_device_range(S, nS, lo, 2, INT_MAX, 128000000, g["q"], 54321)
        st = hw.join_device(R, S, hw.BloomFilterArgs(hw.BLOCKED, g["m"], 1, g["B"]))
        tot[0] += st.filtered
        tot[1] += st.matches
        del S
    assert tuple(tot) == (g["k1_filtered"], g["results"])


@pytest.mark.parametrize("row", GOLD["F1_published"],
                         ids=lambda r: f"{r['variant']}-q{r['q']}-m{r['m']}-k{r['k']}-B{r['B']}")
def test_published_thesis_rows(hw, full_scale, row):
    R, S_for = full_scale
    st = hw.join_device(R, S_for(row["q"]),
                        hw.BloomFilterArgs(VAR[row["variant"]], row["m"], row["k"], row["B"]))
    assert (st.filtered, st.matches) == (row["filtered"], row["results"])


@pytest.mark.parametrize("case", FILT["cases"], ids=lambda c: f"v{c['variant']}-m{c['m']}-k{c['k']}-B{c['B']}")
def test_filter_bytes_identical_to_reference(hw, cuda, orc, case):
    R = orc.gen_keys(FILT["r"], FILT["nthreads"], FILT["r"], FILT["r"], 1.0, 7)
    S = orc.gen_keys(FILT["s"], FILT["nthreads"], INT_MAX, FILT["r"], FILT["q"], 8)
    dR = to_dev(cuda, np.stack([R, np.arange(R.size, dtype=np.int32)], 1))
    dS = to_dev(cuda, np.stack([S, np.arange(S.size, dtype=np.int32)], 1))
    st = hw.join_device(dR, dS, hw.BloomFilterArgs(case["variant"], case["m"], case["k"], case["B"]))
    assert st.filtered == case["filtered"]
    bm = hw.export_filter(case["m"])
    assert hashlib.sha256(bm.tobytes()).hexdigest() == case["sha256"]


def oracle_check(hw, cuda, orc, Rk, Sk, args, nthr=4):
    R = np.stack([Rk.astype(np.int32), np.arange(Rk.size, dtype=np.int32)], 1)
    S = np.stack([Sk.astype(np.int32), np.arange(Sk.size, dtype=np.int32)], 1)
    st = hw.join_device(to_dev(cuda, R.reshape(-1, 2)), to_dev(cuda, S.reshape(-1, 2)), args)
    if args is None:
        res, filt, _ = orc.bpro(R, S, nthr, 0, 0, 0, 0, use_bloom=False)
    else:
        res, filt, _ = orc.bpro(R, S, nthr, args.variant, args.m, args.k, args.B)
    assert (st.filtered, st.matches) == (filt, res), (st, filt, res)
    return st


ARGS = [None, ("blocked", 1 << 20, 1, 1024), ("blocked", 1 << 22, 3, 512), ("basic", 1 << 20, 1, 0),
        ("basic", 1 << 20, 3, 0), ("sectorized", 1 << 20, 1, 1024), ("sectorized", 1 << 22, 4, 512),
        ("blocked", 1 << 16, 2, 4), ("blocked", 1 << 31, 2, 512), ("blocked", 64, 1, 32),
        ("basic", 1 << 31, 2, 0), ("basic", 64, 3, 0)]


def mk(hw, a):
    return None if a is None else hw.BloomFilterArgs.from_flag(a[0], a[1], a[2], a[3] or 1024)


@pytest.mark.parametrize("a", ARGS, ids=str)
def test_edge_sizes(hw, cuda, orc, a):
    args = mk(hw, a)
    rng = np.random.default_rng(3)
    for nR, nS in [(0, 1000), (1000, 0), (1, 1), (1, 5000), (7, 33), (4097, 4099), (100003, 400009)]:
        Rk = rng.permutation(nR).astype(np.int64) + 1
        Sk = rng.integers(0, 2 * max(nR, 1) + 2, size=nS)
        oracle_check(hw, cuda, orc, Rk, Sk, args)


@pytest.mark.parametrize("variant", ["blocked", "sectorized"])
@pytest.mark.parametrize("B", [8, 16, 32, 64, 256, 1024])
@pytest.mark.parametrize("k", [1, 2, 3])
def test_packed_words_every_block_size(hw, cuda, orc, variant, B, k):
    """Packed partition words (FMT_PACKED: first bit-in-block in the low log2B bits, code digits
    above, so the low log2(m/F) bits are the slice bit) for every block size the slice path takes
    (8 <= B <= F), k = 1 (KIND_BLOCK_PK1) and k >= 2 (KIND_BLOCK_PKK), against the oracle."""
    rng = np.random.default_rng(11 + B + k)
    Rk = rng.permutation(60000).astype(np.int64) + 1
    Sk = rng.integers(0, 240000, size=300000)
    oracle_check(hw, cuda, orc, Rk, Sk, hw.BloomFilterArgs.from_flag(variant, 1 << 21, k, B))


@pytest.mark.parametrize("a", ARGS[:6], ids=str)
def test_duplicates_negatives_and_extremes(hw, cuda, orc, a):
    args = mk(hw, a)
    rng = np.random.default_rng(4)
    Rk = np.concatenate([rng.integers(-3000, 3000, size=60000),
                         np.array([INT_MAX, -INT_MAX - 1, 0, -1, 42] * 3)])
    Sk = np.concatenate([rng.integers(-4000, 4000, size=500000),
                         np.array([INT_MAX, -INT_MAX - 1, 0, -1, 42, 43] * 7)])
    oracle_check(hw, cuda, orc, Rk, Sk, args)


@pytest.mark.parametrize("a", ARGS[:4], ids=str)
def test_skewed_probe_side(hw, cuda, orc, a):
    """Zipf-like skew: a few hot keys carry most of S (one partition gets most of the work)."""
    args = mk(hw, a)
    rng = np.random.default_rng(5)
    nR = 200000
    Rk = rng.permutation(nR) + 1
    ranks = rng.zipf(1.3, size=3000000)
    Sk = np.where(ranks <= nR, ranks, rng.integers(nR + 1, 10 * nR, size=ranks.size))
    oracle_check(hw, cuda, orc, Rk, Sk, args)
    Sk1 = np.full(1000000, 77)  # every S tuple on one key
    st = oracle_check(hw, cuda, orc, Rk, Sk1, args)
    assert st.matches == Sk1.size


@pytest.mark.parametrize("m,k", [(1 << 20, 5), (1 << 24, 8), (1 << 16, 17), (1 << 20, 256),
                                 (1 << 20, 257), (1 << 16, 300), (64, 9), (1 << 32, 4)], ids=str)
def test_basic_multi_pass_bits(hw, cuda, orc, m, k):
    """Basic k >= 2 (one bit per pass, Engine::enqueue_basic_kk): odd and even pass counts, k at and
    above the scatter grid (k > 256: the bit positions come from k_bitpos, not the fused position
    scatter), and tiny R whose k * |R| position ranges cross several multiples of |R| per workgroup."""
    args = hw.BloomFilterArgs(hw.BASIC, m, k, 1024)
    rng = np.random.default_rng(k)
    for nR, nS in [(0, 3000), (1, 1), (3, 5000), (37, 101), (4097, 40999), (100003, 400009)]:
        Rk = rng.permutation(nR).astype(np.int64) + 1
        Sk = rng.integers(0, 3 * max(nR, 1) + 2, size=nS)
        oracle_check(hw, cuda, orc, Rk, Sk, args)
    assert hw.join_device(to_dev(cuda, np.zeros((8, 2))), to_dev(cuda, np.zeros((8, 2))), args).mode == 2


def test_hot_build_key_chunked_join(hw, cuda, orc):
    """One key repeated in R beyond the LDS table capacity: the join processes R in pieces."""
    Rk = np.concatenate([np.full(20000, 5), np.arange(100, 50000)])
    Sk = np.concatenate([np.full(3000, 5), np.arange(0, 60000)])
    st = oracle_check(hw, cuda, orc, Rk, Sk, mk(hw, ("blocked", 1 << 20, 1, 1024)))
    assert st.matches == 20000 * 3001 + (50000 - 100)


def test_repeatable_and_buffer_reuse(hw, cuda, f3):
    R, S = f3
    a = hw.BloomFilterArgs(hw.BLOCKED, 1 << 24, 1, 1024)
    first = hw.join_device(R, S, a)
    small = hw.join_device(R[:1000], S[:5000], a)  # shrink, then grow again
    again = hw.join_device(R, S, a)
    assert (first.filtered, first.matches) == (again.filtered, again.matches)
    assert small.matches <= 5000


def test_async_joins_back_to_back(hw, cuda, f3):
    """hwbrj_join_device_async x3 then hwbrj_join_wait_all: every join's counts are the golden's.
    Async joins record no phase events (counts only); a synchronous join after them measures its
    phases again."""
    g = GOLD["F3_grid"]
    R, S = f3
    args = hw.BloomFilterArgs(hw.BLOCKED, g["m"], 1, 1024)
    for _ in range(3):
        hw.join_device_async(R, S, args)
    sts = hw.join_wait_all()
    assert [(st.filtered, st.matches) for st in sts] == [(g["rows"]["1024"][0], g["results"])] * 3
    st = sts[-1]
    assert st.ms_total == 0 and st.ms_probe == 0
    st = hw.join_device(R, S, args)
    assert (st.filtered, st.matches) == (g["rows"]["1024"][0], g["results"])
    assert st.ms_total > 0 and st.ms_probe > 0 and st.ms_s_scatter > 0
    assert st.ms_surv == 0  # (fused into the probe: no boundary of its own)
    parts = st.ms_r_scatter + st.ms_r_index + st.ms_build + st.ms_s_scatter + st.ms_s_index + st.ms_probe + st.ms_join
    assert abs(parts - st.ms_total) <= 1e-3 * st.ms_total + 1e-3


def test_generate_device_matches_host(hw, cuda):
    for (n, nthr, maxid, thr, q) in [(1000000, 2, 1000000, 1000000, 1.0), (3000001, 3, INT_MAX, 100000, 0.01)]:
        d = dev_rel(hw, cuda, n, maxid, thr, q, 9, nthr).cpu().numpy()
        h = hw.generate_host(n, nthr, maxid, thr, q, 9, 8)
        assert np.array_equal(d, h)
        part = cuda.empty((n // 3, 2), dtype=cuda.int32, device="cuda")
        hw.generate_device_range(part, n, n // 2, nthr, maxid, thr, q, 9)
        assert np.array_equal(part.cpu().numpy(), h[n // 2: n // 2 + n // 3])


def test_bpro_host_boundary_stdout(hw, capfd):
    """BPRO over host relation_t (H2D inside), stdout lines of the reference (run.py regexes)."""
    g = GOLD["F3_grid"]
    R = hw.Relation(hw.generate_host(g["r"], 2, g["r"], g["r"], 1.0, 1))
    S = hw.Relation(hw.generate_host(g["s"], 2, INT_MAX, g["r"], g["q"], 2))
    res = hw.BPRO(R, S, 4, hw.BloomFilterArgs(hw.BLOCKED, g["m"], 1, 1024))
    out = capfd.readouterr().out
    assert res.totalresults == g["results"] and res.nthreads == 4
    assert f"S-tuples after filter: {g['rows']['1024'][0]}" in out
    assert "TOTAL-TIME-USECS, TOTAL-TUPLES, NSEC-PER-TUPLE:" in out
    assert "PARTITION-TIME-USECS, PROBE-TIME-USECS, JOIN-TIME-USECS:" in out
    res = hw.PRO(R, S, 2)
    assert res.totalresults == g["results"]
    a = hw.BloomFilterArgs(hw.BLOCKED, g["m"], 1, 1024)
    for fn in (hw.BPRH, hw.BPRHO, hw.BRJ):  # the other join_init_run entries: same counts
        assert fn(R, S, 2, a).totalresults == g["results"]
    for fn in (hw.PRH, hw.PRHO, hw.RJ):
        assert fn(R, S, 2).totalresults == g["results"]


@pytest.fixture(scope="module")
def gen3(hw):
    """The rand()-driven relations of SURVEY.md s8c F3 (bit-exact reference generators, host)."""
    g = json.load(open(os.path.join(HERE, "golden", "survey_counts.json")))["F3_generators"]
    kw = dict(r_seed=g["r_seed"], s_seed=g["s_seed"], host_threads=8)
    return g, {
        "nonunique": hw.reference_relations(g["r"], g["s"], g["nonunique"]["q"], non_unique=True, **kw),
        "fullrange": hw.reference_relations(g["r"], g["s"], 0.01, full_range=True, **kw),
        "zipf": hw.reference_relations(g["r"], g["s"], skew=g["zipf"]["z"], **kw),
    }


@pytest.mark.parametrize("mode", ["nonunique", "zipf"])
def test_generator_goldens(hw, cuda, gen3, mode):
    g, rels = gen3
    R, S = rels[mode]
    row = g[mode]
    st = hw.join_device(to_dev(cuda, R), to_dev(cuda, S), hw.BloomFilterArgs(hw.BLOCKED, g["m"], row["k"], g["B"]))
    assert (st.filtered, st.matches) == (row["filtered"], row["results"])


@pytest.mark.parametrize("mode", ["nonunique", "fullrange", "zipf"])
@pytest.mark.parametrize("a", [None, ("basic", 1 << 24, 1, 0), ("blocked", 1 << 24, 3, 512),
                               ("sectorized", 1 << 24, 2, 1024)], ids=str)
def test_generator_relations_vs_oracle(hw, cuda, orc, gen3, mode, a):
    """Duplicate build keys (non-unique / full-range R) and heavy probe skew (Zipf S)."""
    R, S = gen3[1][mode]
    args = mk(hw, a)
    st = hw.join_device(to_dev(cuda, R), to_dev(cuda, S), args)
    if args is None:
        res, filt, _ = orc.bpro(R, S, 8, 0, 0, 0, 0, use_bloom=False)
    else:
        res, filt, _ = orc.bpro(R, S, 8, args.variant, args.m, args.k, args.B)
    assert (st.filtered, st.matches) == (filt, res)


def test_cli_generator_flags_end_to_end(hw):
    g = json.load(open(os.path.join(HERE, "golden", "survey_counts.json")))["F3_generators"]
    row = g["nonunique"]
    out = subprocess.run([hw.CLI_PATH, "-a", "PRO", "-r", str(g["r"]), "-s", str(g["s"]), "-q", str(row["q"]),
                          "--non-unique", "-b", "blocked", "-m", str(g["m"]), "-k", "1"],
                         capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stdout + out.stderr
    assert f"S-tuples after filter: {row['filtered']}" in out.stdout
    assert f"[INFO ] Results = {row['results']}. DONE." in out.stdout
    out = subprocess.run([hw.CLI_PATH, "-a", "PRHO", "-r", str(g["r"]), "-s", str(g["s"] // 4), "-z", "0.75",
                          "-b", "blocked", "-m", str(g["m"]), "-k", "1"],
                         capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stdout + out.stderr
    assert f"[INFO ] Results = {g['s'] // 4}. DONE." in out.stdout


def test_cli_end_to_end(hw):
    g = GOLD["F3_grid"]
    out = subprocess.run([hw.CLI_PATH, "-a", "PRO", "-r", str(g["r"]), "-s", str(g["s"]), "-q", "0.01",
                          "-b", "blocked", "-m", str(g["m"]), "-k", "1", "-n", "2"],
                         capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stdout + out.stderr
    assert f"S-tuples after filter: {g['rows']['1024'][0]}" in out.stdout
    assert f"[INFO ] Results = {g['results']}. DONE." in out.stdout


def test_bench_two_ranks(hw):
    """bench.py's N > 1 path end to end (torch.distributed.run, 2 ranks, S sharded, counts
    all-reduced), rehearsed on one GPU: HWBRJ_BENCH_SHARED_GPU=1 puts both ranks on it with gloo."""
    import socket
    g = GOLD["F3_grid"]
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    root = os.path.dirname(HERE)
    env = dict(os.environ, HWBRJ_BENCH_SHARED_GPU="1")
    out = subprocess.run(["python", "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                          "--master-addr", "127.0.0.1", "--master-port", str(port),
                          os.path.join(root, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
                          "-r", str(g["r"]), "-s", str(g["s"]), "-m", str(g["m"])],
                         capture_output=True, text=True, timeout=300, env=env, cwd=root)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-2000:]
    line = json.loads([x for x in out.stdout.splitlines() if x.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["scaling"] == "strong" and line["dist"]["world_size_seen"] == 2
    assert (line["parity"]["filtered"], line["parity"]["matches"]) == (g["rows"]["1024"][0], g["results"])
    per = line["parity"]["per_rank"]  # two S shards: their counts sum to the golden
    assert len(per) == 2 and [sum(c) for c in zip(*per)] == [g["rows"]["1024"][0], g["results"]]
    # the other designs on the same ranks: the broadcast needs a GPU per rank,
    # the partitioned join runs over the torch transport; its per-rank counts sum to the golden
    alt = line["alt_designs"]
    assert "skipped" in alt["bcast"]
    for name in ("partitioned", "partitioned_async"):  # (torch gloo callbacks: ranks share the GPU)
        part = alt[name]
        assert len(part["per_rank"]) == 2 and part["sum"] == [g["rows"]["1024"][0], g["results"]], (name, part)
        assert part["ms"] > 0


def test_bench_rccl_process_group(hw):
    """bench.py under torch.distributed.run with the RCCL ("nccl") process group on the one GPU
    (HWBRJ_BENCH_DIST=1 at world 1): the init, barriers and reductions of the N > 1 path over RCCL."""
    import socket
    g = GOLD["F3_grid"]
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    root = os.path.dirname(HERE)
    env = dict(os.environ, HWBRJ_BENCH_DIST="1")
    env.pop("HWBRJ_BENCH_SHARED_GPU", None)
    out = subprocess.run(["python", "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
                          "--master-addr", "127.0.0.1", "--master-port", str(port),
                          os.path.join(root, "bench.py"), "--gpus", "1", "--steps", "2", "--warmup", "1",
                          "-r", str(g["r"]), "-s", str(g["s"]), "-m", str(g["m"]), "--no-cpu-baseline"],
                         capture_output=True, text=True, timeout=300, env=env, cwd=root)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-2000:]
    line = json.loads([x for x in out.stdout.splitlines() if x.startswith("{")][-1])
    assert (line["parity"]["filtered"], line["parity"]["matches"]) == (g["rows"]["1024"][0], g["results"])
    assert line["scaling"] == "strong" and line["dist"] == {"world_size_seen": 1, "backend": "nccl",
                                                            "shared_gpu_rehearsal": False}
    # the other designs on the same rank over the library's RCCL communicator
    for name in ("bcast", "partitioned", "partitioned_async"):
        leg = line["alt_designs"][name]
        assert leg.get("sum") == [g["rows"]["1024"][0], g["results"]] and leg["ms"] > 0, (name, leg)
        assert leg["per_rank"] == [leg["sum"]]


def _sorted_pairs(p):
    p = np.asarray(p).reshape(-1, 2)
    return p[np.lexsort((p[:, 1], p[:, 0]))]


@pytest.mark.parametrize("case", ["pkfk", "dups", "nonunique", "edge"])
def test_materialized_pairs_vs_oracle(hw, cuda, orc, gen3, case):
    """JOIN_RESULT_MATERIALIZE: the multiset of {R.payload, S.payload} pairs equals the oracle's."""
    rng = np.random.default_rng(11)
    if case == "pkfk":
        R = orc.relation(1000000, 2, 1000000, 1000000, 1.0, 1)
        S = orc.relation(16000000, 2, INT_MAX, 1000000, 0.01, 2)
    elif case == "dups":
        Rk = np.concatenate([rng.integers(-3000, 3000, size=60000), [INT_MAX, -INT_MAX - 1, -1] * 3])
        Sk = np.concatenate([rng.integers(-4000, 4000, size=500000), [INT_MAX, -INT_MAX - 1, -1] * 5])
        R = np.stack([Rk, rng.integers(-2**31, 2**31, size=Rk.size)], 1).astype(np.int32)
        S = np.stack([Sk, rng.integers(-2**31, 2**31, size=Sk.size)], 1).astype(np.int32)
    elif case == "nonunique":
        R, S = gen3[1]["nonunique"]
    else:
        R = np.array([[5, 1], [5, 2]], dtype=np.int32)
        S = np.array([[5, 7], [6, 8], [5, 9]], dtype=np.int32)
    for args in (hw.BloomFilterArgs(hw.BLOCKED, 1 << 24, 1, 1024), None):
        st, pairs, _ = hw.join_materialize_device(to_dev(cuda, R), to_dev(cuda, S), args)
        want = orc.join_pairs(R, S)
        assert st.matches == want.shape[0] == pairs.shape[0]
        assert np.array_equal(_sorted_pairs(pairs.cpu().numpy()), _sorted_pairs(want))


def test_materialize_empty_sides(hw, cuda):
    e = np.empty((0, 2), dtype=np.int32)
    one = np.array([[1, 1]], dtype=np.int32)
    for R, S in [(e, one), (one, e)]:
        st, pairs, _ = hw.join_materialize_device(to_dev(cuda, R), to_dev(cuda, S), None)
        assert st.matches == 0 and pairs.shape[0] == 0


def test_bpro_materialized_result_list(hw, orc):
    """Host BPRO with materialization fills result_t.resultlist with the reference's chained
    buffers (src/tuple_buffer.h); the pairs equal the oracle's."""
    R = hw.generate_host(300000, 2, 300000, 300000, 1.0, 5)
    S = hw.generate_host(3000000, 2, INT_MAX, 300000, 0.5, 6)
    hw.set_materialize(True)
    try:
        res = hw.BPRO(hw.Relation(R), hw.Relation(S), 4, hw.BloomFilterArgs(hw.BLOCKED, 1 << 22, 2, 512))
    finally:
        hw.set_materialize(False)
    want = orc.join_pairs(R, S)
    assert res.totalresults == want.shape[0] == res.pairs.shape[0] > 1024 * 1024
    assert np.array_equal(_sorted_pairs(res.pairs), _sorted_pairs(want))


@pytest.mark.parametrize("split", ["700", "5000"])
def test_join_skew_split_forced(hw, cuda, orc, gen3, split, hook):
    """The join's skew split (extra parts over a job's probe items) forced on every job: the counts
    and materialized pairs still equal the oracle's (Zipf S; non-unique R takes the hash path)."""
    hook(hw.HOOK_JOIN_SPLIT, split)
    for mode in ("zipf", "nonunique"):
        R, S = gen3[1][mode]
        S = S[:4000000]
        for args in (hw.BloomFilterArgs(hw.BLOCKED, 1 << 24, 1, 1024), None):
            st = hw.join_device(to_dev(cuda, R), to_dev(cuda, S), args)
            res, filt, _ = orc.bpro(R, S, 8, 1 if args else 0, 1 << 24, 1, 1024, args is not None)
            assert (st.filtered, st.matches) == (filt, res)


def test_join_key_formats_across_launches(hw, cuda, orc):
    """3-byte join keys (pack3): a probe item whose survivors overflow its LDS stage
    keeps 32-bit survivor runs, so a launch can hold both formats (the mixed join), and the Engine
    stops packing after a join that had such items (pack3_hint_). At the north star's filter size the
    stage holds 2592 survivors. Here |S| = 2^24 over 1024 partitions and 256 scatter regions: a
    partition has ~640 chunks (~26 words each), i.e. a full 384-chunk probe item of ~9800 words and
    a last one of ~6600. With 32 % members the full items overflow the stage and the last ones do
    not (a mixed launch); with 1 % none overflows. The sequence low, low (packed), mid (mixed
    launch), mid (32-bit), low (32-bit), low (packed again) must count what the oracle counts every
    time, and the path each join took (hwbrj_stats_t.join_keys, unstaged_items) must be that
    sequence (round 4's 21 % members never overflowed a stage)."""
    rng = np.random.default_rng(23)
    nR, nS = 1 << 20, 1 << 24
    Rk = rng.permutation(nR).astype(np.int64) + 1
    outside = lambda n: rng.integers(2 * nR, INT_MAX, size=n)  # never in R
    S_lo = np.concatenate([rng.integers(1, nR + 1, size=nS // 100), outside(nS - nS // 100)])
    S_mid = np.concatenate([rng.integers(1, nR + 1, size=nS * 32 // 100), outside(nS - nS * 32 // 100)])
    rng.shuffle(S_lo)
    rng.shuffle(S_mid)
    args = hw.BloomFilterArgs(hw.BLOCKED, 1 << 30, 1, 1024)
    want = {}
    for name, Sk in (("lo", S_lo), ("mid", S_mid)):
        R = np.stack([Rk.astype(np.int32), np.arange(nR, dtype=np.int32)], 1)
        S = np.stack([Sk.astype(np.int32), np.arange(nS, dtype=np.int32)], 1)
        res, filt, _ = orc.bpro(R, S, 8, args.variant, args.m, args.k, args.B)
        assert res == int(np.isin(Sk, Rk).sum())
        want[name] = (filt, res, to_dev(cuda, R), to_dev(cuda, S))
    seq = [("lo", hw.JOIN_KEYS_PACKED), ("lo", hw.JOIN_KEYS_PACKED), ("mid", hw.JOIN_KEYS_MIXED),
           ("mid", hw.JOIN_KEYS_32), ("lo", hw.JOIN_KEYS_32), ("lo", hw.JOIN_KEYS_PACKED)]
    hw.join_device(want["lo"][2], want["lo"][3], args)  # (a packing join before the sequence)
    for name, keys in seq:
        filt, res, dR, dS = want[name]
        st = hw.join_device(dR, dS, args)
        assert (st.filtered, st.matches) == (filt, res), (name, st)
        assert st.join_keys == keys, (name, st)
        # 18-bit keys whenever packed (hash_shift 14 at F = 1024, 16 subs), else 32-bit codes
        assert st.join_key_bits == (32 if keys == hw.JOIN_KEYS_32 else 18), (name, st)
        # unstaged items: some in every mid join (packed or not), none in a lo join
        assert (st.unstaged_items > 0) == (name == "mid"), (name, st)


@pytest.mark.parametrize("cfg,bits", [(("blocked", 1 << 24, 1, 1024), 18), (("sectorized", 1 << 24, 2, 512), 18),
                                      (("blocked", 1 << 24, 1, 1 << 17), 24), (("blocked", 1 << 22, 2, 1 << 15), 24),
                                      (None, 18)], ids=str)
def test_join_key_widths(hw, cuda, orc, cfg, bits):
    """The packed join-key width follows the geometry (join_key_bits): 18 bits where the join keys are
    v = code >> 14 (F = 1024 with 16 subs, or fewer partitions with 2^(14 - log2F) subs: the bitmap
    path's keys), 24 bits where fewer subs leave wider keys (m / B = 128 blocks: F = 128 partitions
    of 2 subs, hash_shift 8, the hash-table path), each counted as the oracle counts, synchronously
    and through back-to-back async joins (both widths in one run). (A join whose probe items
    overflowed their stage turns packing off for the next one: the first join of each side may run
    32-bit codes, the ones after it pack.)"""
    rng = np.random.default_rng(bits + (cfg[1] if cfg else 0))
    nR, nS = 1000003, 6000011
    Rk = rng.permutation(nR).astype(np.int64) + 1
    Sk = rng.integers(1, 40 * nR, size=nS)
    R = np.stack([Rk.astype(np.int32), np.arange(nR, dtype=np.int32)], 1)
    S = np.stack([Sk.astype(np.int32), np.arange(nS, dtype=np.int32)], 1)
    args = mk(hw, cfg)
    if args is None:
        res, filt, _ = orc.bpro(R, S, 8, 0, 0, 0, 0, use_bloom=False)
    else:
        res, filt, _ = orc.bpro(R, S, 8, args.variant, args.m, args.k, args.B)
    dR, dS = to_dev(cuda, R), to_dev(cuda, S)
    for _ in range(2):
        st = hw.join_device(dR, dS, args)
        assert (st.filtered, st.matches) == (filt, res), st
    assert st.join_key_bits == bits and st.unstaged_items == 0, st
    other = (hw.BloomFilterArgs(hw.BLOCKED, 1 << 24, 1, 1 << 17) if bits == 18
             else hw.BloomFilterArgs(hw.BLOCKED, 1 << 24, 1, 1024))
    ost = hw.join_device(dR, dS, other)
    for a in (args, other, args):
        hw.join_device_async(dR, dS, a)
    sts = hw.join_wait_all()
    assert [(x.filtered, x.matches) for x in sts] == [(filt, res), (ost.filtered, ost.matches), (filt, res)]
    assert {sts[0].join_key_bits, sts[1].join_key_bits} == {18, 24}, sts
