"""CPU tests of the drop-in boundary: libhwbrj.so loads and exports every symbol include/hwbrj.h
declares, the host-side pieces (hashes, generator, argument checks, CLI parsing) agree with the
oracle. No GPU compute here."""
import json
import os
import re
import subprocess

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
GOLD = json.load(open(os.path.join(HERE, "golden", "survey_counts.json")))
KATS = json.load(open(os.path.join(HERE, "golden", "ref_kats.json")))
INT_MAX = 2**31 - 1


def declared_functions():
    src = open(os.path.join(ROOT, "include", "hwbrj.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    src = re.sub(r"^\s*#.*$", "", src, flags=re.M)  # preprocessor lines (#error text, macros)
    # (function-pointer members, "int (*f)(...);", are not exported functions)
    names = re.findall(r"\b([A-Za-z_][A-Za-z0-9_]*)\s*\((?!\s*\*)[^;{]*\)\s*;", src)
    return sorted(set(n for n in names if n not in ("if", "while", "for", "sizeof")))


def test_library_exports_every_declared_symbol(hw):
    names = declared_functions()
    assert {"BPRO", "PRO", "assert_args", "hwbrj_join_device"} <= set(names)
    out = subprocess.run(["nm", "-D", "--defined-only", hw.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    missing = [n for n in names if n not in exported]
    assert not missing, missing


def test_struct_layouts_match_reference(hw):
    import ctypes
    # src/types.h:37-63, src/bloom_filter.h:50-55 on x86-64
    assert ctypes.sizeof(hw._Tuple) == 8
    assert ctypes.sizeof(hw._Relation) == 16
    assert ctypes.sizeof(hw._Result) == 24
    assert ctypes.sizeof(hw._BloomArgs) == 32
    assert hw.BASIC == 0 and hw.BLOCKED == 1
    # src/tuple_buffer.h:27-40 (chained result buffers of JOIN_RESULT_MATERIALIZE)
    assert ctypes.sizeof(hw._TupleBuffer) == 16 and ctypes.sizeof(hw._ChainedTupleBuffer) == 40
    assert ctypes.sizeof(hw._ThreadResult) == 24


def test_stats_layout_matches_header(hw, tmp_path):
    """hwbrj_stats_t as the C compiler lays it out (include/hwbrj.h) equals the ctypes mirror,
    including the join key format fields at its end."""
    import ctypes
    src = tmp_path / "st.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "hwbrj.h"\nint main(void) {\n'
                   '  printf("%zu %zu %zu %zu %zu %d %d %d\\n", sizeof(hwbrj_stats_t), offsetof(hwbrj_stats_t, '
                   'ms_join_probe), offsetof(hwbrj_stats_t, join_keys), offsetof(hwbrj_stats_t, '
                   'unstaged_items), offsetof(hwbrj_stats_t, join_key_bits), HWBRJ_JOIN_KEYS_32, '
                   'HWBRJ_JOIN_KEYS_PACKED, HWBRJ_JOIN_KEYS_MIXED);\n'
                   '  return 0;\n}\n')
    exe = tmp_path / "st"
    subprocess.run(["gcc", "-std=gnu11", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                    "-o", str(exe), str(src)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True,
                                          check=True).stdout.split()]
    S = hw._Stats
    assert got == [ctypes.sizeof(S), S.ms_join_probe.offset, S.join_keys.offset,
                   S.unstaged_items.offset, S.join_key_bits.offset, hw.JOIN_KEYS_32, hw.JOIN_KEYS_PACKED,
                   hw.JOIN_KEYS_MIXED]


def test_host_hashes_match_reference_kats(hw):
    for row in KATS["kats"]:
        assert hw.hash_crc(42, row["key"]) == row["crc32c"]
        assert hw.hash_crapwow(42, row["key"]) == row["crapwow"]
        assert hw.hash_crc(7, row["key"]) == row["crc32c_seed7"]


@pytest.mark.parametrize("n,nthr,maxid,thr,q", [
    (1000000, 2, 1000000, 1000000, 1.0),
    (16000000, 2, INT_MAX, 1000000, 0.01),
    (2000000, 3, INT_MAX, 250000, 0.001),
    (1000, 7, INT_MAX, 100, 0.5),
    (4095, 1, INT_MAX, 4095, 0.0),
    (100, 16, 100, 100, 1.0),
    (50000, 5, INT_MAX, 333, 1.0),
])
def test_host_generator_is_reference_multiset(hw, orc, n, nthr, maxid, thr, q):
    t = hw.generate_host(n, nthr, maxid, thr, q, 99, 4)
    assert np.array_equal(t[:, 1], np.arange(n, dtype=np.int64).astype(np.int32))
    want = np.sort(orc.gen_keys(n, nthr, maxid, thr, q))
    assert np.array_equal(np.sort(t[:, 0]), want)


def test_host_generator_seeds_permute(hw):
    a = hw.generate_host(100000, 2, 100000, 100000, 1.0, 1, 2)
    b = hw.generate_host(100000, 2, 100000, 100000, 1.0, 2, 2)
    assert not np.array_equal(a[:, 0], b[:, 0])
    assert np.array_equal(np.sort(a[:, 0]), np.sort(b[:, 0]))


@pytest.mark.parametrize("variant,m,B", [(1, 1 << 20, 512), (1, 3 << 20, 512), (1, 1 << 20, 48),
                                         (1, 1 << 10, 2048), (0, 1 << 20, 48), (0, 7, 1),
                                         (2, 1 << 20, 64), (1, 1 << 20, 0)])
def test_assert_args_matches_reference_rules(hw, orc, variant, m, B):
    ref_invalid = bool(orc.lib().orc_bloom_args_invalid(min(variant, 1), m, B))
    assert hw.assert_args(hw.BloomFilterArgs(variant, m, 1, B)) == (not ref_invalid)


def test_from_flag_mirrors_cli_parsing(hw):
    assert hw.BloomFilterArgs.from_flag("no", 1, 1) is None
    assert hw.BloomFilterArgs.from_flag("blocked", 1 << 20, 2).variant == hw.BLOCKED
    assert hw.BloomFilterArgs.from_flag("basic", 1 << 20, 2).variant == hw.BASIC
    assert hw.BloomFilterArgs.from_flag("whatever", 1 << 20, 2).variant == hw.BASIC  # main.c:692
    assert hw.BloomFilterArgs.from_flag("sectorized", 1 << 20, 2).variant == hw.SECTORIZED


def test_cli_help_and_errors(hw):
    cli = hw.CLI_PATH
    out = subprocess.run([cli, "-h"], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0 and "--bloom-filter" in out.stdout
    out = subprocess.run([cli, "-a", "NPO"], capture_output=True, text=True, timeout=60)
    assert "does not exist" in out.stdout
    # src/bloom_filter.c:25-34: invalid filter arguments print and exit(1)
    out = subprocess.run([cli, "-b", "blocked", "-m", "1000", "-r", "10", "-s", "10"],
                         capture_output=True, text=True, timeout=60)
    assert out.returncode == 1 and "m must be a power of 2" in out.stdout


def test_package_refuses_without_library(tmp_path):
    # the product path must fail loudly when the HIP library is missing (no CPU fallback)
    code = ("import sys, os; sys.path.insert(0, %r); import hwbloomradixjoin_amd as hw; "
            "hw.LIB_PATH = os.path.join(%r, 'nope.so'); hw._LIB = None\n"
            "try:\n    hw.lib()\nexcept ImportError as e:\n    print('RAISED', e)\n") % (ROOT, str(tmp_path))
    out = subprocess.run(["python3", "-c", code], capture_output=True, text=True, timeout=120)
    assert "RAISED" in out.stdout


def test_rccl_binding_draws_unique_id(hw):
    """The native RCCL transport binds librccl.so.1 at first use (hwbrj_comm.cpp) and draws the
    128-byte ncclUniqueId a multi-GPU job hands to every rank (no GPU needed for the id)."""
    import ctypes
    a, b = (ctypes.c_uint8 * 128)(), (ctypes.c_uint8 * 128)()
    assert hw.lib().hwbrj_comm_unique_id(a) == 0, hw.lib().hwbrj_last_error()
    assert hw.lib().hwbrj_comm_unique_id(b) == 0
    assert any(bytes(a)) and bytes(a) != bytes(b)


def test_write_relation_format(hw, tmp_path):
    """hwbrj_write_relation: src/generator.c:250-263's file, byte for byte as its fprintf writes it
    ("#KEY, VAL" header, "%d %d" lines), negative and extreme values included."""
    import numpy as np
    rng = np.random.default_rng(5)
    t = np.stack([rng.integers(-2**31, 2**31, size=5000), rng.integers(-2**31, 2**31, size=5000)], 1)
    t[:4] = [[0, 0], [-1, 2**31 - 1], [-2**31, -2**31], [2**31 - 1, -7]]
    f = tmp_path / "R.tbl"
    hw.write_relation(t.astype(np.int32), str(f))
    want = "#KEY, VAL\n" + "".join(f"{k} {p}\n" for k, p in t.tolist())
    assert f.read_text() == want
    hw.write_relation(np.zeros((0, 2), dtype=np.int32), str(f))
    assert f.read_text() == "#KEY, VAL\n"


def test_product_build_reports_no_knobs(hw):
    """hwbrj_version() names every compile-time switch and dev environment knob that differs from
    the product default: the in-tree build reports none."""
    v = hw.version()
    assert v.startswith("hwbloomradixjoin_amd ") and "(gfx950)" in v
    assert "knobs" not in v, v


def test_ablations_need_dev_build(tmp_path):
    """A results-invalid ablation cannot slip into a product build: hwbrj_kernels.hip refuses
    HWBRJ_ABL_* / HWBRJ_STAMPS unless HWBRJ_DEV_BUILD is defined (preprocessing only)."""
    src = os.path.join(ROOT, "hwbloomradixjoin_amd", "csrc", "hwbrj_kernels.hip")
    inc = ["-I", os.path.join(ROOT, "hwbloomradixjoin_amd", "csrc"), "-I", os.path.join(ROOT, "include")]
    base = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-std=c++17", "-E", "-o", str(tmp_path / "k.i")] + inc
    r = subprocess.run(base + ["-DHWBRJ_ABL_NOCRC", src], capture_output=True, text=True)
    assert r.returncode != 0 and "dev builds only" in r.stderr, r.stderr[-2000:]
    r = subprocess.run(base + ["-DHWBRJ_ABL_NOCRC", "-DHWBRJ_DEV_BUILD", src], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]


def test_bench_uses_pmc_traffic_only_for_the_profiled_library(tmp_path, hw):
    """bench.py's roofline.traffic comes from profiles/pmc_traffic.json only when that file was
    profiled on this configuration AND on a library with the same stamp."""
    import importlib.util
    import json as _json
    spec = importlib.util.spec_from_file_location("bench", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    key = [1, 2, 0.01, "blocked", 1 << 30, 1, 1024]
    f = tmp_path / "pmc.json"
    f.write_text(_json.dumps({"config_key": key, "library": hw.version(), "phases": {}}))
    pm, note = bench.load_pmc(str(f), key, hw.version())
    assert pm is not None and "this library" in note
    pm, note = bench.load_pmc(str(f), key, hw.version() + " knobs: X")
    assert pm is None and "not used" in note
    pm, note = bench.load_pmc(str(f), key[:-1] + [512], hw.version())
    assert pm is None
    assert "src " in hw.version()


def test_bench_modeled_join_key_bytes():
    """modeled_bytes prices the join's runs at the key format the join reported
    (hwbrj_stats_t.join_keys, join_key_bits): join_key_bits / 8 bytes per key for packed and mixed
    runs (2.25 for the north star's 18-bit keys), else 4."""
    import importlib.util
    from types import SimpleNamespace as NS
    spec = importlib.util.spec_from_file_location("bench", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    assert bench.join_key_bytes(NS(join_keys=1, join_key_bits=18)) == 2.25  # packed (the north star)
    assert bench.join_key_bytes(NS(join_keys=1, join_key_bits=24)) == 3.0
    assert bench.join_key_bytes(NS(join_keys=2, join_key_bits=18)) == 2.25  # mixed
    assert bench.join_key_bytes(NS(join_keys=0, join_key_bits=32)) == 4.0  # 32-bit codes
    mb = bench.modeled_bytes(10, 20, 5, 0, 4.0, 3.0)
    assert mb["join_codes_R"] == 60.0 and mb["survivors"] == 30.0


def test_write_result_relation_reference_order(hw, tmp_path):
    """hwbrj_write_result_relation emits the pairs in write_result_relation's order
    (src/tuple_buffer.h:205-231): per thread, the newest chained buffer first, every buffer from its
    last pair to its first (cb_begin_backwards / cb_read_backwards, :58-90). Thread 0 holds a
    partly filled newest buffer (3 pairs) and a full older one; thread 1 one pair."""
    import ctypes
    n_old = hw._CB_TUPLES
    old = np.stack([np.arange(n_old), -np.arange(n_old)], 1).astype(np.int32)
    new = np.array([[7, 70], [8, 80], [9, 90]], dtype=np.int32)
    one = np.array([[5, 50]], dtype=np.int32)
    TP = ctypes.POINTER(hw._Tuple)
    b_old = hw._TupleBuffer(old.ctypes.data_as(TP), None)
    b_new = hw._TupleBuffer(new.ctypes.data_as(TP), ctypes.pointer(b_old))
    b_one = hw._TupleBuffer(one.ctypes.data_as(TP), None)
    c0 = hw._ChainedTupleBuffer(ctypes.pointer(b_new), None, None, 3, 0, 0, 2)
    c1 = hw._ChainedTupleBuffer(ctypes.pointer(b_one), None, None, 1, 0, 0, 1)
    tl = (hw._ThreadResult * 2)(hw._ThreadResult(n_old + 3, ctypes.addressof(c0), 0),
                                hw._ThreadResult(1, ctypes.addressof(c1), 1))
    res = hw._Result(n_old + 4, ctypes.addressof(tl), 2)
    out = tmp_path / "Out.tbl"
    assert hw.lib().hwbrj_write_result_relation(ctypes.addressof(res), str(out).encode()) == 0
    got = np.loadtxt(out, dtype=np.int64, ndmin=2)
    want = np.concatenate([new[::-1], old[::-1], one]).astype(np.int64)
    assert got.shape == want.shape and np.array_equal(got, want)


def test_prof_summary_phase_labels():
    """tools/prof_summary.py (the per-phase PMC traffic bench.py's roofline.traffic comes from)
    takes the last join between two k_join dispatches (a join's last kernel) and labels plan /
    list-fill kernels by the side of the scatter before them, whichever side the Engine runs first."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("prof_summary", os.path.join(ROOT, "tools", "prof_summary.py"))
    ps = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ps)
    one = ["k_scatter_s", "k_plan", "k_list_fill", "k_scatter_r", "k_plan", "k_list_fill", "k_build",
           "k_probe", "k_join_split", "k_join"]
    names = ["k_gen"] + one + ["__amd_rocclr_copyBuffer"] + one + ["k_copy_bw"]
    idx = ps.last_join(names)
    assert [names[i] for i in idx] == ["__amd_rocclr_copyBuffer"] + one
    assert ps.label(names, idx) == ["other", "s_scatter", "s_index", "s_index", "r_scatter", "r_index",
                                    "r_index", "build", "probe", "join", "join"]
    r_first = ["k_scatter_r", "k_plan", "k_list_fill", "k_build", "k_scatter_s", "k_plan", "k_list_fill"]
    assert ps.label(r_first, range(len(r_first))) == ["r_scatter", "r_index", "r_index", "build",
                                                      "s_scatter", "s_index", "s_index"]
