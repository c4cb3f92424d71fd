"""The drop-in boundary as the reference's own callers see it.

- CPU: a C translation unit that includes the reference's headers (src/types.h, bloom_filter.h,
  parallel_radix_join.h, parallel_radix_join_bloom.h, as src/main.c does) together with
  include/hwbrj.h compiles without edits and links BPRO / hwbrj_BPRO from libhwbrj.so. Skipped
  when /root/reference is absent (the GPU box has no copy of it).
- GPU: the five regexes of the reference's harness (measurements/run.py:109-129, restated below)
  parse the CLI's stdout, and the four that concern the operator parse host BPRO's stdout.
"""
import os
import re
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
REF_SRC = "/root/reference/src"
INT_MAX = 2**31 - 1

# measurements/run.py:109-129 (parse_result), verbatim patterns
RUN_PY_S_SIZE = r"relation S with size = [\d.]+ MiB, #tuples = (\d+) : OK"
RUN_PY_FILTERED = r"S-tuples after filter: (\d+)\n"
RUN_PY_CYCLES = r"RUNTIME TOTAL, BUILD, PART \(cycles\):\W+(\d+)\W+(\d+)\W+(\d+)"
RUN_PY_TIME = r"TOTAL-TIME-USECS, TOTAL-TUPLES, NSEC-PER-TUPLE:\W+([\d.]+)\W+(\d+)\W+([\d.]+)"
RUN_PY_PHASES = r"PARTITION-TIME-USECS, PROBE-TIME-USECS, JOIN-TIME-USECS:\W+([\d.]+)\W+([\d.]+)\W+([\d.]+)"


def parse_like_run_py(out, with_s_line=True):
    """measurements/run.py:parse_result's searches; a failing search raises there (AttributeError
    on None.group), so every pattern must match."""
    d = {}
    if with_s_line:
        m = re.search(RUN_PY_S_SIZE, out)
        assert m, out[-2000:]
        d["s_size"] = int(m.group(1))
    m = re.search(RUN_PY_FILTERED, out)
    d["filtered"] = int(m.group(1)) if m else None
    for key, pat in (("cycles", RUN_PY_CYCLES), ("time", RUN_PY_TIME), ("phases", RUN_PY_PHASES)):
        m = re.search(pat, out)
        assert m, (key, out[-2000:])
        d[key] = m.groups()
    return d


C_MAIN = r"""
#include <stdio.h>
#include <stddef.h>
%(pre)s
#include "hwbrj.h"
%(post)s
/* what src/main.c does with these types (:304, :390-393, :473-478) */
typedef result_t *(*JoinBloom)(relation_t *, relation_t *, int, bloom_filter_args_t *);
typedef result_t *(*Join)(relation_t *, relation_t *, int);
int main(void) {
    bloom_filter_args_t a;
    a.variant = BLOCKED; a.m = 1 << 24; a.k = 1; a.B = 1024;
    JoinBloom jb[] = {BPRO, hwbrj_BPRO, BPRH, BPRHO, BRJ};
    Join j[] = {PRO, hwbrj_PRO, PRH, PRHO, RJ};
    printf("%%zu %%zu %%zu %%zu %%d %%d %%d %%d\n", sizeof(tuple_t), sizeof(relation_t),
           sizeof(result_t), sizeof(bloom_filter_args_t), (int) BASIC, (int) BLOCKED,
           (int) HWBRJ_SECTORIZED, jb[0] != 0 && jb[1] != 0 && j[0] != 0 && j[1] != 0 && a.B == 1024);
    return 0;
}
"""

REF_HEADERS = ('#include "types.h"\n#include "bloom_filter.h"\n#include "parallel_radix_join.h"\n'
               '#include "parallel_radix_join_bloom.h"')


def _compile_and_run(hw, tmp_path, name, pre, post, include_ref):
    src = tmp_path / f"{name}.c"
    src.write_text(C_MAIN % {"pre": pre, "post": post})
    exe = tmp_path / name
    pkg = os.path.dirname(hw.LIB_PATH)
    cmd = ["gcc", "-std=gnu11", "-Wall", "-Werror", "-o", str(exe), str(src),
           "-I", os.path.join(ROOT, "include")]
    if include_ref:
        cmd += ["-I", REF_SRC]
    cmd += ["-L", pkg, "-lhwbrj", f"-Wl,-rpath,{pkg}"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    return r.stdout.split()


@pytest.mark.skipif(not os.path.isdir(REF_SRC), reason="the reference is not present (GPU box)")
@pytest.mark.parametrize("order", ["reference_first", "types_after_hwbrj"])
def test_reference_headers_and_hwbrj_h_in_one_unit(hw, tmp_path, order):
    """src/main.c includes types.h, bloom_filter.h and the join headers (src/main.c:254-264);
    adding #include "hwbrj.h" after them must compile with no other edit, and
    link BPRO / hwbrj_BPRO against libhwbrj.so. types.h may also come after hwbrj.h."""
    if order == "reference_first":
        out = _compile_and_run(hw, tmp_path, order, REF_HEADERS, "", True)
    else:
        out = _compile_and_run(hw, tmp_path, order, "", '#include "types.h"\n#include "parallel_radix_join.h"', True)
    assert out == ["8", "16", "24", "32", "0", "1", "2", "1"], out


def test_hwbrj_h_alone_compiles_as_c(hw, tmp_path):
    out = _compile_and_run(hw, tmp_path, "alone", "", "", False)
    assert out == ["8", "16", "24", "32", "0", "1", "2", "1"], out


def test_run_py_regexes_on_a_reference_shaped_sample():
    """The restated patterns parse the reference's own output shape (src/main.c:433-480,
    src/parallel_radix_join_bloom.c:1253, :1531-1544): a sample built from its format strings."""
    def cfmt(fmt, *args):  # the C format strings, with Python's conversions
        return fmt.replace("%llu", "%d").replace("lf", "f") % args
    sample = ("[INFO ] Creating relation R with size = 7.629 MiB, #tuples = 1000000 : OK \n"
              "[INFO ] Creating relation S with size = 122.070 MiB, #tuples = 16000000 : OK \n"
              "[INFO ] Running join algorithm PRO ...\n"
              "S-tuples after filter: 1073970\n"
              + cfmt("RUNTIME TOTAL, BUILD, PART (cycles): \n%llu \t %llu \t %llu\n", 1, 2, 3)
              + cfmt("TOTAL-TIME-USECS, TOTAL-TUPLES, NSEC-PER-TUPLE: \n%.4lf \t %llu \t %.4lf\n", 1.5, 160000, 0.1)
              + cfmt("PARTITION-TIME-USECS, PROBE-TIME-USECS, JOIN-TIME-USECS: \n%.4lf \t %.4lf\t %.4lf\n", 1.0, 0.2, 0.5)
              + "[INFO ] Results = 160000. DONE.\n")
    d = parse_like_run_py(sample)
    assert d["s_size"] == 16000000 and d["filtered"] == 1073970
    assert d["time"][1] == "160000"


@pytest.mark.gpu
def test_cli_stdout_parses_with_run_py_regexes(hw):
    """The CLI's stdout through run.py's five searches: S size, S-tuples after filter, the three
    timing blocks; TOTAL-TUPLES is Results (src/parallel_radix_join_bloom.c:1536-1539)."""
    import json
    g = json.load(open(os.path.join(HERE, "golden", "survey_counts.json")))["F3_grid"]
    out = subprocess.run([hw.CLI_PATH, "-a", "PRO", "-r", str(g["r"]), "-s", str(g["s"]), "-q", "0.01",
                          "-b", "blocked", "-m", str(g["m"]), "-k", "1", "-n", "2"],
                         capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    d = parse_like_run_py(out.stdout)
    assert d["s_size"] == g["s"]
    assert d["filtered"] == g["rows"]["1024"][0]
    assert int(d["time"][1]) == g["results"]
    tot, part, join = float(d["time"][0]), float(d["phases"][0]), float(d["phases"][2])
    assert tot > 0 and abs(part + join - tot) <= 0.01 * tot + 1.0
    # PRO without a filter: no "S-tuples after filter" line, the rest parses
    out = subprocess.run([hw.CLI_PATH, "-a", "PRO", "-r", "1000000", "-s", "16000000", "-q", "1.0"],
                         capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    d = parse_like_run_py(out.stdout)
    assert d["filtered"] is None and int(d["time"][1]) == 16000000


@pytest.mark.gpu
def test_host_bpro_stdout_parses_with_run_py_regexes(hw, capfd):
    """Host BPRO prints what the reference's join prints (the filter count and the timing block,
    src/parallel_radix_join_bloom.c:1253, :1509-1547): run.py's four operator patterns match."""
    import json
    g = json.load(open(os.path.join(HERE, "golden", "survey_counts.json")))["F3_grid"]
    R = hw.Relation(hw.generate_host(g["r"], 2, g["r"], g["r"], 1.0, 1))
    S = hw.Relation(hw.generate_host(g["s"], 2, INT_MAX, g["r"], g["q"], 2))
    capfd.readouterr()
    res = hw.BPRO(R, S, 2, hw.BloomFilterArgs(hw.BLOCKED, g["m"], 1, 1024))
    d = parse_like_run_py(capfd.readouterr().out, with_s_line=False)
    assert res.totalresults == g["results"] == int(d["time"][1])
    assert d["filtered"] == g["rows"]["1024"][0]
