"""Register use and per-barrier-interval instruction mix of kernels in a gfx950 .s file (dev tool).

    hipcc -O3 --offload-arch=gfx950 --cuda-device-only -S -o /tmp/k.s hwbrj_kernels.hip
    python tools/isa_mix.py /tmp/k.s <kernel-name-substring> [--mix]
"""
import collections
import re
import sys


def main():
    path, sub = sys.argv[1], sys.argv[2]
    s = open(path).read()
    for b in s.split("  - .agpr_count")[1:]:
        name = re.search(r"\.name:\s+(\S+)", b).group(1)
        if sub in name:
            def field(k):
                return re.search(r"\." + k + r":\s+(\d+)", b).group(1)
            print(f"{name[:64]:64s} vgpr={field('vgpr_count')} spill={field('vgpr_spill_count')} "
                  f"sgpr_spill={field('sgpr_spill_count')}")
    if "--mix" not in sys.argv:
        return
    for m in re.finditer(r"^(_Z\S*" + re.escape(sub) + r"\S*):", s, re.M):
        a = m.start()
        e = s.index(".Lfunc_end", a)
        body = s[a:e].splitlines()
        idx = [i for i, l in enumerate(body) if "s_barrier" in l]
        print(m.group(1))
        for j in range(len(idx) - 1):
            c = collections.Counter()
            for l in body[idx[j]:idx[j + 1]]:
                t = l.strip().split()
                if not t or t[0][0] in ";.":
                    continue
                op = t[0]
                key = ("waitcnt" if op.startswith("s_waitcnt") else "salu" if op.startswith("s_") else
                       "valu" if op.startswith("v_") else "lds" if op.startswith("ds_") else
                       "vmem" if op.startswith(("buffer_", "global_", "scratch_")) else op)
                c[key] += 1
            print(f"   lines {idx[j]}-{idx[j + 1]}: {dict(c)}")


if __name__ == "__main__":
    main()
