"""Static instruction counts per source section of one kernel, from a gfx950 assembly listing built
with -DMCPT_ISA_MARKERS (hipcc -S --cuda-device-only): every instruction is attributed to the last
'; MCPT_SEC <name>' marker before it in the listing (block layout follows the source closely; the
attribution is approximate where the scheduler moves instructions across a marker).

  python tools/isa_sections.py kernels_markers.s _ZN8mcpt_dev7k_shadeILb0EEEvNS_9ShadeArgsE
"""
import collections
import re
import sys


def sections(path, sym):
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith(sym + ":"))
    cur = "entry"
    cnt = collections.defaultdict(lambda: collections.Counter())
    for l in lines[start + 1:]:
        if l.startswith(".Lfunc_end"):
            break
        m = re.search(r"MCPT_SEC (\w+)", l)
        if m:
            cur = m.group(1)
            continue
        s = l.strip()
        if not s or s.startswith((";", ".")) or s.endswith(":"):
            continue
        op = s.split()[0]
        kind = ("valu" if op.startswith("v_") else "salu" if op.startswith("s_") else
                "vmem" if op.startswith(("global_", "scratch_", "buffer_", "flat_")) else
                "lds" if op.startswith("ds_") else "other")
        cnt[cur][kind] += 1
        if op.startswith(("v_div_scale_f32", "v_rcp_iflag", "v_div_scale_f64", "v_mul_lo_u32", "v_mul_hi_u32",
                          "v_rcp_f64", "v_sqrt")):
            cnt[cur][op.split("_e")[0]] += 1
    return cnt


if __name__ == "__main__":
    for name, c in sections(sys.argv[1], sys.argv[2]).items():
        extra = " ".join(f"{k}={v}" for k, v in sorted(c.items()) if k not in ("valu", "salu", "vmem", "lds", "other"))
        print(f"{name:12s} valu {c['valu']:4d} salu {c['salu']:4d} vmem {c['vmem']:3d} lds {c['lds']:3d}  {extra}")
