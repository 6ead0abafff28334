"""Static instruction counts per source section of one kernel, from a gfx950 assembly listing built
with -DMCPT_ISA_MARKERS (hipcc -S --cuda-device-only): every instruction is attributed to the last
'; MCPT_SEC <name>' marker before it in the listing (block layout follows the source closely; the
attribution is approximate where the scheduler moves instructions across a marker).  Section names
that end in digits continue the section of that name (t_node2: the rest of t_node after a branch).

--rare OPCODE...: basic blocks holding one of these opcodes are counted under 'rare' (branches that
the measured rays never take: the infinite-inverse slab (v_sub_f32: the fast path subtracts with
packed adds), the fp64 division fallback (v_div_scale_f64), scratch stack entries).

  python tools/isa_sections.py kernels_markers.s _ZN8mcpt_dev7k_shadeILb0EEEvNS_9ShadeArgsE
"""
import argparse
import collections
import re


def blocks(path, sym):
    """[(section, block label, Counter)] in listing order."""
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith(sym + ":"))
    cur, out = "entry", []
    blk = None
    for l in lines[start + 1:]:
        if l.startswith(".Lfunc_end"):
            break
        m = re.search(r"MCPT_SEC (\w+)", l)
        if m:
            cur = re.sub(r"\d+$", "", m.group(1))
            blk = None
            continue
        mb = re.match(r"^(\.LBB\d+_\d+):|^; %bb\.(\d+):", l)
        if mb:
            blk = None
            label = mb.group(1) or f"bb.{mb.group(2)}"
            out.append((cur, label, collections.Counter()))
            blk = out[-1][2]
            continue
        s = l.strip()
        if not s or s.startswith((";", ".")) or s.endswith(":"):
            continue
        if blk is None:
            out.append((cur, "(cont)", collections.Counter()))
            blk = out[-1][2]
        op = s.split()[0]
        kind = ("valu" if op.startswith("v_") else "salu" if op.startswith("s_") else
                "vmem" if op.startswith(("global_", "scratch_", "buffer_", "flat_")) else
                "lds" if op.startswith("ds_") else "other")
        blk[kind] += 1
        blk["op:" + op.split("_e32")[0].split("_e64")[0]] += 1
    return out


def sections(path, sym, rare=()):
    cnt = collections.defaultdict(collections.Counter)
    for sec, _, c in blocks(path, sym):
        if rare and any(k.startswith("op:" + r) for k in c for r in rare):
            sec = "rare"
        cnt[sec].update(c)
    return cnt


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("sym")
    ap.add_argument("--rare", nargs="*", default=[])
    a = ap.parse_args()
    for name, c in sections(a.asm, a.sym, a.rare).items():
        hot = ("v_div_scale_f32", "v_rcp_iflag_f32", "v_div_scale_f64", "v_mul_lo_u32", "v_mul_hi_u32", "v_rcp_f64",
               "v_sqrt_f32")
        extra = " ".join(f"{k}={c['op:' + k]}" for k in hot if c["op:" + k])
        print(f"{name:12s} valu {c['valu']:4d} salu {c['salu']:4d} vmem {c['vmem']:3d} lds {c['lds']:3d}  {extra}")
