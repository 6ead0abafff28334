"""Per-basic-block instruction counts of one kernel in a gfx950 assembly listing (hipcc -S
--cuda-device-only): VALU (v_*), SALU (s_*), vector memory (global_/scratch_/buffer_), LDS (ds_).
Used for the static side of the k_trace / k_shade VALU attribution:

  python tools/isa_blocks.py kernels.s _ZN8mcpt_dev7k_traceILi2ELi8ELb0EEEvNS_9TraceArgsE
"""
import re
import sys


def blocks(path, sym):
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith(sym + ":"))
    out, cur = [], None
    for i in range(start + 1, len(lines)):
        l = lines[i]
        if l.startswith(".Lfunc_end") or l.startswith("\t.section"):
            break
        m = re.match(r"^(\.LBB\d+_\d+):|^; %bb\.(\d+):", l)
        if m:
            cur = {"name": m.group(1) or f"bb.{m.group(2)}", "line": i - start + 1, "valu": 0, "salu": 0, "vmem": 0,
                   "lds": 0}
            out.append(cur)
            continue
        s = l.strip()
        if not s or s.startswith(";") or s.startswith(".") or cur is None:
            continue
        op = s.split()[0]
        if op.startswith("v_"):
            cur["valu"] += 1
        elif op.startswith("s_"):
            cur["salu"] += 1
        elif op.startswith(("global_", "scratch_", "buffer_", "flat_")):
            cur["vmem"] += 1
        elif op.startswith("ds_"):
            cur["lds"] += 1
    return out


if __name__ == "__main__":
    for b in blocks(sys.argv[1], sys.argv[2]):
        print(f"{b['name']:12s} line {b['line']:5d}  valu {b['valu']:3d} salu {b['salu']:3d} vmem {b['vmem']:2d} lds {b['lds']:2d}")
