"""k_trace VALU attribution: static VALU instructions per
section of the kernel's loop (the -DMCPT_ISA_MARKERS listing, tools/isa_sections.py) times the
section's executions in the counting build's phase counts (bench.py roofline.k_trace_phases.counts:
one frame), against the measured SQ_INSTS_VALU of the product kernel per frame.

  python tools/trace_attrib.py km.s bench.json [--valu 78.8e9] [--sym k_traceILi2ELi8ELb0]

A section's static count is an upper bound on what one execution issues: exec-masked branches that
no lane of the wave takes are skipped (s_cbranch_execz).  Sections marked 'rare' (the slab of a ray
with an infinite inverse component, the fp64 division fallback of the triangle test) are counted as
never executed."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import isa_sections  # noqa: E402

# section -> which phase count multiplies it
PER = {"t_node": "node_iters", "t_pop": "pop_iters", "t_tri": "tri_phases", "t_top": "trips", "t_trip": "trips",
       "t_end": "trips", "t_finish": "finish_trips", "t_refill": "refills", "rare": None}
WHAT = {"t_node": "pair step: child-pair slab test, cull keys, push, leaf parking",
        "t_pop": "stack pop (LDS / scratch entries, re-test against the cut)",
        "t_tri": "triangle phase: one Moller-Trumbore test per parked leaf, hit update, leaf advance",
        "t_top": "loop top: idle-lane ballot, refill decision",
        "t_trip": "trip bookkeeping and register moves before the node phase",
        "t_end": "trip end: loop back-edge moves",
        "t_finish": "ray finish: result store, occluder-cache record (any hit)",
        "t_refill": "refill: hand-out atomic, entry search, ray loads, 1/d, culling scale",
        "rare": "infinite-inverse slab, fp64 division fallback (not executed on these rays)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("bench_json")
    ap.add_argument("--sym", default="_ZN8mcpt_dev7k_traceILi2ELi8ELb0EEEvNS_9TraceArgsE")
    ap.add_argument("--valu", type=float, default=78.8e9, help="measured SQ_INSTS_VALU per frame (PMC pass)")
    ap.add_argument("--rare", nargs="*", default=["v_sub_f32", "v_div_scale_f64", "scratch_"],
                    help="opcodes whose basic blocks are never executed on the measured rays (isa_sections.py)")
    a = ap.parse_args()
    sec = isa_sections.sections(a.asm, a.sym, rare=a.rare)
    d = json.load(open(a.bench_json))
    counts = d["roofline"]["k_trace_phases"]["counts"]
    rows, tot = [], 0.0
    for name, c in sec.items():
        key = PER.get(name)
        n = counts.get(key, 0) if key else 0
        v = c["valu"] * n
        tot += v
        rows.append((name, c["valu"], key, n, v))
    print(f"{'section':10s} {'static':>6s} {'x count':>14s} {'':>12s} {'VALU (G)':>9s} {'share':>6s}")
    for name, st, key, n, v in sorted(rows, key=lambda r: -r[4]):
        print(f"{name:10s} {st:6d} {str(key):>14s} {n/1e6:10.1f} M {v/1e9:9.2f} {v/max(tot,1):6.3f}  {WHAT.get(name, '')}")
    print(f"estimate {tot/1e9:.2f} G VALU per frame (upper bound per section); measured {a.valu/1e9:.2f} G: "
          f"ratio {tot/a.valu:.3f}")


if __name__ == "__main__":
    main()
