"""Two pipelines on one GPU (round 6 probe): does running two halves of the frame concurrently, each
in its own context and HIP stream, fill the idle issue slots of one kernel with another's work?

The frame's 64-px tiles are split (tx + ty) mod 2 between two contexts on device 0 (compact path
state, as two ranks of the strong split would hold it).  Timed: the whole frame in one context at
the bench's slots; the two halves one after the other; the two halves at once from two host
threads (ctypes releases the GIL, each context syncs only its own stream).  Timing only: the
halves' films are those of the strong split (tests/test_gpu.py covers their parity).

Usage: python tools/overlap_probe.py [--config 2] [--slots 24 48] [--frames 2] [--out f.json]
"""
import argparse
import json
import os
import sys
import threading
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mc-path-tracer_amd"))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--slots", type=int, nargs="+", default=[24, 48])
    ap.add_argument("--tile", type=int, default=64)
    ap.add_argument("--frames", type=int, default=2)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    import mcpt
    from mcpt import parallel

    import bench

    rc = mcpt.CONFIGS[args.config]
    W, H = rc.width, rc.height
    scene = mcpt.build_config_scene(args.config)
    cam = mcpt.config_camera(rc)

    def tracer():
        pt = mcpt.PathTracer(0, mcpt.default_config(spp=rc.spp, max_depth=rc.max_depth))
        pt.upload_scene(scene)
        pt.set_camera(cam)
        return pt

    res = {"what": __doc__.split("\n\n")[1].replace("\n", " "), "config": args.config, "runs": []}
    base = bench.BENCH_SLOTS[args.config]
    one = tracer()
    one.set_path_slots(base)
    one.resize(W, H, 256, 256)

    def timed(fn):
        t0 = time.perf_counter()
        fn()
        return (time.perf_counter() - t0) * 1e3

    def one_frame():
        one.clear()
        one.render()
    one_frame()
    t_one = [timed(one_frame) for _ in range(args.frames)]
    res["one_context_ms"] = [round(x, 2) for x in t_one]
    print(json.dumps({"one_context_ms": res["one_context_ms"], "slots": base}), flush=True)

    halves = [tracer(), tracer()]
    for slots in args.slots:
        for r, pt in enumerate(halves):
            pt.set_compact_paths(True)
            pt.set_path_slots(1)
            pt.resize(W, H, args.tile, args.tile)
            pt.set_tiles(parallel.tiles_for_rank(r, 2, W, H, args.tile))
            pt.set_path_slots(slots)

        def half(pt):
            pt.clear()
            pt.render()

        def seq():
            for pt in halves:
                half(pt)

        def conc():
            th = [threading.Thread(target=half, args=(pt,)) for pt in halves]
            for t in th:
                t.start()
            for t in th:
                t.join()
        seq()
        conc()
        t_seq = [timed(seq) for _ in range(args.frames)]
        t_conc = [timed(conc) for _ in range(args.frames)]
        run = {"slots_per_half": slots, "tile": args.tile, "sequential_ms": [round(x, 2) for x in t_seq],
               "concurrent_ms": [round(x, 2) for x in t_conc],
               "concurrent_vs_one_context": round(min(t_one) / min(t_conc), 4)}
        res["runs"].append(run)
        print(json.dumps(run), flush=True)
    for pt in halves + [one]:
        pt.close()
    if args.out:
        json.dump(res, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
