"""One rank's share of a strong-split frame on one GPU, rendered a few times (for a kernel trace of
the per-iteration costs):

  rocprofv3 --kernel-trace -d gpurun_out/rk -o rk --output-format csv -- \\
      python3 tools/rank_frames.py --config 2 --world 8 --rank 0 --frames 3

Prints per frame the wall time, iterations and the library's kernel times (events)."""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mc-path-tracer_amd"))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--frames", type=int, default=3)
    ap.add_argument("--slots", type=int, default=None)
    a = ap.parse_args()
    import bench
    import mcpt
    from mcpt import parallel

    rc = mcpt.CONFIGS[a.config]
    args = argparse.Namespace(config=a.config, slots=a.slots)
    pt, _, _ = bench.make_tracer(0, args, rc, rc.spp)
    tile = bench.part_tile(a.world)
    W, H = rc.width, rc.height
    base = a.slots or bench.BENCH_SLOTS[a.config]
    slots = parallel.strong_slots(base, a.world, W, H, rc.spp, tile) if a.world > 1 else base
    tiles = bench.tiles_for(a.rank, a.world, W, H, tile)
    if a.world > 1:
        pt.set_compact_paths(True)
        pt.set_path_slots(1)
        pt.resize(W, H, tile, tile)
        pt.set_tiles(tiles)
        pt.set_path_slots(slots)
    else:
        pt.set_path_slots(slots)
        pt.resize(W, H, tile, tile)
    for f in range(a.frames + 1):
        pt.clear()
        t0 = time.perf_counter()
        st = pt.render()
        dt = time.perf_counter() - t0
        rc_ = pt.ray_counts()  # traversed vs resolved (occluder cache) since the clear
        print(json.dumps({"frame": f, "warmup": f == 0, "wall_ms": round(dt * 1e3, 3), "iterations": st.iterations,
                          "ms_shade": round(st.ms_shade, 3), "ms_trace": round(st.ms_extend, 3), "rays": st.rays,
                          "slots": slots, "tiles": len(tiles), "ray_counts": rc_,
                          "occ_resolved_frac": round(rc_["any_hit_occluder_cache"] / max(1, rc_["any_hit"]), 4),
                          "knobs": {k: v for k, v in os.environ.items() if k.startswith("MCPT_")}}), flush=True)
    pt.close()


if __name__ == "__main__":
    main()
