"""Multi-GPU rehearsal on one GPU: render each rank's tile partition alone and time it.

For N in (2, 4, 8), rank r's share of the frame -- the tiles with (tx + ty) mod N == r -- is
rendered to the config's spp with the strong split's path slots (mcpt/parallel.py strong_slots) and
the rank's own compact path state (mcpt_set_compact_paths, as bench.py's ranks hold it), one rank
after the other on one device, with the device memory the rank's context holds.  The slowest partition sets an N-GPU frame's time, so
max / mean of the per-rank times is the strong split's load imbalance.
Tile sizes 256 (the reference's Film tile, Film.cu:17) and 64 (bench.MULTI_TILE) are compared:
results do not depend on the tiling (keyed RNG), only the balance does.  The whole frame on one
"rank" (N = 1, the config's bench slots) is timed too, so efficiency = t_1 / (N max_r t_r), and at
64 px tiles the base slot count is compared with the strong split's (--slot-choices).

Usage: python tools/partition_rehearsal.py [--configs 2 4 5] [--tiles 64] [--out profiles/partition_r05.json]
"""
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
    ap.add_argument("--configs", type=int, nargs="+", default=[2, 4, 5])
    ap.add_argument("--tiles", type=int, nargs="+", default=[64])
    ap.add_argument("--spp", type=int, default=None, help="override every config's spp (C5's 4096 spp frame: ~50 s)")
    ap.add_argument("--slot-choices", default="strong,base",
                    help="at the smallest tile: strong_slots and/or base, and explicit counts (e.g. strong,base,96)")
    ap.add_argument("--worlds", type=int, nargs="+", default=[2, 4, 8])
    ap.add_argument("--out", default=os.path.join(REPO, "profiles", "partition_r05.json"))
    args = ap.parse_args()
    import torch

    import mcpt
    from mcpt import parallel

    import bench

    def used_gb():  # device memory in use (every allocation of this process: the library's hipMallocs)
        free, total = torch.cuda.mem_get_info(0)
        return round((total - free) / 1e9, 2)

    res = {"what": __doc__.split("\n\n")[1].replace("\n", " "), "runs": []}
    for cid in args.configs:
        rc = mcpt.CONFIGS[cid]
        spp = args.spp or rc.spp
        scene = mcpt.build_config_scene(cid)
        cam = mcpt.config_camera(rc)
        pt = mcpt.PathTracer(0, mcpt.default_config(spp=spp, max_depth=rc.max_depth))
        pt.upload_scene(scene)
        pt.set_camera(cam)
        W, H = rc.width, rc.height
        base = bench.BENCH_SLOTS[cid]

        def frame_ms(tiles):
            pt.set_tiles(tiles)
            pt.clear()
            t0 = time.perf_counter()
            st = pt.render()
            return (time.perf_counter() - t0) * 1e3, st.rays

        pt.set_path_slots(base)
        pt.resize(W, H, 256, 256)
        frame_ms(None)  # warmup
        t1, rays1 = frame_ms(None)
        res["runs"].append({"config": cid, "frame": [W, H], "spp": spp, "world": 1, "tile": 256, "slots": base,
                            "per_rank_ms": [round(t1, 2)], "rays": rays1, "device_used_gb": used_gb()})
        print(json.dumps(res["runs"][-1]), flush=True)
        for world in args.worlds:
            choices = []
            for tile in args.tiles:
                choices.append((tile, parallel.strong_slots(base, world, W, H, spp, tile)))
            if "base" in args.slot_choices and base != choices[-1][1]:
                choices.append((min(args.tiles), base))
            for c in args.slot_choices.split(","):  # explicit slot counts at the smallest tile
                if c.isdigit() and all(int(c) != sl for _, sl in choices):
                    choices.append((min(args.tiles), int(c)))
            for tile, slots in choices:
                # bench.py's rank layout: compact path state, film at one slot, the tiles, then the slots
                pt.set_compact_paths(True)
                pt.set_path_slots(1)
                pt.resize(W, H, tile, tile)
                ms, rays, px, mem = [], [], [], []
                for r in range(world):
                    tiles = parallel.tiles_for_rank(r, world, W, H, tile)
                    pt.set_tiles(tiles)
                    pt.set_path_slots(slots)
                    if r == 0:  # warmup: the first launches of this slot / tile layout
                        frame_ms(tiles)
                    t, ry = frame_ms(tiles)
                    ms.append(t)
                    rays.append(ry)
                    mem.append(used_gb())
                    px.append(sum(min(tile, W - tx * tile) * min(tile, H - ty * tile) for tx, ty in tiles))
                    pt.set_path_slots(1)  # the next rank's tiles are allocated at one slot first
                pt.set_compact_paths(False)
                mean = sum(ms) / len(ms)
                run = {"config": cid, "frame": [W, H], "spp": spp, "world": world, "tile": tile, "slots": slots,
                       "path_state": "compact (the rank's tiles)", "per_rank_device_used_gb": mem,
                       "per_rank_ms": [round(x, 2) for x in ms], "per_rank_pixels": px, "per_rank_rays": rays,
                       "max_over_mean": round(max(ms) / mean, 4), "ideal_ms": round(mean, 2),
                       "max_ms": round(max(ms), 2), "efficiency_vs_one_gpu": round(t1 / (world * max(ms)), 4)}
                res["runs"].append(run)
                print(json.dumps(run), flush=True)
        pt.close()
    with open(args.out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
