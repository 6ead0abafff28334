"""bench.py -- Mray/s (extend+shade) of the MI355X wavefront path tracer on BASELINE config 2.

Workload (BASELINE.json configs[1]): 1920x1080, 256 spp, depth 5, MIS on, env importance sampling,
Cornell-box + 5 spheres proxy for the missing scene_show_off_spheres.glb lit by
night_free_Env.hdr.  A *step* is one wavefront iteration (the reference's wavefront_pathtrace,
wavefront_kernels.cu:377-442: logic+generate+material -> extend -> shadow) over every pixel the
rank owns; paths are in steady state after the warmup.  Three paths are in flight per pixel
(mcpt_set_path_slots: slot k renders samples k, k+3, ...; same per-sample results, films equal to
fp32 summation order -- tests/test_gpu.py::test_path_slots_*): 6.2 M paths per iteration amortise
each launch's ramp-up and drain (+15 % over one path per pixel, measured).  value = (extension + shadow + BRDF
visibility rays of all ranks) / (max over ranks of the timed wall time).

Multi-GPU: one process per GPU (torch.distributed.run), weak scaling: the film is 1920 x 1080*N
pixels of the same 16:9 view (the config-2 camera; N-fold vertical supersampling), and 256x256
tiles are dealt to ranks by (tx + ty) mod N, so every rank owns ~one 1080p frame of pixels with
the same image content (sky / geometry mix) as the 1-GPU run.  No collective runs inside the timed region (tiles are independent); the RCCL gather of
the film is a separate, untimed step (mcpt/parallel.py).
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "mc-path-tracer_amd"))

HBM_PEAK = 8.0e12  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
L2_PEAK = 34.5e12  # aggregate L2 bandwidth over the 8 XCDs (MI355X_MICROARCH.md, L2 section)
# SURVEY.md 8(d) algorithmic bytes per unit of work
B_EXT_STATE = 65      # extend: queue 4 + ray 24 + len 4 read, len/found/pos/n/mat 33 written
B_ANY_STATE = 33      # shadow: queue 4 + ray 24 + light id 4 read, visible 1 written
B_NODE = 32           # per BVH node box visited (a child-pair fetch visits 2)
B_TRI = 36            # per ray/triangle test
B_HIT = 40            # per closest hit: 3 normals + material id
B_SHADE = 195 + 172   # logic + material per path-bounce
B_GEN = 49            # generate per new sample


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-spp", type=int, default=12, help="spp of the full-frame CPU-oracle sample")
    ap.add_argument("--gather", action="store_true", help="RCCL-gather the film after timing (N>1)")
    ap.add_argument("--no-full-frame", action="store_true", help="skip the untimed-by-value full 256-spp frame")
    ap.add_argument("--slots", type=int, default=int(os.environ.get("MCPT_BENCH_SLOTS", "3")),
                    help="paths in flight per pixel (mcpt_set_path_slots)")
    return ap.parse_args()


def tiles_for(rank, world, W, H, tile):
    nx, ny = (W + tile - 1) // tile, (H + tile - 1) // tile
    return [(tx, ty) for ty in range(ny) for tx in range(nx) if (tx + ty) % world == rank]


KERNEL_SOURCES = ("mc-path-tracer_amd/csrc/kernels.hip", "mc-path-tracer_amd/csrc/kernels.hpp",
                  "mc-path-tracer_amd/csrc/device/mcpt_core.hpp", "mc-path-tracer_amd/csrc/runtime.cpp",
                  "mc-path-tracer_amd/csrc/host/scene.cpp", "mc-path-tracer_amd/csrc/host/proxies.cpp")


def source_hash():
    """Hash of the kernel and scene sources: stamps the PMC summaries (tools/pmc.py) so that a
    summary taken on other code is recognised as stale (the GPU box has no .git)."""
    import hashlib

    h = hashlib.sha256()
    for f in KERNEL_SOURCES:
        with open(os.path.join(REPO, f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def pmc_summary(config, slots):
    """The newest committed rocprofv3 PMC summary (profiles/pmc_*.json) and whether it was
    measured on this code (source hash) and this workload (config, path slots)."""
    files = sorted(glob.glob(os.path.join(REPO, "profiles", "pmc_*.json")))
    if not files:
        return None, "no PMC summary in profiles/"
    try:
        d = json.load(open(files[-1]))
    except Exception as e:  # noqa: BLE001
        return None, f"unreadable PMC summary: {e}"
    stamp = d.get("stamp", {})
    why = []
    if stamp.get("source_hash") != source_hash():
        why.append("kernel sources changed since it was taken")
    if stamp.get("config") != config or stamp.get("slots") != slots:
        why.append(f"taken on config {stamp.get('config')} / {stamp.get('slots')} slots")
    return d, ("; ".join(why) or None)


def pmc_traffic(summary, kernel_prefix):
    """Per-iteration HBM bytes of a stage from a PMC summary: the sum over the stage's kernels
    (each launched once per iteration) of their bytes per launch."""
    if not summary:
        return None
    got = [v.get("hbm_bytes_per_launch") for k, v in summary.get("kernels", {}).items()
           if any(k.startswith(p) or k.startswith("void " + p) for p in kernel_prefix)]
    return int(sum(got)) if got and None not in got else None


def cpu_baseline(scene_arrays, cam, W, H, spp, max_depth):
    """Oracle (scalar C port of the reference kernels) on the host cores: the full frame at a few spp."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle_py  # checker/baseline only

    threads = min(16, os.cpu_count() or 1)
    t = time.perf_counter()
    _, _, cnt = oracle_py.render(scene_arrays, cam, W, H, spp=spp, max_depth=max_depth, nthreads=threads)
    dt = time.perf_counter() - t
    rays = cnt["extend_rays"] + cnt["shadow_rays"] + cnt["vis_rays"]
    return {"value": round(rays / dt / 1e6, 3), "unit": "Mray/s", "cores": threads, "kind": "port",
            "sample": f"oracle/ (scalar C restatement of the reference kernels, -O2, literal stack traversal, "
                      f"{threads} std threads over 256x256 tiles): the full {W}x{H} frame at {spp} spp, "
                      f"{rays} rays in {dt:.1f} s"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world == 1 and os.environ.get("MCPT_BENCH_NO_TORCH") == "1":
        torch = None
    else:
        import torch

    dist = None
    # MCPT_BENCH_BACKEND=gloo + MCPT_BENCH_SHARE_GPU=1: rehearse the N-rank path on a 1-GPU box
    # (every rank on device local % ndev, host-side collectives); the driver's runs use RCCL.
    backend = os.environ.get("MCPT_BENCH_BACKEND", "nccl")
    if world > 1:
        import torch.distributed as dist

        if os.environ.get("MCPT_BENCH_SHARE_GPU") == "1":
            local = local % torch.cuda.device_count()
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    import numpy as np

    import mcpt

    rc = mcpt.CONFIGS[args.config]
    W, H = rc.width, rc.height * world
    scene = mcpt.build_config_scene(args.config)
    cam = mcpt.config_camera(rc, rc.width, rc.height)  # the 1080p view at any N (see docstring)
    pt = mcpt.PathTracer(local, mcpt.default_config(spp=rc.spp, max_depth=rc.max_depth))
    pt.upload_scene(scene)
    pt.set_camera(cam)
    pt.set_path_slots(args.slots)
    pt.resize(W, H)
    my_tiles = tiles_for(rank, world, W, H, 256)
    pt.set_tiles(my_tiles)

    pt.iterate(args.warmup)
    if dist:
        dist.barrier()
    if torch:
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    st = pt.iterate(args.steps)  # returns after its stream has drained
    if torch:
        torch.cuda.synchronize()
    if dist:
        dist.barrier()
    dt = time.perf_counter() - t0

    rays = st.rays
    # The literal workload once through, outside `value`: clear the film and render every
    # pixel the rank owns to spp completion (startup and tail iterations included).
    full = None
    if not args.no_full_frame:
        pt.clear()
        if torch:
            torch.cuda.synchronize()
        t1 = time.perf_counter()
        fs = pt.render()
        dt_full = time.perf_counter() - t1
        full = [dt_full, float(fs.rays), float(fs.iterations)]
    if dist:
        v = torch.tensor([dt, float(rays)], dtype=torch.float64, device="cuda" if backend == "nccl" else "cpu")
        mx = v.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        dist.all_reduce(v, op=dist.ReduceOp.SUM)
        dt_all, rays_all = float(mx[0]), float(v[1])
        if full:
            f = torch.tensor(full, dtype=torch.float64, device=v.device)
            fmax = f.clone()
            dist.all_reduce(fmax, op=dist.ReduceOp.MAX)
            dist.all_reduce(f, op=dist.ReduceOp.SUM)
            full = [float(fmax[0]), float(f[1]), float(fmax[2])]
    else:
        dt_all, rays_all = dt, float(rays)

    if args.gather and dist:
        from mcpt import parallel

        parallel.gather_film(pt, rank, world)

    if rank != 0:
        if dist:
            dist.barrier()
            dist.destroy_process_group()
        return

    K = args.steps
    # logical bytes per SURVEY.md 8(d): state bytes per ray/path-bounce + BVH bytes per visit
    b_ext = B_EXT_STATE * st.extend_rays + 2 * B_NODE * st.ext_nodes + B_TRI * st.ext_tests + B_HIT * st.ext_hits
    b_any = B_ANY_STATE * (st.shadow_rays + st.vis_rays) + 2 * B_NODE * st.any_nodes + B_TRI * st.any_tests
    b_shd = B_SHADE * st.shadow_rays + B_GEN * (st.extend_rays - st.shadow_rays)
    # dominant kernel by summed HIP-event time over the timed region (same stream as the kernels);
    # k_trace traces the extension (closest-hit) and any-hit rays of an iteration in one launch
    kern = {"k_trace": st.ms_extend + st.ms_shadow, "k_shade": st.ms_shade}
    names = {"k_trace": ("mcpt_dev::k_trace(", "mcpt_dev::k_trace<"), "k_shade": ("mcpt_dev::k_shade<", "mcpt_dev::k_material<")}
    dom = max(kern, key=kern.get)
    byts = b_ext + b_any if dom == "k_trace" else b_shd
    state = (B_EXT_STATE * st.extend_rays + B_ANY_STATE * (st.shadow_rays + st.vis_rays)) if dom == "k_trace" else b_shd
    per_launch = byts / K
    avg_ms = kern[dom] / K
    achieved = per_launch / (avg_ms * 1e-3)
    # measured HBM bytes per launch from the committed PMC summary, used only when it was taken
    # on this code and workload (tools/pmc.py stamps it)
    summary, stale = pmc_summary(args.config, args.slots)
    fresh = summary if stale is None else None
    traffic = pmc_traffic(fresh, names[dom])
    frac = achieved / HBM_PEAK
    roof = {"bound": "hbm", "kernel": dom, "achieved": round(achieved / 1e9, 1), "peak": HBM_PEAK / 1e9, "unit": "GB/s",
            "frac": round(frac, 4), "traffic": traffic, "avg_launch_ms": round(avg_ms, 4),
            "algorithmic_bytes_per_launch": int(per_launch),
            "state_only_frac": round(state / K / (avg_ms * 1e-3) / HBM_PEAK, 4),
            "per_ray": {"ext_pair_nodes": round(st.ext_nodes / max(1, st.extend_rays), 2),
                        "ext_tri_tests": round(st.ext_tests / max(1, st.extend_rays), 2),
                        "any_pair_nodes": round(st.any_nodes / max(1, st.shadow_rays + st.vis_rays), 2),
                        "any_tri_tests": round(st.any_tests / max(1, st.shadow_rays + st.vis_rays), 2)}}
    # What binds, from the numbers: SURVEY 8(d)'s logical bytes count every BVH node and triangle
    # fetch; above the HBM peak they can only have come from the caches (L2 / MALL)
    binding = []
    if frac > 1.0:
        binding.append(f"not HBM: the logical bytes run at {frac:.2f}x the HBM peak, so the node and triangle "
                       f"fetches are cache-served ({achieved / L2_PEAK:.2f} of the 34.5 TB/s aggregate L2 rate)")
        roof["l2_frac"] = round(achieved / L2_PEAK, 4)
    if traffic is not None:
        tf = traffic / (avg_ms * 1e-3) / HBM_PEAK
        roof["traffic_GBps"] = round(traffic / (avg_ms * 1e-3) / 1e9, 1)
        roof["traffic_frac"] = round(tf, 4)
        binding.append(f"measured HBM traffic {tf:.2f} of peak")
        if tf > 0.6:
            binding.append("HBM-bound by measured traffic")
    elif stale:
        roof["pmc_stale"] = stale
    if frac > 1.0 and (traffic is None or traffic / (avg_ms * 1e-3) / HBM_PEAK < 0.6):
        binding.append("the traversal is bound by its divergent issue / gather-latency mix (DESIGN.md section 4)")
    roof["binding"] = "; ".join(binding) if binding else "hbm"
    # the streaming stages (logic + generate + material: k_shade and k_material) on their own,
    # by SURVEY 8(d) state bytes and by the PMC traffic
    t_shd = st.ms_shade / K * 1e-3
    roof["shade_stages"] = {"ms_per_iteration": round(st.ms_shade / K, 4),
                            "state_bytes_per_iteration": int(b_shd / K),
                            "state_frac": round(b_shd / K / t_shd / HBM_PEAK, 4)}
    shd_traffic = pmc_traffic(fresh, names["k_shade"])
    if shd_traffic is not None:
        roof["shade_stages"]["traffic"] = shd_traffic
        roof["shade_stages"]["traffic_frac"] = round(shd_traffic / t_shd / HBM_PEAK, 4)
    # measured HBM ceiling on this device (hand-written dwordx4 copy) beside the spec peak
    copy = pt.hbm_copy_gbps(1 << 30, 20)
    roof["measured_copy_GBps"] = round(copy, 1)
    # whole-pipeline form: all logical bytes of both kernels over their summed time
    t_pipe = (st.ms_extend + st.ms_shadow + st.ms_shade) * 1e-3
    roof["pipeline_frac"] = round((b_ext + b_any + b_shd) / t_pipe / HBM_PEAK, 4)
    hbm_meas = [pmc_traffic(fresh, p) for p in names.values()]
    if all(h is not None for h in hbm_meas):  # measured HBM bytes per iteration (fresh PMC summary)
        roof["pipeline_hbm_frac_measured"] = round(sum(hbm_meas) * K / t_pipe / HBM_PEAK, 4)
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(scene.arrays(), cam, W, H, args.cpu_spp, rc.max_depth)
    value = rays_all / dt_all / 1e6
    out = {
        "metric": "Mray/s (extend+shade) at 1080p x256spp depth5; fraction of HBM roofline",
        "value": round(value, 2),
        "unit": "Mray/s",
        "n_gpus": world,
        "steps": K,
        "warmup": args.warmup,
        "ms_per_step": round(dt_all * 1e3 / K, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic",
        "config": {
            "workload": "BASELINE config 2: Cornell-box + 5 spheres proxy (scene_show_off_spheres.glb missing), "
                        f"night_free_Env.hdr env IS, {rc.width}x{rc.height} per GPU, {rc.spp} spp, depth {rc.max_depth}, MIS",
            "frame": [W, H],
            "tiles": "256x256, rank = (tx+ty) mod N",
            "step": "one wavefront iteration (shade+extend+shadow) over the rank's pixels x path slots, steady state",
            "rays_per_step": int(rays_all / K),
            "rays_per_step_rank0": {"extend": round(st.extend_rays / K), "shadow": round(st.shadow_rays / K),
                                    "visibility": round(st.vis_rays / K)},
            "parallelism": f"tiles{world}",
            "path_slots": args.slots,
            "device": pt.device_name,
        },
        "stage_ms_per_step": {k: round(v / K, 4) for k, v in kern.items()},
        "roofline": roof,
        "cpu_baseline": cpu,
    }
    if full:
        out["full_frame"] = {"seconds": round(full[0], 4), "rays": int(full[1]), "iterations": int(full[2]),
                             "mray_s": round(full[1] / full[0] / 1e6, 2),
                             "what": f"film cleared, every pixel rendered to {rc.spp} spp (max over ranks; host "
                                     "syncs every 32 iterations, startup and tail included)"}
    print(json.dumps(out), flush=True)
    pt.close()
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
