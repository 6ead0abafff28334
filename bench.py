"""bench.py -- Mray/s (extend+shade) of the MI355X wavefront path tracer on BASELINE config 2.

Workload (BASELINE.json configs[1]): 1920x1080, 256 spp, depth 5, MIS on, env importance sampling,
Cornell-box + 5 spheres proxy for the missing scene_show_off_spheres.glb lit by
night_free_Env.hdr.  A *step* is one whole frame, the literal workload of the metric: the film is
cleared (g_clear_dfilm, wavefront_kernels.cu:55-76) and every pixel the rank owns is rendered to
256 spp by repeated wavefront iterations (wavefront_pathtrace, wavefront_kernels.cu:377-442:
logic+generate+material -> extend -> shadow), startup and tail iterations included.  value =
(extension + shadow + BRDF visibility rays of all ranks) / (max over ranks of the timed wall time).
BENCH_SLOTS[config] paths are in flight per pixel (mcpt_set_path_slots; 24 on config 2); films equal
the one-path-per-pixel oracle's within the north star's 1e-4 (tests/test_bench_layout.py runs
this exact layout).  `--steady` reports the steady-state iteration rate beside it.

Multi-GPU: one process per GPU.  `--gpus N` without an external launcher starts
the N ranks itself (torch.distributed.run, before anything touches the GPU); under a launcher
WORLD_SIZE must equal N.  Film tiles are dealt to ranks by (tx + ty) mod N (64 x 64 tiles for
N > 1: MULTI_TILE), and every rank holds path state for its own tiles only
(mcpt_set_compact_paths).
  --scaling strong (default): `value` is the metric's own frame (1920 x 1080 for config 2; 3840 x
      2160 for --config 4) split over the ranks, path slots scaled by the rank's pixel share
      (parallel.strong_slots) so every GPU keeps the one-GPU run's paths in flight;
  --scaling weak: `value` is a 1920 x 1080*N frame of the same view (N-fold vertical
      supersampling): every rank owns ~one 1080p frame of pixels with the 1-GPU run's sky /
      geometry mix.
An N>1 run also times the other split as a sub-object ("weak" / "strong"; --no-weak / --no-strong
skip it).  After timing, the strong frame is gathered into rank 0's device film (mcpt/parallel.py:
point-to-point RCCL sends over xGMI) and rank 0 re-renders every other rank's tiles alone and
compares them with the gathered pixels bit for bit (--no-gather / --no-verify-gather skip these).
No collective runs inside a timed region: tiles are independent.
"""
from __future__ import annotations

import argparse
import glob
import re
import json
import os
import socket
import subprocess
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
# Path slots (paths in flight per pixel) per BASELINE config: the measured best of the
# whole-frame sweeps (round 3, DESIGN.md section 2: config 2 at 3/8/16/24/32 slots
# 7287/7856/8064/8095/8081 Mray/s; round 5 at the round-5 kernels, profiles/ab_r05_slots.txt:
# config 2 20/24/32 289.1/287.2/292.3 ms per frame, config 3 32/48/64 252.4/251.8/248.4 ms,
# config 4 16/24/32 5.82/5.75/5.75 s, config 5 (1024 spp) 16/24 11.85/11.72 s); the parity
# tests and smoke() run the same layout.
BENCH_SLOTS = {1: 16, 2: 24, 3: 64, 4: 24, 5: 24}
STEP = "frame"  # what one step is; stamped into the PMC summaries (tools/pmc.py)

# MCPT_* environment knobs.  Every one that is set is stamped into the bench
# line (config.knobs).  These change what is measured -- the culling, the launch geometry, the tree,
# the occluder table, the library or the rank layout -- so a run with any of them set is marked
# "not the product" (config.product = false, with the reasons); the rest only select host-side
# options that do not change a device result or a launch (build threads of the host SAH).
NON_PRODUCT_KNOBS = {
    "MCPT_CULL": "culling switched (0: no culling, the reference-order traversal)",
    "MCPT_CULL_PLANE": "axis-plane culling bound switched",
    "MCPT_TRACE_WAVES": "k_trace launch geometry (waves per CU)",
    "MCPT_TRACE_PARTS": "k_trace hand-out partitions",
    "MCPT_REFILL_MIN": "k_trace refill threshold",
    "MCPT_TRI_MIN": "k_trace triangle-phase threshold",
    "MCPT_MAT_BLOCKS_PER_CU": "k_material grid",
    "MCPT_SHADE_GRID": "k_shade grid",
    "MCPT_SHADE_WGS": "k_shade grid (absolute)",
    "MCPT_NO_BLOCK_DONE": "k_shade finished-block skip off",
    "MCPT_SIBLING_LAYOUT": "BVH sibling layout",
    "MCPT_BVH_WIDTH": "BVH node width forced",
    "MCPT_BVH_ISOLATE": "BVH isolation of unbounded triangles switched",
    "MCPT_GPU_BVH": "device-built BVH instead of the host SAH",
    "MCPT_ENV_GUIDES": "env CDF search guides switched",
    "MCPT_OCC_G": "occluder-table origin grid",
    "MCPT_OCC_B": "occluder-table direction bins",
    "MCPT_OCC_PREFILL": "occluder-table pre-fill at upload switched",
    "MCPT_WORK_COUNTERS": "counting k_trace build in the timed frames",
    "MCPT_LIB": "another libmcpt build",
    "MCPT_BENCH_SLOTS": "path slots overridden",
    "MCPT_BENCH_BACKEND": "collective backend overridden (rehearsal)",
    "MCPT_BENCH_SHARE_GPU": "ranks share one GPU (rehearsal)",
}


def knobs(environ=None):
    """Every MCPT_* variable set in the environment (they reach the library through getenv)."""
    env = os.environ if environ is None else environ
    return {k: env[k] for k in sorted(env) if k.startswith("MCPT_")}


def product_check(args, kn):
    """(product, reasons): whether the line measures the product as shipped -- no knob of
    NON_PRODUCT_KNOBS set, the config's own spp and path slots."""
    why = [f"{k}={v}: {NON_PRODUCT_KNOBS[k]}" for k, v in kn.items() if k in NON_PRODUCT_KNOBS]
    why += [f"{k}={v}: unknown knob" for k, v in kn.items() if k not in NON_PRODUCT_KNOBS and k not in NEUTRAL_KNOBS]
    if getattr(args, "spp", None):
        why.append(f"--spp {args.spp}: not the config's spp")
    if getattr(args, "slots", None) and "MCPT_BENCH_SLOTS" not in kn and args.slots != BENCH_SLOTS.get(args.config):
        why.append(f"--slots {args.slots}: not the config's path slots ({BENCH_SLOTS.get(args.config)})")
    return not why, why


NEUTRAL_KNOBS = {"MCPT_BVH_THREADS", "MCPT_DIST_TIMEOUT_S"}  # host build threads; the collectives' timeout


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5, help="timed frames")
    ap.add_argument("--warmup", type=int, default=1, help="untimed frames before the timed ones")
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--scaling", choices=("weak", "strong"), default="strong",
                    help="N>1: which split `value` reports (the other is timed as a sub-object)")
    ap.add_argument("--spp", type=int, default=None, help="override the config's spp (not the BASELINE workload)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-spp", type=int, default=12, help="spp of the full-frame CPU-oracle sample")
    ap.add_argument("--no-strong", action="store_true",
                    help="N>1 with --scaling weak: skip the strong split of the config's own frame (the sub-object)")
    ap.add_argument("--no-weak", action="store_true",
                    help="N>1 with --scaling strong: skip the weak 1920 x 1080N frame (the sub-object)")
    ap.add_argument("--no-gather", action="store_true",
                    help="N>1: skip the frame-end gather of the strong frame into rank 0's device film (RCCL)")
    ap.add_argument("--no-verify-gather", action="store_true",
                    help="N>1: skip checking the gathered frame against rank 0 rendering it alone (bit for bit)")
    ap.add_argument("--no-work-counters", action="store_true",
                    help="skip rank 0's extra untimed frame with the counting k_trace build (the roofline's per-ray "
                         "node / triangle figures are then absent); the rocprofv3 passes use it")
    ap.add_argument("--steady", action="store_true",
                    help="also time 60 steady-state iterations (outside value; off by default so that every "
                         "k_trace launch of the process belongs to a timed or warmup frame, as rocprofv3 sees it)")
    ap.add_argument("--slots", type=int, default=int(os.environ["MCPT_BENCH_SLOTS"]) if "MCPT_BENCH_SLOTS" in os.environ else None,
                    help="paths in flight per pixel (mcpt_set_path_slots); default BENCH_SLOTS[config]")
    return ap.parse_args(argv)


# Film tile of the multi-GPU partition.  The rank of tile (tx, ty) is (tx + ty) mod N; with the
# reference's 256 x 256 tiles (Film.cu:17) a 1080p frame is 8 x 5 tiles, and at N = 8 each rank's
# five tiles form one diagonal: the slowest partition took 1.74x the mean (one GPU timing each
# partition alone, profiles/partition_r04.json).  64 x 64 tiles (510 of them) give 1.03 at N = 8,
# 1.006 at N = 4.  Results do not depend on the tiling (keyed RNG); one rank keeps 256.
MULTI_TILE = 64


def part_tile(world):
    return 256 if world == 1 else MULTI_TILE


def tiles_for(rank, world, W, H, tile):
    nx, ny = (W + tile - 1) // tile, (H + tile - 1) // tile
    return [(tx, ty) for ty in range(ny) for tx in range(nx) if (tx + ty) % world == rank]


def frame_size(rc, world, scaling):
    """The rendered frame: the config's view, N-fold taller under weak scaling."""
    return (rc.width, rc.height * world) if scaling == "weak" else (rc.width, rc.height)


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


def stamp_spp(config, args_text):
    """The spp a profiled bench command ran at: its --spp, else the config's."""
    m = __import__("re").search(r"--spp[ =](\d+)", args_text or "")
    if m:
        return int(m.group(1))
    import mcpt

    return mcpt.CONFIGS[config].spp


def pmc_summary(config, slots, kind="pmc", spp=None):
    """The newest committed rocprofv3 summary of this config (kind "pmc": FETCH/WRITE traffic,
    "pmcdetail": SQ/TCC counters; profiles/<kind>_rNN.json for config 2, <kind>_c<config>_rNN.json
    for the others) and whether it was measured on this code (source hash) and this workload
    (config, path slots, step, spp: a launch's traffic depends on the spp through the path mix)."""
    pre = f"{kind}_r" if config == 2 else f"{kind}_c{config}_r"
    # <kind>_rNN.json only: variant summaries (<kind>_rNNoccoff.json: a knob set) are not the product's
    files = sorted(f for f in glob.glob(os.path.join(REPO, "profiles", f"{pre}*.json"))
                   if re.fullmatch(r"\d+\.json", os.path.basename(f)[len(pre):]))
    if not files:
        return None, f"no {kind} summary in profiles/"
    try:
        d = json.load(open(files[-1]))
    except Exception as e:  # noqa: BLE001
        return None, f"unreadable {kind} summary: {e}"
    stamp = d.get("stamp", {})
    why = []
    if stamp.get("source_hash") != source_hash():
        why.append("kernel sources changed since it was taken")
    if stamp.get("config") != config or stamp.get("slots") != slots:
        why.append(f"taken on config {stamp.get('config')} / {stamp.get('slots')} slots")
    if stamp.get("step", "iteration") != STEP:
        why.append(f"taken with {stamp.get('step', 'iteration')} steps")
    if spp is not None and "spp" in stamp and stamp["spp"] != spp:
        why.append(f"taken at {stamp['spp']} spp")
    judged = lambda k: {x: v for x, v in k.items() if x not in NEUTRAL_KNOBS}  # noqa: E731
    if "knobs" in stamp and judged(stamp["knobs"]) != judged(knobs()):
        why.append(f"taken with knobs {judged(stamp['knobs'])}")
    return d, ("; ".join(why) or None)


def _timed_kernel(name, kernel_prefix):
    """A summary entry of one of the timed frames' kernels: the prefix matches, and it is not
    k_trace's work-counting instantiation (k_trace<W, S, true>, launched only in the extra
    counting frame)."""
    hit = any(name.startswith(p) or name.startswith("void " + p) for p in kernel_prefix)
    return hit and not (name.split("(")[0].endswith(", true>") and "k_trace<" in name)


def pmc_traffic(summary, kernel_prefix):
    """Per-iteration HBM bytes of a stage from a PMC summary: the sum over the stage's kernels
    (each launched once per iteration) of their bytes per launch."""
    if not summary:
        return None
    got = [v.get("hbm_bytes_per_launch") for k, v in summary.get("kernels", {}).items() if _timed_kernel(k, kernel_prefix)]
    return int(sum(got)) if got and None not in got else None


def pmc_detail(summary, kernel_prefix):
    """Counter ratios of one kernel from a fresh pmcdetail summary (tools/pmc_detail.py)."""
    if not summary:
        return None
    for k, v in summary.get("kernels", {}).items():
        if _timed_kernel(k, kernel_prefix):
            return v.get("ratios")
    return None


def cpu_threads():
    """Host threads for the CPU baseline: the cores this process may run on, capped at the GPU
    box's per-GPU CPU share (OMP_NUM_THREADS, 16 there; os.cpu_count() shows the whole host)."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    share = os.environ.get("OMP_NUM_THREADS")
    if share and share.isdigit() and int(share) > 0:
        n = min(n, int(share))
    return max(1, n)


def cpu_baseline(scene_arrays, cam, W, H, spp, max_depth):
    """Oracle (scalar C port of the reference kernels) on the host cores: the full frame at a few spp."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle_py  # checker/baseline only

    threads = cpu_threads()
    t = time.perf_counter()
    _, _, cnt = oracle_py.render(scene_arrays, cam, W, H, spp=spp, max_depth=max_depth, nthreads=threads)
    dt = time.perf_counter() - t
    rays = cnt["extend_rays"] + cnt["shadow_rays"] + cnt["vis_rays"]
    return {"value": round(rays / dt / 1e6, 3), "unit": "Mray/s", "cores": threads, "kind": "port",
            "host_cpus": os.cpu_count(),
            "sample": f"oracle/ (scalar C restatement of the reference kernels, -O2, literal stack traversal, "
                      f"{threads} std threads over 256x256 tiles = every core this process may use, capped at "
                      f"the box's per-GPU share OMP_NUM_THREADS; host has {os.cpu_count()} CPUs): the full "
                      f"{W}x{H} frame at {spp} spp, {rays} rays in {dt:.1f} s"}


def spawn_ranks(args):
    """`--gpus N` without a launcher: start N ranks with torch.distributed.run as a child process
    (nothing has touched the GPU yet) and exit with its status."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.run(cmd, env=env).returncode


class Acc:
    """Sum of StageStats over frames."""
    KEYS = ("extend_rays", "shadow_rays", "vis_rays", "iterations", "ms_shade", "ms_extend",
            "ext_nodes", "ext_tests", "ext_hits", "any_nodes", "any_tests", "any_hits")

    RAYS = ("extension", "extension_traversed", "any_hit", "any_hit_traversed", "any_hit_occluder_cache")

    def __init__(self):
        for k in self.KEYS:
            setattr(self, k, 0)
        self.occ = 0  # any-hit rays the occluder cache resolved in k_material (not traced by k_trace)
        self.counts = dict.fromkeys(self.RAYS, 0)  # mcpt_debug_ray_counts, summed over frames

    def add(self, st):
        for k in self.KEYS:
            setattr(self, k, getattr(self, k) + getattr(st, k))

    @property
    def rays(self):
        return int(self.extend_rays + self.shadow_rays + self.vis_rays)


def roofline(st, ms_trace, ms_shade, config, slots, work=None, spp=None):
    """roofline object of the dominant kernel (k_trace) and of the shading stages.

    achieved = SURVEY.md 8(d)'s algorithmic bytes that live in HBM: the per-ray state (65 B per
    extension ray, 33 B per any-hit ray) times the rays of a launch, over the launch time.  The
    traversal's node and triangle bytes (8(d)'s B_bvh) are reported separately as cache-served
    bytes: they run at several times the HBM peak, so they come from L1 / L2 / MALL (their own
    roof is the L2's).  traffic = measured HBM bytes per launch from the committed rocprofv3 PMC
    summary (profiles/pmc_r*.json) when it was taken on this code and workload.  bound = the
    resource with the highest measured utilisation (HBM traffic, L2 bytes, VALU issue), or
    "latency" when none reaches 0.5.  work: the traversal work counters (node steps, triangle
    tests, hits) of one extra, untimed frame rendered with mcpt_set_work_counters on (the counting
    k_trace build is slower, so the timed frames run without it); st's own counters otherwise."""
    n = max(1, st.iterations)
    w = work if work is not None else st
    wn = max(1, w.iterations)
    w_occ = getattr(w, "occ", 0)
    w_ext, w_any = w.extend_rays, w.shadow_rays + w.vis_rays - w_occ
    avg_s = ms_trace / n * 1e-3
    ext_q = st.extend_rays
    any_all = st.shadow_rays + st.vis_rays
    occ = getattr(st, "occ", 0)
    any_q = any_all - occ  # any-hit rays k_trace traced (the occluder cache resolved the rest)
    state = (B_EXT_STATE * ext_q + B_ANY_STATE * any_q) / n
    bvh = (2 * B_NODE * (w.ext_nodes + w.any_nodes) + B_TRI * (w.ext_tests + w.any_tests) + B_HIT * w.ext_hits) / wn
    achieved = state / avg_s if avg_s > 0 else 0.0
    names = {"k_trace": ("mcpt_dev::k_trace<",), "shade": ("mcpt_dev::k_shade<", "mcpt_dev::k_material<")}
    summary, stale = pmc_summary(config, slots, spp=spp)
    fresh = summary if stale is None else None
    detail, dstale = pmc_summary(config, slots, "pmcdetail", spp=spp)
    dfresh = detail if dstale is None else None
    traffic = pmc_traffic(fresh, names["k_trace"])
    roof = {"bound": None, "kernel": "k_trace", "achieved": round(achieved / 1e9, 1), "peak": HBM_PEAK / 1e9,
            "unit": "GB/s", "frac": round(achieved / HBM_PEAK, 4), "traffic": traffic,
            "avg_launch_ms": round(ms_trace / n, 4), "launches": int(n),
            "algorithmic_bytes_per_launch": int(state),
            "algorithmic": "SURVEY 8(d) per-ray state bytes (65 B extension, 33 B any-hit) x rays per launch",
            "cache_served": {"bytes_per_launch": int(bvh), "GBps": round(bvh / avg_s / 1e9, 1) if avg_s > 0 else 0.0,
                             "l2_peak_GBps": L2_PEAK / 1e9, "l2_frac": round(bvh / avg_s / L2_PEAK, 4) if avg_s > 0 else 0.0,
                             "what": "SURVEY 8(d) B_bvh: 64 B per child-pair node step, 36 B per triangle "
                                     "test, 40 B per closest hit (logical; served by L1/L2/MALL)"},
            "per_ray": {"ext_pair_nodes": round(w.ext_nodes / max(1, w_ext), 2),
                        "ext_tri_tests": round(w.ext_tests / max(1, w_ext), 2),
                        "any_pair_nodes": round(w.any_nodes / max(1, w_any), 2),
                        "any_tri_tests": round(w.any_tests / max(1, w_any), 2),
                        "any_resolved_by_occluder_cache": round(occ / max(1, any_all), 4),
                        "counted_on": "one extra untimed frame, counting k_trace build" if work is not None
                                      else "the timed frames"}}
    util = {"l2": roof["cache_served"]["l2_frac"]}
    if traffic is not None and avg_s > 0:
        roof["traffic_GBps"] = round(traffic / avg_s / 1e9, 1)
        roof["traffic_frac"] = round(traffic / avg_s / HBM_PEAK, 4)
        util["hbm"] = roof["traffic_frac"]
    else:
        roof["pmc_stale"] = stale
        util["hbm"] = roof["frac"]
    r = with_valu_useful(pmc_detail(dfresh, names["k_trace"]))
    if r:
        roof["counters"] = r
        if "valu_useful" in r:
            util["valu"] = r["valu_useful"]
    elif dstale:
        roof["counters_stale"] = dstale
    roof["utilisation"] = util
    top = max(util, key=util.get)
    roof["bound"] = top if util[top] >= 0.5 else "latency"
    why = [f"{k} {v:.2f}" for k, v in sorted(util.items(), key=lambda kv: -kv[1])]
    roof["binding"] = (f"utilisation {', '.join(why)}" +
                       (f" (valu: busy {r['valu_busy']:.2f} x lane utilisation {r['lane_util']:.2f})"
                        if r and "valu_useful" in r else "") +
                       (f"; waves wait on memory {r['wait_frac']:.2f} of their cycles" if r and "wait_frac" in r else ""))
    # the streaming stages (logic + generate + material: k_shade and k_material) on their own
    t_shd = ms_shade / n * 1e-3
    b_shd = (B_SHADE * st.shadow_rays + B_GEN * max(0, st.extend_rays - st.shadow_rays)) / n
    shade = {"ms_per_iteration": round(ms_shade / n, 4), "state_bytes_per_iteration": int(b_shd),
             "state_frac": round(b_shd / t_shd / HBM_PEAK, 4) if t_shd > 0 else None}
    shd_traffic = pmc_traffic(fresh, names["shade"])
    if shd_traffic is not None and t_shd > 0:
        shade["traffic"] = shd_traffic
        shade["traffic_frac"] = round(shd_traffic / t_shd / HBM_PEAK, 4)
    per = {k: with_valu_useful(pmc_detail(dfresh, (p,))) for k, p in (("k_shade", "mcpt_dev::k_shade<"),
                                                                       ("k_material", "mcpt_dev::k_material<"))}
    per = {k: v for k, v in per.items() if v}
    if per:
        shade["counters"] = per
    roof["shade_stages"] = shade
    return roof


def with_valu_useful(r):
    """Counter ratios with valu_useful = valu_busy x lane_util: the share of the VALU's lane-cycles
    doing a lane's work (busy alone counts an instruction with most lanes masked off as busy)."""
    if not r:
        return r
    r = dict(r)
    if "valu_busy" in r and "lane_util" in r:
        r["valu_useful"] = round(r["valu_busy"] * r["lane_util"], 4)
    return r


def trace_phases(work):
    """k_trace's lane utilisation split by loop phase, from the counting frame's phase counts
    (mcpt_debug_trace_profile): node phase = node steps / (64 x node-phase wave iterations),
    triangle phase = triangle tests / (64 x triangle phases), and the lanes idle / parked at a
    trip's start (after the refill)."""
    ph = getattr(work, "phases", None) if work is not None else None
    if not ph or not ph.get("trips"):
        return None
    trips = ph["trips"]
    node_steps = work.ext_nodes + work.any_nodes
    return {"node_phase_lane_util": round(node_steps / max(1, 64 * ph["node_iters"]), 4),
            "tri_phase_lane_util": round(ph["tri_lanes"] / max(1, 64 * ph["tri_phases"]), 4),
            "node_iters_per_trip": round(ph["node_iters"] / trips, 3),
            "tri_phases_per_trip": round(ph["tri_phases"] / trips, 4),
            "refills_per_trip": round(ph["refills"] / trips, 4),
            "lanes_refilled_per_refill": round(ph["refill_lanes"] / max(1, ph["refills"]), 2),
            "trip_start_lanes": {"node_work": round(ph["trip_node_lanes"] / (64 * trips), 4),
                                 "parked_leaf": round(ph["trip_leaf_lanes"] / (64 * trips), 4),
                                 "idle": round(ph["trip_idle_lanes"] / (64 * trips), 4)},
            "counts": ph,
            "what": "counting k_trace build, one untimed frame: wave iterations of the node-phase loop (per trip "
                    "the busiest lane's steps) and triangle phases, with the lanes doing work in each"}


def extend_shade(st, frame_s, steps, config, slots, spp=None):
    """The metric's own roofline fraction: the whole wavefront step (extend + shade: k_shade,
    k_material, k_trace) against 8 TB/s, per frame.  state: SURVEY.md 8(d)'s algorithmic bytes
    (465 B per path-bounce split as logic+material 367 per continuing path-bounce, extend 65 per
    extension ray, shadow 33 per any-hit ray, generate 49 per new sample); traffic: the committed
    PMC summary's HBM bytes per launch of each kernel x launches per frame (when its stamp matches
    this code and workload)."""
    K = max(1, steps)
    it = st.iterations / K
    gen = max(0, st.extend_rays - st.shadow_rays)
    state = (B_SHADE * st.shadow_rays + B_GEN * gen + B_EXT_STATE * st.extend_rays +
             B_ANY_STATE * (st.shadow_rays + st.vis_rays)) / K
    out = {"frame_s": round(frame_s, 5), "iterations_per_frame": round(it, 1),
           "state_bytes_per_frame": int(state), "state_GBps": round(state / frame_s / 1e9, 1),
           "state_frac": round(state / frame_s / HBM_PEAK, 4)}
    summary, stale = pmc_summary(config, slots, spp=spp)
    if stale is None:
        per = [pmc_traffic(summary, (p,)) for p in ("mcpt_dev::k_trace<", "mcpt_dev::k_shade<", "mcpt_dev::k_material<")]
        if None not in per:
            traffic = sum(per) * it
            out.update({"traffic_bytes_per_frame": int(traffic), "traffic_GBps": round(traffic / frame_s / 1e9, 1),
                        "traffic_frac": round(traffic / frame_s / HBM_PEAK, 4),
                        "traffic_per_kernel_per_launch": dict(zip(("k_trace", "k_shade", "k_material"), per))})
    else:
        out["pmc_stale"] = stale
    return out


def dev_of(backend):
    return "cuda" if backend == "nccl" else "cpu"


def timed_frames(pt, steps, warmup, dist, torch):
    """warmup untimed frames, then `steps` frames timed between barrier + synchronize on both
    sides.  A frame: the film cleared and every pixel of the rank's tile set rendered to spp."""
    for _ in range(warmup):
        pt.clear()
        pt.render()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    st = Acc()
    for _ in range(steps):
        pt.clear()
        st.add(pt.render())  # returns after its stream has drained
        st.occ += pt.occ_stats()[0]  # host copies of the frame's counters (no device call)
        for k, v in pt.ray_counts().items():
            st.counts[k] += v
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    return time.perf_counter() - t0, st


def rank_times(dist, dev, dt, rays, world, torch):
    """Every rank's (seconds, rays) of its timed frames, on every rank (all_gather)."""
    mine = torch.tensor([dt, float(rays)], dtype=torch.float64, device=dev)
    allr = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(allr, mine)
    t = [float(a[0]) for a in allr]
    r = [float(a[1]) for a in allr]
    mean = sum(t) / len(t)
    return {"seconds": [round(x, 4) for x in t], "mray_s": [round(b / a / 1e6, 1) for a, b in zip(t, r)],
            "max_over_mean": round(max(t) / mean, 4) if mean > 0 else None}


def set_layout(pt, rc, rank, world, kind, spp, args):
    """Film, tile set and path slots of one split.  kind "strong": the config's own frame over the
    ranks, slots scaled by the rank's pixel share (parallel.strong_slots); "weak": 1920 x 1080N at the
    base slots.  N > 1: compact path state (the rank's tiles only, mcpt_set_compact_paths), allocated
    film first (one slot), then the tile set, then the slots -- never slots x the whole frame."""
    from mcpt import parallel

    W, H = frame_size(rc, world, kind)
    tile = part_tile(world)
    base = args.slots or BENCH_SLOTS[args.config]
    slots = parallel.strong_slots(base, world, W, H, spp, tile) if kind == "strong" else base
    tiles = tiles_for(rank, world, W, H, tile)
    if world == 1:
        pt.set_path_slots(slots)
        pt.resize(W, H, tile, tile)
        pt.set_tiles(tiles)
    else:
        pt.set_compact_paths(True)
        pt.set_path_slots(1)
        pt.resize(W, H, tile, tile)
        pt.set_tiles(tiles)
        pt.set_path_slots(slots)
    return {"frame": [W, H], "tile": tile, "slots": slots, "tiles": tiles,
            "path_pixels_rank": len(tiles) * tile * tile if world > 1 else W * H}


def run_split(pt, rc, rank, world, dist, backend, kind, spp, args, torch):
    """One split timed (warmup + steps frames): its layout, the rank's own timing, every rank's
    (seconds, Mray/s) and the job's value (all ranks' rays / the max-over-ranks time)."""
    lay = set_layout(pt, rc, rank, world, kind, spp, args)
    dt, st = timed_frames(pt, args.steps, args.warmup, dist, torch)
    out = {"kind": kind, "layout": lay, "dt": dt, "st": st, "dt_all": dt, "rays_all": float(st.rays), "per_rank": None}
    if dist:
        per = rank_times(dist, dev_of(backend), dt, st.rays, world, torch)
        out["per_rank"] = per
        out["dt_all"] = max(per["seconds"])
        out["rays_all"] = sum(b * a * 1e6 for a, b in zip(per["seconds"], per["mray_s"]))
    return out


def split_summary(run, args, world):
    """The JSON sub-object of a split that is not the headline."""
    lay = run["layout"]
    return {"frame": lay["frame"], "slots": lay["slots"], "spp": run["spp"], "steps": args.steps,
            "ms_per_frame": round(run["dt_all"] * 1e3 / args.steps, 3),
            "mray_s": round(run["rays_all"] / run["dt_all"] / 1e6, 2), "per_rank": run["per_rank"],
            "tile": lay["tile"], "path_pixels_per_rank": lay["path_pixels_rank"],
            "tiles_per_rank": [len(tiles_for(r, world, lay["frame"][0], lay["frame"][1], lay["tile"]))
                               for r in range(world)]}


def gather_and_verify(pt, rc, rank, world, dist, spp, args, torch):
    """The strong frame's frame-end gather into rank 0's device film (point-to-point sends over
    RCCL / xGMI), outside any timed region, and its check: rank 0 re-renders every other rank's
    tiles alone (same path slots, so the same summation order) and compares them with the gathered
    pixels bit for bit.  The film must hold the strong layout (set_layout)."""
    import numpy as np

    from mcpt import parallel

    W, H = rc.width, rc.height
    tile = part_tile(world)
    out = {}
    pt.clear()
    pt.render()  # the film the gather moves: one whole strong frame
    torch.cuda.synchronize()
    dist.barrier()
    tg = time.perf_counter()
    parallel.gather_film_to_root(pt, rank, world, tile)
    torch.cuda.synchronize()
    out["gather_s"] = round(time.perf_counter() - tg, 4)
    out["gather_backend"] = dist.get_backend()
    if not args.no_verify_gather and rank == 0:
        Lg, sg = pt.film()  # the gathered frame
        ok, covered = True, 0
        for r in range(world):
            tr = tiles_for(r, world, W, H, tile)
            if not tr:
                continue
            if r:
                pt.set_tiles(tr)  # compact: re-allocates for rank r's tiles and clears the film
                pt.render()
            Lr, sr = pt.film() if r else (Lg, sg)
            m = np.zeros((H, W), bool)
            for tx, ty in tr:
                m[ty * tile:(ty + 1) * tile, tx * tile:(tx + 1) * tile] = True
            ok = ok and bool(np.array_equal(Lg[m].view(np.uint32), Lr[m].view(np.uint32)) and np.array_equal(sg[m], sr[m]))
            covered += int(m.sum())
        out["gather_equals_rerendered_tiles"] = bool(ok and covered == W * H and int(sg.sum()) > 0)
        out["verify"] = "rank 0 re-rendered every other rank's tiles alone; gathered pixels equal bit for bit"
    dist.barrier()
    return out


def make_tracer(local, args, rc, spp):
    """The product path tracer on device `local` with the config's scene and camera."""
    import mcpt

    scene = mcpt.build_config_scene(args.config)
    cam = mcpt.config_camera(rc, rc.width, rc.height)  # the config's view at any N (see docstring)
    pt = mcpt.PathTracer(local, mcpt.default_config(spp=spp, max_depth=rc.max_depth))
    # MCPT_GPU_BVH=ploc|lbvh: the device-built tree (A/B of tree quality; films do not depend on the tree)
    pt.upload_scene(scene, gpu_bvh=os.environ.get("MCPT_GPU_BVH") or False)
    pt.set_camera(cam)
    return pt, scene, cam


def dist_timeout_s():
    """Timeout of every collective of an N > 1 run (MCPT_DIST_TIMEOUT_S, default 600 s): a rank that
    fails or stalls in a step after the timed frames makes the others' collectives raise instead
    of hanging, so rank 0 still prints the headline line."""
    return float(os.environ.get("MCPT_DIST_TIMEOUT_S", "600"))


def guarded(fn, *a, **kw):
    """fn's result and None, or None and the error text: a step after the headline's timed frames
    (the gather, its check, the other split) must not take the already-measured line with it."""
    try:
        return fn(*a, **kw), None
    except Exception as e:  # noqa: BLE001
        return None, f"{type(e).__name__}: {e}"[:600]


def agree(dist, dev, ok, torch):
    """Every rank's verdict on the step just run (a MIN all-reduce of the ok flags); False on any
    rank that failed, and wherever the collective itself fails or times out."""
    try:
        t = torch.tensor([1.0 if ok else 0.0], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        return bool(float(t[0]) > 0.5)
    except Exception:  # noqa: BLE001
        return False


def main(argv=None, tracer=make_tracer, torch_mod=None):
    """tracer(local, args, rc, spp) -> (pt, scene, cam) and torch_mod are test seams: the gloo tests
    run the multi-rank flow on the CPU with a stand-in tracer (tests/test_bench_robust.py)."""
    args = parse(argv)
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(spawn_ranks(args))
    world = int(env_world or "1")
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: launch one rank per GPU "
              f"(or run without a launcher and let --gpus start the ranks)", file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if torch_mod is None:
        import torch
    else:
        torch = torch_mod

    dist = None
    # MCPT_BENCH_BACKEND=gloo + MCPT_BENCH_SHARE_GPU=1: rehearse the N-rank path on a 1-GPU box
    # (every rank on device local % ndev, host-side collectives); the driver's runs use RCCL.
    backend = os.environ.get("MCPT_BENCH_BACKEND", "nccl")
    if world > 1:
        import datetime

        import torch.distributed as dist

        if os.environ.get("MCPT_BENCH_SHARE_GPU") == "1":
            local = local % torch.cuda.device_count()
        torch.cuda.set_device(local)
        timeout = datetime.timedelta(seconds=dist_timeout_s())
        if backend == "nccl":
            # a timed-out RCCL collective raises in the waiting call (instead of the watchdog
            # aborting the process), so guarded() can record it and rank 0 still prints its line
            os.environ.setdefault("TORCH_NCCL_BLOCKING_WAIT", "1")
            dist.init_process_group("nccl", device_id=torch.device("cuda", local), timeout=timeout)
        else:
            dist.init_process_group(backend, timeout=timeout)

    import mcpt

    rc = mcpt.CONFIGS[args.config]
    spp = args.spp or rc.spp
    pt, scene, cam = tracer(local, args, rc, spp)

    # the headline split (value); N = 1: the config's frame on one GPU (both splits are that frame)
    head = run_split(pt, rc, rank, world, dist, backend, args.scaling, spp, args, torch)
    head["spp"] = spp
    dt, st = head["dt"], head["st"]
    dt_all, rays_all = head["dt_all"], head["rays_all"]
    slots, W, H, tile = head["layout"]["slots"], head["layout"]["frame"][0], head["layout"]["frame"][1], head["layout"]["tile"]

    # steady state (outside `value`): iterations with every pixel's paths in flight
    steady = None
    if args.steady:
        pt.clear()
        pt.iterate(30)
        t1 = time.perf_counter()
        ss = pt.iterate(60)
        steady = [time.perf_counter() - t1, float(ss.rays), float(ss.ms_extend), float(ss.ms_shade)]
        if dist:
            f = torch.tensor(steady, dtype=torch.float64, device=dev_of(backend))
            fmax = f.clone()
            dist.all_reduce(fmax, op=dist.ReduceOp.MAX)
            dist.all_reduce(f, op=dist.ReduceOp.SUM)
            steady = [float(fmax[0]), float(f[1]), float(steady[2]), float(steady[3])]

    # traversal work counters (node steps, triangle tests, hits) from one more, untimed frame with
    # the counting k_trace build (mcpt_set_work_counters): they feed the roofline's per-ray figures.
    # --no-work-counters skips it (rocprofv3 passes: every launch then belongs to a timed or warmup frame)
    work = None
    if rank == 0 and not args.no_work_counters:
        pt.set_work_counters(True)
        pt.clear()
        work = Acc()
        work.add(pt.render())
        work.occ = pt.occ_stats()[0]
        work.phases = pt.trace_profile()
        pt.set_work_counters(False)
    per_rank = head["per_rank"]
    # The steps after the headline's timed frames (the gather and its check, the other split) run
    # guarded: an error on any rank lands in the line's gather.error / <split>.error, every rank
    # agrees on it before the next step (which is then skipped), and rank 0 prints the line anyway.
    gather = None
    extras_ok = True
    dev = dev_of(backend)
    if dist and args.scaling == "strong" and not args.no_gather:
        gather, err = guarded(gather_and_verify, pt, rc, rank, world, dist, spp, args, torch)
        extras_ok = agree(dist, dev, err is None, torch)
        if err or not extras_ok:
            gather = {"error": err or "failed on another rank"}
    other = None
    other_kind = "weak" if args.scaling == "strong" else "strong"
    skip_other = args.no_weak if other_kind == "weak" else args.no_strong
    if dist and not skip_other:
        if not extras_ok:
            other = {"error": "skipped: the gather failed"}
        else:
            orun, err = guarded(run_split, pt, rc, rank, world, dist, backend, other_kind, spp, args, torch)
            extras_ok = agree(dist, dev, err is None, torch)
            if err or not extras_ok:
                other = {"error": err or "failed on another rank"}
            else:
                orun["spp"] = spp
                other = split_summary(orun, args, world)
                if other_kind == "strong" and not args.no_gather:
                    g, err = guarded(gather_and_verify, pt, rc, rank, world, dist, spp, args, torch)
                    extras_ok = agree(dist, dev, err is None, torch)
                    other.update(g if err is None and extras_ok else {"gather_error": err or "failed on another rank"})

    if rank != 0:
        if dist:
            finish_dist(dist)
        return

    K = args.steps
    roof = roofline(st, st.ms_extend, st.ms_shade, args.config, slots, work, spp=spp)
    roof["extend_shade"] = extend_shade(st, dt_all / K, K, args.config, slots, spp=spp)
    tp = trace_phases(work)
    if tp:
        roof["k_trace_phases"] = tp
    roof["measured_copy_GBps"] = round(pt.hbm_copy_gbps(1 << 30, 20), 1)  # one-pass dwordx4 copy ceiling
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(scene.arrays(), cam, W, H, args.cpu_spp, rc.max_depth)
    value = rays_all / dt_all / 1e6
    kn = knobs()
    prod, not_prod = product_check(args, kn)
    names = {2: "Cornell-box + 5 spheres proxy (scene_show_off_spheres.glb missing), night_free_Env.hdr",
             3: "deep-BVH proxy, 871,416 tris (scene_show_off_dragon.glb missing), night_free_Env.hdr",
             4: "Suzanne x2 Loop-subdivided, 251,904 tris (scene_show_off_head.glb missing), HDR_029",
             5: "2 M-tri displaced-icosphere proxy (greek_sculpture.glb missing), night_free_Env.hdr",
             1: "sphere.glb, HDR_029"}
    out = {
        "metric": "Mray/s (extend+shade) at 1080p x256spp depth5; fraction of HBM roofline",
        "value": round(value, 2),
        "unit": "Mray/s",
        "n_gpus": world,
        "steps": K,
        "warmup": args.warmup,
        "ms_per_step": round(dt_all * 1e3 / K, 3),
        "higher_is_better": True,
        "scaling": args.scaling,
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic",
        "config": {
            "workload": f"BASELINE config {args.config}: {names[args.config]}, env IS, "
                        f"{W}x{H} frame, {spp} spp, depth {rc.max_depth}, MIS"
                        + (" (spp overridden: not the BASELINE workload)" if args.spp else ""),
            "frame": [W, H],
            "spp": spp,
            "tiles": f"{tile}x{tile}, rank = (tx+ty) mod N",
            "split": ("one GPU: the config's frame" if world == 1 else
                      f"{args.scaling}: " + ("the config's own frame split over the ranks (the metric's frame)"
                                             if args.scaling == "strong" else
                                             f"a {W}x{H} frame (1080p per rank, N-fold vertical supersampling)")),
            "path_state": ("full frame" if world == 1 else
                           f"compact: the rank's tiles only, {head['layout']['path_pixels_rank']} pixels x {slots} slots"),
            "step": "one whole frame: film cleared, every pixel the rank owns rendered to spp "
                    "(all wavefront iterations: shade + extend + shadow)",
            "rays_per_step": int(rays_all / K),
            "rays_traversed_per_step_rank0": {
                "extension": int(st.counts["extension_traversed"] / K),
                "extension_resolved_in_place": int((st.counts["extension"] - st.counts["extension_traversed"]) / K),
                "any_hit": int(st.counts["any_hit_traversed"] / K),
                "any_hit_resolved_in_place": int((st.counts["any_hit"] - st.counts["any_hit_traversed"] -
                                                  st.counts["any_hit_occluder_cache"]) / K),
                "any_hit_occluder_cache": int(st.counts["any_hit_occluder_cache"] / K),
                "what": "rays k_trace traversed; the rest of rays_per_step were resolved where they were made "
                        "(NaN / zero direction or a root-box miss; an any-hit ray occluded by its cell's cached "
                        "triangle): counted as rays, as the reference traces them",
                "mray_s_traversed": round((st.counts["extension_traversed"] + st.counts["any_hit_traversed"]) /
                                          dt / 1e6, 2)},
            "rays_per_step_rank0": {"extension": int(st.extend_rays / K), "shadow": int(st.shadow_rays / K),
                                    "visibility": int(st.vis_rays / K)},
            "iterations_per_step_rank0": round(st.iterations / K, 1),
            "parallelism": f"tiles{world}",
            "path_slots": slots,
            "occluder_cache": pt.occ_stats()[1],  # any-hit occluder cache: same results
            "device": pt.device_name,
            "knobs": kn,  # every MCPT_* variable set (see NON_PRODUCT_KNOBS)
            "product": prod,
        },
        "stage_ms_per_step": {"k_trace": round(st.ms_extend / K, 3), "k_shade+k_material": round(st.ms_shade / K, 3)},
        "roofline": roof,
        "cpu_baseline": cpu,
    }
    if not prod:
        out["config"]["not_product"] = not_prod
        out["config"]["workload"] += " [NOT THE PRODUCT: " + "; ".join(not_prod) + "]"
    if steady:
        out["steady_state"] = {"mray_s": round(steady[1] / steady[0] / 1e6, 2),
                               "ms_per_iteration": round(steady[0] * 1e3 / 60, 4),
                               "k_trace_ms": round(steady[2] / 60, 4), "shade_ms": round(steady[3] / 60, 4),
                               "what": "60 wavefront iterations after 30, every pixel's path slots in flight "
                                       "(rank 0's kernel times; rays and time over all ranks)"}
    if per_rank:
        out["per_rank"] = per_rank
    if gather:
        out["gather"] = gather
    if other:
        out[other_kind] = other
    print(json.dumps(out), flush=True)
    pt.close()
    if dist:
        finish_dist(dist)


def finish_dist(dist):
    """Final barrier and teardown; after a failed step either may raise (the line is printed)."""
    try:
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        print(f"bench.py: process group teardown: {type(e).__name__}: {e}", file=sys.stderr)


if __name__ == "__main__":
    main()
