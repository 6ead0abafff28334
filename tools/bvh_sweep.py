"""Pipeline A/B over BVH builders: same config, same seed -> the film must be bit-identical for every
tree (hits are tree-independent); compares the per-iteration trace / shade time in steady state.
usage: python tools/bvh_sweep.py [config] [warmup] [iters]"""
import hashlib, os, sys, time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "mc-path-tracer_amd")]
import numpy as np, mcpt

cid = int(sys.argv[1]) if len(sys.argv) > 1 else 2
warm = int(sys.argv[2]) if len(sys.argv) > 2 else 30
iters = int(sys.argv[3]) if len(sys.argv) > 3 else 30
rc = mcpt.CONFIGS[cid]
variants = [dict()]
for nb in (32, 64, 128):
    for ct in (0.25, 0.5):
        for mp in (1, 8):
            variants.append(dict(builder="sah3", buckets=nb, trav_cost=ct, isect_cost=1.0, max_prims=mp))
pt = mcpt.PathTracer(0, mcpt.default_config(spp=rc.spp, max_depth=rc.max_depth))
pt.set_camera(mcpt.config_camera(rc))
ref_hash = None
for kw in variants:
    s = mcpt.Scene(); s.make_proxy(cid, mcpt.ASSET_DIR)
    t = time.time(); s.build(**kw); bt = time.time() - t
    pt.upload_scene(s)
    pt.resize(rc.width, rc.height)
    pt.iterate(warm)
    st = pt.iterate(iters)
    Ld, smp = pt.film()
    h = hashlib.md5(Ld.tobytes() + smp.tobytes()).hexdigest()[:10]
    ref_hash = ref_hash or h
    n = len(s.arrays()["nprims"])
    rays = st.extend_rays + st.shadow_rays + st.vis_rays
    print(f"{str(kw):95s} nodes {n:8d} build {bt:5.2f}s [{h}{'' if h == ref_hash else ' MISMATCH'}] "
          f"trace {st.ms_extend / iters:.4f} shade {st.ms_shade / iters:.4f} ms/iter "
          f"{rays / (st.ms_extend + st.ms_shade) / 1e3:.0f} Mray/s  ext nodes/ray {st.ext_nodes / max(1, st.extend_rays):.2f} "
          f"tests/ray {st.ext_tests / max(1, st.extend_rays):.2f} any nodes/ray {st.any_nodes / max(1, st.shadow_rays + st.vis_rays):.2f}",
          flush=True)
