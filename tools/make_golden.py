"""Generate tests/golden/ fixtures from the CPU oracle (oracle/).

The reference itself cannot be built or run here: its kernels need CUDA 11.8,
MSVC, OpenGL and assimp binaries, and its RNG is clock64()-seeded.  These vectors therefore pin
the oracle against regressions and let the GPU path be diffed field by field; their inputs
(sphere.glb, Cube.glb, HDR_029_Sky_Cloudy_Env.hdr) are the reference's own asset files.
Run: python tools/make_golden.py
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "mc-path-tracer_amd"), os.path.join(REPO, "oracle"), os.path.join(REPO, "tests")]
import mcpt  # noqa: E402
import oracle_py as op  # noqa: E402
import stage_fixtures as sf  # noqa: E402

OUT = os.environ.get("GOLDEN_OUT", os.path.join(REPO, "tests", "golden"))


def rays(n, seed, box=3.0):
    rng = np.random.default_rng(seed)
    ro = rng.uniform(-box, box, (n, 3)).astype(np.float32)
    rd = rng.normal(size=(n, 3)).astype(np.float32)
    rd /= np.linalg.norm(rd, axis=1, keepdims=True)
    # aim half of them at the origin so that they hit
    tgt = rng.uniform(-0.5, 0.5, (n // 2, 3)).astype(np.float32)
    d = tgt - ro[: n // 2]
    rd[: n // 2] = d / np.linalg.norm(d, axis=1, keepdims=True)
    return ro, rd


def main():
    os.makedirs(OUT, exist_ok=True)
    s1 = mcpt.build_config_scene(1)
    a1 = s1.arrays()
    cube = mcpt.Scene()
    cube.load_glb(os.path.join(mcpt.ASSET_DIR, "Cube.glb"))
    cube.set_env_hdr(os.path.join(mcpt.ASSET_DIR, "HDR_029_Sky_Cloudy_Env.hdr"), 1)
    cube.build(8)
    ac = cube.arrays()
    # film fixture: config 1 at 64x64, 4 spp, depth 3
    cam = mcpt.config_camera(mcpt.CONFIGS[1], 64, 64)
    Ld, smp, cnt = op.render(a1, cam, 64, 64, spp=4, max_depth=3)
    np.savez_compressed(os.path.join(OUT, "film_c1_64x64_s4_d3.npz"), Ld=Ld, samples=smp,
                        counters=np.array([cnt[k] for k in ("extend_rays", "shadow_rays", "vis_rays")], np.uint64),
                        inv_view_proj=np.array(cam.inv_view_proj, np.float32),
                        inv_view=np.array(cam.inv_view, np.float32))
    # film fixture: Cube (axis-aligned normals -> NaN frames), 32x32, 2 spp, depth 5
    camc = mcpt.make_camera((0.0, 0.0, 4.0), aspect=1.0)
    Lc, sc_, cc = op.render(ac, camc, 32, 32, spp=2, max_depth=5)
    np.savez_compressed(os.path.join(OUT, "film_cube_32x32_s2_d5.npz"), Ld=Lc, samples=sc_,
                        counters=np.array([cc[k] for k in ("extend_rays", "shadow_rays", "vis_rays")], np.uint64))
    # trace fixtures: 256 rays per scene, closest + any
    for name, arr in (("c1", a1), ("cube", ac)):
        ro, rd = rays(256, 7)
        pt, nm, tri = op.trace_closest(arr, ro, rd)  # tri: triangle ids (scene order, any BVH)
        vis = op.trace_any(arr, ro, rd)
        np.savez_compressed(os.path.join(OUT, f"trace_{name}_256.npz"), ro=ro, rd=rd, pos_t=pt, nrm_mat=nm, tri=tri, vis=vis)
    for suffix in sf.SCENES:
        stage_vectors(suffix)
    print("golden fixtures written to", OUT)


def stage_vectors(suffix):
    """Per-stage golden vectors of one fixture scene
    (stage_fixtures.SCENES; round 6 added config 2's proxy): inputs from tests/stage_fixtures.py,
    outputs from the oracle's stage restatements, diffed field by field against mcpt_stage_run by
    tests/test_gpu.py::test_stage_golden_vectors.  `python tools/make_golden.py --stages c2` writes
    one scene's vectors only."""
    cid = sf.SCENES[suffix]
    s = sf.stage_scene(mcpt, cid)
    a = s.arrays()
    cam = sf.stage_camera(mcpt, cid)
    W, H = sf.FILM
    kw = dict(max_depth=sf.DEPTH, rr_depth=sf.RR)
    for name, st in (("logic", sf.logic_state(len(a["mat"]))), ("generate", sf.logic_state(len(a["mat"]), True))):
        out = op.stage_logic(a, cam, W, H, st, sf.SPP, **kw)
        np.savez_compressed(os.path.join(OUT, f"stage_{name}_{suffix}.npz"), **{"in_" + k: v for k, v in st.items()},
                            **{"out_" + k: v for k, v in out.items()})
    st = sf.material_state(a, op.trace_closest, cid)
    out = op.stage_material(a, st, **kw)
    np.savez_compressed(os.path.join(OUT, f"stage_material_{suffix}.npz"), **{"in_" + k: v for k, v in st.items()},
                        **{"out_" + k: v for k, v in out.items()})


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--stages":
        os.makedirs(OUT, exist_ok=True)
        for suffix in sys.argv[2:]:
            stage_vectors(suffix)
    else:
        main()
