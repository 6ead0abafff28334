"""GPU parity tests: the gfx950 HIP path (through the C ABI) against the CPU oracle.

Bar: bitwise for hit indices / visibility / sample counts; radiance within the north star's
1e-4 relative fp32 tolerance |g - c| <= 1e-4 * max(|g|, |c|) + 1e-7 (the kernels and the oracle
share IEEE op order, so in practice films are bitwise equal and the tests also report that).
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu
RTOL = 1e-4


def film_close(g, c):
    tol = RTOL * np.maximum(np.abs(g), np.abs(c)) + 1e-7
    ok = (np.abs(g - c) <= tol) | (np.isnan(g) & np.isnan(c))
    return bool(ok.all()), int((~ok).sum())


def make_pt(mcpt, scene, cam, W, H, spp, depth, tile=256):
    pt = mcpt.PathTracer(0, mcpt.default_config(spp=spp, max_depth=depth, tile=tile))
    pt.upload_scene(scene)
    pt.set_camera(cam)
    pt.resize(W, H, tile, tile)
    return pt


def random_rays(n, seed, box=3.0):
    rng = np.random.default_rng(seed)
    ro = rng.uniform(-box, box, (n, 3)).astype(np.float32)
    rd = rng.normal(size=(n, 3)).astype(np.float32)
    rd /= np.linalg.norm(rd, axis=1, keepdims=True)
    t = rng.uniform(-0.8, 0.8, (n // 2, 3)).astype(np.float32)
    d = t - ro[: n // 2]
    rd[: n // 2] = d / np.linalg.norm(d, axis=1, keepdims=True)
    return ro, rd


@pytest.mark.parametrize("which", ["scene_c1", "scene_c2", "scene_cube"])
def test_trace_parity_random_rays(request, mcpt_mod, oracle, which):
    s, a = request.getfixturevalue(which)
    pt = mcpt_mod.PathTracer(0)
    pt.upload_scene(s)
    ro, rd = random_rays(100000, 21)
    # edge cases: NaN and zero directions, origins on the surface, grazing directions
    ro[:4] = [[0, 0, 5], [0, 0, 5], [0, 0, 5], [0, 0, 1]]
    rd[:4] = [[np.nan, 0, -1], [0, 0, 0], [0, 0, -1], [1, 0, 0]]
    gp, gn, gt = pt.trace_closest(ro, rd)
    op_, on, ot = oracle.trace_closest(a, ro, rd)
    assert np.array_equal(gt, ot)
    assert np.array_equal(gp.view(np.uint32), op_.view(np.uint32))
    assert np.array_equal(gn.view(np.uint32), on.view(np.uint32))
    assert np.array_equal(pt.trace_any(ro, rd), oracle.trace_any(a, ro, rd))
    pt.close()


def test_trace_parity_deep_bvh(mcpt_mod, oracle, scene_c3):
    """Config-3 proxy (871,416 triangles, SAH depth 25): bitwise closest/any hits vs the oracle."""
    s, a = scene_c3
    pt = mcpt_mod.PathTracer(0)
    pt.upload_scene(s)
    ro, rd = random_rays(20000, 5, box=2.5)
    ro[:, 1] += 1.0  # the proxy is centred at (0, 1, 0)
    gp, gn, gt = pt.trace_closest(ro, rd)
    op_, on, ot = oracle.trace_closest(a, ro, rd)
    assert np.array_equal(gt, ot)
    assert np.array_equal(gp.view(np.uint32), op_.view(np.uint32))
    assert np.array_equal(gn.view(np.uint32), on.view(np.uint32))
    assert np.array_equal(pt.trace_any(ro, rd), oracle.trace_any(a, ro, rd))
    assert (gt >= 0).mean() > 0.3  # the rays do hit the surface
    pt.close()


def test_config3_1080p_band_parity(mcpt_mod, oracle, scene_c3):
    """Config 3 (deep BVH) at 1080p, 1 spp on the GPU; a band of rows through the proxy's
    silhouette re-executed by the oracle matches bit for bit."""
    rc = mcpt_mod.CONFIGS[3]
    W, H = rc.width, rc.height
    cam = mcpt_mod.config_camera(rc)
    pt = make_pt(mcpt_mod, scene_c3[0], cam, W, H, 1, rc.max_depth)
    st = pt.render()
    Ld, smp = pt.film()
    assert st.live_paths == 0 and np.all(smp[:-1, :-1] == 1)
    r0, r1 = 600, 604
    rL, rs, _ = oracle.render(scene_c3[1], cam, W, H, 1, rc.max_depth, rows=(r0, r1))
    assert np.array_equal(smp[r0:r1], rs[r0:r1])
    ok, nbad = film_close(Ld[r0:r1], rL[r0:r1])
    assert ok, f"{nbad} radiance values differ"
    pt.close()


def test_trace_golden_fixtures(mcpt_mod, scene_c1, scene_cube):
    for name, (s, _) in (("c1", scene_c1), ("cube", scene_cube)):
        g = np.load(os.path.join(GOLDEN, f"trace_{name}_256.npz"))
        pt = mcpt_mod.PathTracer(0)
        pt.upload_scene(s)
        p, n, t = pt.trace_closest(g["ro"], g["rd"])
        assert np.array_equal(t, g["tri"])
        assert np.array_equal(p.view(np.uint32), g["pos_t"].view(np.uint32))
        assert np.array_equal(n.view(np.uint32), g["nrm_mat"].view(np.uint32))
        assert np.array_equal(pt.trace_any(g["ro"], g["rd"]), g["vis"])
        pt.close()


def test_film_golden_c1(mcpt_mod, scene_c1):
    g = np.load(os.path.join(GOLDEN, "film_c1_64x64_s4_d3.npz"))
    cam = mcpt_mod.config_camera(mcpt_mod.CONFIGS[1], 64, 64)
    pt = make_pt(mcpt_mod, scene_c1[0], cam, 64, 64, 4, 3)
    st = pt.render()
    Ld, smp = pt.film()
    assert np.array_equal(smp, g["samples"])
    ok, nbad = film_close(Ld, g["Ld"])
    assert ok, f"{nbad} radiance values differ"
    assert np.array_equal(Ld.view(np.uint32), g["Ld"].view(np.uint32))
    assert [st.extend_rays, st.shadow_rays, st.vis_rays] == list(g["counters"])
    pt.close()


def test_film_golden_cube_nan_frames(mcpt_mod, scene_cube):
    """Cube.glb: exactly axis-aligned normals -> NaN gram_schmidt frames (Appendix A.9)."""
    g = np.load(os.path.join(GOLDEN, "film_cube_32x32_s2_d5.npz"))
    cam = mcpt_mod.make_camera((0.0, 0.0, 4.0), aspect=1.0)
    pt = make_pt(mcpt_mod, scene_cube[0], cam, 32, 32, 2, 5)
    st = pt.render()
    Ld, smp = pt.film()
    assert np.array_equal(smp, g["samples"])
    assert film_close(Ld, g["Ld"])[0]
    assert [st.extend_rays, st.shadow_rays, st.vis_rays] == list(g["counters"])
    pt.close()


def test_config1_full_parity(mcpt_mod, oracle, scene_c1):
    """BASELINE config 1 in full: sphere.glb + HDR_029, 256x256, 16 spp, depth 3."""
    rc = mcpt_mod.CONFIGS[1]
    cam = mcpt_mod.config_camera(rc)
    pt = make_pt(mcpt_mod, scene_c1[0], cam, rc.width, rc.height, rc.spp, rc.max_depth)
    st = pt.render()
    Ld, smp = pt.film()
    rL, rs, cnt = oracle.render(scene_c1[1], cam, rc.width, rc.height, rc.spp, rc.max_depth)
    assert np.array_equal(smp, rs)
    ok, nbad = film_close(Ld, rL)
    assert ok, f"{nbad} radiance values differ"
    assert (st.extend_rays, st.shadow_rays, st.vis_rays) == (cnt["extend_rays"], cnt["shadow_rays"], cnt["vis_rays"])
    pt.close()


def test_config2_parity_small(mcpt_mod, oracle, scene_c2):
    rc = mcpt_mod.CONFIGS[2]
    W, H = 160, 90
    cam = mcpt_mod.config_camera(rc, W, H)
    pt = make_pt(mcpt_mod, scene_c2[0], cam, W, H, 3, rc.max_depth)
    pt.render()
    Ld, smp = pt.film()
    rL, rs, _ = oracle.render(scene_c2[1], cam, W, H, 3, rc.max_depth)
    assert np.array_equal(smp, rs)
    assert film_close(Ld, rL)[0]
    pt.close()


def test_config2_1080p_band_parity_and_properties(mcpt_mod, oracle, scene_c2):
    """Full 1080p frame at 2 spp on the GPU; a band of rows re-executed by the oracle must match
    bit for bit (rows are independent), and frame-wide invariants hold."""
    rc = mcpt_mod.CONFIGS[2]
    W, H = rc.width, rc.height
    cam = mcpt_mod.config_camera(rc)
    pt = make_pt(mcpt_mod, scene_c2[0], cam, W, H, 2, rc.max_depth)
    pt.set_work_counters(True)  # the counting k_trace build: same hits, StageStats work counters filled
    st = pt.render()
    Ld, smp = pt.film()
    assert np.all(smp[:-1, :-1] == 2) and np.all(smp[-1] == 0) and np.all(smp[:, -1] == 0)
    assert st.live_paths == 0
    # traversal work counters: per traced ray, a handful of node pairs and triangle tests
    rays_any = st.shadow_rays + st.vis_rays
    assert 1.0 < st.ext_nodes / st.extend_rays < 64.0 and 0.1 < st.ext_tests / st.extend_rays < 32.0
    assert 1.0 < st.any_nodes / rays_any < 64.0 and 0.1 < st.any_tests / rays_any < 32.0
    assert 0 < st.ext_hits <= st.extend_rays and st.any_hits <= rays_any
    r0, r1 = 532, 548
    rL, rs, _ = oracle.render(scene_c2[1], cam, W, H, 2, rc.max_depth, rows=(r0, r1))
    assert np.array_equal(smp[r0:r1], rs[r0:r1])
    assert film_close(Ld[r0:r1], rL[r0:r1])[0]
    # determinism: a second context reproduces the frame bit for bit
    pt2 = make_pt(mcpt_mod, scene_c2[0], cam, W, H, 2, rc.max_depth)
    st2 = pt2.render()
    L2, s2 = pt2.film()
    assert np.array_equal(L2.view(np.uint32), Ld.view(np.uint32)) and st2.rays == st.rays
    pt.close()
    pt2.close()


def test_tile_partition_invariance(mcpt_mod, scene_c2):
    """The multi-GPU contract on one device: rendering tile subsets separately (as ranks would)
    gives the same film as one pass; so does the reference-style one-tile-per-step loop."""
    rc = mcpt_mod.CONFIGS[2]
    W, H, T = 200, 120, 64
    cam = mcpt_mod.config_camera(rc, W, H)
    full = make_pt(mcpt_mod, scene_c2[0], cam, W, H, 2, 5, tile=T)
    full.render()
    L0, s0 = full.film()
    from mcpt import parallel

    # 1/2/4/8 (and 3) tile partitions on one device, bit-identical
    for nparts in (2, 3, 4, 8):
        parts = make_pt(mcpt_mod, scene_c2[0], cam, W, H, 2, 5, tile=T)
        for r in range(nparts):
            parts.set_tiles(parallel.tiles_for_rank(r, nparts, W, H, T))
            parts.render()
        L1, s1 = parts.film()
        parts.close()
        assert np.array_equal(L0.view(np.uint32), L1.view(np.uint32)) and np.array_equal(s0, s1), nparts
    # reference orchestration: one tile per wavefront_pathtrace call, round-robin (Film.cu:94-103)
    ref = make_pt(mcpt_mod, scene_c2[0], cam, W, H, 2, 5, tile=T)
    nx, ny = parallel.tile_grid(W, H, T)
    for it in range(40 * nx * ny):
        t = it % (nx * ny)
        ref.step(t % nx, t // nx)
    L2, s2 = ref.film()
    assert np.array_equal(L0.view(np.uint32), L2.view(np.uint32)) and np.array_equal(s0, s2)
    for p in (full, ref):
        p.close()


@pytest.mark.parametrize("slots", [2, 4])
def test_path_slots_config1_parity(mcpt_mod, oracle, scene_c1, slots):
    """mcpt_set_path_slots: S paths in flight per pixel, slot k running samples k, k+S, ... with the
    same per-sample RNG keys, so every sample contributes exactly what it does with one path per
    pixel; only the summation order of the film differs.  BASELINE config 1 in full against the
    oracle: sample counts and ray counts exact, radiance within the north star's 1e-4."""
    rc = mcpt_mod.CONFIGS[1]
    cam = mcpt_mod.config_camera(rc)
    pt = mcpt_mod.PathTracer(0, mcpt_mod.default_config(spp=rc.spp, max_depth=rc.max_depth))
    pt.upload_scene(scene_c1[0])
    pt.set_camera(cam)
    pt.set_path_slots(slots)  # before resize: allocated once
    pt.resize(rc.width, rc.height)
    st = pt.render()
    Ld, smp = pt.film()
    rL, rs, cnt = oracle.render(scene_c1[1], cam, rc.width, rc.height, rc.spp, rc.max_depth)
    assert np.array_equal(smp, rs)
    ok, nbad = film_close(Ld, rL)
    assert ok, f"{nbad} radiance values differ"
    assert (st.extend_rays, st.shadow_rays, st.vis_rays) == (cnt["extend_rays"], cnt["shadow_rays"], cnt["vis_rays"])
    assert st.iterations < 7 * rc.spp  # slots run their samples concurrently
    # the readers (tonemap, device read) see the resolved film
    with np.errstate(invalid="ignore", divide="ignore"):
        c = (Ld / smp[..., None].astype(np.float32)) * np.float32(1.0)
        v = np.float32(255) * (c / (c + np.float32(1.0)))
    want = np.where(np.isfinite(v) & (v >= 0), v, 0).astype(np.uint32).astype(np.uint8)
    assert np.array_equal(pt.tonemap(1.0)[..., :3], want)
    pt.close()


def test_path_slots_ragged_and_resize(mcpt_mod, oracle, scene_c2):
    """Slots with spp not a multiple of S (slot 2 of 3 runs one sample fewer), slots changed after
    resize (re-allocates, clears), and spp=1 with 4 slots bit-identical to one slot."""
    rc = mcpt_mod.CONFIGS[2]
    W, H = 160, 90
    cam = mcpt_mod.config_camera(rc, W, H)
    pt = make_pt(mcpt_mod, scene_c2[0], cam, W, H, 4, rc.max_depth)
    pt.render()
    pt.set_path_slots(3)
    assert pt.film()[1].max() == 0  # cleared by the re-allocation
    pt.render()
    Ld, smp = pt.film()
    rL, rs, _ = oracle.render(scene_c2[1], cam, W, H, 4, rc.max_depth)
    assert np.array_equal(smp, rs)
    assert film_close(Ld, rL)[0]
    one = make_pt(mcpt_mod, scene_c2[0], cam, W, H, 1, rc.max_depth)
    one.render()
    four = make_pt(mcpt_mod, scene_c2[0], cam, W, H, 1, rc.max_depth)
    four.set_path_slots(4)
    four.render()
    (a, sa), (b, sb) = one.film(), four.film()
    assert np.array_equal(sa, sb) and np.array_equal(a.view(np.uint32), b.view(np.uint32))
    with pytest.raises(mcpt_mod.McptError):
        pt.set_path_slots(0)
    for p in (pt, one, four):
        p.close()


@pytest.mark.parametrize("which", ["scene_c2", "scene_cube", "scene_c1", "scene_c3"])
def test_occluder_cache_same_film(request, mcpt_mod, which):
    """The any-hit occluder cache (kernels.hip occ_hit1) decides only which any-hit rays skip the
    traversal: a cached triangle counts only under its own leaf box with the traversal's slab
    arithmetic and cull, so every ray it resolves is one the traversal finds occluded too.  Films
    and ray counts with the cache (default; it starts empty with every film clear and fills during
    the frame) and without it (MCPT_OCC_G=0 at upload) are bit-identical, frame after frame; on the
    closed config-2 box and the cube (flat, axis-aligned leaf boxes) it resolves rays."""
    scene = request.getfixturevalue(which)[0]
    W, H = 160, 90
    if which == "scene_cube":
        cam = mcpt_mod.make_camera((0.3, 0.1, 3.0), aspect=W / H)
    else:
        cam = mcpt_mod.config_camera(mcpt_mod.CONFIGS[int(which[-1])], W, H)

    def run(env):
        old = os.environ.get("MCPT_OCC_G")
        if env is None:
            os.environ.pop("MCPT_OCC_G", None)
        else:
            os.environ["MCPT_OCC_G"] = env
        try:
            pt = make_pt(mcpt_mod, scene, cam, W, H, 24, 5, tile=64)
        finally:
            if old is None:
                os.environ.pop("MCPT_OCC_G", None)
            else:
                os.environ["MCPT_OCC_G"] = old
        pt.set_path_slots(2)
        out = []
        for _ in range(2):
            pt.clear()
            st = pt.render()
            L, smp = pt.film()
            out.append((L.copy(), smp.copy(), (st.extend_rays, st.shadow_rays, st.vis_rays), pt.occ_stats()))
        pt.close()
        return out

    off, on = run("0"), run(None)
    assert off[0][3] == (0, False) and on[0][3][1]
    for a in on + off[1:]:
        assert np.array_equal(a[0].view(np.uint32), off[0][0].view(np.uint32))
        assert np.array_equal(a[1], off[0][1]) and a[2] == off[0][2]
    resolved = on[1][3][0]
    # the table is emptied with each film clear, so both frames start cold; which rays it resolves
    # depends on the order the traversal's records land in (racy stores), never the films
    assert abs(on[0][3][0] - resolved) <= 0.05 * max(resolved, 20)
    print(f"{which}: any-hit rays {sum(off[0][2][1:])}, resolved by the cache {resolved}")
    if which in ("scene_c2", "scene_cube"):
        assert resolved > 0


@pytest.mark.parametrize("shade_wgs", [None, "3"])
def test_finished_blocks_skip_and_reset(mcpt_mod, scene_c2, shade_wgs, monkeypatch):
    """k_shade's block done flags (ShadeArgs::blk_done): once a film is complete, further
    iterations trace nothing and leave it bit for bit; a film clear resets the flags, so the
    re-render equals the first one; turning a camera change into a stale film does too.  A
    render with the flags off (MCPT_NO_BLOCK_DONE, new context) gives the same film.  With
    shade_wgs = 3 (MCPT_SHADE_WGS) k_shade runs the 256 shading blocks on 3 workgroups, ~86 per
    workgroup (the virtual-block loop and its done-flag prefetch); the film equals the one-pass
    grid's (MCPT_SHADE_GRID=0)."""
    import os

    if shade_wgs:
        monkeypatch.setenv("MCPT_SHADE_WGS", shade_wgs)
    else:
        monkeypatch.setenv("MCPT_SHADE_GRID", "0")
    rc = mcpt_mod.CONFIGS[2]
    W, H, T = 200, 120, 64
    cam = mcpt_mod.config_camera(rc, W, H)
    pt = make_pt(mcpt_mod, scene_c2[0], cam, W, H, 3, 5, tile=T)
    pt.set_path_slots(2)
    pt.render()
    L0, s0 = pt.film()
    st = pt.iterate(5)
    assert st.rays == 0
    L1, s1 = pt.film()
    assert np.array_equal(L0.view(np.uint32), L1.view(np.uint32)) and np.array_equal(s0, s1)
    pt.clear()
    pt.render()
    L2, s2 = pt.film()
    assert np.array_equal(L0.view(np.uint32), L2.view(np.uint32)) and np.array_equal(s0, s2)
    pt.set_camera(mcpt_mod.make_camera((0.3, 0.1, 3.0), aspect=W / H))  # stale film: cleared by the next call
    pt.render()
    pt.set_camera(cam)
    pt.render()
    L3, s3 = pt.film()
    assert np.array_equal(L0.view(np.uint32), L3.view(np.uint32)) and np.array_equal(s0, s3)
    pt.close()
    os.environ["MCPT_NO_BLOCK_DONE"] = "1"
    try:
        off = make_pt(mcpt_mod, scene_c2[0], cam, W, H, 3, 5, tile=T)
    finally:
        del os.environ["MCPT_NO_BLOCK_DONE"]
    off.set_path_slots(2)
    off.render()
    L4, s4 = off.film()
    off.close()
    assert np.array_equal(L0.view(np.uint32), L4.view(np.uint32)) and np.array_equal(s0, s4)


def test_path_slots_partition_invariance(mcpt_mod, scene_c2):
    """With 2 path slots, tile subsets rendered separately (as ranks would) and the reference's
    one-tile-per-call orchestration give the batch film bit for bit (same slot order per pixel)."""
    rc = mcpt_mod.CONFIGS[2]
    W, H, T = 200, 120, 64
    cam = mcpt_mod.config_camera(rc, W, H)
    from mcpt import parallel

    pts = [make_pt(mcpt_mod, scene_c2[0], cam, W, H, 3, 5, tile=T) for _ in range(3)]
    for p in pts:
        p.set_path_slots(2)
    full, parts, ref = pts
    full.render()
    for r in range(2):
        parts.set_tiles(parallel.tiles_for_rank(r, 2, W, H, T))
        parts.render()
    nx, ny = parallel.tile_grid(W, H, T)
    for it in range(40 * nx * ny):
        t = it % (nx * ny)
        ref.step(t % nx, t // nx)
    (L0, s0), (L1, s1), (L2, s2) = full.film(), parts.film(), ref.film()
    assert s0[: H - 1, : W - 1].min() == 3
    for L, sm in ((L1, s1), (L2, s2)):
        assert np.array_equal(L0.view(np.uint32), L.view(np.uint32)) and np.array_equal(s0, sm)
    for p in pts:
        p.close()


def test_degenerate_and_ragged_films(mcpt_mod, oracle, scene_c1):
    """Edge cases of the film/tile contract against the oracle: 1x1 and 2x2 films (the last row
    and column are never rendered, wavefront_kernels.cu:110), spp = 0, ragged non-square tiles,
    a tile larger than the film, with 1 and 2 path slots; bad sizes are rejected."""
    rc = mcpt_mod.CONFIGS[1]
    cases = [(1, 1, 2, 256, 256), (2, 2, 3, 256, 256), (70, 50, 2, 48, 32), (100, 60, 2, 512, 512), (33, 17, 0, 16, 8)]
    for W, H, spp, tw, th in cases:
        cam = mcpt_mod.config_camera(rc, W, H)
        rL, rs, cnt = oracle.render(scene_c1[1], cam, W, H, spp, rc.max_depth)
        for slots in (1, 2):
            pt = mcpt_mod.PathTracer(0, mcpt_mod.default_config(spp=spp, max_depth=rc.max_depth))
            pt.upload_scene(scene_c1[0])
            pt.set_camera(cam)
            pt.set_path_slots(slots)
            pt.resize(W, H, tw, th)
            st = pt.render()
            Ld, smp = pt.film()
            assert st.live_paths == 0
            assert np.array_equal(smp, rs), (W, H, spp, tw, th, slots)
            assert film_close(Ld, rL)[0], (W, H, spp, tw, th, slots)
            if slots == 1:
                assert np.array_equal(Ld.view(np.uint32), np.asarray(rL, np.float32).reshape(Ld.shape).view(np.uint32))
            assert (st.extend_rays, st.shadow_rays, st.vis_rays) == (cnt["extend_rays"], cnt["shadow_rays"], cnt["vis_rays"])
            pt.close()
    pt = mcpt_mod.PathTracer(0)
    for bad in ((0, 4, 256, 256), (4, 0, 256, 256), (4, 4, 0, 256), (64, 64, 1 << 14, 1 << 14)):
        with pytest.raises(mcpt_mod.McptError):
            pt.resize(*bad)
    pt.close()


def test_tonemap_matches_draw_to_surface(mcpt_mod, scene_c1):
    cam = mcpt_mod.config_camera(mcpt_mod.CONFIGS[1], 64, 64)
    pt = make_pt(mcpt_mod, scene_c1[0], cam, 64, 64, 2, 3)
    pt.render()
    Ld, smp = pt.film()
    img = pt.tonemap(1.5)
    with np.errstate(invalid="ignore", divide="ignore"):
        c = (Ld / smp[..., None].astype(np.float32)) * np.float32(1.5)
        c = c / (c + np.float32(1.0))
        v = np.float32(255) * c
    want = np.where(np.isfinite(v) & (v >= 0), v, 0).astype(np.uint32).astype(np.uint8)  # NaN -> 0 (:18)
    assert np.array_equal(img[..., :3], want) and np.all(img[..., 3] == 255)
    pt.close()


def test_errors_are_reported(mcpt_mod):
    pt = mcpt_mod.PathTracer(0)
    with pytest.raises(mcpt_mod.McptError, match="no scene"):
        pt.iterate(1)
    with pytest.raises(mcpt_mod.McptError):
        pt.trace_closest(np.zeros((1, 3), np.float32), np.ones((1, 3), np.float32))
    pt.close()


def test_film_writers(mcpt_mod, scene_c1, tmp_path):
    """mcpt_film_write_png / _pfm on a rendered film: PNG == tonemap RGB, PFM == Ld / samples."""
    from test_image_io import read_pfm, read_png

    rc = mcpt_mod.CONFIGS[1]
    W, H = 64, 48
    cam = mcpt_mod.config_camera(rc, W, H)
    pt = make_pt(mcpt_mod, scene_c1[0], cam, W, H, 4, rc.max_depth)
    pt.render()
    Ld, smp = pt.film()
    pt.write_png(tmp_path / "f.png", 1.5)
    pt.write_pfm(tmp_path / "f.pfm")
    assert np.array_equal(read_png(tmp_path / "f.png"), pt.tonemap(1.5)[..., :3])
    want = np.where(smp[..., None] > 0, Ld / np.maximum(smp, 1)[..., None].astype(np.float32), 0).astype(np.float32)
    assert np.array_equal(read_pfm(tmp_path / "f.pfm"), want)
    pt.close()


@pytest.mark.parametrize("which", ["scene_c1", "scene_c2"])
def test_fixed_mode_parity(request, mcpt_mod, oracle, which):
    """Quality mode (MCPT_FLAG_FIXED) on the GPU against the oracle's fixed mode, with Russian
    roulette active (depth 5 > rr_depth 3)."""
    s, a = request.getfixturevalue(which)
    rc = mcpt_mod.CONFIGS[1 if which == "scene_c1" else 2]
    W, H = 96, 64
    cam = mcpt_mod.config_camera(rc, W, H)
    pt = mcpt_mod.PathTracer(0, mcpt_mod.default_config(spp=3, max_depth=5, fixed=True))
    pt.upload_scene(s)
    pt.set_camera(cam)
    pt.resize(W, H)
    pt.render()
    Ld, smp = pt.film()
    rL, rs, _ = oracle.render(a, cam, W, H, 3, 5, fixed=True)
    assert np.array_equal(smp, rs)
    ok, nbad = film_close(Ld, rL)
    assert ok, f"{nbad} radiance values differ"
    pt.close()


def test_fixed_mode_delta_light_parity(mcpt_mod, oracle):
    """Fixed mode with a directional (delta) light: selection pdf 1/2 and MIS weight 1."""
    from test_fixed_mode import cube_scene

    s = cube_scene(mcpt_mod, with_dir_light=True)
    a = s.arrays()
    cam = mcpt_mod.make_camera((0.5, 0.7, 3.0))
    W = H = 48
    for fixed in (False, True):
        pt = mcpt_mod.PathTracer(0, mcpt_mod.default_config(spp=4, max_depth=5, fixed=fixed))
        pt.upload_scene(s)
        pt.set_camera(cam)
        pt.resize(W, H)
        pt.render()
        Ld, smp = pt.film()
        rL, rs, _ = oracle.render(a, cam, W, H, 4, 5, fixed=fixed)
        assert np.array_equal(smp, rs)
        assert film_close(Ld, rL)[0]
        pt.close()


@pytest.mark.parametrize("builder", ["ploc", "lbvh"])
@pytest.mark.parametrize("which", ["scene_c1", "scene_c2", "scene_cube", "scene_c3"])
def test_gpu_bvh_same_hits(request, mcpt_mod, oracle, which, builder):
    """GPU-built BVHs (mcpt_scene_upload_gpu_bvh, PLOC and linear BVH): hits bit-identical to the
    oracle, which traverses the host SAH tree -- the traversal's result does not depend on the tree."""
    s, a = request.getfixturevalue(which)
    pt = mcpt_mod.PathTracer(0)
    pt.upload_scene(s, gpu_bvh=builder)
    assert pt.last_build_ms > 0
    n = 20000 if which == "scene_c3" else 100000
    ro, rd = random_rays(n, 31, box=2.5)
    if which == "scene_c3":
        ro[:, 1] += 1.0
    ro[:4] = [[0, 0, 5], [0, 0, 5], [0, 0, 5], [0, 0, 1]]
    rd[:4] = [[np.nan, 0, -1], [0, 0, 0], [0, 0, -1], [1, 0, 0]]
    gp, gn, gt = pt.trace_closest(ro, rd)
    op_, on, ot = oracle.trace_closest(a, ro, rd)
    assert np.array_equal(gt, ot)
    assert np.array_equal(gp.view(np.uint32), op_.view(np.uint32))
    assert np.array_equal(gn.view(np.uint32), on.view(np.uint32))
    assert np.array_equal(pt.trace_any(ro, rd), oracle.trace_any(a, ro, rd))
    pt.close()


@pytest.mark.parametrize("builder", ["ploc", "lbvh"])
def test_gpu_bvh_film_parity(mcpt_mod, oracle, scene_c2, builder):
    rc = mcpt_mod.CONFIGS[2]
    W, H = 160, 90
    cam = mcpt_mod.config_camera(rc, W, H)
    pt = mcpt_mod.PathTracer(0, mcpt_mod.default_config(spp=3, max_depth=rc.max_depth))
    pt.upload_scene(scene_c2[0], gpu_bvh=builder)
    pt.set_camera(cam)
    pt.resize(W, H)
    pt.render()
    Ld, smp = pt.film()
    rL, rs, _ = oracle.render(scene_c2[1], cam, W, H, 3, rc.max_depth)
    assert np.array_equal(smp, rs)
    assert np.array_equal(Ld.view(np.uint32), rL.view(np.uint32))
    pt.close()


def test_cpp_example_batch_equals_reference_orchestration(tmp_path):
    """examples/mcpt_render (C++ over the C ABI only): config 1 at 4 spp in batch mode and in the
    reference's one-tile-per-call orchestration write bit-identical PFM films."""
    import subprocess

    from conftest import REPO
    from test_image_io import read_pfm, read_png

    exe = os.path.join(REPO, "examples", "mcpt_render")
    if not os.path.exists(exe):
        subprocess.run(["make", "-C", REPO, "example"], check=True, capture_output=True)
    env = dict(os.environ, MCPT_ASSETS=os.path.join(REPO, "assets"))
    for mode, extra in (("batch", []), ("tile", ["--tiles-per-call"])):
        r = subprocess.run([exe, "1", "4", str(tmp_path / mode)] + extra, capture_output=True, text=True, env=env,
                           timeout=300)
        assert r.returncode == 0, r.stdout + r.stderr
    a, b = read_pfm(tmp_path / "batch.pfm"), read_pfm(tmp_path / "tile.pfm")
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
    assert read_png(tmp_path / "batch.png").shape == (256, 256, 3)


def test_film_observes_camera_and_scene(mcpt_mod):
    """Film::update -> clear() (Film.cu:278-281) on Camera::update / Scene::notify: a different
    camera or a scene re-upload clears the film before the next iteration; the same camera does
    not; MCPT_FLAG_NO_AUTO_CLEAR leaves clearing to the caller."""
    from test_fixed_mode import cube_scene

    s = cube_scene(mcpt_mod, False)
    cam = mcpt_mod.make_camera((0.5, 0.7, 3.0))
    cam2 = mcpt_mod.make_camera((0.4, 0.7, 3.0))
    W = H = 32
    for auto in (True, False):
        pt = mcpt_mod.PathTracer(0, mcpt_mod.default_config(spp=2, max_depth=3, auto_clear=auto))
        pt.upload_scene(s)
        pt.set_camera(cam)
        pt.resize(W, H)
        pt.render()
        full = pt.film()[1].copy()
        assert full[: H - 1, : W - 1].min() == 2
        pt.set_camera(cam)  # unchanged camera: no notification
        pt.iterate(1)
        assert np.array_equal(pt.film()[1], full)
        pt.set_camera(cam2)
        pt.iterate(1)
        smp = pt.film()[1]
        if auto:
            assert smp.max() <= 1 and smp.sum() < full.sum()
        else:
            assert np.array_equal(smp, full)
        if auto:
            pt.render()
            pt.upload_scene(s)  # re-upload notifies the film
            pt.iterate(1)
            assert pt.film()[1].max() <= 1
        pt.close()


def test_device_division_is_ieee(mcpt_mod):
    """The kernels divide by a shared fp64 reciprocal (mcpt_core.hpp Recip/quot3); on the device
    that must equal IEEE fp32 division bit for bit: random pairs over the whole exponent range,
    special values, and the hardest cases (a/b within ~2^-49 of a rounding midpoint)."""
    g = np.random.default_rng(5)
    n = 1 << 20
    a = g.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32).view(np.float32)
    b = g.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32).view(np.float32)
    # near-1 quotients and signed zeros / infinities / NaN / subnormals
    c = g.uniform(0.5, 2.0, n).astype(np.float32)
    d = g.uniform(0.5, 2.0, n).astype(np.float32)
    sp = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 1e-45, -1e-40, 3.4e38, 1.0, -1.0], np.float32)
    sa, sb = np.meshgrid(sp, sp)
    # hard cases: A = (M B + 1) / 2^25 with M an odd 25-bit integer, so a/b sits 1/(M B) above a midpoint
    B = (g.integers(0, 1 << 23, 4 * n) | (1 << 23) | 1).astype(np.uint64)
    inv = B.copy()
    for _ in range(6):
        inv = (inv * (2 - B * inv)) & 0xFFFFFFFF
    M = (-inv) & 0x1FFFFFF
    ok = (M >> 24) == 1
    A = (M * B + 1) >> 25
    ok &= (((M * B + 1) & 0x1FFFFFF) == 0) & (A >= (1 << 23)) & (A < (1 << 24))
    e = g.integers(-60, 60, ok.sum())
    ha = np.ldexp(A[ok].astype(np.float64), e).astype(np.float32)
    hb = np.ldexp(B[ok].astype(np.float64), e).astype(np.float32)
    assert ha.size > 100000
    aa = np.concatenate([a, c, sa.ravel(), ha])
    bb = np.concatenate([b, d, sb.ravel(), hb])
    pt = mcpt_mod.PathTracer(0)
    got = pt.debug_quot(aa, bb)
    with np.errstate(all="ignore"):
        ref = aa / bb
    nan = np.isnan(ref)
    assert np.array_equal(np.isnan(got), nan)
    assert np.array_equal(got[~nan].view(np.uint32), ref[~nan].view(np.uint32))
    pt.close()


def test_hbm_copy_ceiling(mcpt_mod):
    """mcpt_debug_hbm_copy: the measured copy ceiling the bench reports beside the 8 TB/s spec."""
    pt = mcpt_mod.PathTracer(0)
    g = pt.hbm_copy_gbps(256 << 20, 5)
    assert 1000.0 < g < 8000.0
    with pytest.raises(mcpt_mod.McptError):
        pt.hbm_copy_gbps(16, 1)
    pt.close()


def test_sah3_tree_same_results(mcpt_mod, oracle, scene_c2):
    """The GPU on an SAH3 tree (multi-triangle leaves) == the oracle on the reference builder's
    tree: vertex-grazing rays and a config-2 film band."""
    from test_oracle import grazing_rays

    a0 = mcpt_mod.build_config_scene(2, builder="reference").arrays()
    s1 = mcpt_mod.build_config_scene(2, builder="sah3", buckets=16, trav_cost=2.0, isect_cost=1.0, max_prims=8)
    assert s1.arrays()["nprims"].max() > 1
    pt = mcpt_mod.PathTracer(0, mcpt_mod.default_config(spp=2, max_depth=5))
    pt.upload_scene(s1)
    ro, rd = grazing_rays(a0, 200000, 2)
    gp, gn, gt = pt.trace_closest(ro, rd)
    op_, on, ot = oracle.trace_closest(a0, ro, rd)
    assert np.array_equal(gt, ot)
    assert np.array_equal(gp.view(np.uint32), op_.view(np.uint32))
    assert np.array_equal(gn.view(np.uint32), on.view(np.uint32))
    assert np.array_equal(pt.trace_any(ro, rd), oracle.trace_any(a0, ro, rd))
    rc = mcpt_mod.CONFIGS[2]
    W, H = 160, 90
    cam = mcpt_mod.config_camera(rc, W, H)
    pt.set_camera(cam)
    pt.resize(W, H)
    pt.render()
    Ld, smp = pt.film()
    rL, rs, _ = oracle.render(a0, cam, W, H, 2, 5)
    assert np.array_equal(smp, rs)
    assert np.array_equal(Ld.view(np.uint32), np.asarray(rL).reshape(Ld.shape).view(np.uint32))
    pt.close()


@pytest.mark.parametrize("nparts", [1, 3, 12, 64])
def test_trace_partitions_trace_every_ray(mcpt_mod, oracle, scene_c2, nparts):
    """k_trace work partitions: waves start on a partition of their die and, once it is drained,
    join the others, so any partition count traces every queued ray.  12 partitions on 8 dies
    leaves four with no home waves at all (drained only by joining waves); 3 does not divide the
    64 shards evenly; 64 is one shard each.  Films, ray counts and the per-launch drain check
    (k_accumulate) must not change."""
    rc = mcpt_mod.CONFIGS[2]
    W, H = 320, 180
    cam = mcpt_mod.config_camera(rc, W, H)
    ref = make_pt(mcpt_mod, scene_c2[0], cam, W, H, 3, rc.max_depth)
    st_ref = ref.render()
    L_ref, s_ref = ref.film()
    pt = make_pt(mcpt_mod, scene_c2[0], cam, W, H, 3, rc.max_depth)
    pt.set_trace_partitions(nparts)
    st = pt.render()  # raises if a launch left rays untraced
    L, s = pt.film()
    assert np.array_equal(s, s_ref) and st.rays == st_ref.rays
    assert np.array_equal(L.view(np.uint32), L_ref.view(np.uint32))
    # the single-shard trace API (mcpt_stage_run) under the same partition count
    ro, rd = random_rays(50000, 9)
    _, _, gt = pt.trace_closest(ro, rd)
    assert np.array_equal(gt, oracle.trace_closest(scene_c2[1], ro, rd)[2])
    assert np.array_equal(pt.trace_any(ro, rd), oracle.trace_any(scene_c2[1], ro, rd))
    with pytest.raises(mcpt_mod.McptError):
        pt.set_trace_partitions(65)
    pt.close()
    ref.close()


@pytest.mark.parametrize("knob", ["MCPT_REFILL_MIN=1", "MCPT_REFILL_MIN=64", "MCPT_TRI_MIN=0", "MCPT_TRI_MIN=64"])
def test_trace_schedule_knobs_same_film(mcpt_mod, scene_c2, knob):
    """k_trace's refill threshold (idle lanes before a wave takes new rays; per instantiation by
    default, launch_trace) and triangle-phase threshold only schedule work: at their extremes
    the film, sample counts and ray counts are bit-identical to the defaults'.  Both knobs are
    read when the context is created."""
    rc = mcpt_mod.CONFIGS[2]
    W, H = 320, 180
    cam = mcpt_mod.config_camera(rc, W, H)
    ref = make_pt(mcpt_mod, scene_c2[0], cam, W, H, 3, rc.max_depth)
    st_ref = ref.render()
    L_ref, s_ref = ref.film()
    ref.close()
    var, val = knob.split("=")
    old = os.environ.get(var)
    os.environ[var] = val
    try:
        pt = make_pt(mcpt_mod, scene_c2[0], cam, W, H, 3, rc.max_depth)
    finally:
        if old is None:
            os.environ.pop(var, None)
        else:
            os.environ[var] = old
    st = pt.render()
    L, s = pt.film()
    assert np.array_equal(s, s_ref) and st.rays == st_ref.rays
    assert np.array_equal(L.view(np.uint32), L_ref.view(np.uint32))
    pt.close()


def test_node_layouts_same_hits(mcpt_mod, oracle, scene_c2):
    """Pair-node numberings 0 (depth-first), 1 (sibling pairs, depth-first), 2 (breadth-first) and
    3 (line pairs with pad nodes) are layout only: bit-identical hits and visibility, also through
    4-wide nodes collapsed from layout 3's pairs; out-of-range MCPT_SIBLING_LAYOUT values are
    ignored (the size-based default, 2 for config 2's small tree)."""
    s, a = scene_c2
    ro, rd = random_rays(100000, 33)
    ref = None
    old = os.environ.get("MCPT_SIBLING_LAYOUT")
    try:
        for layout, width in (("0", None), ("1", None), ("2", None), ("3", None), ("3", "4"), ("4", None), ("x", None)):
            os.environ["MCPT_SIBLING_LAYOUT"] = layout
            if width:
                os.environ["MCPT_BVH_WIDTH"] = width
            try:
                pt = mcpt_mod.PathTracer(0)
                pt.upload_scene(s)
            finally:
                os.environ.pop("MCPT_BVH_WIDTH", None)
            got = mcpt_mod.lib().mcpt_debug_node_layout(pt.h)
            assert got == (int(layout) if layout in "0123" else 2)
            p, n, t = pt.trace_closest(ro, rd)
            v = pt.trace_any(ro, rd)
            if ref is None:
                ref = (p, n, t, v)
                assert np.array_equal(t, oracle.trace_closest(a, ro, rd)[2])
            else:
                assert np.array_equal(t, ref[2]) and np.array_equal(v, ref[3])
                assert np.array_equal(p.view(np.uint32), ref[0].view(np.uint32))
                assert np.array_equal(n.view(np.uint32), ref[1].view(np.uint32))
            pt.close()
    finally:
        if old is None:
            os.environ.pop("MCPT_SIBLING_LAYOUT", None)
        else:
            os.environ["MCPT_SIBLING_LAYOUT"] = old


def test_path_slots_rejected_count_keeps_film(mcpt_mod, scene_c1):
    """mcpt_set_path_slots checks W*H*slots < 2^31 before touching the film: a rejected count
    leaves the slot count and the accumulated film in place; an accepted one clears it."""
    W, H = 8192, 4096  # 2^25 pixels: 64 slots would be 2^31 paths
    cam = mcpt_mod.config_camera(mcpt_mod.CONFIGS[1], W, H)
    pt = make_pt(mcpt_mod, scene_c1[0], cam, W, H, 1, 1)
    pt.set_tiles([(0, 0)])
    pt.iterate(3)
    Ld0, s0 = pt.film()
    assert s0[:256, :256].sum() > 0
    with pytest.raises(mcpt_mod.McptError):
        pt.set_path_slots(64)  # rejected up front
    Ld1, s1 = pt.film()
    assert np.array_equal(s1, s0) and np.array_equal(Ld1.view(np.uint32), Ld0.view(np.uint32))
    pt.set_path_slots(2)
    _, s2 = pt.film()
    assert s2.sum() == 0  # accepted change: film cleared
    pt.close()


def test_ploc_small_and_degenerate_inputs(mcpt_mod, oracle):
    """PLOC on 1, 2, 3 and 37 triangles, and on many coincident (identical) triangles: equal
    union areas everywhere, so only the index tie-break orders the pairs; hits match the oracle."""
    rng = np.random.default_rng(5)
    for ntri, same in ((1, False), (2, False), (3, False), (37, False), (300, True)):
        v = rng.uniform(-1, 1, (ntri, 3, 3)).astype(np.float32)
        if same:
            v[:] = v[0]
        s = mcpt_mod.Scene()
        nrm = np.tile(np.float32([0, 0, 1]), (ntri, 1))
        s.add_mesh(v[:, 0], v[:, 1], v[:, 2], nrm, nrm, nrm, (0.5, 0.5, 0.5))
        s.set_env_color((1, 1, 1), 1.0)
        s.build(8)
        a = s.arrays()
        pt = mcpt_mod.PathTracer(0)
        pt.upload_scene(s, gpu_bvh="ploc")
        ro, rd = random_rays(20000, ntri, box=2.0)
        assert np.array_equal(pt.trace_closest(ro, rd)[2], oracle.trace_closest(a, ro, rd)[2])
        assert np.array_equal(pt.trace_any(ro, rd), oracle.trace_any(a, ro, rd))
        pt.close()


@pytest.mark.parametrize("compact", [False, True])
@pytest.mark.parametrize("slots", [1, 2])
def test_native_gather_equals_one_pass(mcpt_mod, scene_c2, slots, compact):
    """mcpt_gather (C ABI): three contexts render the interleaved tile partition of a frame
    ((tx + ty) mod 3, as three GPUs would) and the root gathers the others' tiles; the root's film
    then equals the single-context frame bit for bit (path slots resolved before the copy).
    compact: every context holds path state for its own tiles only (mcpt_set_compact_paths)."""
    from mcpt import parallel

    rc = mcpt_mod.CONFIGS[2]
    W, H, T = 300, 200, 64
    cam = mcpt_mod.config_camera(rc, W, H)
    full = make_pt(mcpt_mod, scene_c2[0], cam, W, H, 2, 5, tile=T)
    full.set_path_slots(slots)
    full.render()
    L_full, s_full = full.film()
    parts = []
    for r in range(3):
        pt = make_pt(mcpt_mod, scene_c2[0], cam, W, H, 2, 5, tile=T)
        if compact:
            pt.set_compact_paths(True)
        pt.set_path_slots(slots)
        pt.set_tiles(parallel.tiles_for_rank(r, 3, W, H, T))
        pt.render()
        parts.append(pt)
    _, s0 = parts[0].film()
    assert 0 < (s0 > 0).sum() < (s_full > 0).sum()  # the root alone has only its own tiles
    mcpt_mod.gather(parts, root=0)
    L, s = parts[0].film()
    assert np.array_equal(s, s_full)
    assert np.array_equal(L.view(np.uint32), L_full.view(np.uint32))
    with pytest.raises(mcpt_mod.McptError):
        mcpt_mod.gather([parts[0], parts[0]], root=0)  # a context listed twice
    for pt in parts + [full]:
        pt.close()


@pytest.mark.parametrize("compact", [False, True])
def test_native_gather_with_a_context_without_tiles(mcpt_mod, scene_c2, compact):
    """More contexts than tiles: a 2 x 1-tile film over three contexts leaves the third
    with an empty tile set.  In the compact layout its path state is empty, and set_tiles, film
    clears, the film readers and render launch nothing (no zero-sized grid).  The gather still
    equals the one-context frame bit for bit.  Tiles gathered into the root cannot become its own
    before a film clear (their sample counts would restart while their radiance accumulates)."""
    from mcpt import parallel

    rc = mcpt_mod.CONFIGS[2]
    W, H, T = 100, 50, 64
    cam = mcpt_mod.config_camera(rc, W, H)
    full = make_pt(mcpt_mod, scene_c2[0], cam, W, H, 2, 5, tile=T)
    full.set_path_slots(2)
    full.render()
    L_full, s_full = full.film()
    parts = []
    for r in range(3):
        pt = make_pt(mcpt_mod, scene_c2[0], cam, W, H, 2, 5, tile=T)
        if compact:
            pt.set_compact_paths(True)
        pt.set_path_slots(2)
        pt.set_tiles(parallel.tiles_for_rank(r, 3, W, H, T))
        pt.clear()
        pt.render()
        parts.append(pt)
    assert parallel.tiles_for_rank(2, 3, W, H, T) == []
    L2, s2 = parts[2].film()  # the empty context's film: all zero
    assert not s2.any() and not L2.any()
    mcpt_mod.gather(parts, root=0)
    L, s = parts[0].film()
    assert np.array_equal(s, s_full) and np.array_equal(L.view(np.uint32), L_full.view(np.uint32))
    if not compact:
        with pytest.raises(mcpt_mod.McptError):
            parts[0].set_tiles([(0, 0), (1, 0)])  # (1, 0) holds pixels gathered from context 1
        parts[0].clear()
        parts[0].set_tiles([(0, 0), (1, 0)])
    for pt in parts + [full]:
        pt.close()


@pytest.mark.parametrize("shade_wgs", [None, "2"])
def test_compact_paths_layout(mcpt_mod, scene_c2, shade_wgs, monkeypatch):
    """mcpt_set_compact_paths: path state over the tile set only (a multi-GPU rank's 1/N).  Films are
    the full layout's bit for bit: the whole tile set in a scrambled order, a partition's tiles with 3
    path slots, the reference's one-tile-per-call loop over the set's tiles, and a partition packed
    and unpacked into a compact root (the RCCL gather's two halves).  Tiles outside the set are
    rejected by mcpt_wavefront_step, duplicates by mcpt_set_tiles; path slots keep the set.  With
    shade_wgs = 2 (MCPT_SHADE_WGS) the compact contexts run k_shade's shading blocks on two
    workgroups (the bounded grid's loop over tile-set blocks and their done flags)."""
    from mcpt import parallel

    rc = mcpt_mod.CONFIGS[2]
    W, H, T = 200, 120, 64  # ragged: the last tile row and column overhang the film
    cam = mcpt_mod.config_camera(rc, W, H)
    full = make_pt(mcpt_mod, scene_c2[0], cam, W, H, 2, 5, tile=T)  # the default grid
    full.set_path_slots(3)
    full.render()
    L0, s0 = full.film()
    if shade_wgs:  # every context created from here on
        monkeypatch.setenv("MCPT_SHADE_WGS", shade_wgs)
    nx, ny = parallel.tile_grid(W, H, T)
    every = [(tx, ty) for ty in range(ny) for tx in range(nx)]
    rng = np.random.default_rng(5)
    scrambled = [every[i] for i in rng.permutation(len(every))]
    pt = make_pt(mcpt_mod, scene_c2[0], cam, W, H, 2, 5, tile=T)
    pt.set_compact_paths(True)
    pt.set_path_slots(3)
    pt.set_tiles(scrambled)
    pt.render()
    L1, s1 = pt.film()
    assert np.array_equal(L0.view(np.uint32), L1.view(np.uint32)) and np.array_equal(s0, s1)
    # one rank of three: its own tiles equal the full frame's, the rest of the film is zero
    mine = parallel.tiles_for_rank(1, 3, W, H, T)
    pt.set_tiles(mine)
    pt.set_path_slots(2)  # keeps the tile set (compact layout)
    pt.set_path_slots(3)
    pt.render()
    L2, s2 = pt.film()
    own = np.zeros((H, W), bool)
    for tx, ty in mine:
        own[ty * T:(ty + 1) * T, tx * T:(tx + 1) * T] = True
    assert np.array_equal(s2[own], s0[own]) and not s2[~own].any()
    assert np.array_equal(L2[own].view(np.uint32), L0[own].view(np.uint32)) and not L2[~own].any()
    # the reference orchestration (one tile per call) over the set's tiles, one slot
    ref = make_pt(mcpt_mod, scene_c2[0], cam, W, H, 2, 5, tile=T)
    ref.set_compact_paths(True)
    ref.set_tiles(mine)
    for it in range(40 * len(mine)):
        ref.step(*mine[it % len(mine)])
    L3, s3 = ref.film()
    full.set_path_slots(1)
    full.render()
    Lf1, sf1 = full.film()
    assert np.array_equal(s3[own], sf1[own]) and np.array_equal(L3[own].view(np.uint32), Lf1[own].view(np.uint32))
    other = next(t for t in every if t not in mine)
    with pytest.raises(mcpt_mod.McptError):
        ref.step(*other)
    with pytest.raises(mcpt_mod.McptError):
        ref.set_tiles([mine[0], mine[0]])
    # pack on this rank, unpack into a compact root that owns the other tiles (mcpt/parallel.py's
    # gather without the transport): the root's film is then the whole frame
    import ctypes as C

    import torch

    root = make_pt(mcpt_mod, scene_c2[0], cam, W, H, 2, 5, tile=T)
    root.set_compact_paths(True)
    root.set_path_slots(3)
    root.set_tiles([t for t in every if t not in mine])
    root.render()
    n = C.c_uint32()
    lib = mcpt_mod.lib()
    assert lib.mcpt_film_pack_tiles(pt.h, None, C.byref(n)) == 0 and n.value == len(mine) * T * T
    buf = torch.empty((n.value, 4), dtype=torch.float32, device="cuda")
    assert lib.mcpt_film_pack_tiles(pt.h, C.c_void_p(buf.data_ptr()), C.byref(n)) == 0
    xy = np.ascontiguousarray(mine, np.uint32).reshape(-1, 2)
    assert lib.mcpt_film_unpack_tiles(root.h, C.c_void_p(buf.data_ptr()), xy.ctypes.data_as(C.POINTER(C.c_uint32)),
                                      len(mine)) == 0
    L4, s4 = root.film()
    assert np.array_equal(L0.view(np.uint32), L4.view(np.uint32)) and np.array_equal(s0, s4)
    root.clear()  # a film clear empties the unpacked pixels too
    _, s5 = root.film()
    assert not s5.any()
    for p in (full, pt, ref, root):
        p.close()


@pytest.mark.parametrize("gpu_bvh", [False, "ploc"])
@pytest.mark.parametrize("which", ["scene_c1", "scene_c2", "scene_cube", "scene_c3"])
def test_quad_nodes_same_hits(request, mcpt_mod, oracle, which, gpu_bvh):
    """4-wide nodes (the default for trees beyond L2; MCPT_BVH_WIDTH=4 forces them here): the
    collapse copies boxes, never recomputes them, so hits stay bit-identical to the oracle's."""
    s, a = request.getfixturevalue(which)
    old = os.environ.get("MCPT_BVH_WIDTH")
    os.environ["MCPT_BVH_WIDTH"] = "4"
    try:
        pt = mcpt_mod.PathTracer(0)
        pt.upload_scene(s, gpu_bvh=gpu_bvh)
    finally:
        if old is None:
            os.environ.pop("MCPT_BVH_WIDTH", None)
        else:
            os.environ["MCPT_BVH_WIDTH"] = old
    n = 20000 if which == "scene_c3" else 100000
    ro, rd = random_rays(n, 41, box=2.5)
    if which == "scene_c3":
        ro[:, 1] += 1.0
    ro[:4] = [[0, 0, 5], [0, 0, 5], [0, 0, 5], [0, 0, 1]]
    rd[:4] = [[np.nan, 0, -1], [0, 0, 0], [0, 0, -1], [1, 0, 0]]
    gp, gn, gt = pt.trace_closest(ro, rd)
    op_, on, ot = oracle.trace_closest(a, ro, rd)
    assert np.array_equal(gt, ot)
    assert np.array_equal(gp.view(np.uint32), op_.view(np.uint32))
    assert np.array_equal(gn.view(np.uint32), on.view(np.uint32))
    assert np.array_equal(pt.trace_any(ro, rd), oracle.trace_any(a, ro, rd))
    if which == "scene_c2":  # a film through the 4-wide traversal
        rc = mcpt_mod.CONFIGS[2]
        W, H = 160, 90
        cam = mcpt_mod.config_camera(rc, W, H)
        pt.close()
        os.environ["MCPT_BVH_WIDTH"] = "4"
        try:
            pt = make_pt(mcpt_mod, s, cam, W, H, 3, rc.max_depth)
        finally:
            if old is None:
                os.environ.pop("MCPT_BVH_WIDTH", None)
            else:
                os.environ["MCPT_BVH_WIDTH"] = old
        pt.render()
        Ld, smp = pt.film()
        rL, rs, _ = oracle.render(a, cam, W, H, 3, rc.max_depth)
        assert np.array_equal(smp, rs)
        assert np.array_equal(Ld.view(np.uint32), rL.view(np.uint32))
    pt.close()


def _nan_equal(x, y):
    """bitwise, except that NaNs only need to be NaN on both sides (x86's 0/0 is -NaN, gfx950's +NaN;
    the tables' consumers only compare against them)"""
    return bool(((x.view(np.uint32) == y.view(np.uint32)) | (np.isnan(x) & np.isnan(y))).all())


def _env_only(a, tex):
    b = dict(a)
    b["env_tex"] = np.ascontiguousarray(tex, np.float32)
    for k in ("env_marginal_y", "env_conds_y", "env_pdf"):
        b[k] = np.zeros(0, np.float32)
    return b


@pytest.mark.parametrize("shape", ["c2", (77, 300), (77, 301), (512, 1024), "zeros", "spike"])
def test_env_tables_built_on_device_equal_oracle(mcpt_mod, oracle, scene_c2, shape):
    """build_environment_light (light_initialization_kernels.cu:3-161) on the device: marginal,
    conditional and pdf tables equal the oracle's or_env_build for the config-2 map and synthetic
    ones (odd sizes, an all-zero map whose tables are NaN, one dominant texel)."""
    _, a = scene_c2
    rng = np.random.default_rng(5)
    if shape == "c2":
        tex = a["env_tex"]
    elif shape == "zeros":
        tex = np.zeros((64, 128, 4), np.float32)
    elif shape == "spike":
        tex = rng.uniform(0, 0.01, (128, 256, 4)).astype(np.float32)
        tex[40, 17, :3] = 5e4
    else:
        tex = (rng.lognormal(0, 2, shape + (4,)) * (rng.uniform(size=shape + (1,)) > 0.2)).astype(np.float32)
    H, W = tex.shape[:2]
    pt = mcpt_mod.PathTracer(0)
    pt.upload_scene(mcpt_mod.desc_from_arrays(_env_only(a, tex)))
    got = pt.env_tables(W, H)
    ref = oracle.env_build(tex)
    assert got["device_built"]
    for k in ("marginal_y", "conds_y", "pdf"):
        assert _nan_equal(got[k], ref[k]), k
    # guides: on for real maps (row 0 is NaN throughout: 0 / (denom * 0)), off for the NaN tables
    assert got["guides"] == (shape != "zeros")
    assert pt.last_env_build_ms > 0
    pt.close()


def test_env_device_tables_same_film(mcpt_mod, scene_c2):
    """Config-2 film with the HRDI tables built on the device equals the host-table film bit for bit
    (and host tables uploaded as given read back unchanged)."""
    s, a = scene_c2
    rc = mcpt_mod.CONFIGS[2]
    W, H = 160, 90
    cam = mcpt_mod.config_camera(rc, W, H)
    films = []
    for desc in (s, mcpt_mod.desc_from_arrays(_env_only(a, a["env_tex"]))):
        pt = make_pt(mcpt_mod, desc, cam, W, H, 4, rc.max_depth)
        t = pt.env_tables(a["env_tex"].shape[1], a["env_tex"].shape[0])
        assert t["guides"]
        if desc is s:
            assert not t["device_built"]
            for k in ("marginal_y", "conds_y", "pdf"):
                assert np.array_equal(t[k].view(np.uint32), a["env_" + k].view(np.uint32))
        pt.render()
        films.append(pt.film())
        pt.close()
    (L0, s0), (L1, s1) = films
    assert np.array_equal(s0, s1) and np.array_equal(L0.view(np.uint32), L1.view(np.uint32))


def _same(a, b):
    a, b = np.asarray(a), np.asarray(b)
    if a.dtype.kind == "f":
        return bool(np.array_equal(a.view(np.uint32), b.view(np.uint32)) or
                    np.array_equal(np.isnan(a), np.isnan(b)) and np.array_equal(a[~np.isnan(a)], b[~np.isnan(b)]))
    return bool(np.array_equal(a, b))


@pytest.mark.parametrize("scene", ["c1dir", "c2"])
@pytest.mark.parametrize("stage", ["logic", "generate", "material"])
def test_stage_golden_vectors(mcpt_mod, oracle, stage, scene):
    """Per-stage golden vectors: mcpt_stage_run runs the product's
    k_shade (LOGIC / GENERATE: wf_logic + wf_generate, wavefront_kernels.cu:90-251) or k_material
    (MATERIAL: light choice + wf_mat_mix, :207-213, 295-375) on the fixture's path state; every
    output field equals the oracle's stage restatement (tools/make_golden.py) bit for bit, on two
    fixture scenes (config 1's sphere, config 2's room; stage_fixtures.SCENES).  Rays the kernels
    resolve in place because they cannot hit the scene are checked against the oracle's traversal
    instead of a queue entry."""
    import stage_fixtures as sf

    cid = sf.SCENES[scene]
    g = np.load(os.path.join(GOLDEN, f"stage_{stage}_{scene}.npz"))
    inp = {k[3:]: g[k] for k in g.files if k.startswith("in_")}
    ref = {k[4:]: g[k] for k in g.files if k.startswith("out_")}
    s = sf.stage_scene(mcpt_mod, cid)
    a = s.arrays()
    pt = mcpt_mod.PathTracer(0, mcpt_mod.default_config(spp=sf.SPP, max_depth=sf.DEPTH, rr_depth=sf.RR))
    pt.upload_scene(s)
    pt.set_camera(sf.stage_camera(mcpt_mod, cid))
    got = pt.stage(stage, inp, film=sf.FILM if stage != "material" else None)
    pt.close()
    _check_stage(stage, got, ref, a, oracle)


@pytest.mark.gpu
def test_stage_logic_rejects_inconsistent_sample_index(mcpt_mod):
    """The device derives a path's sample count from the sample index its flags word carries (a dead
    path keeps its next one: DESIGN.md section 3), so LOGIC input where a live path's index differs
    from its samples -- a state neither the reference nor the oracle produces -- fails loudly; dead
    paths come back with the interface's F_DEAD-only flags."""
    import stage_fixtures as sf

    s = sf.stage_scene(mcpt_mod)
    a = s.arrays()
    pt = mcpt_mod.PathTracer(0, mcpt_mod.default_config(spp=sf.SPP, max_depth=sf.DEPTH, rr_depth=sf.RR))
    pt.upload_scene(s)
    pt.set_camera(sf.stage_camera(mcpt_mod))
    inp = sf.logic_state(len(a["mat"]))
    live = np.flatnonzero((inp["flags"] & 1) == 0)
    bad = dict(inp)
    bad["samples"] = inp["samples"].copy()
    bad["samples"][live[0]] += 1
    with pytest.raises(mcpt_mod.McptError):
        pt.stage("logic", bad, film=sf.FILM)
    got = pt.stage("logic", inp, film=sf.FILM)
    dead = (got["flags"] & 1) == 1
    assert dead.any() and np.all(got["flags"][dead] == 1)
    pt.close()


def _check_stage(stage, got, ref, a, oracle):
    """mcpt_stage_run outputs against the oracle's stage restatement, field by field, bit for bit."""
    if stage in ("logic", "generate"):
        for k in ("flags", "samples", "Ld"):
            assert _same(got[k], ref[k]), k
        cont = (ref["queued"] & 2) > 0
        assert np.array_equal((got["queued"] & 2) > 0, cont)
        assert _same(got["beta"][cont, :3], ref["beta"][cont, :3])
        gen = (ref["queued"] & 1) > 0
        assert gen.sum() > 50 and (stage == "generate" or cont.sum() > 50)
        assert _same(got["ray_o"][gen], ref["ray_o"][gen]) and _same(got["ray_d"][gen], ref["ray_d"][gen])
        queued = (got["queued"] & 1) > 0
        assert not queued[~gen].any()
        resolved = gen & ~queued  # camera rays missing the scene: resolved in place, never queued
        assert np.all(got["hit_tri"][resolved] == -1)
        if resolved.any():
            assert np.all(oracle.trace_closest(a, ref["ray_o"][resolved], ref["ray_d"][resolved])[2] == -1)
    else:
        for k in ("flags", "ray_o", "ray_d", "beta", "nee0", "nee1"):
            assert _same(got[k], ref[k]), k
        q = got["queued"]
        ext_resolved = (q & 1) == 0
        if ext_resolved.any():
            assert np.all(got["hit_tri"][ext_resolved] == -1)
            assert np.all(oracle.trace_closest(a, ref["ray_o"][ext_resolved], ref["ray_d"][ext_resolved])[2] == -1)
        for bit, vk, o_k, d_k in ((4, 0, "light_o", "light_d"), (8, 1, "bvis_o", "bvis_d")):
            drawn = ~np.isnan(ref[o_k][:, 0])
            qd = (q & bit) > 0
            assert not qd[~drawn].any()
            assert _same(got[o_k][qd], ref[o_k][qd]) and _same(got[d_k][qd], ref[d_k][qd])
            res = drawn & ~qd  # resolved in place: visible
            assert np.all(got["vis"][res, vk] == 1)
            if res.any():
                assert np.all(oracle.trace_any(a, ref[o_k][res], ref[d_k][res]) == 1)
        assert (q & 4).sum() > 50 and (q & 8).sum() > 20 and np.isnan(ref["bvis_o"][:, 0]).sum() > 50


@pytest.mark.parametrize("stage", ["logic", "generate", "material"])
def test_stage_fixed_mode_vs_oracle(mcpt_mod, oracle, stage):
    """The quality-mode integrator (MCPT_FLAG_FIXED, Appendix A) stage by stage: the same fixture
    states through mcpt_stage_run on a FIXED context, against the oracle's stage restatement in
    fixed mode computed here (no committed vector: the mode is an alternative, not reference
    parity).  RR survivors reweighted, 1/N light pick, delta-light MIS weight 1, clamped env cells."""
    import stage_fixtures as sf

    s = sf.stage_scene(mcpt_mod)
    a = s.arrays()
    cam = sf.stage_camera(mcpt_mod)
    kw = dict(max_depth=sf.DEPTH, rr_depth=sf.RR, fixed=True)
    if stage == "material":
        inp = sf.material_state(a, oracle.trace_closest)
        ref = oracle.stage_material(a, inp, **kw)
    else:
        inp = sf.logic_state(len(a["mat"]), stage == "generate")
        ref = oracle.stage_logic(a, cam, sf.FILM[0], sf.FILM[1], inp, sf.SPP, **kw)
    pt = mcpt_mod.PathTracer(0, mcpt_mod.default_config(spp=sf.SPP, max_depth=sf.DEPTH, rr_depth=sf.RR, fixed=True))
    pt.upload_scene(s)
    pt.set_camera(cam)
    got = pt.stage(stage, inp, film=sf.FILM if stage != "material" else None)
    pt.close()
    _check_stage(stage, got, ref, a, oracle)


def test_bvh_without_containment_disables_cull_and_cache(mcpt_mod, oracle, scene_c2):
    """A caller-supplied BVH whose boxes do not contain their subtrees (here: an interior node's box
    shrunk by a fifth per side, so some of its triangles stick out): the occluder cache's lemma
    and the culling bound both assume containment, so mcpt_scene_upload turns
    both off.  Hits then still equal the oracle's traversal of the same boxes, and films are
    bit-identical with the cache requested (default) and switched off (MCPT_OCC_G=0)."""
    _, a0 = scene_c2
    a = {k: (v.copy() if isinstance(v, np.ndarray) else v) for k, v in a0.items()}
    inner = np.nonzero(a["nprims"] == 0)[0]
    n = int(inner[1])  # an interior node below the root
    lo, hi = a["bmin"].reshape(-1, 3)[n].copy(), a["bmax"].reshape(-1, 3)[n].copy()
    ext = hi - lo
    a["bmin"].reshape(-1, 3)[n] = lo + 0.2 * ext
    a["bmax"].reshape(-1, 3)[n] = hi - 0.2 * ext
    d = mcpt_mod.desc_from_arrays(a)
    pt = mcpt_mod.PathTracer(0)
    pt.upload_scene(d)
    ro, rd = random_rays(100000, 33)
    gp, gn, gt = pt.trace_closest(ro, rd)
    op_, on, ot = oracle.trace_closest(a, ro, rd)
    assert np.array_equal(gt, ot)
    assert np.array_equal(gp.view(np.uint32), op_.view(np.uint32))
    assert np.array_equal(pt.trace_any(ro, rd), oracle.trace_any(a, ro, rd))
    pt.close()

    W, H = 160, 90
    cam = mcpt_mod.config_camera(mcpt_mod.CONFIGS[2], W, H)

    def run(env):
        old = os.environ.get("MCPT_OCC_G")
        if env is None:
            os.environ.pop("MCPT_OCC_G", None)
        else:
            os.environ["MCPT_OCC_G"] = env
        try:
            p = make_pt(mcpt_mod, d, cam, W, H, 24, 5, tile=64)
        finally:
            if old is None:
                os.environ.pop("MCPT_OCC_G", None)
            else:
                os.environ["MCPT_OCC_G"] = old
        p.set_path_slots(2)
        p.clear()
        st = p.render()
        L, smp = p.film()
        out = (L.copy(), smp.copy(), (st.extend_rays, st.shadow_rays, st.vis_rays), p.occ_stats())
        p.close()
        return out

    off, on = run("0"), run(None)
    assert on[3] == (0, False), "the occluder cache must be off for a BVH that breaks containment"
    assert np.array_equal(on[0].view(np.uint32), off[0].view(np.uint32))
    assert np.array_equal(on[1], off[1]) and on[2] == off[2]
