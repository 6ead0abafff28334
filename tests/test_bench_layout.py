"""Parity at the bench's own layout, for every GPU BASELINE config.

bench.py renders each config's full frame with BENCH_SLOTS path slots per pixel (several paths
in flight per pixel, each slot accumulating its own samples).  Here the GPU renders exactly that
layout -- full resolution, the bench's slot count, the config's depth -- to high sample counts
(config 1 whole, 16 spp at its 16 slots; 256 spp for configs 2 and 3, as benched; 16 spp for
configs 4 and 5 over the whole frame, and their full 1024 / 4096 spp on ten tiles spread over the
frame, test_full_spp_tiles_against_oracle), and a band of rows re-executed by the oracle (one path per pixel, the
reference's layout: wavefront_kernels.cu:90-375) must agree: sample counts exactly, radiance within
the north star's 1e-4 relative (the slots only change the film's summation order).  High sample
indices, Russian roulette at depth and the slots' interleaved sample chains are all exercised.
"""
import os
import sys
import time

import numpy as np
import pytest

from conftest import REPO

sys.path.insert(0, REPO)
import bench  # noqa: E402  (BENCH_SLOTS: the layout under test is the bench's)

pytestmark = pytest.mark.gpu
RTOL = 1e-4


def film_close(g, c):
    tol = RTOL * np.maximum(np.abs(g), np.abs(c)) + 1e-7
    ok = (np.abs(g - c) <= tol) | (np.isnan(g) & np.isnan(c))
    return bool(ok.all()), int((~ok).sum())


@pytest.mark.parametrize("cid,spp,rows", [(1, 16, (0, 255)), (2, 256, (536, 540)), (3, 256, (600, 604)),
                                          (4, 16, (1078, 1082)), (5, 16, (2046, 2049))],
                         ids=["config1", "config2", "config3", "config4", "config5"])
def test_bench_layout_band_parity(request, mcpt_mod, oracle, cid, spp, rows):
    rc = mcpt_mod.CONFIGS[cid]
    slots = bench.BENCH_SLOTS[cid]
    if cid in (1, 2, 3):
        scene, arrays = request.getfixturevalue(f"scene_c{cid}")
    else:
        scene = mcpt_mod.build_config_scene(cid)
        arrays = scene.arrays()
    cam = mcpt_mod.config_camera(rc)
    pt = mcpt_mod.PathTracer(0, mcpt_mod.default_config(spp=spp, max_depth=rc.max_depth))
    pt.upload_scene(scene)
    pt.set_camera(cam)
    pt.set_path_slots(slots)
    pt.resize(rc.width, rc.height)
    t0 = time.perf_counter()
    st = pt.render()
    t_gpu = time.perf_counter() - t0
    assert st.live_paths == 0
    Ld, smp = pt.film()
    pt.close()
    # every rendered pixel has all its samples (last row / column never rendered: :110)
    assert np.all(smp[:-1, :-1] == spp) and not smp[-1].any() and not smp[:, -1].any()
    r0, r1 = rows
    t0 = time.perf_counter()
    rL, rs, cnt = oracle.render(arrays, cam, rc.width, rc.height, spp, rc.max_depth, rows=(r0, r1))
    t_cpu = time.perf_counter() - t0
    assert np.array_equal(smp[r0:r1], rs[r0:r1])
    ok, nbad = film_close(Ld[r0:r1], rL[r0:r1])
    assert ok, f"{nbad} radiance values differ"
    assert np.isfinite(Ld[r0:r1]).all() and Ld[r0:r1].max() > 0
    # RR and the deepest vertices were reached in the band (the oracle counts the rays it traced)
    assert cnt["extend_rays"] > (r1 - r0) * (rc.width - 1) * spp
    print(f"config {cid}: {rc.width}x{rc.height} {spp} spp {slots} slots: GPU frame {t_gpu:.2f} s "
          f"({st.rays / t_gpu / 1e6:.0f} Mray/s), oracle rows {r0}-{r1} {t_cpu:.1f} s")


def test_bench_layout_config2_scattered_rows(mcpt_mod, oracle, scene_c2):
    """The benched frame itself (config 2, 1080p, 256 spp, the bench's slots) against the oracle
    on eight single rows spread from the top edge to the last rendered row: sky-only rows, the
    box walls, the spheres and the floor, each with its own path-length mix."""
    rc = mcpt_mod.CONFIGS[2]
    scene, arrays = scene_c2
    cam = mcpt_mod.config_camera(rc)
    pt = mcpt_mod.PathTracer(0, mcpt_mod.default_config(spp=rc.spp, max_depth=rc.max_depth))
    pt.upload_scene(scene)
    pt.set_camera(cam)
    pt.set_path_slots(bench.BENCH_SLOTS[2])
    pt.resize(rc.width, rc.height)
    pt.render()
    Ld, smp = pt.film()
    pt.close()
    for r in (0, 135, 270, 405, 675, 810, 945, rc.height - 2):
        rL, rs, _ = oracle.render(arrays, cam, rc.width, rc.height, rc.spp, rc.max_depth, rows=(r, r + 1))
        assert np.array_equal(smp[r], rs[r]), r
        ok, nbad = film_close(Ld[r:r + 1], rL[r:r + 1])
        assert ok, f"row {r}: {nbad} radiance values differ"


@pytest.mark.parametrize("cid,tiles", [(4, [(7, 4), (3, 2), (0, 0), (14, 8), (10, 6), (5, 7)]),
                                       (5, [(8, 8), (0, 0), (15, 15), (4, 11)])], ids=["config4", "config5"])
def test_full_spp_tiles_against_oracle(mcpt_mod, oracle, cid, tiles):
    """Configs 4 and 5 at their full sample counts -- 1024 spp depth 8, 4096 spp depth 12 -- at the
    bench's path slots (24: slot k renders samples k, k + 24, ..., 42-43 / 170-171 of them, sample
    indices up to 4095 keyed into the RNG, wavefront_kernels.cu:124,219-222) on whole 256 x 256
    tiles (mcpt_set_tiles) spread over the frame -- corners, the centre, sky and geometry, the
    bottom-right tiles with the never-rendered last row and column (:110) and config 4's partial
    bottom tile row -- two rows of each tile against the oracle (the one tile alone: part=(tx + ty,
    a modulus larger than any tx + ty))."""
    rc = mcpt_mod.CONFIGS[cid]
    scene = mcpt_mod.build_config_scene(cid)
    arrays = scene.arrays()
    cam = mcpt_mod.config_camera(rc)
    pt = mcpt_mod.PathTracer(0, mcpt_mod.default_config(spp=rc.spp, max_depth=rc.max_depth))
    pt.upload_scene(scene)
    pt.set_camera(cam)
    pt.set_path_slots(bench.BENCH_SLOTS[cid])
    pt.resize(rc.width, rc.height)
    pt.set_tiles(tiles)
    t0 = time.perf_counter()
    st = pt.render()
    t_gpu = time.perf_counter() - t0
    Ld, smp = pt.film()
    pt.close()
    big = rc.width // 256 + rc.height // 256 + 2
    W, H = rc.width, rc.height
    lit = 0
    for tx, ty in tiles:
        y0, y1, x0, x1 = ty * 256, min((ty + 1) * 256, H), tx * 256, min((tx + 1) * 256, W)
        want = np.full((y1 - y0, x1 - x0), rc.spp, np.uint32)
        if y1 == H:
            want[-1] = 0  # the last row and column are never rendered (wavefront_kernels.cu:110)
        if x1 == W:
            want[:, -1] = 0
        assert np.array_equal(smp[y0:y1, x0:x1], want)
        for r in (y0 + 40, min(y0 + 200, H - 2)):
            t0 = time.perf_counter()
            rL, rs, cnt = oracle.render(arrays, cam, W, H, rc.spp, rc.max_depth, rows=(r, r + 1), part=(tx + ty, big))
            t_cpu = time.perf_counter() - t0
            cols = slice(x0, x1)
            assert np.array_equal(smp[r, cols], rs[r, cols]) and rs[r].sum() == want[r - y0].sum()
            ok, nbad = film_close(Ld[r, cols], rL[r, cols])
            assert ok, f"config {cid} tile {(tx, ty)} row {r}: {nbad} radiance values differ"
            lit += int(Ld[r, cols].max() > 0)
            print(f"config {cid} tile {(tx, ty)} row {r}: {rc.spp} spp, {cnt['extend_rays']} oracle extension rays "
                  f"({t_cpu:.1f} s); GPU tiles {t_gpu:.2f} s, {st.rays} rays")
    assert lit >= len(tiles)  # most checked rows carry light
