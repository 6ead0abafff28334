"""CPU tests: pin the oracle (oracle/) before trusting it.

Pins available for this reference (no tests, no golden vectors, not buildable here):
  * its only self-check, sum(env pdf) ~= 1 (light_initialization_kernels.cu:113-133);
  * the README BRDF formulas (README.md:74-124) evaluated independently in float64 numpy;
  * lowerbias32 (cuda_math/Random.cu:5-13) re-derived in numpy;
  * glibc float64 transcendentals for the deterministic replacements of CUDA fast-math;
  * brute-force ray casting (no BVH) for the traversal;
  * committed golden fixtures (tests/golden, tools/make_golden.py) against regressions.
"""
import os

import numpy as np
import pytest

from conftest import ASSETS, GOLDEN

pytestmark = []


def ulp_diff(a, b):
    a = np.asarray(a, np.float32).view(np.int32).astype(np.int64)
    b = np.asarray(b, np.float32).view(np.int32).astype(np.int64)
    a = np.where(a < 0, -(a & 0x7FFFFFFF), a)
    b = np.where(b < 0, -(b & 0x7FFFFFFF), b)
    return np.abs(a - b)


# ---------------------------------------------------------------- RNG
def np_lowerbias32(x):
    x = np.asarray(x, np.uint64) & 0xFFFFFFFF
    x ^= x >> 16
    x = (x * 0xA812D533) & 0xFFFFFFFF
    x ^= x >> 15
    x = (x * 0xB278E4AD) & 0xFFFFFFFF
    x ^= x >> 17
    return x


def py_splitmix64(z):
    M = (1 << 64) - 1
    z = (z + 0x9E3779B97F4A7C15) & M
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M
    return z ^ (z >> 31)


def test_lowerbias32_matches_reference_formula(oracle):
    xs = np.random.default_rng(0).integers(0, 2**32, 2000, dtype=np.uint64)
    want = np_lowerbias32(xs)
    got = np.array([oracle.lib().or_lowerbias32(int(x)) for x in xs], np.uint64)
    assert np.array_equal(got, want)


def test_keyed_rng_appendix_b(oracle):
    seed = 0x5EED2026
    for pixel, sample, ln, slot in [(0, 0, 0, 0), (12345, 7, 3, 9), (2**31, 255, 13, 15), (99, 1, 1, 1)]:
        s = py_splitmix64((pixel << 32 | sample) ^ seed)
        key = (s ^ (s >> 32)) & 0xFFFFFFFF
        d = int(np_lowerbias32((key + (ln * 16 + slot) * 0x9E3779B9) & 0xFFFFFFFF))
        want = np.float32(np.float64(d) * 2.0**-32)   # Random.cu:34 double scaling, float return
        assert oracle.lib().or_rand(seed, pixel, sample, ln, slot) == want
    # rand_float can round to exactly 1.0f (draw = 0xFFFFFFFF)
    assert np.float32(np.float64(0xFFFFFFFF) * 2.0**-32) == np.float32(1.0)


# ---------------------------------------------------------------- transcendentals
@pytest.mark.parametrize("fn,ref,lo,hi,bound", [
    ("or_sinf", np.sin, -10.0, 10.0, 4), ("or_cosf", np.cos, -10.0, 10.0, 4),
    ("or_asinf", np.arcsin, -1.0, 1.0, 3), ("or_acosf", np.arccos, -1.0, 1.0, 3)])
def test_transcendentals_vs_glibc(oracle, fn, ref, lo, hi, bound):
    xs = np.random.default_rng(1).uniform(lo, hi, 20000).astype(np.float32)
    f = getattr(oracle.lib(), fn)
    got = np.array([f(float(x)) for x in xs], np.float32)
    want = ref(xs.astype(np.float64)).astype(np.float32)
    # absolute error near zeros of sin/cos, ULPs elsewhere
    big = np.abs(want) > 1e-3
    assert ulp_diff(got[big], want[big]).max() <= bound
    assert np.abs(got - want).max() < 2e-6


def test_atan2_vs_glibc_and_special_cases(oracle):
    rng = np.random.default_rng(2)
    y = rng.normal(size=20000).astype(np.float32)
    x = rng.normal(size=20000).astype(np.float32)
    f = oracle.lib().or_atan2f
    got = np.array([f(float(a), float(b)) for a, b in zip(y, x)], np.float32)
    want = np.arctan2(y.astype(np.float64), x.astype(np.float64)).astype(np.float32)
    assert np.abs(got - want).max() < 1e-6
    assert f(0.0, 1.0) == 0.0 and f(1.0, 0.0) == np.float32(np.pi / 2) and f(-1.0, 0.0) == -np.float32(np.pi / 2)
    assert f(0.0, -1.0) == np.float32(np.pi) and f(-0.0, -1.0) == -np.float32(np.pi)
    assert np.isnan(f(float("nan"), 1.0)) and np.isnan(oracle.lib().or_sinf(float("nan")))


# ---------------------------------------------------------------- BRDF vs README formulas
def readme_brdf(base, n, wi, wo, r=1.0, m=0.0, f0s=0.04):
    """README.md:74-124 (GGX NDF, Schlick-GGX G with k = a/2, Schlick F), float64; the reference
    folds the cosine into f (dMaterial.cu:275, :340) and clamps with eps = 1e-5."""
    eps = 1e-5
    n, wi, wo = (np.asarray(v, np.float64) for v in (n, wi, wo))
    h = (wo + wi) / np.linalg.norm(wo + wi)
    a = r * r
    a2 = a * a
    ndh = max(n @ h, eps)
    D = a2 / (np.pi * max(ndh * ndh * (a2 - 1) + 1, eps) ** 2)
    k = a / 2

    def g1(v):
        nv = max(n @ v, eps)
        return nv / max(nv * (1 - k) + k, eps)

    f0 = np.full(3, f0s) * (1 - m) + np.asarray(base, np.float64) * m
    F = f0 + (1 - f0) * (1 - max(h @ wo, 0.0)) ** 5
    ndwi, ndwo = max(n @ wi, eps), max(n @ wo, eps)
    spec = D * g1(wi) * g1(wo) * F * ndwi / max(4 * ndwo * ndwi, eps)
    diff = (1 - F) * (1 - m) * np.asarray(base, np.float64) * ndwi / np.pi
    pdf_spec = D * max(h @ n, eps) / max(4 * max(wo @ h, eps), eps)
    return spec, diff, pdf_spec, 1 / (2 * np.pi)


@pytest.mark.parametrize("rough,metal", [(1.0, 0.0), (0.5, 0.0), (0.3, 1.0), (0.8, 0.5)])
def test_brdf_matches_readme(oracle, rough, metal):
    rng = np.random.default_rng(3)
    for _ in range(200):
        n = rng.normal(size=3); n /= np.linalg.norm(n)
        wi = rng.normal(size=3); wi /= np.linalg.norm(wi)
        wo = rng.normal(size=3); wo /= np.linalg.norm(wo)
        if n @ wi < 0.05 or n @ wo < 0.05:
            continue
        base = rng.uniform(0.05, 1.0, 3)
        params = np.array([*base, 0.04, 0.04, 0.04, rough, metal], np.float32)
        out = np.zeros(8, np.float32)
        f32 = lambda v: np.asarray(v, np.float32)
        oracle.lib().or_brdf_eval(oracle.fptr(params), oracle.fptr(f32(n)), oracle.fptr(f32(wi)), oracle.fptr(f32(wo)), oracle.fptr(out))
        spec, diff, ps, pd = readme_brdf(base.astype(np.float32), f32(n), f32(wi), f32(wo), np.float32(rough), np.float32(metal))
        np.testing.assert_allclose(out[0:3], spec, rtol=2e-4, atol=1e-7)
        np.testing.assert_allclose(out[3:6], diff, rtol=2e-4, atol=1e-7)
        np.testing.assert_allclose(out[6], ps, rtol=2e-4)
        np.testing.assert_allclose(out[7], pd, rtol=1e-6)


def test_power_heuristic(oracle):
    ph = oracle.lib().or_power_heuristic
    assert ph(1.0, 1.0) == np.float32(0.5)
    assert ph(3.0, 4.0) == np.float32(9.0 / 25.0)
    assert ph(2.0, 0.0) == 1.0 and ph(0.0, 2.0) == 0.0
    assert np.isnan(ph(0.0, 0.0))          # 0/0: fails 'weight > 0' in wf_logic


def test_upper_bound_semantics(oracle):
    ub = lambda lst, v: oracle.lib().or_upper_bound(oracle.fptr(np.asarray(lst, np.float32)), len(lst), v)
    lst = [0.0, 0.1, 0.1, 0.5, 1.0]
    assert ub(lst, -1.0) == 0 and ub(lst, 0.0) == 1 and ub(lst, 0.1) == 3 and ub(lst, 0.3) == 3
    assert ub(lst, 1.0) == 5 and ub(lst, 2.0) == 5
    nan_row = [float("nan")] * 4     # conditional row 0 (sin(0)=0 -> 0/0): x = -1 quirk
    assert ub(nan_row, 0.5) == 0


# ---------------------------------------------------------------- env light tables
def test_env_tables_reference_selfcheck(scene_c1, oracle):
    """g_test (light_initialization_kernels.cu:113-133) prints sum(pdf) ~= 1."""
    _, a = scene_c1
    assert abs(float(a["env_pdf"].sum(dtype=np.float64)) - 1.0) < 1e-3
    assert abs(float(a["env_marginal_y"][-1]) - 1.0) < 1e-3
    assert a["env_marginal_y"][0] == 0.0           # sin(0) row: y >= 0 always when sampling
    rows = a["env_conds_y"][1:, -1]
    assert np.all(np.abs(rows - 1.0) < 1e-3)
    assert np.all(np.isnan(a["env_conds_y"][0]))   # 0/(denom*0): reference quirk kept


def test_env_tables_product_equals_oracle_bitwise(scene_c1, scene_c2, oracle):
    for _, a in (scene_c1, scene_c2):
        e = oracle.env_build(a["env_tex"])
        for k in ("marginal_y", "conds_y", "pdf"):
            assert np.array_equal(e[k].view(np.uint32), a["env_" + k].view(np.uint32)), k


def decode_hdr_py(path):
    """Independent Radiance RGBE decoder (stb_image semantics: rgb * 2^(e-136))."""
    b = open(path, "rb").read()
    p = b.index(b"\n\n") + 2
    e = b.index(b"\n", p)
    _, H, _, W = b[p:e].split()
    H, W = int(H), int(W)
    p = e + 1
    out = np.zeros((H, W, 3), np.float32)
    for y in range(H):
        assert b[p] == 2 and b[p + 1] == 2
        p += 4
        sc = np.zeros((4, W), np.uint8)
        for c in range(4):
            x = 0
            while x < W:
                n = b[p]; p += 1
                if n > 128:
                    sc[c, x:x + n - 128] = b[p]; p += 1; x += n - 128
                else:
                    sc[c, x:x + n] = np.frombuffer(b[p:p + n], np.uint8); p += n; x += n
        ex = sc[3].astype(np.int32)
        f = np.where(ex > 0, np.ldexp(np.float32(1.0), ex - 136), 0).astype(np.float32)
        out[y] = (sc[:3].T.astype(np.float32) * f[:, None])
    return out


def test_hdr_decode_matches_independent_decoder(scene_c1):
    _, a = scene_c1
    ref = decode_hdr_py(os.path.join(ASSETS, "HDR_029_Sky_Cloudy_Env.hdr"))
    assert a["env_tex"].shape == (256, 512, 4)
    assert np.array_equal(a["env_tex"][..., :3], ref)
    assert np.all(a["env_tex"][..., 3] == 0)


# ---------------------------------------------------------------- scene loading / BVH
def test_sphere_glb(scene_c1):
    _, a = scene_c1
    assert len(a["mat"]) == 960
    for k in ("v0", "v1", "v2"):
        r = np.linalg.norm(a[k], axis=1)
        assert r.max() <= 1.0 + 1e-6 and r.min() > 0.99
    for k in ("n0", "n1", "n2"):
        assert np.abs(np.linalg.norm(a[k], axis=1) - 1).max() < 1e-5
    assert np.array_equal(a["mat_params"][0], np.array([1, 1, 1, .04, .04, .04, 1, 0], np.float32))


def test_bvh_structure(scene_c2):
    s, a = scene_c2
    n = len(a["nprims"])
    leaves = a["nprims"] > 0
    assert a["nprims"].max() <= 8
    covered = np.zeros(len(a["mat"]), np.int32)
    for o, c in zip(a["offset"][leaves], a["nprims"][leaves]):
        covered[o:o + c] += 1
    assert np.all(covered == 1)                     # every triangle in exactly one leaf
    inner = np.where(~leaves)[0]
    for i in inner[:500]:                            # children contained in parent box
        for ch in (i + 1, a["offset"][i]):
            assert np.all(a["bmin"][ch] >= a["bmin"][i]) and np.all(a["bmax"][ch] <= a["bmax"][i])
    assert s.bvh_depth <= 64 and n == 2 * leaves.sum() - 1


def random_rays(n, seed, box=3.0):
    rng = np.random.default_rng(seed)
    ro = rng.uniform(-box, box, (n, 3)).astype(np.float32)
    rd = rng.normal(size=(n, 3)).astype(np.float32)
    rd /= np.linalg.norm(rd, axis=1, keepdims=True)
    t = rng.uniform(-0.5, 0.5, (n // 2, 3)).astype(np.float32)
    d = t - ro[: n // 2]
    rd[: n // 2] = d / np.linalg.norm(d, axis=1, keepdims=True)
    return ro, rd


@pytest.mark.parametrize("which", ["scene_c1", "scene_c2", "scene_cube"])
def test_traversal_equals_brute_force(request, oracle, which):
    _, a = request.getfixturevalue(which)
    ro, rd = random_rays(4000, 11)
    p0, n0, t0 = oracle.trace_closest(a, ro, rd, 0)
    p1, n1, t1 = oracle.trace_closest(a, ro, rd, 1)
    assert np.array_equal(t0, t1) and np.array_equal(p0.view(np.uint32), p1.view(np.uint32))
    assert np.array_equal(n0.view(np.uint32), n1.view(np.uint32))
    assert (t0 >= 0).mean() > 0.2
    assert np.array_equal(oracle.trace_any(a, ro, rd, 0), oracle.trace_any(a, ro, rd, 1))


def test_closest_hit_geometry(scene_c1, oracle):
    """Hits lie on the unit sphere along the ray, normals are unit and face the ray."""
    _, a = scene_c1
    ro = np.tile(np.array([[0, 0, 5]], np.float32), (500, 1))
    tgt = np.random.default_rng(4).uniform(-0.6, 0.6, (500, 3)).astype(np.float32)
    rd = (tgt - ro) / np.linalg.norm(tgt - ro, axis=1, keepdims=True)
    pt, nm, tri = oracle.trace_closest(a, ro, rd)
    hit = tri >= 0
    assert hit.mean() > 0.9
    r = np.linalg.norm(pt[hit, :3], axis=1)        # flat facets of a 960-tri tessellation
    assert r.min() > 0.985 and r.max() < 1.0 + 1e-5
    np.testing.assert_allclose(pt[hit, :3], ro[hit] + rd[hit] * pt[hit, 3:4], atol=1e-5)
    assert np.all((nm[hit, :3] * rd[hit]).sum(1) < 0)


def test_backface_culling(oracle, scene_c1):
    _, a = scene_c1
    # from inside the sphere every triangle is back-facing (Triangle.cu:7,20 TEST_CULL)
    ro = np.zeros((100, 3), np.float32)
    rd = np.random.default_rng(5).normal(size=(100, 3)).astype(np.float32)
    rd /= np.linalg.norm(rd, axis=1, keepdims=True)
    _, _, tri = oracle.trace_closest(a, ro, rd)
    assert np.all(tri == -1)


def test_nan_direction_is_miss_and_visible(oracle, scene_c1):
    _, a = scene_c1
    ro = np.array([[0, 0, 5]] * 3, np.float32)
    rd = np.array([[np.nan, 0, -1], [0, np.nan, -1], [0, 0, 0]], np.float32)
    _, _, tri = oracle.trace_closest(a, ro, rd)
    assert np.all(tri == -1)
    assert np.all(oracle.trace_any(a, ro, rd) == 1)


# ---------------------------------------------------------------- golden fixtures
def test_golden_film_c1(scene_c1, oracle, mcpt_mod):
    g = np.load(os.path.join(GOLDEN, "film_c1_64x64_s4_d3.npz"))
    cam = mcpt_mod.config_camera(mcpt_mod.CONFIGS[1], 64, 64)
    assert np.array_equal(np.array(cam.inv_view_proj, np.float32), g["inv_view_proj"])
    _, a = scene_c1
    Ld, smp, cnt = oracle.render(a, cam, 64, 64, spp=4, max_depth=3)
    assert np.array_equal(Ld.view(np.uint32), g["Ld"].view(np.uint32))
    assert np.array_equal(smp, g["samples"])
    assert [cnt["extend_rays"], cnt["shadow_rays"], cnt["vis_rays"]] == list(g["counters"])
    # reference edge semantics: last row / column never rendered (wavefront_kernels.cu:110)
    assert np.all(smp[:-1, :-1] == 4) and np.all(smp[-1] == 0) and np.all(smp[:, -1] == 0)


def test_golden_film_cube_nan_frames(scene_cube, oracle, mcpt_mod):
    g = np.load(os.path.join(GOLDEN, "film_cube_32x32_s2_d5.npz"))
    cam = mcpt_mod.make_camera((0.0, 0.0, 4.0), aspect=1.0)
    _, a = scene_cube
    Ld, smp, cnt = oracle.render(a, cam, 32, 32, spp=2, max_depth=5)
    assert np.array_equal(Ld.view(np.uint32), g["Ld"].view(np.uint32))
    assert np.array_equal(smp, g["samples"])


def test_golden_traces(oracle, scene_c1, scene_cube):
    for name, (_, a) in (("c1", scene_c1), ("cube", scene_cube)):
        g = np.load(os.path.join(GOLDEN, f"trace_{name}_256.npz"))
        pt, nm, tri = oracle.trace_closest(a, g["ro"], g["rd"])
        assert np.array_equal(tri, g["tri"])  # triangle ids (scene order): independent of the BVH
        assert np.array_equal(pt.view(np.uint32), g["pos_t"].view(np.uint32))
        assert np.array_equal(nm.view(np.uint32), g["nrm_mat"].view(np.uint32))
        assert np.array_equal(oracle.trace_any(a, g["ro"], g["rd"]), g["vis"])


def test_tile_order_invariance_oracle(scene_c1, oracle, mcpt_mod):
    """Keyed RNG: results do not depend on tile size / order (partition invariance)."""
    _, a = scene_c1
    cam = mcpt_mod.config_camera(mcpt_mod.CONFIGS[1], 48, 40)
    A = oracle.render(a, cam, 48, 40, spp=2, max_depth=3, tile=256, nthreads=1)
    B = oracle.render(a, cam, 48, 40, spp=2, max_depth=3, tile=16, nthreads=4)
    assert np.array_equal(A[0].view(np.uint32), B[0].view(np.uint32)) and np.array_equal(A[1], B[1])


def grazing_rays(a, n, seed):
    """Rays passing within ~1e-7..3e-6 (relative) of random triangle vertices, from 0.3-2 units
    away: where Moller-Trumbore can accept a line just outside the triangle's own box (the cases
    that made results depend on leaf grouping before the own-box check: ~0.7% of these rays)."""
    g = np.random.default_rng(seed)
    T = len(a["mat"])
    ti, k = g.integers(0, T, n), g.integers(0, 3, n)
    V = np.stack([a["v0"], a["v1"], a["v2"]], 1)[ti, k].astype(np.float64)
    off = g.normal(size=(n, 3))
    off /= np.linalg.norm(off, axis=1, keepdims=True)
    tgt = V + off * np.abs(V).max(1, keepdims=True) * 10.0 ** g.uniform(-7.5, -5.5, (n, 1))
    d = g.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    o = tgt - d * g.uniform(0.3, 2.0, (n, 1))
    return o.astype(np.float32), d.astype(np.float32)


@pytest.mark.parametrize("cfg", [dict(builder="sah3", buckets=32, trav_cost=1.0, isect_cost=1.0, max_prims=8),
                                 dict(builder="sah3", buckets=8, trav_cost=4.0, isect_cost=1.0, max_prims=8)])
def test_results_do_not_depend_on_the_bvh(mcpt_mod, oracle, scene_c2, cfg):
    """Hits and films are the same for any tree: the reference builder's one-triangle leaves and
    SAH3's multi-triangle leaves (own-box check + triangle-id ties, oracle/mcpt_oracle.c)."""
    s0 = mcpt_mod.build_config_scene(2, builder="reference")
    a0 = s0.arrays()
    s1 = mcpt_mod.build_config_scene(2, **cfg)
    a1 = s1.arrays()
    assert len(a1["nprims"]) < len(a0["nprims"]) and a1["nprims"].max() > 1  # really a different tree
    ro, rd = grazing_rays(a0, 50000, 1)
    r0 = oracle.trace_closest(a0, ro, rd)
    r1 = oracle.trace_closest(a1, ro, rd)
    for x, y in zip(r0, r1):
        assert np.array_equal(np.asarray(x).view(np.uint32), np.asarray(y).view(np.uint32))
    assert np.array_equal(oracle.trace_any(a0, ro, rd), oracle.trace_any(a1, ro, rd))
    rc = mcpt_mod.CONFIGS[2]
    cam = mcpt_mod.config_camera(rc, 64, 36)
    f0 = oracle.render(a0, cam, 64, 36, spp=2, max_depth=5)
    f1 = oracle.render(a1, cam, 64, 36, spp=2, max_depth=5)
    assert np.array_equal(f0[0].view(np.uint32), f1[0].view(np.uint32)) and np.array_equal(f0[1], f1[1])


@pytest.mark.parametrize("builder", ["reference", "sah3"])
def test_threaded_host_bvh_build_is_identical(mcpt_mod, monkeypatch, builder):
    """The host SAH builds split the top of the tree serially and build the subtrees below on
    worker threads (scene.cpp Builder::build_parallel); every split depends on its range alone,
    so the flattened arrays equal the one-thread build bit for bit (config 4 proxy, 252K tris)."""
    out = []
    for threads in ("1", "8"):
        monkeypatch.setenv("MCPT_BVH_THREADS", threads)
        s = mcpt_mod.Scene().make_proxy(4)
        s.build(builder=builder)
        out.append((s.arrays(), s.bvh_depth))
    (a, da), (b, db) = out
    assert da == db
    for k in ("v0", "v1", "v2", "n0", "n1", "n2", "mat", "bmin", "bmax", "offset", "nprims", "axis", "tri_id"):
        assert np.array_equal(a[k], b[k]), k


def _pixels_changed(a, b):
    (La, sa, _), (Lb, sb, _) = a, b
    px = np.any(La.view(np.uint32) != Lb.view(np.uint32), axis=2) | (sa != sb)
    return int(px.sum())


def test_literal_leaf_rule_deviation(mcpt_mod, oracle, scene_c1, scene_cube, scene_c2):
    """Quantifies deviation 4 of DESIGN.md section 5.  The oracle (and the GPU) add an own-box
    slab test inside multi-triangle leaves and break exact-t ties by triangle id, so results do
    not depend on the tree; the reference tests every leaf primitive and keeps the first visited
    (Triangle.cu:170-179).  traversal=2 is that literal rule.  Measured: it changes no pixel of
    the golden films, of config 1 / config 2 renders, on either tree; only rays built to graze
    triangle vertices see a different closest hit (counted below), and there the literal result
    depends on how a builder grouped triangles into leaves -- why it cannot be the contract."""
    counts = {}
    cam1 = mcpt_mod.config_camera(mcpt_mod.CONFIGS[1], 64, 64)
    camc = mcpt_mod.make_camera((0.0, 0.0, 4.0), aspect=1.0)
    rc2 = mcpt_mod.CONFIGS[2]
    cam2 = mcpt_mod.config_camera(rc2, 160, 90)
    s1r = mcpt_mod.build_config_scene(1, builder="reference").arrays()
    s2r = mcpt_mod.build_config_scene(2, builder="reference").arrays()
    for name, a, cam, W, H, spp, d in (("c1_golden_sah3", scene_c1[1], cam1, 64, 64, 4, 3),
                                       ("cube_golden_sah3", scene_cube[1], camc, 32, 32, 2, 5),
                                       ("c2_160x90_sah3", scene_c2[1], cam2, 160, 90, 3, 5),
                                       ("c1_reference_tree", s1r, cam1, 64, 64, 4, 3),
                                       ("c2_160x90_reference_tree", s2r, cam2, 160, 90, 3, 5)):
        base = oracle.render(a, cam, W, H, spp, d)
        lit = oracle.render(a, cam, W, H, spp, d, traversal=2)
        counts[name] = (_pixels_changed(base, lit), (W - 1) * (H - 1))
    # adversarial rays grazing triangle vertices (where the two rules can differ at all)
    ro, rd = grazing_rays(scene_c2[1], 50000, 1)
    t0 = oracle.trace_closest(scene_c2[1], ro, rd)[2]
    t2 = oracle.trace_closest(scene_c2[1], ro, rd, traversal=2)[2]
    counts["c2_grazing_rays_sah3"] = (int((t0 != t2).sum()), len(ro))
    print("pixels (rays) changed by the literal leaf rule:", counts)
    assert counts["c1_reference_tree"][0] == 0 and counts["c2_160x90_reference_tree"][0] == 0
    for name, (n, tot) in counts.items():
        assert n <= 0.01 * tot, (name, n, tot)


@pytest.mark.parametrize("scene", ["c1dir", "c2"])
@pytest.mark.parametrize("stage", ["logic", "generate", "material"])
def test_stage_golden_vectors_oracle(mcpt_mod, oracle, stage, scene):
    """The oracle's stage restatements (or_stage_logic / or_stage_material, sharing logic_core,
    mis_terms, pick_light and mat_mix_core with the full render) reproduce the committed per-stage
    golden vectors bit for bit (regression pin; the GPU side is tests/test_gpu.py)."""
    import stage_fixtures as sf

    cid = sf.SCENES[scene]
    g = np.load(os.path.join(GOLDEN, f"stage_{stage}_{scene}.npz"))
    inp = {k[3:]: g[k] for k in g.files if k.startswith("in_")}
    a = sf.stage_scene(mcpt_mod, cid).arrays()
    kw = dict(max_depth=sf.DEPTH, rr_depth=sf.RR)
    if stage == "material":
        out = oracle.stage_material(a, inp, **kw)
    else:
        out = oracle.stage_logic(a, sf.stage_camera(mcpt_mod, cid), *sf.FILM, inp, sf.SPP, **kw)
    for k, v in out.items():
        ref = g["out_" + k]
        assert np.array_equal(np.asarray(v).view(np.uint8), ref.view(np.uint8)), k


def test_udiv_small_exact():
    """k_shade's udiv_small (kernels.hip): floor(n / d) from the truncated fp32 product n * RN32(1/d)
    plus one correction, for every sample index n < 2^19 (kMaxSpp) and path-slot count d <= 256
    (the ABI's range) -- the float estimate is never above the quotient and at most one below."""
    n = np.arange(1 << 19, dtype=np.uint32)
    nf = n.astype(np.float32)
    for d in range(1, 257):
        r = np.float32(1.0) / np.float32(d)
        q = (nf * r).astype(np.uint32)  # v_mul_f32 (RN) then v_cvt_u32_f32 (toward zero)
        q = q + ((n - q * np.uint32(d)) >= d).astype(np.uint32)
        assert np.array_equal(q, n // np.uint32(d)), d


def test_traversal_study_model_consistency(oracle, scene_c2):
    """The round-6 traversal study (oracle/trav_model.c or_model_study / or_lru_sim, tools/trav_study.py,
    DESIGN.md section 4) records what the model's traversal does without changing it: its hits and
    visibility equal or_model_trace's, every pair step fetches one line, the origin-box steps are a
    subset of the steps, and the LRU model is sane (a cache that holds every line misses exactly
    once per distinct line; a one-line cache misses on every change of line)."""
    import numpy as np
    _, a = scene_c2
    rng = np.random.default_rng(3)
    n = 2000
    ro = rng.uniform(-0.9, 0.9, (n, 3)).astype(np.float32)
    rd = rng.normal(size=(n, 3)).astype(np.float32)
    rd /= np.linalg.norm(rd, axis=1, keepdims=True)
    m = oracle.model_margins(a)
    tri, t, vis, _ = oracle.model_trace(a, ro, rd, 2, m)
    nn = len(a["nprims"])
    pair_line = (np.arange(nn) >> 1).astype(np.int32)  # any numbering will do here
    for kind in (0, 1):
        st = oracle.model_study(a, ro, rd, 2, kind, pair_line, nn, margins=m)
        hit = st["hit"].astype(bool)
        assert np.array_equal(hit, (tri >= 0) if kind == 0 else (vis == 0))
        assert np.all(st["origin_steps"] <= st["steps"]) and st["steps"].sum() > n
        interior_lines = (np.diff(st["off"]) >= st["steps"]).all()
        assert interior_lines
        lines, off = st["lines"], st["off"]
        distinct = len(np.unique(lines))
        assert oracle.lru_sim(lines, off, 1, 1 << 16, 16) == distinct  # everything fits: cold misses only
        one = oracle.lru_sim(lines, off, 1, 1, 1)
        changes = sum(1 + int((np.diff(lines[off[i]:off[i + 1]]) != 0).sum()) if off[i + 1] > off[i] else 0
                      for i in range(n))
        # rays back to back through one line: a miss on every change, the first of each ray
        # only when it differs from the previous ray's last line
        assert changes - n <= one <= changes
