"""The traversal's box culling against the reference's cull-free traversal, on adversarial rays.

The reference visits every box the infinite line crosses (Bounds3f.h:114-153, Triangle.cu:144-243);
the product skips boxes by the bound of mcpt_core.hpp "conservative box culling" (DESIGN.md
section 5).  The round-3 rule (behind the origin by an absolute 1e-5, beyond (1 + 2^-8) t_best)
was not a bound: Moller-Trumbore's fp32 t strays further than 2^-8 for rays that graze a large
triangle, and the absolute threshold does not follow the scene's scale.

CPU tests: the bound itself on grazing (ray, triangle) pairs evaluated with the oracle's exact
fp32 operation order; a model of the product's traversal (oracle/trav_model.c) under the round-4
rule against the oracle on adversarial rays (tests/adversarial.py: corner, near-origin and grazing
rays on C2's walls, C3's ground quad, an axis-aligned floor with objects resting on it; C2 at
x1e-3 / x1 / x1e3); and the round-3 rule, which the same rays catch.
GPU tests: the product's k_trace (closest and any hit) against the oracle on >= 1 M such rays.
"""
import os

import numpy as np
import pytest

from adversarial import adversarial_rays, triangle_pools

U = 2.0 ** -24


def scaled_scene(mcpt, cid, scale=1.0):
    s = mcpt.Scene()
    s.make_proxy(cid, mcpt.ASSET_DIR)
    if scale != 1.0:
        s.transform(np.diag([scale, scale, scale, 1.0]).astype(np.float32).T.reshape(16))
    s.build(**mcpt.DEFAULT_BVH)
    return s


def floor_scene(mcpt):
    """An exactly axis-aligned 10 x 10 floor at y = 0 (no proxy rotation) with a sphere and a cube
    resting on it: the contact lines are where a grazing ray meets two surfaces at nearly one t."""
    s = mcpt.Scene()
    v = np.array([[-5, 0, -5], [5, 0, -5], [5, 0, 5], [-5, 0, 5]], np.float32)
    # wound so that e1 x e2 = +y: rays coming down are front-facing (d . (e1 x e2) < 0, Triangle.cu:20)
    v0 = np.array([v[0], v[0]]); v1 = np.array([v[2], v[3]]); v2 = np.array([v[1], v[2]])
    n = np.tile(np.array([[0, 1, 0]], np.float32), (2, 1))
    s.add_mesh(v0, v1, v2, n, n, n, (0.7, 0.7, 0.7))
    for name, sc, t in (("sphere.glb", 0.5, (0.0, 0.5, 0.0)), ("Cube.glb", 0.3, (1.2, 0.3, 0.4))):
        m = np.diag([sc, sc, sc, 1.0]).astype(np.float32)
        m[:3, 3] = t
        s.load_glb(os.path.join(mcpt.ASSET_DIR, name), m.T.reshape(16))
    s.set_env_color((0.8, 0.8, 0.8))
    s.build(**mcpt.DEFAULT_BVH)
    return s


# ---- the bound on single (ray, triangle) pairs ---------------------------------------------
def mt_fp32(o, d, p0, e1, e2):
    """tri_intersect's fp32 expressions (oracle/mcpt_oracle.c:582-600, Triangle.cu:9-64) in the
    same operation order; returns accepted, D, N (fp32 values) -- t' = N / D."""
    f = np.float32

    def cross(a, b):
        return np.stack([a[:, 1] * b[:, 2] - a[:, 2] * b[:, 1], a[:, 2] * b[:, 0] - a[:, 0] * b[:, 2],
                         a[:, 0] * b[:, 1] - a[:, 1] * b[:, 0]], 1)

    def dot(a, b):
        return (a[:, 0] * b[:, 0] + a[:, 1] * b[:, 1]) + a[:, 2] * b[:, 2]

    pvec = cross(d, e2)
    det = dot(e1, pvec)
    tvec = o - p0
    u = dot(tvec, pvec)
    qvec = cross(tvec, e1)
    v = dot(d, qvec)
    nn = dot(e2, qvec)
    ok = (det.astype(np.float64) >= np.float64(f(1e-6))) & (u >= 0) & (u <= det) & (v >= 0) & ((u + v) <= det)
    return ok, det, nn


def test_cull_bound_on_grazing_pairs(mcpt_mod):
    """For every accepted grazing (ray, triangle) pair: the point o + t' d lies within
    omega_T + beta_T |o - p0| (per axis) of the triangle's own box, the inequality every cull
    decision of mcpt_core.hpp rests on (beta_T, omega_T as the product computes them)."""
    rng = np.random.default_rng(5)
    checked = 0
    worst = 0.0
    for cid in (2, 3):
        a = mcpt_mod.build_config_scene(cid).arrays()
        big, anyt = triangle_pools(a)
        for pool in (big, anyt):
            m = 400000
            T = pool[rng.integers(0, len(pool), m)]
            v0, v1, v2 = (np.asarray(a[k], np.float32)[T] for k in ("v0", "v1", "v2"))
            e1, e2 = v1 - v0, v2 - v0
            n = np.cross(e1.astype(np.float64), e2.astype(np.float64))
            area2 = np.linalg.norm(n, axis=1)
            n /= area2[:, None]
            # |cos| from the det threshold's own angle (det = |e1 x e2| |cos|, Triangle.cu:20: the
            # noisiest rays it accepts) up to 100x it, and log-uniform in [1e-7, 1e-2]
            c = np.where(rng.random(m) < 0.5, 1e-6 / area2 * 10.0 ** rng.uniform(-0.3, 2, m),
                         10.0 ** rng.uniform(-7, -2, m))
            c = np.minimum(c, 0.5)
            r = rng.normal(size=(m, 3))
            tau = r - np.sum(r * n, 1, keepdims=True) * n
            tau /= np.linalg.norm(tau, axis=1, keepdims=True)
            d = (tau * np.sqrt(1 - c * c)[:, None] - c[:, None] * n).astype(np.float32)
            bu, bv = rng.random(m), rng.random(m)
            flip = bu + bv > 1
            bu[flip], bv[flip] = 1 - bu[flip], 1 - bv[flip]
            q = v0 + bu[:, None] * e1 + bv[:, None] * e2
            # bary slightly outside too: noise may still accept
            q = q + (rng.normal(size=(m, 3)) * 1e-3 * np.linalg.norm(e1, axis=1, keepdims=True)).astype(np.float32)
            dist = rng.uniform(0.01, 4.0, m)
            o = (q - dist[:, None] * d).astype(np.float32)
            ok, det, nn = mt_fp32(o, d, v0, e1, e2)
            tp = nn.astype(np.float64) / det.astype(np.float64)
            P = o.astype(np.float64) + tp[:, None] * d.astype(np.float64)
            lo = np.minimum(np.minimum(v0, v1), v2).astype(np.float64)
            hi = np.maximum(np.maximum(v0, v1), v2).astype(np.float64)
            w = np.maximum(np.maximum(lo - P, P - hi), 0.0).max(axis=1)
            n1 = np.linalg.norm(e1.astype(np.float64), axis=1)
            n2 = np.linalg.norm(e2.astype(np.float64), axis=1)
            beta = 28.3 * U * n1 * n2 / np.float64(np.float32(1e-6)) * (1 + 1 / 512) + 1.01 * U
            omega = 2.1 * U * np.maximum(n1, n2)
            bound = omega + beta * np.linalg.norm(o.astype(np.float64) - v0.astype(np.float64), axis=1)
            sel = ok & np.isfinite(tp)
            assert (w[sel] <= bound[sel]).all(), f"bound violated on {(w[sel] > bound[sel]).sum()} pairs"
            checked += int(sel.sum())
            if sel.any():
                worst = max(worst, float((w[sel] / bound[sel]).max()))
    assert checked > 200000, checked
    print(f"{checked} accepted grazing pairs, largest w / bound = {worst:.3g}")


def test_plane_bound_on_grazing_pairs():
    """Axis-plane triangles (mcpt_core.hpp cull_plane_b: walls, floors, box faces): for every
    accepted pair, the point o + t' d lies within omega_T + 1.01 u |tvec| + b_T (|tvec| + |t'| |d|)
    of the triangle's box, b_T = 15.0003 u |e1| |e2| / G', whatever the angle -- rays down to
    |cos| = 1e-9, far below the det threshold's own angle for large triangles, which the general
    bound (28.3 u |e1| |e2| / 1e-6) cannot cover.  Right-angled, general and thin triangles
    (|e1| |e2| / G up to ~1e3), sizes 1e-3 .. 1e3, planes off the origin, every axis."""
    rng = np.random.default_rng(11)
    checked, worst = 0, 0.0
    for rep in range(6):
        m = 300000
        ax = rng.integers(0, 3, m)
        size = 10.0 ** rng.uniform(-3, 3, m)
        kind = rng.integers(0, 3, m)
        # in-plane edge vectors (a, c) of e1, e2: right angle, general, thin
        e1p = np.stack([size, np.zeros(m)], 1)
        e2p = np.where((kind == 0)[:, None], np.stack([np.zeros(m), size * rng.uniform(0.2, 5, m)], 1),
                       rng.normal(size=(m, 2)) * size[:, None])
        thin = kind == 2
        e2p[thin] = e1p[thin] * rng.uniform(0.3, 2, thin.sum())[:, None] + \
            np.stack([np.zeros(thin.sum()), size[thin] * 10.0 ** rng.uniform(-3, -1, thin.sum())], 1)
        rot = rng.uniform(0, 2 * np.pi, m)
        cr, sr = np.cos(rot), np.sin(rot)
        def rotp(e):
            return np.stack([cr * e[:, 0] - sr * e[:, 1], sr * e[:, 0] + cr * e[:, 1]], 1)
        e1p, e2p = rotp(e1p), rotp(e2p)
        off = rng.normal(size=(m, 3)) * size[:, None] * 10.0 ** rng.uniform(-1, 2, m)[:, None]
        v0 = off.astype(np.float32)
        v1 = v0.copy(); v2 = v0.copy()
        ia, ic = (ax + 1) % 3, (ax + 2) % 3
        r = np.arange(m)
        v1[r, ia] += e1p[:, 0].astype(np.float32); v1[r, ic] += e1p[:, 1].astype(np.float32)
        v2[r, ia] += e2p[:, 0].astype(np.float32); v2[r, ic] += e2p[:, 1].astype(np.float32)
        e1, e2 = v1 - v0, v2 - v0
        assert (e1[r, ax] == 0).all() and (e2[r, ax] == 0).all()
        nrm = np.zeros((m, 3)); nrm[r, ax] = 1.0
        n64 = np.cross(e1.astype(np.float64), e2.astype(np.float64))
        nrm *= np.sign(n64[r, ax])[:, None]  # d . (e1 x e2) < 0 below: det > 0 (front face)
        c = 10.0 ** rng.uniform(-9, -0.5, m)
        tau = rng.normal(size=(m, 3)); tau[r, ax] = 0.0
        tau /= np.linalg.norm(tau, axis=1, keepdims=True)
        d = (tau * np.sqrt(1 - c * c)[:, None] - c[:, None] * nrm).astype(np.float32)
        bu, bv = rng.random(m), rng.random(m)
        flip = bu + bv > 1
        bu[flip], bv[flip] = 1 - bu[flip], 1 - bv[flip]
        q = v0 + bu[:, None] * e1 + bv[:, None] * e2
        dist = size * 10.0 ** rng.uniform(-4, 3, m)
        o = (q - dist[:, None] * d).astype(np.float32)
        ok, det, nn = mt_fp32(o, d, v0, e1, e2)
        tq = nn.astype(np.float64) / det.astype(np.float64)
        P = o.astype(np.float64) + tq[:, None] * d.astype(np.float64)
        lo = np.minimum(np.minimum(v0, v1), v2).astype(np.float64)
        hi = np.maximum(np.maximum(v0, v1), v2).astype(np.float64)
        w = np.maximum(np.maximum(lo - P, P - hi), 0.0).max(axis=1)
        n1 = np.linalg.norm(e1.astype(np.float64), axis=1)
        n2 = np.linalg.norm(e2.astype(np.float64), axis=1)
        A1 = e1[r, ia].astype(np.float64); C1 = e1[r, ic].astype(np.float64)
        A2 = e2[r, ia].astype(np.float64); C2 = e2[r, ic].astype(np.float64)
        g = np.abs(A1 * C2 - C1 * A2)
        gp = g - 5.0002 * U * (np.abs(A1 * C2) + np.abs(C1 * A2))
        b = 15.0003 * U * n1 * n2 / gp
        tv = np.linalg.norm(o.astype(np.float64) - v0.astype(np.float64), axis=1)
        bound = 2.1 * U * np.maximum(n1, n2) + 1.01 * U * tv + b * (tv + np.abs(tq) * np.linalg.norm(d.astype(np.float64), axis=1))
        sel = ok & np.isfinite(tq) & (gp > 0.5 * g)
        assert (w[sel] <= bound[sel]).all(), f"bound violated on {(w[sel] > bound[sel]).sum()} pairs"
        checked += int(sel.sum())
        worst = max(worst, float((w[sel] / bound[sel]).max()))
    assert checked > 500000, checked
    print(f"{checked} accepted axis-plane pairs, largest w / bound = {worst:.3g}")


# ---- the traversal model on adversarial rays ------------------------------------------------
SCENES = [("c2", 1.0), ("c2", 1e3), ("c2", 1e-3), ("c3", 1.0), ("floor", 1.0)]


@pytest.fixture(scope="module")
def adv_scenes(mcpt_mod, scene_c3):
    out = {}
    for name, sc in SCENES:
        if name == "c3":
            a = scene_c3[1]
        elif name == "floor":
            a = floor_scene(mcpt_mod).arrays()
        else:
            a = scaled_scene(mcpt_mod, 2, sc).arrays()
        out[(name, sc)] = a
    return out


@pytest.mark.parametrize("name,scale", SCENES)
def test_round4_cull_model_equals_reference(oracle, adv_scenes, name, scale):
    """The round-4 rule (mode 2 of oracle/trav_model.c, the product's keep_box) gives the
    reference's closest hit and visibility on every adversarial ray; mode 0 (no culling) is the
    model's own check against the oracle."""
    a = adv_scenes[(name, scale)]
    n = 120000 if name == "c3" else 300000
    ro, rd = adversarial_rays(a, n, seed=11, scale=scale)
    _, _, otri = oracle.trace_closest(a, ro, rd)
    ovis = oracle.trace_any(a, ro, rd)
    m = oracle.model_margins(a)
    assert m["contained"]
    pos_t, _, _ = oracle.trace_closest(a, ro, rd)
    for mode in (0, 2):
        tri, t, vis, boxes = oracle.model_trace(a, ro, rd, mode, m)
        assert np.array_equal(tri, otri), f"mode {mode}: {(tri != otri).sum()} closest hits differ"
        assert np.array_equal(t.view(np.uint32), pos_t[:, 3].view(np.uint32))
        assert np.array_equal(vis, ovis), f"mode {mode}: {(vis != ovis).sum()} visibilities differ"


def test_round3_cull_rule_is_caught(oracle, adv_scenes):
    """The round-3 rule (mode 1) differs from the reference on the adversarial rays of the
    x1e3 config-2 scene: its absolute 1e-5 behind-origin threshold is below the fp32 noise of t
    there.  (This is the hole the round-4 bound closes; kept as evidence that the rays find it.)"""
    a = adv_scenes[("c2", 1e3)]
    ro, rd = adversarial_rays(a, 300000, seed=7, scale=1e3)
    _, _, otri = oracle.trace_closest(a, ro, rd)
    ovis = oracle.trace_any(a, ro, rd)
    tri, _, vis, _ = oracle.model_trace(a, ro, rd, 1)
    assert (tri != otri).sum() + (vis != ovis).sum() > 0


def test_cull_margins_monotone_and_scale_free(oracle, adv_scenes):
    """Margins: a node's W is the max of its subtree's (so an ancestor passes wherever a leaf
    does: the occluder cache's lemma); the walls (sqrt3 beta >= 1/2) are never culled, the
    sphere triangles are."""
    a = adv_scenes[("c2", 1.0)]
    m = oracle.model_margins(a)
    nw, off, npr = m["node_w"], a["offset"], a["nprims"]
    for i in np.nonzero(npr == 0)[0]:
        assert nw[i] >= nw[i + 1] and nw[i] >= nw[off[i]]
    big, _ = triangle_pools(a, n_big=10)
    assert np.isinf(m["tri_w"][big]).all()
    assert np.isfinite(m["tri_w"]).mean() > 0.99


# ---- the finite-margin far cut ------------------------------------------
# adversarial_rays' corner rays graze the 16 largest triangles, whose margins are infinite on C2:
# they never exercise a finite far cut.  far_cut_rays grazes the bounded triangles (finite W'_T)
# with S anywhere or adjacent to T.  At x1e3 no C2 triangle is bounded (|e1||e2| grows against the
# fixed det threshold 1e-6), at x1e-3 every one is (the walls included).
FAR_SCENES = [("c2", 1.0), ("c2", 1e-3), ("c3", 1.0), ("c4", 1.0)]
FAR_RAYS = int(os.environ.get("MCPT_TEST_FAR_RAYS", "1000000"))  # per scene (a soak raises it)


@pytest.fixture(scope="module")
def far_scenes(mcpt_mod, adv_scenes):
    out = dict(adv_scenes)
    out[("c4", 1.0)] = mcpt_mod.build_config_scene(4).arrays()
    return out


@pytest.mark.parametrize("name,scale", FAR_SCENES)
def test_far_cut_model_equals_reference(oracle, far_scenes, name, scale):
    """1 M far-cut rays per scene through the model of the product's traversal (trav_model.c mode
    2: the round-4 bound, finite margins on the grazed triangles) against the oracle's cull-free
    reference traversal: closest triangle, t and visibility bit for bit.  Most closest hits are on
    a bounded triangle (the far cut of its leaf decided between candidates at nearly one t)."""
    from adversarial import bounded_pool, engaged, far_cut_rays

    a = far_scenes[(name, scale)]
    assert len(bounded_pool(a)) > 0
    ro, rd = far_cut_rays(a, FAR_RAYS, seed=41, scale=scale)
    assert len(ro) == FAR_RAYS
    th = max(1, min(8, os.cpu_count() or 1))
    pos_t, _, otri = oracle.trace_closest(a, ro, rd, nthreads=th)
    ovis = oracle.trace_any(a, ro, rd, nthreads=th)
    m = oracle.model_margins(a)
    assert m["contained"]
    tri, t, vis, _ = oracle.model_trace(a, ro, rd, 2, m, nthreads=th)
    assert np.array_equal(tri, otri), f"{(tri != otri).sum()} closest hits differ"
    assert np.array_equal(t.view(np.uint32), pos_t[:, 3].view(np.uint32))
    assert np.array_equal(vis, ovis), f"{(vis != ovis).sum()} visibilities differ"
    e = engaged(a, ro, rd, otri)
    assert e > 0.5, e
    print(f"{name} x{scale}: {FAR_RAYS} far-cut rays, {e:.3f} with a bounded closest hit, 0 differ")


# ---- a round-5 candidate, modelled on the CPU ---------------
SAFE_C = 1e-3


def test_safe_ray_bound_on_grazing_pairs():
    """For rays with |d . m^| >= c |d| (m = e2 x e1) the det is either rejected or >= |d| K,
    K = c |m| - 7.0712 u |e1| |e2|, so the accepted point lies within omega + beta |tvec| of the
    triangle's box with beta = 28.3 u |e1| |e2| / K + 1.01 u -- no det threshold, and finite for
    config 2's walls (the general bound is not).  Checked on config 2/3's largest triangles for rays
    at |cos| in [c, 30 c], the band where the bound is tightest."""
    import mcpt

    rng = np.random.default_rng(23)
    checked, worst = 0, 0.0
    for cid in (2, 3):
        a = mcpt.build_config_scene(cid).arrays()
        big, _ = triangle_pools(a, n_big=12)
        m = 300000
        T = big[rng.integers(0, len(big), m)]
        v0, v1, v2 = (np.asarray(a[k], np.float32)[T] for k in ("v0", "v1", "v2"))
        e1, e2 = v1 - v0, v2 - v0
        mvec = np.cross(e2.astype(np.float64), e1.astype(np.float64))
        mm = np.linalg.norm(mvec, axis=1)
        mh = mvec / mm[:, None]
        c = SAFE_C * 10.0 ** rng.uniform(0, np.log10(30), m)
        r = rng.normal(size=(m, 3))
        tang = r - np.sum(r * mh, 1, keepdims=True) * mh
        tang /= np.linalg.norm(tang, axis=1, keepdims=True)
        d = (tang * np.sqrt(1 - c * c)[:, None] + c[:, None] * mh).astype(np.float32)  # front-facing
        bu, bv = rng.random(m), rng.random(m)
        flip = bu + bv > 1
        bu[flip], bv[flip] = 1 - bu[flip], 1 - bv[flip]
        q = v0 + bu[:, None] * e1 + bv[:, None] * e2
        q = q + (rng.normal(size=(m, 3)) * 1e-3).astype(np.float32)
        o = (q - rng.uniform(0.01, 4.0, m)[:, None] * d).astype(np.float32)
        ok, det, nn = mt_fp32(o, d, v0, e1, e2)
        tp = nn.astype(np.float64) / det.astype(np.float64)
        P = o.astype(np.float64) + tp[:, None] * d.astype(np.float64)
        lo = np.minimum(np.minimum(v0, v1), v2).astype(np.float64)
        hi = np.maximum(np.maximum(v0, v1), v2).astype(np.float64)
        w = np.maximum(np.maximum(lo - P, P - hi), 0.0).max(axis=1)
        n1 = np.linalg.norm(e1.astype(np.float64), axis=1)
        n2 = np.linalg.norm(e2.astype(np.float64), axis=1)
        K = SAFE_C * mm - 7.0712 * U * n1 * n2
        beta = 28.3 * U * n1 * n2 / K + 1.01 * U
        bound = 2.1 * U * np.maximum(n1, n2) + beta * np.linalg.norm(o.astype(np.float64) - v0.astype(np.float64), axis=1)
        sel = ok & np.isfinite(tp) & (K > 0)
        assert (w[sel] <= bound[sel]).all(), f"bound violated on {(w[sel] > bound[sel]).sum()} pairs"
        checked += int(sel.sum())
        worst = max(worst, float((w[sel] / bound[sel]).max()))
    assert checked > 200000, checked
    print(f"{checked} accepted pairs at |cos| in [c, 30c], largest w / bound = {worst:.3g}")


@pytest.mark.parametrize("name,scale", [("c2", 1.0), ("c2", 1e3), ("c2", 1e-3)])
def test_safe_ray_margins_model_equals_reference(oracle, adv_scenes, name, scale):
    """Mode 6 of oracle/trav_model.c (the walls' finite margins for rays at |cos| >= 1e-3 to every
    wall plane, no culling for the others) against the cull-free reference, on the adversarial rays
    plus grazing rays in the band [5e-4, 2e-2] around the switch; and its box tests against mode 2's."""
    from adversarial import grazing_rays

    a = adv_scenes[(name, scale)]
    ro, rd = adversarial_rays(a, 200000, seed=31, scale=scale)
    big, _ = triangle_pools(a)
    o2, d2 = grazing_rays(a, 100000, 37, big, scale, band=(5e-4, 2e-2))
    ro, rd = np.concatenate([ro, o2]), np.concatenate([rd, d2])
    _, _, otri = oracle.trace_closest(a, ro, rd)
    ovis = oracle.trace_any(a, ro, rd)
    pos_t, _, _ = oracle.trace_closest(a, ro, rd)
    m6 = oracle.model_margins(a, safe_c=SAFE_C)
    assert np.isfinite(m6["tri_w"][big[:10]]).all()  # the walls are bounded for safe rays
    tri, t, vis, boxes6 = oracle.model_trace(a, ro, rd, 6, m6, safe_c=SAFE_C)
    assert np.array_equal(tri, otri), f"{(tri != otri).sum()} closest hits differ"
    assert np.array_equal(t.view(np.uint32), pos_t[:, 3].view(np.uint32))
    assert np.array_equal(vis, ovis), f"{(vis != ovis).sum()} visibilities differ"
    _, _, _, boxes2 = oracle.model_trace(a, ro, rd, 2, oracle.model_margins(a))
    print(f"box tests: mode 2 {boxes2}, mode 6 {boxes6}")


# ---- the product on the GPU -----------------------------------------------------------------
GPU_SCENES = [("c2", 1.0, 1000000), ("c2", 1e3, 1000000), ("c2", 1e-3, 1000000), ("c3", 1.0, 1000000),
              ("floor", 1.0, 1000000), ("c5", 1.0, 500000), ("c4", 1.0, 1000000)]
# far-cut rays (finite margins) on every scene with bounded triangles; tiny: the 2-entry LDS stack
# instantiation (mcpt_debug_tiny_lds_stack), so that scratch stack entries carry adversarial rays
GPU_FAR = [("c2", 1.0, False), ("c2", 1e-3, False), ("c3", 1.0, False), ("c4", 1.0, False), ("c5", 1.0, False),
           ("c2", 1.0, True), ("c4", 1.0, True), ("c5", 1.0, True)]


def _gpu_scene(mcpt_mod, request, name, scale):
    if name == "c3":
        return request.getfixturevalue("scene_c3")
    if name == "floor":
        s = floor_scene(mcpt_mod)
    elif name in ("c4", "c5"):
        s = mcpt_mod.build_config_scene(int(name[1]))
    else:
        s = scaled_scene(mcpt_mod, 2, scale)
    return s, s.arrays()


def _gpu_vs_oracle(mcpt_mod, oracle, s, a, ro, rd, tiny=False):
    pt = mcpt_mod.PathTracer(0)
    pt.upload_scene(s)
    if tiny:
        pt.set_tiny_lds_stack(True)
    gp, gn, gt = pt.trace_closest(ro, rd)
    gv = pt.trace_any(ro, rd)
    pt.close()
    th = max(1, min(8, os.cpu_count() or 1))
    op_, on, ot = oracle.trace_closest(a, ro, rd, nthreads=th)
    ov = oracle.trace_any(a, ro, rd, nthreads=th)
    bad = np.nonzero((gt != ot) | (gv != ov))[0]
    assert len(bad) == 0, f"{len(bad)} of {len(ro)} rays differ, first {bad[:5]}"
    assert np.array_equal(gp.view(np.uint32), op_.view(np.uint32))
    assert np.array_equal(gn.view(np.uint32), on.view(np.uint32))
    return ot, ov


@pytest.mark.gpu
@pytest.mark.parametrize("name,scale,n", GPU_SCENES)
def test_gpu_cull_adversarial(mcpt_mod, oracle, request, name, scale, n):
    """k_trace (persistent traversal, pair or 4-wide nodes, conservative culls) against the
    oracle's cull-free reference traversal on adversarial rays: closest-hit triangle, t, position,
    normal and any-hit visibility bit for bit.  C5 (2 M triangles) runs the 4-wide nodes."""
    s, a = _gpu_scene(mcpt_mod, request, name, scale)
    n = n * int(os.environ.get("MCPT_TEST_CULL_SCALE", "1"))  # a soak multiplies the ray counts
    ro, rd = adversarial_rays(a, n, seed=23, scale=scale)
    ot, ov = _gpu_vs_oracle(mcpt_mod, oracle, s, a, ro, rd)
    print(f"{name} x{scale}: {n} rays, {(ot >= 0).mean():.3f} hit, {(ov == 0).mean():.3f} occluded, 0 differ")


@pytest.mark.gpu
@pytest.mark.parametrize("name,scale,tiny", GPU_FAR)
def test_gpu_far_cut_adversarial(mcpt_mod, oracle, request, name, scale, tiny):
    """k_trace on 1 M far-cut rays (tests/adversarial.py far_cut_rays: the grazed triangle bounded,
    S anywhere or adjacent, crossings within t_S (1 +- 2^-6) and (1 +- 2^-12)) against the oracle's
    cull-free traversal, bit for bit: C2 (pairs, 8-entry stack), C3 and C5 (4-wide), C4 (pairs,
    deep 10-entry stack: k_trace<2,10>); tiny = the 2-entry LDS stack with scratch entries."""
    from adversarial import engaged, far_cut_rays

    s, a = _gpu_scene(mcpt_mod, request, name, scale)
    ro, rd = far_cut_rays(a, FAR_RAYS, seed=43, scale=scale)
    ot, ov = _gpu_vs_oracle(mcpt_mod, oracle, s, a, ro, rd, tiny)
    print(f"{name} x{scale} tiny={tiny}: {len(ro)} far-cut rays, {engaged(a, ro, rd, ot):.3f} bounded closest hits, "
          f"{(ov == 0).mean():.3f} occluded, 0 differ")
