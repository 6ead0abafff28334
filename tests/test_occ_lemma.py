"""The lemma the any-hit occluder cache rests on (kernels.hip occ_test / occ_hit1):
with the traversal's fp32 slab arithmetic (pair_slab: per axis min/max of (plane - o) * inv, then
max3 of the entries and min3 of the exits), a box that contains another never has a later entry or
an earlier exit, so if the leaf box of a cached triangle passes the slab test and keep_box's cull,
every ancestor box (which contains it) passes too and the traversal reaches that leaf.

numpy float32 operations round to nearest like the gfx950 VALU ops, so this checks the same
arithmetic on the host over many random and degenerate (flat, touching, huge) boxes.  CPU only.
"""
import numpy as np

K_HUGE = np.float32(1e32)
K_CULL_ABS = np.float32(1e-5)
K_CULL_REL = np.float32(1.0 / 256.0)


def slab(mn, mx, o, inv):
    """pair_slab's arithmetic for one box (rows of float32 vectors)."""
    a = (mn - o) * inv
    b = (mx - o) * inv
    t0 = np.maximum(np.maximum(np.minimum(a[:, 0], b[:, 0]), np.minimum(a[:, 1], b[:, 1])), np.minimum(a[:, 2], b[:, 2]))
    t1 = np.minimum(np.minimum(np.maximum(a[:, 0], b[:, 0]), np.maximum(a[:, 1], b[:, 1])), np.maximum(a[:, 2], b[:, 2]))
    return t0, t1


def passes(t0, t1):
    cut = K_HUGE + K_HUGE * K_CULL_REL  # an any-hit ray's cut
    return (t0 <= t1) & ~(t1 < -K_CULL_ABS) & ~(t0 > cut)


def _cases(rng, n, scale):
    o = (rng.standard_normal((n, 3)) * scale).astype(np.float32)
    d = rng.standard_normal((n, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True).astype(np.float32)
    inv = (np.float32(1.0) / d).astype(np.float32)
    c = (rng.standard_normal((n, 3)) * scale).astype(np.float32)
    h = np.abs(rng.standard_normal((n, 3)) * scale * 0.1).astype(np.float32)
    h[rng.random((n, 3)) < 0.2] = 0  # flat boxes (axis-aligned triangles)
    mn, mx = c - h, c + h
    g0 = np.abs(rng.standard_normal((n, 3)) * scale * 0.05).astype(np.float32)
    g1 = np.abs(rng.standard_normal((n, 3)) * scale * 0.05).astype(np.float32)
    g0[rng.random((n, 3)) < 0.3] = 0  # ancestors that share a plane with the leaf
    g1[rng.random((n, 3)) < 0.3] = 0
    return o, inv, mn, mx, mn - g0, mx + g1


def test_slab_interval_monotone_in_the_box():
    rng = np.random.default_rng(2026)
    for scale in (1.0, 1e-3, 1e4):
        o, inv, mn, mx, pmn, pmx = _cases(rng, 200_000, scale)
        assert (pmn <= mn).all() and (pmx >= mx).all()
        t0, t1 = slab(mn, mx, o, inv)
        p0, p1 = slab(pmn, pmx, o, inv)
        assert (p0 <= t0).all() and (p1 >= t1).all()
        leaf = passes(t0, t1)
        assert leaf.any()
        assert passes(p0, p1)[leaf].all()  # a passing leaf box implies a passing ancestor


def test_rays_through_a_box_face_and_touching_boxes():
    """Rays aimed at the flat face of a box (the walls of the closed config-2 box), and ancestors
    that coincide with the leaf: still monotone, and a box equal to the leaf passes equally."""
    rng = np.random.default_rng(7)
    n = 100_000
    mn = np.zeros((n, 3), np.float32)
    mx = np.ones((n, 3), np.float32)
    mx[:, 0] = 0  # the x = 0 wall
    tgt = rng.random((n, 3)).astype(np.float32)
    tgt[:, 0] = 0
    o = (tgt + rng.standard_normal((n, 3)).astype(np.float32)).astype(np.float32)
    d = (tgt - o).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True).astype(np.float32)
    inv = (np.float32(1.0) / d).astype(np.float32)
    t0, t1 = slab(mn, mx, o, inv)
    q0, q1 = slab(mn.copy(), mx.copy(), o, inv)
    assert np.array_equal(passes(t0, t1), passes(q0, q1))
    p0, p1 = slab(mn - np.float32(0.5), mx + np.float32(0.5), o, inv)
    assert passes(p0, p1)[passes(t0, t1)].all()
