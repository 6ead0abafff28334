"""Adversarial rays for the traversal's box culling (round-3 VERDICT, next #1).

The reference visits every box the infinite line crosses (Triangle.cu:144-243, Bounds3f.h:121-153)
and keeps the smallest Moller-Trumbore t (Triangle.cu:9-64).  The product skips boxes that cannot
hold the answer, and the rule is only exact if it accounts for how far Moller-Trumbore's fp32 t
can stray for a ray that grazes a triangle.  These generators aim at exactly that:

  corner   a ray that hits triangle S at t_S and grazes triangle T (|cos| in [1e-6, 1e-3] against
           T's normal) so that it crosses T's plane at t_S (1 + delta), |delta| <= 2^-6: the far
           cut decides between them.  S and T are adjacent walls, the two triangles of a quad,
           a wall and a sphere triangle, ...
  near     origins within 1e-7..1e-4 (scene scale) in front of and behind a triangle, grazing or
           random directions: the behind-origin cut decides.
  grazing  rays that graze a triangle from 0.01..3 scene units away.

Triangles are drawn from the largest ones (walls, ground quads) and from all of them.
"""
from __future__ import annotations

import numpy as np


def _unit(v):
    return v / np.linalg.norm(v, axis=-1, keepdims=True)


def _tri_frames(a, idx):
    v0, v1, v2 = (np.asarray(a[k], np.float64)[idx] for k in ("v0", "v1", "v2"))
    n = np.cross(v1 - v0, v2 - v0)  # e1 x e2: front-facing for Moller-Trumbore (det > 0) iff d . n < 0
    return v0, v1, v2, _unit(n)


def _bary(rng, m):
    u, v = rng.random(m), rng.random(m)
    flip = u + v > 1
    u[flip], v[flip] = 1 - u[flip], 1 - v[flip]
    return u, v


def _tangent(rng, n):
    r = rng.normal(size=n.shape)
    t = r - np.sum(r * n, axis=1, keepdims=True) * n
    return _unit(t)


def _grazing_dir(rng, n, lo=1e-6, hi=1e-3, front=True):
    """Unit direction with |d . n| = c, c log-uniform in [lo, hi]; front-facing (d . n < 0) or not."""
    m = len(n)
    c = 10.0 ** rng.uniform(np.log10(lo), np.log10(hi), m)
    s = -1.0 if front is True else np.where(rng.random(m) < 0.5, -1.0, 1.0)
    tau = _tangent(rng, n)
    d = tau * np.sqrt(1 - c * c)[:, None] + (s * c)[:, None] * n
    return d, c


def triangle_pools(a, n_big=16, seed=0):
    """(big, any): the n_big largest triangles and all triangle indices."""
    v0, v1, v2 = (np.asarray(a[k], np.float64) for k in ("v0", "v1", "v2"))
    area = 0.5 * np.linalg.norm(np.cross(v1 - v0, v2 - v0), axis=1)
    big = np.argsort(-area)[:n_big]
    return big, np.arange(len(area))


def corner_rays(a, m, seed, pool_s, pool_t, scale=1.0):
    rng = np.random.default_rng(seed)
    out_o, out_d = [], []
    have = 0
    for _ in range(50):
        k = 4 * (m - have) + 64
        S = pool_s[rng.integers(0, len(pool_s), k)]
        T = pool_t[rng.integers(0, len(pool_t), k)]
        s0, s1, s2, ns = _tri_frames(a, S)
        t0, _, _, nt = _tri_frames(a, T)
        u, v = _bary(rng, k)
        p = s0 + u[:, None] * (s1 - s0) + v[:, None] * (s2 - s0)
        tS = scale * rng.uniform(0.05, 2.0, k)
        d, c = _grazing_dir(rng, nt)
        # S must be hit front-facing too: flip the tangential part when it is not
        bad = np.sum(d * ns, axis=1) >= 0
        d[bad] = d[bad] - 2 * (d[bad] - np.sum(d[bad] * nt[bad], axis=1, keepdims=True) * nt[bad])
        ok = np.sum(d * ns, axis=1) < 0
        delta = rng.uniform(-2.0 ** -6, 2.0 ** -6, k)
        h = delta * tS * c  # height of p above T's plane: the line crosses it at tS (1 + delta)
        w = nt - np.sum(nt * ns, axis=1, keepdims=True) * ns  # in-plane direction of steepest height change
        wn = np.sum(nt * w, axis=1)
        coplanar = np.abs(wn) < 1e-9
        g = np.sum(nt * (p - t0), axis=1)
        s = np.where(coplanar, 0.0, (h - g) / np.where(coplanar, 1.0, wn))
        p2 = p + s[:, None] * w
        # p2 still inside S (barycentric test in S's plane)
        e1, e2 = s1 - s0, s2 - s0
        q = p2 - s0
        d11, d12, d22 = np.sum(e1 * e1, 1), np.sum(e1 * e2, 1), np.sum(e2 * e2, 1)
        q1, q2 = np.sum(q * e1, 1), np.sum(q * e2, 1)
        den = d11 * d22 - d12 * d12
        bu = (d22 * q1 - d12 * q2) / den
        bv = (d11 * q2 - d12 * q1) / den
        inside = (bu >= 0) & (bv >= 0) & (bu + bv <= 1)
        keep = ok & inside & (S != T) & np.isfinite(p2).all(1)
        o = p2 - tS[:, None] * d
        out_o.append(o[keep])
        out_d.append(d[keep])
        have += int(keep.sum())
        if have >= m:
            break
    o, d = np.concatenate(out_o)[:m], np.concatenate(out_d)[:m]
    return o.astype(np.float32), d.astype(np.float32)


def near_rays(a, m, seed, pool, scale=1.0):
    rng = np.random.default_rng(seed)
    T = pool[rng.integers(0, len(pool), m)]
    v0, v1, v2, n = _tri_frames(a, T)
    u, v = _bary(rng, m)
    q = v0 + u[:, None] * (v1 - v0) + v[:, None] * (v2 - v0)
    h = scale * 10.0 ** rng.uniform(-7, -4, m) * np.where(rng.random(m) < 0.5, -1.0, 1.0)
    o = q + h[:, None] * n
    d, _ = _grazing_dir(rng, n, front=None)
    rnd = rng.random(m) < 0.25  # a quarter with random directions
    d[rnd] = _unit(rng.normal(size=(int(rnd.sum()), 3)))
    return o.astype(np.float32), d.astype(np.float32)


def grazing_rays(a, m, seed, pool, scale=1.0, band=(1e-6, 1e-3)):
    rng = np.random.default_rng(seed)
    T = pool[rng.integers(0, len(pool), m)]
    v0, v1, v2, n = _tri_frames(a, T)
    u, v = _bary(rng, m)
    q = v0 + u[:, None] * (v1 - v0) + v[:, None] * (v2 - v0)
    d, _ = _grazing_dir(rng, n, lo=band[0], hi=band[1])
    t = scale * rng.uniform(0.01, 3.0, m)
    o = q - t[:, None] * d + scale * 1e-5 * rng.normal(size=(m, 3))
    return o.astype(np.float32), d.astype(np.float32)


def adversarial_rays(a, m, seed=0, scale=1.0):
    """m rays: corner (big-big, any-big), near (big, any), grazing (big, any), in equal parts."""
    big, anyt = triangle_pools(a)
    k = m // 6
    parts = [corner_rays(a, k, seed + 1, big, big, scale), corner_rays(a, k, seed + 2, anyt, big, scale),
             near_rays(a, k, seed + 3, big, scale), near_rays(a, k, seed + 4, anyt, scale),
             grazing_rays(a, k, seed + 5, big, scale), grazing_rays(a, m - 5 * k, seed + 6, anyt, scale)]
    o = np.concatenate([p[0] for p in parts])
    d = np.concatenate([p[1] for p in parts])
    return o, d
