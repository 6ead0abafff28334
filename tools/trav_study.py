# Round-6 traversal study, CPU only: the product traversal's model
# (oracle/trav_model.c mode 2) on a config scene's any-hit and closest-hit rays --
#   * pair steps per ray split by outcome (occluded / unoccluded) and the steps whose node box holds
#     the ray's origin;
#   * the 128-B lines the steps fetch under each node numbering (layouts 0 / 1 / 2 of
#     runtime.cpp scene_upload and the candidates below), distinct lines per ray and the misses of a
#     4-MB 16-way LRU (one XCD's L2) over the rays interleaved 16 K at a time.
# Rays: camera rays of the config to first hits, then from those surface points (offset along the
# normal) hemisphere directions (any hit: shadow / visibility rays; closest: the next bounce).
# usage: python tools/trav_study.py [config] [rays] [out.json]
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mc-path-tracer_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import mcpt  # noqa: E402
import oracle_py as op  # noqa: E402


def surface_rays(a, rc, n, seed):
    rng = np.random.default_rng(seed)
    o = np.tile(np.array(rc.position, np.float32), (n, 1))
    # directions inside the camera's frustum (yaw -90: looking down -z, pitch in degrees)
    th = np.tan(np.radians(rc.fovy) / 2)
    x = rng.uniform(-th * rc.width / rc.height, th * rc.width / rc.height, n)
    y = rng.uniform(-th, th, n)
    p = np.radians(rc.pitch)
    d = np.stack([x, y * np.cos(p) + np.sin(p), -np.cos(p) + y * np.sin(p)], 1)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    pt, nrm, tri = op.trace_closest(a, o, d.astype(np.float32), nthreads=8)
    k = tri >= 0
    nn = nrm[k, :3]
    flip = (nn * d[k]).sum(1) > 0  # face the camera
    nn[flip] *= -1
    p0 = pt[k, :3] + nn * 1e-3
    d2 = rng.normal(size=(k.sum(), 3))
    d2 /= np.linalg.norm(d2, axis=1, keepdims=True)
    d2[(d2 * nn).sum(1) < 0] *= -1
    return p0.astype(np.float32), d2.astype(np.float32)


def layouts(a):
    """desc node -> pair index per numbering; expansion pairs appended after the desc pairs."""
    nprims, off = a["nprims"], a["offset"]
    N = len(nprims)
    interior = nprims == 0
    npair = int(interior.sum())
    kids = lambda i: [c for c in (i + 1, int(off[i])) if nprims[c] == 0]  # noqa: E731
    bmin, bmax = a["bmin"].reshape(-1, 3), a["bmax"].reshape(-1, 3)
    ext = np.maximum(bmax - bmin, 0)
    area = ext[:, 0] * ext[:, 1] + ext[:, 1] * ext[:, 2] + ext[:, 2] * ext[:, 0]
    out = {}
    l0 = np.full(N, -1, np.int64)
    l0[interior] = np.arange(npair)
    out["0 depth-first (product, large trees)"] = l0

    def sibling(bfs):
        po = np.full(N, -1, np.int64)
        po[0] = 0
        nxt = 1
        st = [0]
        head = 0
        while (head < len(st)) if bfs else st:
            if bfs:
                i = st[head]; head += 1
            else:
                i = st.pop()
            ks = kids(i)
            for c in ks:
                po[c] = nxt; nxt += 1
            st.extend(ks if bfs else ks[::-1])
        return po
    out["1 sibling pairs, depth-first"] = sibling(False)
    out["2 sibling pairs, breadth-first (product, small trees)"] = sibling(True)

    def vertical(top_pairs=0, pad=True):
        """line = (head, its larger-area interior child); heads depth-first.  top_pairs > 0: the
        first top_pairs nodes breadth-first (a hot block) before the vertical subtrees."""
        po = np.full(N, -1, np.int64)
        nxt = 0
        roots = [0]
        if top_pairs:
            q, h = [0], 0
            while h < len(q) and nxt < top_pairs:
                i = q[h]; h += 1
                po[i] = nxt; nxt += 1
                q.extend(kids(i))
            roots = [i for i in q[h:]]
            nxt += nxt & 1
        st = roots[::-1]
        while st:
            i = st.pop()
            if po[i] >= 0:
                continue
            if pad and nxt & 1:
                nxt += 1
            po[i] = nxt; nxt += 1
            ks = kids(i)
            rest = []
            if ks:
                c = max(ks, key=lambda k: area[k])
                po[c] = nxt; nxt += 1
                rest = [k for k in ks if k != c] + kids(c)
            # push so the larger-area grandchild comes next (depth-first)
            rest.sort(key=lambda k: area[k])
            st.extend(rest)
        return po, nxt
    v, nv = vertical()
    out["V vertical line pairs (head + larger child), padded"] = v
    v2, _ = vertical(pad=False)
    out["V' vertical line pairs, unpadded"] = v2
    h, _ = vertical(top_pairs=16384)
    out["H breadth-first top 16 K pairs + vertical"] = h
    return out, npair


def pair_line_of(a, po):
    """desc node -> line of its pair (interior) or of its expansion block (multi-triangle leaf)."""
    nprims = a["nprims"]
    base = int(po.max()) + 1
    pl = np.zeros(len(nprims), np.int64)
    interior = nprims == 0
    pl[interior] = po[interior] >> 1
    # expansion blocks in desc order of the leaves (runtime.cpp expand): n - 1 pairs each
    multi = nprims > 1
    sizes = np.where(multi, nprims - 1, 0)
    starts = base + np.concatenate([[0], np.cumsum(sizes)[:-1]])
    pl[multi] = starts[multi] >> 1
    top = int(base + sizes.sum())
    return pl.astype(np.int32), (top * 64 + 127) // 128


def morton(p):
    """30-bit Morton code of points over their bounding box."""
    mn, mx = p.min(0), p.max(0)
    q = ((p - mn) / (mx - mn + 1e-9) * 1023).astype(np.uint64)
    code = np.zeros(len(p), np.uint64)
    for b in range(10):
        for k in range(3):
            code |= ((q[:, k] >> np.uint64(b)) & np.uint64(1)) << np.uint64(3 * b + k)
    return code


def main():
    cid = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 60000
    rc = mcpt.CONFIGS[cid]
    t0 = time.time()
    s = mcpt.build_config_scene(cid)
    a = s.arrays()
    print(f"C{cid}: {len(a['mat'])} tris, {len(a['nprims'])} desc nodes, build {time.time() - t0:.1f} s", flush=True)
    ro, rd = surface_rays(a, rc, n, 11)
    m = op.model_margins(a)
    lay, npair = layouts(a)
    res = {"config": cid, "rays": int(len(ro)), "pairs": npair, "rule": "trav_model.c mode 2 (the product's keep_box)",
           "l2_model": "4 MB, 16-way LRU, 128-B lines, rays interleaved 16384 at a time", "kinds": {}}
    for kind, name in ((1, "any_hit"), (0, "closest")):
        r0 = None
        for ln, po in lay.items():
            pl, tl0 = pair_line_of(a, po)
            st = op.model_study(a, ro, rd, 2, kind, pl, tl0, margins=m, cap_per_ray=1024)
            if r0 is None:
                r0 = st
                hit = st["hit"].astype(bool)
                steps, ostp = st["steps"], st["origin_steps"]
                k = {"hit_frac": round(float(hit.mean()), 4),
                     "pair_steps": round(float(steps.mean()), 2),
                     "pair_steps_hit": round(float(steps[hit].mean()), 2) if hit.any() else None,
                     "pair_steps_miss": round(float(steps[~hit].mean()), 2) if (~hit).any() else None,
                     "origin_box_steps": round(float(ostp.mean()), 2),
                     "origin_box_steps_hit": round(float(ostp[hit].mean()), 2) if hit.any() else None,
                     "origin_box_steps_miss": round(float(ostp[~hit].mean()), 2) if (~hit).any() else None,
                     "tri_tests": round(float(st["tris"].mean()), 2), "layouts": {}}
                res["kinds"][name] = k
            off, lines = st["off"], st["lines"]
            distinct = sum(len(np.unique(lines[off[i]:off[i + 1]])) for i in range(0, len(ro), 10)) / len(range(0, len(ro), 10))
            miss = op.lru_sim(lines, off, 16384, 2048, 16)
            k["layouts"][ln] = {"lines_per_ray": round(float(len(lines) / len(ro)), 2),
                                "distinct_lines_per_ray": round(float(distinct), 2),
                                "l2_misses_per_ray": round(miss / len(ro), 3)}
            print(name, ln, k["layouts"][ln], flush=True)
        # ray order: the same rays sorted by the Morton code of their origin (layout 0)
        o = np.argsort(morton(ro), kind="stable")
        pl, tl0 = pair_line_of(a, lay["0 depth-first (product, large trees)"])
        st = op.model_study(a, ro[o], rd[o], 2, kind, pl, tl0, margins=m, cap_per_ray=1024)
        k["l2_misses_per_ray_origin_sorted"] = {str(b): round(op.lru_sim(st["lines"], st["off"], b, 2048, 16) / len(ro), 3)
                                                for b in (4096, 16384)}
        print(name, {x: y for x, y in k.items() if x != "layouts"}, flush=True)
    if len(sys.argv) > 3:
        json.dump(res, open(sys.argv[3], "w"), indent=1)


if __name__ == "__main__":
    main()
