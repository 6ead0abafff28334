"""Inputs of the per-stage golden vectors: the scene and the path
states tools/make_golden.py feeds to the oracle's stage restatements (or_stage_logic /
or_stage_material) and tests/test_gpu.py::test_stage_golden_vectors feeds to mcpt_stage_run.

Scenes (SCENES: fixture suffix -> BASELINE config): sphere.glb + HDR_029 (config 1), and config 2's
proxy (Cornell-style room, spheres of several materials, night_free_Env.hdr), each plus one
directional light, so the light choice picks the env light (HRDI sampling) or the delta light
about half the time each.  Config 2's walls give axis-aligned normals (Appendix A's gram_schmidt
quirk) and its rays start inside the room."""
import numpy as np

SPP, DEPTH, RR = 16, 5, 3
FILM = (17, 17)  # 289 paths, 256 processed (the last row / column never are: :110)
N_MAT = 256


SCENES = {"c1dir": 1, "c2": 2}


def stage_scene(mcpt, cid=1):
    s = mcpt.Scene()
    s.make_proxy(cid)
    s.add_dir_light((-0.3, -1.0, -0.2), (1.0, 0.9, 0.8), 2.0)
    s.build(**mcpt.DEFAULT_BVH)
    return s


def stage_camera(mcpt, cid=1):
    return mcpt.config_camera(mcpt.CONFIGS[cid], *FILM)


def material_state(a, trace_closest, cid=1):
    """256 continuing paths at their closest hits (hit_tri = index into the scene arrays), len 1..5,
    random sample indices and throughputs.  Config 1: rays from a shell aimed into the unit sphere;
    config 2: rays from points inside the room (0.8 of its box) in random directions."""
    rng = np.random.default_rng(2026)
    ro_l, rd_l, tri_l = [], [], []
    inv = np.argsort(a["tri_id"])  # scene triangle id -> array index
    mn, mx = np.asarray(a["bmin"][0], np.float64), np.asarray(a["bmax"][0], np.float64)
    while sum(len(t) for t in tri_l) < N_MAT:
        if cid == 1:
            o = rng.normal(size=(512, 3))
            o = (o / np.linalg.norm(o, axis=1, keepdims=True) * rng.uniform(1.5, 4.0, (512, 1))).astype(np.float32)
            t = rng.uniform(-0.7, 0.7, (512, 3))
        else:
            c, h = (mn + mx) / 2, (mx - mn) / 2 * 0.8
            o = (c + h * rng.uniform(-1.0, 1.0, (512, 3))).astype(np.float32)
            t = o + rng.normal(size=(512, 3))
        d = t - o
        d = (d / np.linalg.norm(d, axis=1, keepdims=True)).astype(np.float32)
        _, _, tri = trace_closest(a, o, d)
        k = tri >= 0
        ro_l.append(o[k]), rd_l.append(d[k]), tri_l.append(inv[tri[k]])
    ro = np.concatenate(ro_l)[:N_MAT]
    rd = np.concatenate(rd_l)[:N_MAT]
    tri = np.concatenate(tri_l)[:N_MAT].astype(np.int32)
    ln = rng.integers(1, DEPTH + 1, N_MAT).astype(np.uint32)
    sidx = rng.integers(0, SPP, N_MAT).astype(np.uint32)
    beta = np.zeros((N_MAT, 4), np.float32)
    beta[:, :3] = rng.uniform(0.05, 1.0, (N_MAT, 3))
    return {"flags": (ln << 1) | (sidx << 13), "hit_tri": tri, "ray_o": ro, "ray_d": rd, "beta": beta}


def logic_state(ntri, dead_all=False):
    """One path per pixel of the 17 x 17 film in every logic case: dead (with and without samples
    left), primary hit / miss (background), deeper vertices with the MIS terms, visibility bits,
    a zero-throughput sample, Russian roulette depths and the depth cap."""
    rng = np.random.default_rng(29 if dead_all else 17)
    n = FILM[0] * FILM[1]
    samples = rng.integers(0, SPP, n).astype(np.uint32)
    ln = rng.integers(1, DEPTH + 2, n).astype(np.uint32)
    cond = rng.integers(0, 16, n).astype(np.uint32)  # bits 9..12: condL, condB, fzero, hasvis
    cond &= np.where(rng.uniform(size=n) < 0.15, 15, 11).astype(np.uint32)  # fzero in ~15 %
    flags = (ln << 1) | (cond << 9) | (samples << 13)
    dead = rng.uniform(size=n) < 0.25
    if dead_all:
        dead[:] = True
        samples = rng.integers(0, SPP + 1, n).astype(np.uint32)  # some pixels complete
    else:
        samples[dead] = rng.integers(0, SPP + 1, dead.sum()).astype(np.uint32)
    flags[dead] = 1
    hit = np.where(rng.uniform(size=n) < 0.75, rng.integers(0, ntri, n), -1).astype(np.int32)
    d = rng.normal(size=(n, 3))
    d = (d / np.linalg.norm(d, axis=1, keepdims=True)).astype(np.float32)
    beta = rng.uniform(0.02, 1.0, (n, 4)).astype(np.float32)
    beta[:, 3] = rng.uniform(0.1, 2.5, n)
    nee0 = rng.uniform(0.0, 3.0, (n, 4)).astype(np.float32)
    nee1 = rng.uniform(0.0, 3.0, (n, 4)).astype(np.float32)
    vis = (rng.uniform(size=(n, 2)) < 0.7).astype(np.uint8)
    Ld = rng.uniform(0.0, 5.0, (n, 3)).astype(np.float32)
    return {"flags": flags, "samples": samples, "hit_tri": hit, "ray_o": np.zeros((n, 3), np.float32), "ray_d": d,
            "beta": beta, "nee0": nee0, "nee1": nee1, "vis": vis, "Ld": Ld}
