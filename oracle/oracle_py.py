"""ctypes binding of liboracle.so -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this.  The
oracle is the CPU restatement of the reference hot path (see mcpt_oracle.h for its pinning
status).  Scenes are passed as the numpy dict produced by ``mcpt.Scene.arrays()`` (plain
arrays, no product objects).
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

ORACLE_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(ORACLE_DIR, "liboracle.so")
_f = C.POINTER(C.c_float)
_i = C.POINTER(C.c_int32)
_u = C.POINTER(C.c_uint32)


class OrScene(C.Structure):
    _fields_ = [("ntri", C.c_int32), ("v0", _f), ("v1", _f), ("v2", _f), ("n0", _f), ("n1", _f), ("n2", _f),
                ("mat", _i), ("nnodes", C.c_int32), ("bmin", _f), ("bmax", _f), ("offset", _i), ("nprims", _i),
                ("axis", _i), ("nmat", C.c_int32), ("mat_params", _f), ("ndir", C.c_int32), ("dir_params", _f),
                ("env_mode", C.c_int32), ("env_color", C.c_float * 3), ("env_ls", C.c_float),
                ("env_w", C.c_int32), ("env_h", C.c_int32), ("env_tex", _f), ("env_marginal_y", _f),
                ("env_conds_y", _f), ("env_pdf", _f), ("tri_id", _i)]


class OrCamera(C.Structure):
    _fields_ = [("inv_view_proj", C.c_float * 16), ("inv_view", C.c_float * 16), ("lens_radius", C.c_float),
                ("focal", C.c_float)]


class OrConfig(C.Structure):
    _fields_ = [("seed", C.c_uint64), ("spp", C.c_int32), ("max_depth", C.c_int32), ("rr_depth", C.c_int32),
                ("tile_w", C.c_int32), ("tile_h", C.c_int32), ("nthreads", C.c_int32), ("traversal", C.c_int32),
                ("row_begin", C.c_int32), ("row_end", C.c_int32), ("fixed", C.c_int32),
                ("tile_mod", C.c_int32), ("tile_rank", C.c_int32)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} missing: build the oracle (make -C oracle)")
        l = C.CDLL(LIB_PATH)
        sig = {
            "or_render": (C.c_int, [C.POINTER(OrScene), C.POINTER(OrCamera), C.POINTER(OrConfig), C.c_int32, C.c_int32,
                                    _f, _u, C.POINTER(C.c_uint64)]),
            "or_trace_closest": (None, [C.POINTER(OrScene), C.c_int32, _f, _f, C.c_int32, _f, _f, _i]),
            "or_trace_any": (None, [C.POINTER(OrScene), C.c_int32, _f, _f, C.c_int32, C.POINTER(C.c_uint8)]),
            "or_env_build": (None, [C.c_int32, C.c_int32, _f, _f, _f, _f, _f, _f]),
            "or_sinf": (C.c_float, [C.c_float]), "or_cosf": (C.c_float, [C.c_float]),
            "or_asinf": (C.c_float, [C.c_float]), "or_acosf": (C.c_float, [C.c_float]),
            "or_atan2f": (C.c_float, [C.c_float, C.c_float]),
            "or_lowerbias32": (C.c_uint32, [C.c_uint32]), "or_splitmix64": (C.c_uint64, [C.c_uint64]),
            "or_rand": (C.c_float, [C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32]),
            "or_env_fetch": (None, [C.POINTER(OrScene), C.c_float, C.c_float, _f]),
            "or_env_pdf": (C.c_float, [C.POINTER(OrScene), C.c_float, C.c_float, C.c_float]),
            "or_env_dir": (None, [C.POINTER(OrScene), C.c_float, C.c_float, _f]),
            "or_brdf_eval": (None, [_f, _f, _f, _f, _f]),
            "or_power_heuristic": (C.c_float, [C.c_float, C.c_float]),
            "or_upper_bound": (C.c_int32, [_f, C.c_int32, C.c_float]),
            "or_gen_ray": (None, [C.POINTER(OrCamera), C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_uint64,
                                  C.c_uint32, C.c_uint32, _f, _f]),
            "or_stage_logic": (None, [C.POINTER(OrScene), C.POINTER(OrCamera), C.POINTER(OrConfig), C.c_int32,
                                      C.c_int32, _u, _u, _i, _f, _f, _f, _f, _f, C.POINTER(C.c_uint8), _f,
                                      C.POINTER(C.c_uint8)]),
            "or_stage_material": (None, [C.POINTER(OrScene), C.POINTER(OrConfig), C.c_int32, _u, _i, _f, _f, _f,
                                         _f, _f, _f, _f, _f, _f]),
            "or_version": (C.c_char_p, []),
            "or_model_margins": (C.c_int32, [C.POINTER(OrScene), _f, _f, _f]),
            "or_model_set_safe": (None, [C.c_double]),
            "or_model_tri_tests": (C.c_uint64, []),
            "or_model_trace": (None, [C.POINTER(OrScene), C.c_int32, _f, _f, C.c_int32, _f, _f, C.c_float, _i, _f,
                                      C.POINTER(C.c_uint8), C.POINTER(C.c_uint64)]),
            "or_model_study": (None, [C.POINTER(OrScene), C.c_int32, _f, _f, C.c_int32, C.c_int32, _f, _f, C.c_float,
                                      _i, C.c_int32, _i, _i, _i, C.POINTER(C.c_uint8), _i, C.c_int64,
                                      C.POINTER(C.c_int64)]),
            "or_lru_sim": (C.c_int64, [_i, C.POINTER(C.c_int64), C.c_int32, C.c_int32, C.c_int32, C.c_int32]),
        }
        for n, (r, a) in sig.items():
            fn = getattr(l, n)
            fn.restype = r
            fn.argtypes = a
        _lib = l
    return _lib


def fptr(a):
    return a.ctypes.data_as(_f)


def scene_struct(a: dict) -> OrScene:
    keep = {}

    def f(k):
        arr = np.ascontiguousarray(a[k], np.float32)
        keep[k] = arr
        return arr.ctypes.data_as(_f) if arr.size else None

    def i(k):
        arr = np.ascontiguousarray(a[k], np.int32)
        keep[k] = arr
        return arr.ctypes.data_as(_i) if arr.size else None

    s = OrScene()
    s.ntri = len(a["mat"])
    s.v0, s.v1, s.v2, s.n0, s.n1, s.n2 = (f(k) for k in ("v0", "v1", "v2", "n0", "n1", "n2"))
    s.mat = i("mat")
    s.nnodes = len(a["nprims"])
    s.bmin, s.bmax = f("bmin"), f("bmax")
    s.offset, s.nprims, s.axis = i("offset"), i("nprims"), i("axis")
    s.nmat = len(a["mat_params"])
    s.mat_params = f("mat_params")
    s.ndir = len(a["dir_params"])
    s.dir_params = f("dir_params")
    s.env_mode = int(a["env_mode"])
    for k in range(3):
        s.env_color[k] = float(a["env_color"][k])
    s.env_ls = float(a["env_ls"])
    tex = np.asarray(a["env_tex"])
    s.env_h, s.env_w = (tex.shape[0], tex.shape[1]) if tex.size else (0, 0)
    s.env_tex, s.env_marginal_y, s.env_conds_y, s.env_pdf = (f(k) for k in ("env_tex", "env_marginal_y", "env_conds_y", "env_pdf"))
    s.tri_id = i("tri_id") if "tri_id" in a and len(a["tri_id"]) else None
    s._keep = keep
    return s


def camera_struct(cam) -> OrCamera:
    c = OrCamera()
    for k in range(16):
        c.inv_view_proj[k] = cam.inv_view_proj[k]
        c.inv_view[k] = cam.inv_view[k]
    c.lens_radius = cam.lens_radius
    c.focal = cam.focal
    return c


def default_threads():
    """Oracle threads: the cores this process may use, at most 16 (the GPU box's per-GPU share)."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def render(arrays: dict, cam, W, H, spp, max_depth=5, rr_depth=3, seed=0x5EED2026, nthreads=None, traversal=0,
           tile=256, rows=None, fixed=False, part=None):
    """Full CPU re-execution of the reference wavefront loop.  Returns (Ld[H,W,3], samples[H,W], counters).
    part=(rank, world) renders only that rank's tiles of the (tx + ty) mod world partition."""
    s = scene_struct(arrays)
    c = camera_struct(cam)
    nthreads = nthreads or default_threads()
    rb, re = rows if rows else (0, 0)
    tr, tm = part if part else (0, 0)
    cfg = OrConfig(seed, spp, max_depth, rr_depth, tile, tile, nthreads, traversal, rb, re, int(fixed), tm, tr)
    Ld = np.zeros(3 * W * H, np.float32)
    samples = np.zeros(W * H, np.uint32)
    cnt = (C.c_uint64 * 6)()
    rc = lib().or_render(C.byref(s), C.byref(c), C.byref(cfg), W, H, fptr(Ld), samples.ctypes.data_as(_u), cnt)
    if rc != 0:
        raise RuntimeError(f"or_render failed: {rc}")
    keys = ("extend_rays", "shadow_rays", "vis_rays", "iterations", "nodes", "tri_tests")
    return Ld.reshape(H, W, 3), samples.reshape(H, W), dict(zip(keys, list(cnt)))


def _chunks(n, nthreads, fn):
    """fn(i0, i1) over [0, n) in nthreads contiguous chunks on a thread pool (ctypes releases the GIL
    during the C call; the ray functions keep no global state).  Results do not depend on nthreads."""
    if nthreads <= 1 or n < 8192:
        return [fn(0, n)]
    from concurrent.futures import ThreadPoolExecutor

    step = (n + nthreads - 1) // nthreads
    with ThreadPoolExecutor(nthreads) as ex:
        return list(ex.map(lambda i: fn(i, min(n, i + step)), range(0, n, step)))


def trace_closest(arrays, ro, rd, traversal=0, nthreads=1):
    s = scene_struct(arrays)
    ro = np.ascontiguousarray(ro, np.float32).reshape(-1, 3)
    rd = np.ascontiguousarray(rd, np.float32).reshape(-1, 3)
    n = len(ro)
    pos_t = np.zeros((n, 4), np.float32)
    nrm = np.zeros((n, 4), np.float32)
    tri = np.zeros(n, np.int32)

    def run(i0, i1):
        lib().or_trace_closest(C.byref(s), i1 - i0, fptr(ro[i0:i1]), fptr(rd[i0:i1]), traversal, fptr(pos_t[i0:i1]),
                               fptr(nrm[i0:i1]), tri[i0:i1].ctypes.data_as(_i))

    _chunks(n, nthreads, run)
    return pos_t, nrm, tri


def trace_any(arrays, ro, rd, traversal=0, nthreads=1):
    s = scene_struct(arrays)
    ro = np.ascontiguousarray(ro, np.float32).reshape(-1, 3)
    rd = np.ascontiguousarray(rd, np.float32).reshape(-1, 3)
    n = len(ro)
    vis = np.zeros(n, np.uint8)

    def run(i0, i1):
        lib().or_trace_any(C.byref(s), i1 - i0, fptr(ro[i0:i1]), fptr(rd[i0:i1]), traversal,
                           vis[i0:i1].ctypes.data_as(C.POINTER(C.c_uint8)))

    _chunks(n, nthreads, run)
    return vis


def model_margins(arrays, safe_c=0.0):
    """Margins of the product culling rule's model (trav_model.c): per desc node, per triangle own
    box, the far coefficient P and whether every node box contains its subtree's vertices.
    safe_c > 0: mode 6's margins (unbounded triangles bounded for rays at |cos| >= safe_c)."""
    lib().or_model_set_safe(float(safe_c))
    s = scene_struct(arrays)
    nw = np.zeros(max(1, s.nnodes), np.float32)
    tw = np.zeros(max(1, s.ntri), np.float32)
    p = np.zeros(1, np.float32)
    ok = lib().or_model_margins(C.byref(s), fptr(nw), fptr(tw), fptr(p))
    lib().or_model_set_safe(0.0)
    return {"node_w": nw, "tri_w": tw, "p": float(p[0]), "contained": bool(ok)}


def model_trace(arrays, ro, rd, mode, margins=None, nthreads=1, safe_c=0.0):
    """trav_model.c: closest (triangle id, t) and any-hit visibility under culling rule `mode`
    (0 none, 1 round 3, 2 round 4, 6 safe-ray margins with unsafe rays unculled, 7 the product's
    dual tree: safe rays on safe-ray margins, unsafe rays on the general ones -- margins["node_w"] /
    ["tri_w"] then hold the general then the safe values, model_margins_dual) and the number of
    boxes tested.  Modes 6 / 7 classify rays by the planes at safe_c.  nthreads > 1 splits the rays
    over threads (not for modes 6 / 7: the safe-ray switch is module state)."""
    s = scene_struct(arrays)
    m = margins or model_margins(arrays)
    ro = np.ascontiguousarray(ro, np.float32).reshape(-1, 3)
    rd = np.ascontiguousarray(rd, np.float32).reshape(-1, 3)
    n = len(ro)
    tri = np.zeros(n, np.int32)
    t = np.zeros(n, np.float32)
    vis = np.zeros(n, np.uint8)

    def run(i0, i1):
        nodes = C.c_uint64(0)
        lib().or_model_trace(C.byref(s), i1 - i0, fptr(ro[i0:i1]), fptr(rd[i0:i1]), mode, fptr(m["node_w"]),
                             fptr(m["tri_w"]), m["p"], tri[i0:i1].ctypes.data_as(_i), fptr(t[i0:i1]),
                             vis[i0:i1].ctypes.data_as(C.POINTER(C.c_uint8)), C.byref(nodes))
        return int(nodes.value)

    if mode in (6, 7):
        lib().or_model_set_safe(float(safe_c))
    try:
        boxes = sum(_chunks(n, 1 if mode in (6, 7) else nthreads, run))
    finally:
        lib().or_model_set_safe(0.0)
    return tri, t, vis, boxes


def model_study(arrays, ro, rd, mode, kind, pair_line, tri_line0, margins=None, cap_per_ray=256):
    """trav_model.c or_model_study: per ray (steps, origin-box steps, triangle tests, hit) and the
    128-B line stream of its traversal under the node numbering pair_line (analysis only)."""
    s = scene_struct(arrays)
    m = margins or model_margins(arrays)
    ro = np.ascontiguousarray(ro, np.float32).reshape(-1, 3)
    rd = np.ascontiguousarray(rd, np.float32).reshape(-1, 3)
    n = len(ro)
    pl = np.ascontiguousarray(pair_line, np.int32)
    steps, osteps, tris = (np.zeros(n, np.int32) for _ in range(3))
    hit = np.zeros(n, np.uint8)
    cap = n * cap_per_ray
    lines = np.zeros(cap, np.int32)
    off = np.zeros(n + 1, np.int64)
    lib().or_model_study(C.byref(s), n, fptr(ro), fptr(rd), mode, kind, fptr(m["node_w"]), fptr(m["tri_w"]), m["p"],
                         pl.ctypes.data_as(_i), int(tri_line0), steps.ctypes.data_as(_i), osteps.ctypes.data_as(_i),
                         tris.ctypes.data_as(_i), hit.ctypes.data_as(C.POINTER(C.c_uint8)), lines.ctypes.data_as(_i),
                         C.c_int64(cap), off.ctypes.data_as(C.POINTER(C.c_int64)))
    if off[-1] > cap:
        raise ValueError("line buffer too small: raise cap_per_ray")
    return {"steps": steps, "origin_steps": osteps, "tris": tris, "hit": hit, "lines": lines[:off[-1]], "off": off}


def lru_sim(lines, off, batch, sets, ways):
    """trav_model.c or_lru_sim: misses of a sets x ways LRU over the rays' line streams."""
    lines = np.ascontiguousarray(lines, np.int32)
    off = np.ascontiguousarray(off, np.int64)
    return int(lib().or_lru_sim(lines.ctypes.data_as(_i), off.ctypes.data_as(C.POINTER(C.c_int64)), len(off) - 1,
                                int(batch), int(sets), int(ways)))


def model_tri_tests():
    """Triangle tests of the last single-threaded model_trace call (both kinds of its rays)."""
    return int(lib().or_model_tri_tests())


def model_margins_dual(arrays, safe_c):
    """Mode 7's margins: the general ones followed by the safe-ray ones (P of the latter, which is
    the larger)."""
    g = model_margins(arrays)
    s = model_margins(arrays, safe_c=safe_c)
    return {"node_w": np.concatenate([g["node_w"], s["node_w"]]), "tri_w": np.concatenate([g["tri_w"], s["tri_w"]]),
            "p": max(g["p"], s["p"]), "contained": g["contained"] and s["contained"], "p_general": g["p"],
            "p_safe": s["p"]}


def env_build(tex: np.ndarray):
    tex = np.ascontiguousarray(tex, np.float32)
    H, W = tex.shape[:2]
    my = np.zeros(H, np.float32)
    mp = np.zeros(H, np.float32)
    cy = np.zeros((H, W), np.float32)
    pdf = np.zeros((H, W), np.float32)
    den = np.zeros(1, np.float32)
    lib().or_env_build(W, H, fptr(tex), fptr(my), fptr(mp), fptr(cy), fptr(pdf), fptr(den))
    return {"marginal_y": my, "marginal_p": mp, "conds_y": cy, "pdf": pdf, "denom": float(den[0])}


def _stage_cfg(spp, max_depth, rr_depth, seed, fixed):
    return OrConfig(seed, spp, max_depth, rr_depth, 256, 256, 1, 0, 0, 0, int(fixed), 0, 0)


def _a(state, k, dt, shape):
    return np.ascontiguousarray(state[k], dt).reshape(shape).copy()


def stage_logic(arrays, cam, W, H, state, spp, max_depth=5, rr_depth=3, seed=0x5EED2026, fixed=False):
    """or_stage_logic: wf_logic + wf_generate over product-form path state (mcpt_path_view fields)."""
    n = W * H
    s = scene_struct(arrays)
    c = camera_struct(cam)
    cfg = _stage_cfg(spp, max_depth, rr_depth, seed, fixed)
    fl, sm = _a(state, "flags", np.uint32, n), _a(state, "samples", np.uint32, n)
    ht = _a(state, "hit_tri", np.int32, n)
    ro = _a(state, "ray_o", np.float32, (n, 3)) if "ray_o" in state else np.zeros((n, 3), np.float32)
    rd, be = _a(state, "ray_d", np.float32, (n, 3)), _a(state, "beta", np.float32, (n, 4))
    n0, n1 = _a(state, "nee0", np.float32, (n, 4)), _a(state, "nee1", np.float32, (n, 4))
    vis, Ld = _a(state, "vis", np.uint8, (n, 2)), _a(state, "Ld", np.float32, (n, 3))
    q = np.zeros(n, np.uint8)
    u8 = C.POINTER(C.c_uint8)
    lib().or_stage_logic(C.byref(s), C.byref(c), C.byref(cfg), W, H, fl.ctypes.data_as(_u), sm.ctypes.data_as(_u),
                         ht.ctypes.data_as(_i), fptr(ro), fptr(rd), fptr(be), fptr(n0), fptr(n1), vis.ctypes.data_as(u8),
                         fptr(Ld), q.ctypes.data_as(u8))
    return {"flags": fl, "samples": sm, "ray_o": ro, "ray_d": rd, "beta": be, "Ld": Ld, "queued": q}


def stage_material(arrays, state, max_depth=5, rr_depth=3, seed=0x5EED2026, fixed=False):
    """or_stage_material: light choice + wf_mat_mix over product-form continuing paths."""
    n = len(state["flags"])
    s = scene_struct(arrays)
    cfg = _stage_cfg(0, max_depth, rr_depth, seed, fixed)
    fl, ht = _a(state, "flags", np.uint32, n), _a(state, "hit_tri", np.int32, n)
    ro, rd = _a(state, "ray_o", np.float32, (n, 3)), _a(state, "ray_d", np.float32, (n, 3))
    be = _a(state, "beta", np.float32, (n, 4))
    n0, n1 = np.zeros((n, 4), np.float32), np.zeros((n, 4), np.float32)
    lo, ld, bo, bd = (np.zeros((n, 3), np.float32) for _ in range(4))
    lib().or_stage_material(C.byref(s), C.byref(cfg), n, fl.ctypes.data_as(_u), ht.ctypes.data_as(_i), fptr(ro),
                            fptr(rd), fptr(be), fptr(n0), fptr(n1), fptr(lo), fptr(ld), fptr(bo), fptr(bd))
    return {"flags": fl, "ray_o": ro, "ray_d": rd, "beta": be, "nee0": n0, "nee1": n1, "light_o": lo, "light_d": ld,
            "bvis_o": bo, "bvis_d": bd}
