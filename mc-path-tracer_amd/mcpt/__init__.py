"""mcpt -- Python view of the MI355X wavefront path-tracing backend (ctypes over include/mcpt.h).

The product is the C ABI in ``libmcpt.so`` (HIP kernels for gfx950 + host C++).  This module
is the thin Python mirror of the reference's host objects, used by tests/ and bench.py:

* :class:`Scene`      -- ``Scene::load`` / ``set_environment_light`` / ``add_light``
                         (CUDA-RayTracer/Scene.h:40-58) plus the BVH build (BVH.cu).
* :class:`PathTracer` -- ``PathTracer::render_image`` (PathTracer.cpp:112-130) and the
                         ``wavefront_pathtrace`` / ``clear_dfilm`` entry points
                         (wavefront_kernels.cuh:18-31), on one device.
* :func:`make_camera` -- ``Camera::update`` matrices (Camera.cu:194-224).

There is no CPU fallback: constructing a :class:`PathTracer` without a gfx950 device raises.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.dirname(_HERE)
REPO_DIR = os.path.dirname(PKG_DIR)
LIB_PATH = os.environ.get("MCPT_LIB") or os.path.join(PKG_DIR, "libmcpt.so")
ASSET_DIR = os.path.join(REPO_DIR, "assets")

MCPT_OK = 0
STAGE_LOGIC, STAGE_GENERATE, STAGE_MATERIAL, STAGE_EXTEND, STAGE_SHADOW = range(5)

_f = C.POINTER(C.c_float)
_i = C.POINTER(C.c_int32)
_u = C.POINTER(C.c_uint32)


class Config(C.Structure):
    _fields_ = [("seed", C.c_uint64), ("spp", C.c_int32), ("max_depth", C.c_int32), ("rr_depth", C.c_int32),
                ("tile_w", C.c_int32), ("tile_h", C.c_int32), ("flags", C.c_int32)]


class SceneDesc(C.Structure):
    _fields_ = [("ntri", C.c_int32), ("v0", _f), ("v1", _f), ("v2", _f), ("n0", _f), ("n1", _f), ("n2", _f),
                ("mat", _i), ("nnodes", C.c_int32), ("bmin", _f), ("bmax", _f), ("offset", _i), ("nprims", _i),
                ("axis", _i), ("nmat", C.c_int32), ("mat_params", _f), ("ndir", C.c_int32), ("dir_params", _f),
                ("env_mode", C.c_int32), ("env_color", C.c_float * 3), ("env_ls", C.c_float),
                ("env_w", C.c_int32), ("env_h", C.c_int32), ("env_tex", _f), ("env_marginal_y", _f),
                ("env_conds_y", _f), ("env_pdf", _f), ("tri_id", _i)]


class Camera(C.Structure):
    _fields_ = [("inv_view_proj", C.c_float * 16), ("inv_view", C.c_float * 16), ("lens_radius", C.c_float),
                ("focal", C.c_float)]


class CameraParams(C.Structure):
    _fields_ = [("position", C.c_float * 3), ("yaw_deg", C.c_float), ("pitch_deg", C.c_float),
                ("fovy_rad", C.c_float), ("aspect", C.c_float), ("znear", C.c_float), ("zfar", C.c_float),
                ("lens_radius", C.c_float), ("focal", C.c_float)]


class StageStats(C.Structure):
    _fields_ = [("extend_rays", C.c_uint64), ("shadow_rays", C.c_uint64), ("vis_rays", C.c_uint64),
                ("iterations", C.c_uint64), ("live_paths", C.c_uint64), ("ms_total", C.c_float),
                ("ms_shade", C.c_float), ("ms_extend", C.c_float), ("ms_shadow", C.c_float),
                ("ext_nodes", C.c_uint64), ("ext_tests", C.c_uint64), ("ext_hits", C.c_uint64),
                ("any_nodes", C.c_uint64), ("any_tests", C.c_uint64), ("any_hits", C.c_uint64)]

    def as_dict(self) -> dict:
        return {k: getattr(self, k) for k, _ in self._fields_}

    @property
    def rays(self) -> int:
        return int(self.extend_rays + self.shadow_rays + self.vis_rays)


class PathView(C.Structure):  # mcpt_path_view: path state at the shading stages' boundary
    _fields_ = [("film_w", C.c_uint32), ("film_h", C.c_uint32), ("flags", _u), ("samples", _u), ("hit_tri", _i),
                ("ray_o", _f), ("ray_d", _f), ("beta", _f), ("nee0", _f), ("nee1", _f),
                ("vis", C.POINTER(C.c_uint8)), ("Ld", _f), ("light_o", _f), ("light_d", _f), ("bvis_o", _f),
                ("bvis_d", _f), ("queued", C.POINTER(C.c_uint8))]


class SoaView(C.Structure):
    _fields_ = [("ray_o", _f), ("ray_d", _f), ("hit_pos_t", _f), ("hit_nrm_mat", _f), ("hit_tri", _i),
                ("visible", C.POINTER(C.c_uint8)), ("steps", _u), ("paths", C.POINTER(PathView))]


# mcpt_path_view fields as numpy: (dtype, values per path)
PATH_FIELDS = {"flags": (np.uint32, 1), "samples": (np.uint32, 1), "hit_tri": (np.int32, 1), "ray_o": (np.float32, 3),
               "ray_d": (np.float32, 3), "beta": (np.float32, 4), "nee0": (np.float32, 4), "nee1": (np.float32, 4),
               "vis": (np.uint8, 2), "Ld": (np.float32, 3), "light_o": (np.float32, 3), "light_d": (np.float32, 3),
               "bvis_o": (np.float32, 3), "bvis_d": (np.float32, 3), "queued": (np.uint8, 1)}
STAGE_BY_NAME = {"logic": STAGE_LOGIC, "generate": STAGE_GENERATE, "material": STAGE_MATERIAL}


def path_view(arrs: dict, n, film=(0, 0)):
    """PathView over numpy arrays (missing fields stay NULL); the arrays are kept on the view."""
    v = PathView()
    v.film_w, v.film_h = film
    keep = {}
    for k, (dt, m) in PATH_FIELDS.items():
        if k in arrs and arrs[k] is not None:
            a = np.ascontiguousarray(arrs[k], dt).reshape(n * m)
            keep[k] = a
            setattr(v, k, a.ctypes.data_as(C.POINTER(np.ctypeslib.as_ctypes_type(dt))))
    v._keep = keep
    return v


# Every symbol declared in include/mcpt.h with its ctypes signature.
ABI = {
    "mcpt_create": (C.c_int, [C.c_int, C.POINTER(Config), C.POINTER(C.c_void_p)]),
    "mcpt_destroy": (None, [C.c_void_p]),
    "mcpt_last_error": (C.c_char_p, [C.c_void_p]),
    "mcpt_scene_upload": (C.c_int, [C.c_void_p, C.POINTER(SceneDesc)]),
    "mcpt_camera_set": (C.c_int, [C.c_void_p, C.POINTER(Camera)]),
    "mcpt_film_resize": (C.c_int, [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32]),
    "mcpt_film_clear": (C.c_int, [C.c_void_p]),
    "mcpt_set_tiles": (C.c_int, [C.c_void_p, _u, C.c_uint32]),
    "mcpt_set_compact_paths": (C.c_int, [C.c_void_p, C.c_int32]),
    "mcpt_debug_tiny_lds_stack": (C.c_int, [C.c_void_p, C.c_int32]),
    "mcpt_set_path_slots": (C.c_int, [C.c_void_p, C.c_uint32]),
    "mcpt_set_trace_partitions": (C.c_int, [C.c_void_p, C.c_uint32]),
    "mcpt_gather": (C.c_int, [C.POINTER(C.c_void_p), C.c_int32, C.c_int32]),
    "mcpt_wavefront_step": (C.c_int, [C.c_void_p, C.c_uint32, C.c_uint32, C.POINTER(StageStats)]),
    "mcpt_iterate": (C.c_int, [C.c_void_p, C.c_uint32, C.POINTER(StageStats)]),
    "mcpt_render": (C.c_int, [C.c_void_p, C.POINTER(StageStats)]),
    "mcpt_stage_run": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(SoaView), C.POINTER(SoaView), C.c_uint32]),
    "mcpt_film_read": (C.c_int, [C.c_void_p, _f, _u]),
    "mcpt_film_read_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p]),
    "mcpt_film_pack_tiles": (C.c_int, [C.c_void_p, C.c_void_p, _u]),
    "mcpt_film_unpack_tiles": (C.c_int, [C.c_void_p, C.c_void_p, _u, C.c_uint32]),
    "mcpt_film_tonemap_rgba8": (C.c_int, [C.c_void_p, C.c_float, C.POINTER(C.c_uint8)]),
    "mcpt_sync": (C.c_int, [C.c_void_p]),
    "mcpt_device_name": (C.c_int, [C.c_void_p, C.c_char_p, C.c_int32]),
    "mcpt_debug_queue_rays": (C.c_int, [C.c_void_p, C.c_int, _f, _f, _u]),
    "mcpt_debug_last_stage_ms": (C.c_float, [C.c_void_p]),
    "mcpt_debug_last_build_ms": (C.c_float, [C.c_void_p]),
    "mcpt_debug_last_env_build_ms": (C.c_float, [C.c_void_p]),
    "mcpt_debug_env_tables": (C.c_int, [C.c_void_p, _f, _f, _f, _i]),
    "mcpt_debug_node_layout": (C.c_int, [C.c_void_p]),
    "mcpt_debug_occ_stats": (C.c_int, [C.c_void_p, C.POINTER(C.c_uint64), C.POINTER(C.c_int32)]),
    "mcpt_debug_ray_counts": (C.c_int, [C.c_void_p, C.POINTER(C.c_uint64)]),
    "mcpt_set_work_counters": (C.c_int, [C.c_void_p, C.c_int32]),
    "mcpt_scene_upload_gpu_bvh": (C.c_int, [C.c_void_p, C.c_void_p]),
    "mcpt_set_gpu_bvh_builder": (C.c_int, [C.c_void_p, C.c_int32]),
    "mcpt_film_size": (C.c_int, [C.c_void_p, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]),
    "mcpt_film_write_png": (C.c_int, [C.c_void_p, C.c_float, C.c_char_p]),
    "mcpt_film_write_pfm": (C.c_int, [C.c_void_p, C.c_char_p]),
    "mcpt_image_write_png": (C.c_int, [C.c_char_p, C.c_uint32, C.c_uint32, C.POINTER(C.c_uint8)]),
    "mcpt_image_write_pfm": (C.c_int, [C.c_char_p, C.c_uint32, C.c_uint32, C.POINTER(C.c_float)]),
    "mcpt_debug_trace_profile": (C.c_int, [C.c_void_p, C.POINTER(C.c_uint64), C.c_int]),
    "mcpt_debug_shade_sections": (C.c_int, [C.c_void_p, C.POINTER(C.c_uint64), C.c_int, C.c_int]),
    "mcpt_scene_build_ex": (C.c_int, [C.c_void_p, C.c_void_p]),
    "mcpt_debug_quot": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p]),
    "mcpt_debug_hbm_copy": (C.c_int, [C.c_void_p, C.c_uint64, C.c_uint32, C.POINTER(C.c_double)]),
    "mcpt_scene_new": (C.c_void_p, []),
    "mcpt_scene_free": (None, [C.c_void_p]),
    "mcpt_scene_load_glb": (C.c_int, [C.c_void_p, C.c_char_p, _f]),
    "mcpt_scene_add_mesh": (C.c_int, [C.c_void_p, C.c_int32, _f, _f, _f, _f, _f, _f, _f]),
    "mcpt_scene_set_env_hdr": (C.c_int, [C.c_void_p, C.c_char_p, C.c_int32]),
    "mcpt_scene_set_env_hdr_ex": (C.c_int, [C.c_void_p, C.c_char_p, C.c_int32, C.c_uint32]),
    "mcpt_scene_set_env_color": (C.c_int, [C.c_void_p, _f, C.c_float]),
    "mcpt_scene_add_dir_light": (C.c_int, [C.c_void_p, _f, _f, C.c_float]),
    "mcpt_scene_transform": (C.c_int, [C.c_void_p, _f]),
    "mcpt_scene_make_proxy": (C.c_int, [C.c_void_p, C.c_int32, C.c_char_p]),
    "mcpt_scene_build": (C.c_int, [C.c_void_p, C.c_int32]),
    "mcpt_scene_get_desc": (C.c_int, [C.c_void_p, C.POINTER(SceneDesc)]),
    "mcpt_scene_bvh_depth": (C.c_int, [C.c_void_p]),
    "mcpt_camera_make": (C.c_int, [C.POINTER(CameraParams), C.POINTER(Camera)]),
}

_lib = None


def lib() -> C.CDLL:
    """Load libmcpt.so (in-tree build).  Raises if it has not been built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} missing: run __graft_entry__.build() (make) first")
        l = C.CDLL(LIB_PATH)
        for name, (res, args) in ABI.items():
            fn = getattr(l, name, None)
            if fn is None and os.environ.get("MCPT_LIB"):
                continue  # an older experimental variant library (tools/gpu/ab_libs.sh)
            if fn is None:
                raise RuntimeError(f"{LIB_PATH} does not export {name}: rebuild it")
            fn.restype = res
            fn.argtypes = args
        _lib = l
    return _lib


class McptError(RuntimeError):
    pass


def _check(rc: int, ctx=None):
    if rc != MCPT_OK:
        msg = lib().mcpt_last_error(ctx)
        raise McptError(f"mcpt error {rc}: {msg.decode() if msg else ''}")


def fptr(a: np.ndarray):
    return a.ctypes.data_as(_f)


class BvhParams(C.Structure):  # mcpt_bvh_params
    _fields_ = [("builder", C.c_int32), ("max_prims", C.c_int32), ("buckets", C.c_int32),
                ("trav_cost", C.c_float), ("isect_cost", C.c_float)]


BVH_REFERENCE, BVH_SAH3 = 0, 1
FLAG_FIXED = 1  # MCPT_FLAG_FIXED: quality-mode integrator
FLAG_NO_AUTO_CLEAR = 2  # MCPT_FLAG_NO_AUTO_CLEAR: camera / scene changes do not clear the film
ENV_DEVICE_TABLES = 1  # MCPT_ENV_DEVICE_TABLES: HRDI tables built on the device at upload


def default_config(spp=16, max_depth=5, rr_depth=3, seed=0x5EED2026, tile=256, fixed=False,
                   auto_clear=True) -> Config:
    flags = (FLAG_FIXED if fixed else 0) | (0 if auto_clear else FLAG_NO_AUTO_CLEAR)
    return Config(seed, spp, max_depth, rr_depth, tile, tile, flags)


def make_camera(position, yaw_deg=-90.0, pitch_deg=0.0, fovy_deg=45.0, aspect=1.0, znear=0.01, zfar=1e4,
                lens_radius=1e-4, focal=35.0) -> Camera:
    """PerspectiveCamera + Camera::update (Camera.cu:194-224) -> dCamera matrices."""
    p = CameraParams((C.c_float * 3)(*position), yaw_deg, pitch_deg, np.float32(np.radians(np.float32(fovy_deg))),
                     aspect, znear, zfar, lens_radius, focal)
    cam = Camera()
    _check(lib().mcpt_camera_make(C.byref(p), C.byref(cam)))
    return cam


def _arr(ptr, n, dtype):
    if n == 0 or not ptr:
        return np.zeros(0, dtype)
    ct = {np.float32: C.c_float, np.int32: C.c_int32}[dtype]
    return np.ctypeslib.as_array(C.cast(ptr, C.POINTER(ct)), shape=(n,)).copy()


class Scene:
    """Host scene builder (Scene.cu) -- owns flat BVH-ordered arrays after build()."""

    def __init__(self):
        self.h = lib().mcpt_scene_new()
        if not self.h:
            raise McptError("mcpt_scene_new failed")

    def __del__(self):
        if getattr(self, "h", None):
            try:
                lib().mcpt_scene_free(self.h)
            except Exception:  # interpreter shutdown
                pass
            self.h = None

    def _ck(self, rc):
        _check(rc)
        return self

    def load_glb(self, path, xform=None):
        xf = None if xform is None else fptr(np.ascontiguousarray(xform, np.float32).reshape(16))
        return self._ck(lib().mcpt_scene_load_glb(self.h, str(path).encode(), xf))

    def add_mesh(self, v0, v1, v2, n0, n1, n2, base_rgb=(1.0, 1.0, 1.0)):
        arrs = [np.ascontiguousarray(a, np.float32).reshape(-1, 3) for a in (v0, v1, v2, n0, n1, n2)]
        bc = np.asarray(base_rgb, np.float32)
        return self._ck(lib().mcpt_scene_add_mesh(self.h, len(arrs[0]), *[fptr(a) for a in arrs], fptr(bc)))

    def set_env_hdr(self, path, mode=1, device_tables=False):
        """EnvironmentLight from an .hdr.  device_tables=True keeps the texture only; the
        light tables are then built on the device at upload (MCPT_ENV_DEVICE_TABLES)."""
        if device_tables:
            return self._ck(lib().mcpt_scene_set_env_hdr_ex(self.h, str(path).encode(), mode, ENV_DEVICE_TABLES))
        return self._ck(lib().mcpt_scene_set_env_hdr(self.h, str(path).encode(), mode))

    def set_env_color(self, rgb, ls=1.0):
        return self._ck(lib().mcpt_scene_set_env_color(self.h, fptr(np.asarray(rgb, np.float32)), ls))

    def add_dir_light(self, direction, rgb, ls=1.0):
        return self._ck(lib().mcpt_scene_add_dir_light(self.h, fptr(np.asarray(direction, np.float32)),
                                                       fptr(np.asarray(rgb, np.float32)), ls))

    def transform(self, xform):
        return self._ck(lib().mcpt_scene_transform(self.h, fptr(np.ascontiguousarray(xform, np.float32).reshape(16))))

    def make_proxy(self, config_id, asset_dir=ASSET_DIR):
        return self._ck(lib().mcpt_scene_make_proxy(self.h, config_id, str(asset_dir).encode()))

    def build(self, max_prims=8, builder="reference", buckets=32, trav_cost=1.0, isect_cost=1.0):
        """BVH + env tables.  builder "reference" = BVHAccel's SAH (mcpt_scene_build); "sah3" =
        binned SAH over all three axes (mcpt_scene_build_ex).  Films do not depend on the tree."""
        if builder == "reference":
            return self._ck(lib().mcpt_scene_build(self.h, max_prims))
        if builder != "sah3":
            raise ValueError(f"unknown builder {builder!r}")
        p = BvhParams(BVH_SAH3, max_prims, buckets, trav_cost, isect_cost)
        return self._ck(lib().mcpt_scene_build_ex(self.h, C.byref(p)))

    def desc(self) -> SceneDesc:
        d = SceneDesc()
        _check(lib().mcpt_scene_get_desc(self.h, C.byref(d)))
        d._owner = self  # keep arrays alive
        return d

    @property
    def bvh_depth(self) -> int:
        return lib().mcpt_scene_bvh_depth(self.h)

    def arrays(self) -> dict:
        """Copies of the built arrays as numpy (for oracles, tests and fixtures)."""
        d = self.desc()
        T, N = d.ntri, d.nnodes
        out = {k: _arr(getattr(d, k), 3 * T, np.float32).reshape(T, 3) for k in ("v0", "v1", "v2", "n0", "n1", "n2")}
        out["mat"] = _arr(d.mat, T, np.int32)
        out["bmin"] = _arr(d.bmin, 3 * N, np.float32).reshape(N, 3)
        out["bmax"] = _arr(d.bmax, 3 * N, np.float32).reshape(N, 3)
        for k in ("offset", "nprims", "axis"):
            out[k] = _arr(getattr(d, k), N, np.int32)
        out["mat_params"] = _arr(d.mat_params, 8 * d.nmat, np.float32).reshape(d.nmat, 8)
        out["dir_params"] = _arr(d.dir_params, 7 * d.ndir, np.float32).reshape(d.ndir, 7)
        out["env_mode"] = d.env_mode
        out["env_color"] = np.array(list(d.env_color), np.float32)
        out["env_ls"] = np.float32(d.env_ls)
        W, H = d.env_w, d.env_h
        out["env_tex"] = _arr(d.env_tex, 4 * W * H, np.float32).reshape(H, W, 4)
        out["env_marginal_y"] = _arr(d.env_marginal_y, H, np.float32)
        # tables are absent (size 0) when left to the device build (set_env_hdr(device_tables=True))
        out["env_conds_y"] = _arr(d.env_conds_y, W * H, np.float32).reshape(H, W) if d.env_conds_y else np.zeros(0, np.float32)
        out["env_pdf"] = _arr(d.env_pdf, W * H, np.float32).reshape(H, W) if d.env_pdf else np.zeros(0, np.float32)
        out["tri_id"] = _arr(d.tri_id, T, np.int32) if d.tri_id else np.arange(T, dtype=np.int32)
        return out


def desc_from_arrays(a: dict) -> SceneDesc:
    """SceneDesc pointing at numpy arrays in ``a`` (kept alive on the returned object)."""
    keep = {}

    def f(k):
        arr = np.ascontiguousarray(a[k], np.float32)
        keep[k] = arr
        return arr.ctypes.data_as(_f) if arr.size else None

    def i(k):
        arr = np.ascontiguousarray(a[k], np.int32)
        keep[k] = arr
        return arr.ctypes.data_as(_i) if arr.size else None

    d = SceneDesc()
    d.ntri = len(a["mat"])
    d.v0, d.v1, d.v2, d.n0, d.n1, d.n2 = (f(k) for k in ("v0", "v1", "v2", "n0", "n1", "n2"))
    d.mat = i("mat")
    d.nnodes = len(a["nprims"])
    d.bmin, d.bmax = f("bmin"), f("bmax")
    d.offset, d.nprims, d.axis = i("offset"), i("nprims"), i("axis")
    d.nmat = len(a["mat_params"])
    d.mat_params = f("mat_params")
    d.ndir = len(a["dir_params"])
    d.dir_params = f("dir_params")
    d.env_mode = int(a["env_mode"])
    for k in range(3):
        d.env_color[k] = float(a["env_color"][k])
    d.env_ls = float(a["env_ls"])
    tex = np.asarray(a["env_tex"])
    d.env_h, d.env_w = (tex.shape[0], tex.shape[1]) if tex.size else (0, 0)
    d.env_tex, d.env_marginal_y, d.env_conds_y, d.env_pdf = (f(k) for k in ("env_tex", "env_marginal_y", "env_conds_y", "env_pdf"))
    d.tri_id = i("tri_id") if "tri_id" in a and len(a["tri_id"]) else None
    d._keep = keep
    return d


class PathTracer:
    """Device context (one GPU): the reference's PathTracer + Film device state."""

    def __init__(self, device=0, config: Config | None = None):
        self.cfg = config or default_config()
        h = C.c_void_p()
        _check(lib().mcpt_create(device, C.byref(self.cfg), C.byref(h)))
        self.h = h
        self.W = self.H = 0

    def close(self):
        if getattr(self, "h", None):
            try:
                lib().mcpt_destroy(self.h)
            except Exception:  # interpreter shutdown
                pass
            self.h = None

    __del__ = close

    def _ck(self, rc):
        _check(rc, self.h)

    @property
    def device_name(self) -> str:
        buf = C.create_string_buffer(256)
        self._ck(lib().mcpt_device_name(self.h, buf, 256))
        return buf.value.decode()

    def upload_scene(self, scene, gpu_bvh=False):
        """mcpt_scene_upload (host BVH from the scene), or with gpu_bvh=True / "ploc" / "lbvh"
        mcpt_scene_upload_gpu_bvh (BVH built on the device, PLOC by default; same hits)."""
        d = scene.desc() if isinstance(scene, Scene) else scene
        if gpu_bvh:
            if gpu_bvh not in (True, "ploc", "lbvh"):
                raise ValueError(f"unknown GPU BVH builder {gpu_bvh!r}")
            # True is the documented default (PLOC), set explicitly: the builder is context state,
            # so an earlier "lbvh" upload must not carry over
            self._ck(lib().mcpt_set_gpu_bvh_builder(self.h, 0 if gpu_bvh == "lbvh" else 1))
            self._ck(lib().mcpt_scene_upload_gpu_bvh(self.h, C.byref(d)))
        else:
            self._ck(lib().mcpt_scene_upload(self.h, C.byref(d)))

    def ray_counts(self) -> dict:
        """Ray counts since the last film clear (mcpt_debug_ray_counts)."""
        v = (C.c_uint64 * 5)()
        if hasattr(lib(), "mcpt_debug_ray_counts") or not os.environ.get("MCPT_LIB"):
            self._ck(lib().mcpt_debug_ray_counts(self.h, v))  # (an older variant library: zeros)
        return dict(zip(("extension", "extension_traversed", "any_hit", "any_hit_traversed", "any_hit_occluder_cache"),
                        [int(x) for x in v]))

    def occ_stats(self):
        """(any-hit rays the occluder cache resolved since the last film clear, cache enabled)."""
        r, e = C.c_uint64(0), C.c_int32(0)
        self._ck(lib().mcpt_debug_occ_stats(self.h, C.byref(r), C.byref(e)))
        return int(r.value), bool(e.value)

    @property
    def last_build_ms(self) -> float:
        return lib().mcpt_debug_last_build_ms(self.h)

    @property
    def last_env_build_ms(self) -> float:
        """Device time of the last HRDI table build at upload (tables not in the desc)."""
        return lib().mcpt_debug_last_env_build_ms(self.h)

    def env_tables(self, W, H) -> dict:
        """The uploaded scene's device HRDI tables (W x H map) and whether they were built on the
        device / the env_cell search guides are on."""
        my = np.zeros(H, np.float32)
        cy = np.zeros((H, W), np.float32)
        pdf = np.zeros((H, W), np.float32)
        fl = C.c_int32(0)
        self._ck(lib().mcpt_debug_env_tables(self.h, fptr(my), fptr(cy), fptr(pdf), C.byref(fl)))
        return {"marginal_y": my, "conds_y": cy, "pdf": pdf, "device_built": bool(fl.value & 1),
                "guides": bool(fl.value & 2)}

    def set_camera(self, cam: Camera):
        self._ck(lib().mcpt_camera_set(self.h, C.byref(cam)))

    def resize(self, W, H, tile_w=256, tile_h=256):
        self._ck(lib().mcpt_film_resize(self.h, W, H, tile_w, tile_h))
        self.W, self.H, self.tile_w, self.tile_h = W, H, tile_w, tile_h

    def clear(self):
        self._ck(lib().mcpt_film_clear(self.h))

    def set_path_slots(self, slots):
        """Paths in flight per pixel (mcpt_set_path_slots); re-allocates and clears the film."""
        self._ck(lib().mcpt_set_path_slots(self.h, slots))

    def set_work_counters(self, on=True):
        """Traversal work counters in StageStats (mcpt_set_work_counters; off by default: the
        counting k_trace build is slower)."""
        if hasattr(lib(), "mcpt_set_work_counters") or not os.environ.get("MCPT_LIB"):
            self._ck(lib().mcpt_set_work_counters(self.h, int(bool(on))))  # (an older variant library counts always)

    def set_trace_partitions(self, nparts=0):
        """k_trace work partitions (mcpt_set_trace_partitions); 0 = the device default, two per XCD."""
        self._ck(lib().mcpt_set_trace_partitions(self.h, nparts))

    def set_compact_paths(self, on=True):
        """Path state over the tile set only (mcpt_set_compact_paths); re-allocates and clears the film.
        In this layout set_tiles re-allocates and clears too."""
        self._ck(lib().mcpt_set_compact_paths(self.h, int(bool(on))))

    def set_tiny_lds_stack(self, on=True):
        """Tests: the traversal's 2-entry LDS stack instantiation (mcpt_debug_tiny_lds_stack)."""
        self._ck(lib().mcpt_debug_tiny_lds_stack(self.h, int(bool(on))))

    def set_tiles(self, tiles=None):
        if tiles is None:
            self._ck(lib().mcpt_set_tiles(self.h, None, 0))
        else:
            t = np.ascontiguousarray(tiles, np.uint32).reshape(-1, 2)
            self._ck(lib().mcpt_set_tiles(self.h, t.ctypes.data_as(_u), len(t)))

    def step(self, tile_x, tile_y) -> StageStats:
        st = StageStats()
        self._ck(lib().mcpt_wavefront_step(self.h, tile_x, tile_y, C.byref(st)))
        return st

    def iterate(self, n) -> StageStats:
        st = StageStats()
        self._ck(lib().mcpt_iterate(self.h, n, C.byref(st)))
        return st

    def render(self) -> StageStats:
        st = StageStats()
        self._ck(lib().mcpt_render(self.h, C.byref(st)))
        return st

    def film(self):
        P = self.W * self.H
        Ld = np.zeros(3 * P, np.float32)
        s = np.zeros(P, np.uint32)
        self._ck(lib().mcpt_film_read(self.h, fptr(Ld), s.ctypes.data_as(_u)))
        return Ld.reshape(self.H, self.W, 3), s.reshape(self.H, self.W)

    def tonemap(self, exposure=1.0):
        out = np.zeros(self.W * self.H * 4, np.uint8)
        self._ck(lib().mcpt_film_tonemap_rgba8(self.h, exposure, out.ctypes.data_as(C.POINTER(C.c_uint8))))
        return out.reshape(self.H, self.W, 4)

    def trace_closest(self, ro, rd, steps=False):
        ro = np.ascontiguousarray(ro, np.float32).reshape(-1, 3)
        rd = np.ascontiguousarray(rd, np.float32).reshape(-1, 3)
        n = len(ro)
        pos_t = np.zeros((n, 4), np.float32)
        nrm = np.zeros((n, 4), np.float32)
        tri = np.zeros(n, np.int32)
        st = np.zeros(n, np.uint32) if steps else None
        vin = SoaView(fptr(ro), fptr(rd), None, None, None, None, None)
        vout = SoaView(None, None, fptr(pos_t), fptr(nrm), tri.ctypes.data_as(_i), None,
                       st.ctypes.data_as(_u) if steps else None)
        self._ck(lib().mcpt_stage_run(self.h, STAGE_EXTEND, C.byref(vin), C.byref(vout), n))
        return (pos_t, nrm, tri, st) if steps else (pos_t, nrm, tri)

    def trace_any(self, ro, rd, steps=False):
        ro = np.ascontiguousarray(ro, np.float32).reshape(-1, 3)
        rd = np.ascontiguousarray(rd, np.float32).reshape(-1, 3)
        n = len(ro)
        vis = np.zeros(n, np.uint8)
        st = np.zeros(n, np.uint32) if steps else None
        vin = SoaView(fptr(ro), fptr(rd), None, None, None, None, None)
        vout = SoaView(None, None, None, None, None, vis.ctypes.data_as(C.POINTER(C.c_uint8)),
                       st.ctypes.data_as(_u) if steps else None)
        self._ck(lib().mcpt_stage_run(self.h, STAGE_SHADOW, C.byref(vin), C.byref(vout), n))
        return (vis, st) if steps else vis

    def stage(self, name, state: dict, film=None) -> dict:
        """mcpt_stage_run of one shading stage ("logic", "generate", "material") over caller path
        state (numpy arrays keyed as mcpt_path_view's fields, n paths); returns every output
        field.  film=(W, H) for logic / generate: path i is pixel (i % W, i // W)."""
        n = len(state["flags"])
        film = film or (0, 0)
        vin = SoaView()
        pin = path_view(state, n, film)
        vin.paths = C.pointer(pin)
        outs = {k: np.zeros((n, m) if m > 1 else n, dt) for k, (dt, m) in PATH_FIELDS.items()}
        vout = SoaView()
        pout = path_view(outs, n, film)
        vout.paths = C.pointer(pout)
        self._ck(lib().mcpt_stage_run(self.h, STAGE_BY_NAME[name], C.byref(vin), C.byref(vout), n))
        return {k: pout._keep[k].reshape(outs[k].shape) for k in outs}

    @property
    def last_stage_ms(self) -> float:
        return lib().mcpt_debug_last_stage_ms(self.h)

    def write_png(self, path, exposure=1.0):
        """Tonemapped film as 8-bit RGB PNG (mcpt_film_write_png)."""
        self._ck(lib().mcpt_film_write_png(self.h, exposure, os.fsencode(path)))

    def write_pfm(self, path):
        """Averaged radiance Ld/samples as float RGB PFM (mcpt_film_write_pfm)."""
        self._ck(lib().mcpt_film_write_pfm(self.h, os.fsencode(path)))

    def trace_profile(self, reset=True):
        """k_trace loop-phase counts of the counting build (mcpt_debug_trace_profile; work counters on)
        since the last film clear or reset, as a dict of wave-summed counts (None: none recorded)."""
        v = (C.c_uint64 * 12)()
        n = lib().mcpt_debug_trace_profile(self.h, v, int(reset))
        names = ("trips", "refills", "refill_lanes", "node_iters", "tri_phases", "tri_lanes", "trip_node_lanes",
                 "trip_leaf_lanes", "trip_idle_lanes", "finish_trips", "pop_iters")
        return {k: int(x) for k, x in zip(names, v)} if n > 0 else None

    def hbm_copy_gbps(self, nbytes=1 << 30, iters=20) -> float:
        """Measured HBM copy ceiling (read + write GB/s) of a hand-written dwordx4 copy kernel."""
        g = C.c_double(0.0)
        self._ck(lib().mcpt_debug_hbm_copy(self.h, nbytes, iters, C.byref(g)))
        return g.value

    def debug_quot(self, a, b):
        """a / b as the kernels divide (shared fp64 reciprocal, mcpt_core.hpp quot3)."""
        a = np.ascontiguousarray(a, np.float32)
        b = np.ascontiguousarray(b, np.float32)
        out = np.empty_like(a)
        self._ck(lib().mcpt_debug_quot(self.h, a.ctypes.data, b.ctypes.data, a.size, out.ctypes.data))
        return out

    def queue_rays(self):
        """Rays of the current extension queue (diagnostics)."""
        n = C.c_uint32(0)
        self._ck(lib().mcpt_debug_queue_rays(self.h, 0, None, None, C.byref(n)))
        ro = np.zeros((n.value, 3), np.float32)
        rd = np.zeros((n.value, 3), np.float32)
        self._ck(lib().mcpt_debug_queue_rays(self.h, 0, fptr(ro), fptr(rd), C.byref(n)))
        return ro[: n.value], rd[: n.value]


def gather(tracers, root=0):
    """mcpt_gather: copy every PathTracer's tile-set pixels into tracers[root]'s film (one process,
    one context per GPU, device-to-device over xGMI)."""
    arr = (C.c_void_p * len(tracers))(*[t.h for t in tracers])
    _check(lib().mcpt_gather(arr, len(tracers), root), tracers[root].h)


@dataclass(frozen=True)
class RenderConfig:
    """BASELINE.json configs."""
    cid: int
    width: int
    height: int
    spp: int
    max_depth: int
    position: tuple
    yaw: float = -90.0
    pitch: float = 0.0
    fovy: float = 45.0


CONFIGS = {
    1: RenderConfig(1, 256, 256, 16, 3, (0.0, 0.0, 4.0)),
    2: RenderConfig(2, 1920, 1080, 256, 5, (0.0, 0.0, 3.5)),
    3: RenderConfig(3, 1920, 1080, 256, 5, (0.0, 1.5, 4.5), pitch=-10.0),
    4: RenderConfig(4, 3840, 2160, 1024, 8, (0.0, 0.0, 2.5)),
    5: RenderConfig(5, 4096, 4096, 4096, 12, (0.0, 1.2, 3.0), pitch=-5.0),
}


def write_png(path, rgba8):
    """Write an (H, W, 4) uint8 buffer as RGB PNG (mcpt_image_write_png; host-only, no GPU)."""
    a = np.ascontiguousarray(rgba8, np.uint8)
    h, w = a.shape[:2]
    rc = lib().mcpt_image_write_png(os.fsencode(path), w, h, a.ctypes.data_as(C.POINTER(C.c_uint8)))
    if rc != 0:
        raise McptError(f"mcpt_image_write_png failed ({rc})")


def write_pfm(path, rgb):
    """Write an (H, W, 3) float buffer as PFM (mcpt_image_write_pfm; host-only, no GPU)."""
    a = np.ascontiguousarray(rgb, np.float32)
    h, w = a.shape[:2]
    rc = lib().mcpt_image_write_pfm(os.fsencode(path), w, h, a.ctypes.data_as(C.POINTER(C.c_float)))
    if rc != 0:
        raise McptError(f"mcpt_image_write_pfm failed ({rc})")


# The build's default BVH: binned SAH over all three axes (mcpt_scene_build_ex).  On config 2 it
# traces ~14% faster than BVHAccel's single-axis 12-bucket SAH; films are identical for any tree.
DEFAULT_BVH = dict(builder="sah3", buckets=128, trav_cost=0.5, isect_cost=1.0, max_prims=8)
# A/B knobs for the builder's cost model (films do not depend on the tree)
for _k, _env, _t in (("trav_cost", "MCPT_BVH_TRAV_COST", float), ("max_prims", "MCPT_BVH_MAX_PRIMS", int),
                     ("builder", "MCPT_BVH_BUILDER", str), ("buckets", "MCPT_BVH_BUCKETS", int),
                     ("isect_cost", "MCPT_BVH_ISECT_COST", float)):
    if os.environ.get(_env):
        DEFAULT_BVH[_k] = _t(os.environ[_env])


def build_config_scene(cid: int, asset_dir=ASSET_DIR, **build_kw) -> Scene:
    """BASELINE config cid's proxy scene, built with DEFAULT_BVH (or ``builder="reference"``, ...)."""
    s = Scene()
    s.make_proxy(cid, asset_dir)
    if (DEFAULT_BVH | build_kw).get("builder") == "reference":
        s.build(max_prims=(DEFAULT_BVH | build_kw).get("max_prims", 8))
    else:
        s.build(**(DEFAULT_BVH | build_kw))
    return s


def config_camera(rc: RenderConfig, width=None, height=None) -> Camera:
    w, h = width or rc.width, height or rc.height
    return make_camera(rc.position, rc.yaw, rc.pitch, rc.fovy, aspect=np.float32(w) / np.float32(h))
