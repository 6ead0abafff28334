"""C-ABI boundary checks that need no GPU: library loads, every declared symbol is exported,
no CPU fallback exists, errors are reported as codes + strings (not exit(99))."""
import ctypes as C
import os
import re

import numpy as np

from conftest import REPO


def declared_symbols():
    src = open(os.path.join(REPO, "include", "mcpt.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(mcpt_[a-z0-9_]+)\s*\(", src)))


def test_every_declared_symbol_is_exported_and_bound(mcpt_mod):
    names = declared_symbols()
    assert len(names) >= 30
    lib = C.CDLL(mcpt_mod.LIB_PATH)
    for n in names:
        assert hasattr(lib, n), f"{n} declared in include/mcpt.h but not exported"
    assert set(names) == set(mcpt_mod.ABI), "ctypes binding out of sync with the header"


def test_no_cpu_fallback(mcpt_mod):
    """Without a gfx950 device the context refuses to exist (MCPT_E_NODEVICE)."""
    import torch

    if torch.cuda.is_available():
        return
    h = C.c_void_p()
    rc = mcpt_mod.lib().mcpt_create(0, None, C.byref(h))
    assert rc == -5 and not h.value
    assert b"no HIP device" in mcpt_mod.lib().mcpt_last_error(None)


def test_scene_errors_are_codes(mcpt_mod):
    s = mcpt_mod.Scene()
    try:
        s.load_glb("/nonexistent.glb")
        raise AssertionError("expected failure")
    except mcpt_mod.McptError as e:
        assert "cannot read" in str(e)
    try:
        s.desc()
        raise AssertionError("expected failure")
    except mcpt_mod.McptError as e:
        assert "not built" in str(e)


def test_camera_matrices(mcpt_mod):
    """glm::lookAt/perspective/inverse restatement: NDC corners map back onto the view frustum."""
    import numpy as np

    cam = mcpt_mod.make_camera((0.0, 0.0, 4.0), -90.0, 0.0, 45.0, aspect=2.0, znear=0.01, zfar=1e4)
    m = np.array(cam.inv_view_proj, np.float64).reshape(4, 4).T      # column-major -> row-major
    near = m @ np.array([0, 0, -1, 1.0])
    far = m @ np.array([0, 0, 1, 1.0])
    near, far = near[:3] / near[3], far[:3] / far[3]
    d = (far - near) / np.linalg.norm(far - near)
    np.testing.assert_allclose(near, [0, 0, 3.99], atol=1e-4)
    np.testing.assert_allclose(d, [0, 0, -1], atol=1e-6)
    top = m @ np.array([0, 1, 1, 1.0])
    top = top[:3] / top[3] - near
    assert abs(np.degrees(np.arctan2(top[1], -top[2])) - 22.5) < 1e-3   # fovy/2
    right = m @ np.array([1, 0, 1, 1.0])
    right = right[:3] / right[3] - near
    np.testing.assert_allclose(right[0] / top[1], 2.0, rtol=1e-5)       # aspect


def test_cpp_example_links_against_the_abi():
    """examples/mcpt_render (C++ over include/mcpt.h only) is built by `make` and resolves every
    mcpt_* symbol it uses from libmcpt.so."""
    import subprocess

    exe = os.path.join(REPO, "examples", "mcpt_render")
    assert os.path.exists(exe)
    out = subprocess.run(["nm", "-D", "--undefined-only", exe], capture_output=True, text=True, check=True).stdout
    used = sorted({l.split()[-1] for l in out.splitlines() if "mcpt_" in l})
    lib = subprocess.run(["nm", "-D", "--defined-only", os.path.join(REPO, "mc-path-tracer_amd", "libmcpt.so")],
                         capture_output=True, text=True, check=True).stdout
    defined = {l.split()[-1] for l in lib.splitlines()}
    assert used and all(u in defined for u in used), [u for u in used if u not in defined]


def test_env_hdr_device_tables_flag(mcpt_mod):
    """mcpt_scene_set_env_hdr_ex(MCPT_ENV_DEVICE_TABLES) keeps the texture and leaves the tables to
    the upload (built on the device); the plain call builds them on the host; bad flags are codes."""
    import os
    hdr = os.path.join(mcpt_mod.ASSET_DIR, "night_free_Env.hdr")
    out = []
    for dev in (False, True):
        s = mcpt_mod.Scene()
        s.set_env_hdr(hdr, 1, device_tables=dev)
        s.build()
        out.append(s.arrays())
    host, dev = out
    assert np.array_equal(host["env_tex"], dev["env_tex"]) and host["env_conds_y"].size > 0
    for k in ("env_marginal_y", "env_conds_y", "env_pdf"):
        assert dev[k].size == 0
    rc = mcpt_mod.lib().mcpt_scene_set_env_hdr_ex(mcpt_mod.Scene().h, hdr.encode(), 1, 6)
    assert rc == -1
