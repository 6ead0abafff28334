"""Quality-mode integrator (mcpt_config.flags = MCPT_FLAG_FIXED) on the oracle:
the fixed quirks change the film in the predicted direction; GPU parity is in test_gpu.py."""
import os

import numpy as np

from conftest import ASSETS


def cube_scene(mcpt_mod, with_dir_light):
    s = mcpt_mod.Scene()
    s.load_glb(os.path.join(ASSETS, "Cube.glb"))
    s.set_env_color([0.25, 0.5, 1.0], 1.0)
    if with_dir_light:
        s.add_dir_light([0.3, -1.0, 0.2], [1.0, 0.9, 0.8], 2.0)
    s.build(8)
    return s


def test_background_added_once(mcpt_mod, oracle):
    """Camera rays that miss everything: the reference adds the env background once per light
    (Appendix A.4), the fixed mode once."""
    s = cube_scene(mcpt_mod, with_dir_light=True)
    a = s.arrays()
    cam = mcpt_mod.make_camera((0.0, 0.0, 4.0), yaw_deg=90.0)  # looking away from the cube
    W = H = 24
    ref, sref, _ = oracle.render(a, cam, W, H, 2, 5)
    fix, sfix, _ = oracle.render(a, cam, W, H, 2, 5, fixed=True)
    assert np.array_equal(sref, sfix)
    m = sref > 0
    bg = np.array([0.25, 0.5, 1.0], np.float32)
    assert np.allclose(fix[m] / sfix[m][:, None], bg, rtol=1e-6)
    assert np.allclose(ref[m] / sref[m][:, None], 2 * bg, rtol=1e-6)  # two lights: env + directional


def test_fixed_mode_changes_only_what_it_fixes(mcpt_mod, oracle, scene_c1):
    rc = mcpt_mod.CONFIGS[1]
    cam = mcpt_mod.config_camera(rc, 48, 48)
    ref, sref, cref = oracle.render(scene_c1[1], cam, 48, 48, 4, rc.max_depth)
    fix, sfix, cfix = oracle.render(scene_c1[1], cam, 48, 48, 4, rc.max_depth, fixed=True)
    fix2, _, _ = oracle.render(scene_c1[1], cam, 48, 48, 4, rc.max_depth, fixed=True)
    assert np.array_equal(sref, sfix)
    assert np.array_equal(fix, fix2)                 # deterministic
    assert not np.array_equal(fix, ref)              # sphere.glb: env IS + Gram-Schmidt + RR differ
    assert np.isfinite(fix).all() and (fix >= 0).all()
