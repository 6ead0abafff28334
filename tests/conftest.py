import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "mc-path-tracer_amd"), os.path.join(REPO, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)
GOLDEN = os.path.join(REPO, "tests", "golden")
ASSETS = os.path.join(REPO, "assets")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) device")


@pytest.fixture(scope="session")
def mcpt_mod():
    import mcpt

    mcpt.lib()
    return mcpt


@pytest.fixture(scope="session")
def oracle():
    import oracle_py

    oracle_py.lib()
    return oracle_py


@pytest.fixture(scope="session")
def scene_c1(mcpt_mod):
    s = mcpt_mod.build_config_scene(1)
    return s, s.arrays()


@pytest.fixture(scope="session")
def scene_c2(mcpt_mod):
    s = mcpt_mod.build_config_scene(2)
    return s, s.arrays()


@pytest.fixture(scope="session")
def scene_c3(mcpt_mod):
    """Config-3 deep-BVH proxy: 871,414-triangle displaced icosphere + ground."""
    s = mcpt_mod.build_config_scene(3)
    return s, s.arrays()


@pytest.fixture(scope="session")
def scene_cube(mcpt_mod):
    """Cube.glb (12 tris, exactly axis-aligned normals: the gram_schmidt NaN-frame case)."""
    s = mcpt_mod.Scene()
    s.load_glb(os.path.join(ASSETS, "Cube.glb"))
    s.set_env_hdr(os.path.join(ASSETS, "HDR_029_Sky_Cloudy_Env.hdr"), 1)
    s.build(8)
    return s, s.arrays()
