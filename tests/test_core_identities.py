"""Host build of the shared numeric core: the exactness identities the GPU fast paths rely on
(dsincos == dsin/dcos, the cheap texel wrap, guided CDF search == upper_bound)."""
import os
import subprocess

from conftest import REPO


def test_core_identities(tmp_path):
    src = os.path.join(REPO, "tests", "native", "core_identities.cpp")
    exe = str(tmp_path / "core_identities")
    subprocess.run(["/opt/rocm/bin/hipcc", "-O2", "-std=c++17", "-ffp-contract=off", "-fno-fast-math",
                    "-I", os.path.join(REPO, "mc-path-tracer_amd", "csrc"), "-I", os.path.join(REPO, "include"),
                    src, "-o", exe], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "bad=0" in r.stdout
