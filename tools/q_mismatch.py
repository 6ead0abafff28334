"""List rays whose GPU closest hit differs from the oracle's (trace parity debugging).
Usage: MCPT_LIB=... python tools/q_mismatch.py [builder] [config]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "mc-path-tracer_amd"), os.path.join(REPO, "oracle"), os.path.join(REPO, "tests")]
import numpy as np  # noqa: E402
import mcpt  # noqa: E402
import oracle_py as op  # noqa: E402
from test_gpu import random_rays  # noqa: E402

builder = sys.argv[1] if len(sys.argv) > 1 else "ploc"
cid = int(sys.argv[2]) if len(sys.argv) > 2 else 1
s = mcpt.build_config_scene(cid)
a = s.arrays()
pt = mcpt.PathTracer(0)
pt.upload_scene(s, gpu_bvh=False if builder == "host" else builder)
ro, rd = random_rays(100000, 31, box=2.5)
ro[:4] = [[0, 0, 5], [0, 0, 5], [0, 0, 5], [0, 0, 1]]
rd[:4] = [[np.nan, 0, -1], [0, 0, 0], [0, 0, -1], [1, 0, 0]]
gp, gn, gt = pt.trace_closest(ro, rd)
op_, on, ot = op.trace_closest(a, ro, rd)
bad = np.nonzero(gt != ot)[0]
print(f"{builder} config {cid}: {len(bad)} of {len(ro)} closest hits differ")
for i in bad[:12]:
    print(f"  ray {i}: o {ro[i].tolist()} d {rd[i].tolist()} gpu tri {gt[i]} t {gp[i][3]:.9g} | oracle tri {ot[i]} t {op_[i][3]:.9g}")
va, vo = pt.trace_any(ro, rd), op.trace_any(a, ro, rd)
badv = np.nonzero(va != vo)[0]
print(f"  any-hit: {len(badv)} differ", [(int(i), int(va[i]), int(vo[i])) for i in badv[:8]])
