"""Experiment: does splitting the frame's tiles over K contexts (own stream each) that iterate
concurrently overlap k_shade of one part with k_trace of another?  Config 2, steady state.
Usage: python tools/overlap_exp.py [K ...]"""
import os
import sys
import threading
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "mc-path-tracer_amd")]
import mcpt  # noqa: E402

rc = mcpt.CONFIGS[2]
scene = mcpt.build_config_scene(2)
cam = mcpt.config_camera(rc, rc.width, rc.height)
W, H = rc.width, rc.height
nx, ny = (W + 255) // 256, (H + 255) // 256
STEPS, WARM = 120, 30


def run(K):
    pts = []
    for k in range(K):
        pt = mcpt.PathTracer(0, mcpt.default_config(spp=rc.spp, max_depth=rc.max_depth))
        pt.upload_scene(scene)
        pt.set_camera(cam)
        pt.set_path_slots(int(os.environ.get("SLOTS", "3")))
        pt.resize(W, H)
        pt.set_tiles([(tx, ty) for ty in range(ny) for tx in range(nx) if (tx + ty) % K == k])
        pt.iterate(WARM)
        pts.append(pt)
    res = [None] * K

    def work(i):
        res[i] = pts[i].iterate(STEPS)

    th = [threading.Thread(target=work, args=(i,)) for i in range(K)]
    t0 = time.perf_counter()
    for t in th:
        t.start()
    for t in th:
        t.join()
    dt = time.perf_counter() - t0
    rays = sum(r.rays for r in res)
    ev = [(r.ms_shade / STEPS, r.ms_extend / STEPS) for r in res]
    print(f"K={K}: {rays / dt / 1e6:8.1f} Mray/s  wall {dt * 1e3 / STEPS:.4f} ms/iter  "
          f"per-ctx event ms (shade, trace): {[(round(a, 4), round(b, 4)) for a, b in ev]}", flush=True)
    for pt in pts:
        pt.close()


for K in [int(a) for a in sys.argv[1:]] or [1, 2, 3, 4]:
    run(K)
