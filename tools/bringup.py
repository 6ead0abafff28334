"""GPU bring-up: trace parity, film parity and a first throughput number in one process."""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "mc-path-tracer_amd"), os.path.join(REPO, "oracle")]
import mcpt  # noqa: E402
import oracle_py as op  # noqa: E402


def log(*a):
    print(*a, flush=True)


def cmp_film(a, b, sa, sb):
    tol = 1e-4 * np.maximum(np.abs(a), np.abs(b)) + 1e-7
    bad = ~(np.abs(a - b) <= tol)
    exact = np.array_equal(a.view(np.uint32), b.view(np.uint32))
    return int(bad.sum()), exact, bool(np.array_equal(sa, sb))


def main():
    s1 = mcpt.build_config_scene(1)
    a1 = s1.arrays()
    pt = mcpt.PathTracer(0, mcpt.default_config(spp=4, max_depth=3))
    log("device", pt.device_name)
    pt.upload_scene(s1)
    rng = np.random.default_rng(1)
    n = 65536
    ro = rng.uniform(-3, 3, (n, 3)).astype(np.float32)
    rd = rng.normal(size=(n, 3)).astype(np.float32)
    rd /= np.linalg.norm(rd, axis=1, keepdims=True)
    t = time.time()
    gp, gn, gt = pt.trace_closest(ro, rd)
    op_, on, ot = op.trace_closest(a1, ro, rd)
    log("closest tri equal", np.array_equal(gt, ot), "hits", (gt >= 0).mean(),
        "pos/t bitwise", np.array_equal(gp.view(np.uint32), op_.view(np.uint32)),
        "nrm bitwise", np.array_equal(gn.view(np.uint32), on.view(np.uint32)), time.time() - t)
    gv = pt.trace_any(ro, rd)
    ov = op.trace_any(a1, ro, rd)
    log("any equal", np.array_equal(gv, ov), gv.mean())
    # film parity C1 64x64 4spp depth 3
    W = H = 64
    cam = mcpt.config_camera(mcpt.CONFIGS[1], W, H)
    pt.set_camera(cam)
    pt.resize(W, H)
    st = pt.render()
    Ld, smp = pt.film()
    rL, rs, cnt = op.render(a1, cam, W, H, spp=4, max_depth=3)
    log("C1 film bad", cmp_film(Ld, rL, smp, rs), "gpu rays", st.extend_rays, st.shadow_rays, st.vis_rays,
        "oracle", cnt)
    pt.close()
    # C2 proxy
    t = time.time()
    s2 = mcpt.build_config_scene(2)
    a2 = s2.arrays()
    log("C2 tris", len(a2["mat"]), "depth", s2.bvh_depth, "build s", time.time() - t)
    rc = mcpt.CONFIGS[2]
    W, H = 192, 108
    pt = mcpt.PathTracer(0, mcpt.default_config(spp=2, max_depth=5))
    pt.upload_scene(s2)
    cam = mcpt.config_camera(rc, W, H)
    pt.set_camera(cam)
    pt.resize(W, H)
    st = pt.render()
    Ld, smp = pt.film()
    t = time.time()
    rL, rs, cnt = op.render(a2, cam, W, H, spp=2, max_depth=5, nthreads=16)
    log("C2 film bad", cmp_film(Ld, rL, smp, rs), "oracle s", time.time() - t, cnt, "gpu", st.as_dict())
    pt.close()
    # throughput at 1080p
    W, H = rc.width, rc.height
    pt = mcpt.PathTracer(0, mcpt.default_config(spp=256, max_depth=5))
    pt.upload_scene(s2)
    pt.set_camera(mcpt.config_camera(rc, W, H))
    pt.resize(W, H)
    pt.iterate(10)
    for k in range(3):
        t = time.time()
        st = pt.iterate(20)
        dt = time.time() - t
        log(f"1080p iter x20: wall {dt*1e3:.1f} ms  rays {st.rays}  {st.rays/dt/1e6:.1f} Mray/s  "
            f"shade {st.ms_shade:.2f} extend {st.ms_extend:.2f} shadow {st.ms_shadow:.2f} ms "
            f"ext {st.extend_rays} sh {st.shadow_rays} vis {st.vis_rays}")
    pt.close()


if __name__ == "__main__":
    main()
