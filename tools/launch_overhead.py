"""Launch-bound regime: per-iteration wall time vs summed kernel time for small frames (config 1,
256x256) -- batch iterations (mcpt_iterate) and the reference's one-tile-per-call loop
(mcpt_wavefront_step, wavefront_kernels.cu:377-442 semantics)."""
import os, sys, time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "mc-path-tracer_amd")]
import mcpt
rc = mcpt.CONFIGS[1]
s = mcpt.build_config_scene(1)
for slots in (1, 16):
    pt = mcpt.PathTracer(0, mcpt.default_config(spp=1 << 20, max_depth=rc.max_depth))
    pt.upload_scene(s); pt.set_camera(mcpt.config_camera(rc)); pt.set_path_slots(slots); pt.resize(rc.width, rc.height)
    pt.iterate(50)
    for n in (1, 32):
        reps = max(1, 64 // n)
        t = time.perf_counter()
        ms = 0.0
        for _ in range(reps):
            st = pt.iterate(n)
            ms += st.ms_shade + st.ms_extend
        dt = (time.perf_counter() - t) / (reps * n)
        print(f"slots {slots:2d} iterate({n:2d}): {dt * 1e6:7.1f} us/iter wall, kernels {ms / (reps * n) * 1e3:7.1f} us/iter")
    pt.close()
pt = mcpt.PathTracer(0, mcpt.default_config(spp=1 << 20, max_depth=rc.max_depth))
pt.upload_scene(s); pt.set_camera(mcpt.config_camera(rc)); pt.resize(rc.width, rc.height)
for _ in range(20):
    pt.step(0, 0)
t = time.perf_counter()
for _ in range(100):
    pt.step(0, 0)
print(f"wavefront_step (one 256x256 tile per call): {(time.perf_counter() - t) / 100 * 1e6:.1f} us/call")
