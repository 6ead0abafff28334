"""k_trace wave lifetimes on steady-state config-2 iterations (needs the -DMCPT_WAVE_TIMES build:
tools/build_variant.sh wt -DMCPT_WAVE_TIMES; run with MCPT_LIB=.../libmcpt_wt.so)."""
import ctypes as C, os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "mc-path-tracer_amd")]
import mcpt
rc = mcpt.CONFIGS[int(os.environ.get("CFG", "2"))]
pt = mcpt.PathTracer(0, mcpt.default_config(spp=rc.spp, max_depth=rc.max_depth))
pt.upload_scene(mcpt.build_config_scene(int(os.environ.get("CFG", "2")))); pt.set_camera(mcpt.config_camera(rc)); pt.set_path_slots(int(os.environ.get("SLOTS", "3"))); pt.resize(rc.width, rc.height)
pt.iterate(30)
L = mcpt.lib()
f = L.mcpt_debug_wave_times
f.restype = C.c_int
f.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.c_int]
W = 16384
for it in range(3):
    st = pt.iterate(1)
    buf = (C.c_uint64 * (4 * W))()
    n = f(pt.h, buf, W)
    a = np.frombuffer(buf, dtype=np.uint64).reshape(-1, 4)[:n].astype(np.int64)
    live = a[:, 1] > 0
    a = a[live]
    t0 = a[:, 0].min()
    s, e = a[:, 0] - t0, a[:, 1] - t0
    T = e.max()
    print(f"iter {it}: waves {len(a)} kernel(10ns ticks) {T}  ms_trace {st.ms_extend:.4f}  start p50/p99/max {np.percentile(s,50):.0f}/{np.percentile(s,99):.0f}/{s.max()}")
    print("   end percentiles (frac of kernel): " + " ".join(f"p{q}={np.percentile(e, q) / T:.3f}" for q in (1, 10, 25, 50, 75, 90, 99)))
    print(f"   mean lifetime frac {((e - s).mean()) / T:.3f}")
    part, dry = a[:, 2], a[:, 3] - t0
    for p in np.unique(part):
        m = part == p
        d = dry[m][a[m, 3] > 0]
        print(f"   part {p}: waves {m.sum()} dry(frac) min/med/max " + (f"{d.min()/T:.3f}/{np.median(d)/T:.3f}/{d.max()/T:.3f}" if len(d) else "-") +
              f"  end min/med/max {e[m].min()/T:.3f}/{np.median(e[m])/T:.3f}/{e[m].max()/T:.3f}")
    # active waves over time
    hist = [(np.sum((s <= t) & (e > t))) for t in np.linspace(0, T, 11)[:-1]]
    print("   live waves at 0%..90%: " + " ".join(str(h) for h in hist))
