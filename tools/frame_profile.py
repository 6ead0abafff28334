"""Per-iteration rays and stage times over one whole config-2 frame (film cleared, every pixel to
spp completion): where the full-frame rate falls below the steady state.
usage: python tools/frame_profile.py [slots] -> gpurun_out/frame_profile.json + a summary"""
import json, os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "mc-path-tracer_amd")]
import mcpt

S = int(sys.argv[1]) if len(sys.argv) > 1 else 3
rc = mcpt.CONFIGS[2]
pt = mcpt.PathTracer(0, mcpt.default_config(spp=rc.spp, max_depth=rc.max_depth))
pt.upload_scene(mcpt.build_config_scene(2))
pt.set_camera(mcpt.config_camera(rc))
pt.set_path_slots(S)
pt.resize(rc.width, rc.height)
pt.clear()
rows = []
for i in range(2000):
    st = pt.iterate(1)
    rows.append([st.rays, st.extend_rays, st.shadow_rays, st.vis_rays, st.ms_extend + st.ms_shadow, st.ms_shade])
    if st.rays == 0:
        break
os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
with open(os.path.join(REPO, "gpurun_out", "frame_profile.json"), "w") as f:
    json.dump({"slots": S, "rows": rows}, f)
rays = sum(r[0] for r in rows)
ms = sum(r[4] + r[5] for r in rows)
print(f"iterations {len(rows)}  rays {rays / 1e9:.3f} G  device ms {ms:.1f}  rate {rays / ms / 1e3:.0f} Mray/s")
n = len(rows)
edges = sorted(set([0, min(n, 4)] + [round(n * k / 8) for k in range(1, 9)]))
for lo, hi in zip(edges[:-1], edges[1:]):
    if hi <= lo:
        continue
    seg = rows[lo:hi]
    r = sum(x[0] for x in seg)
    m = sum(x[4] + x[5] for x in seg)
    print(f"  iters {lo:4d}-{hi:4d}: rays/iter {r / len(seg) / 1e6:6.2f} M  ms/iter {m / len(seg):.3f}  "
          f"rate {r / max(m, 1e-9) / 1e3:6.0f} Mray/s  share of time {m / ms:.3f}")
