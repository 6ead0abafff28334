"""k_trace loop profile on steady-state config-2 iterations (needs the -DMCPT_TRACE_PROF build)."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "mc-path-tracer_amd")]
import mcpt
rc = mcpt.CONFIGS[2]
pt = mcpt.PathTracer(0, mcpt.default_config(spp=256, max_depth=5))
pt.upload_scene(mcpt.build_config_scene(2)); pt.set_camera(mcpt.config_camera(rc)); pt.set_path_slots(int(os.environ.get("SLOTS", "3"))); pt.resize(rc.width, rc.height)
pt.iterate(30)
pt.trace_profile(reset=True)
N = 10
st = pt.iterate(N)
p = pt.trace_profile()
waves = int(os.environ.get("WAVES", "8192"))  # resident waves: 32 per CU x 256 CUs (8-wave child-pair build)
print({k: v / N for k, v in p.items()})
trips = p["trips"] / N
print("per iteration: trips/wave %.0f  node-lane util %.3f  idle-lane frac %.3f  tri phases/trip %.3f  tri lanes/phase %.1f" % (
    trips / waves, p["node_lanes"] / (64 * p["trips"]), p["idle_lanes"] / (64 * p["trips"]), p["tri_phases"] / p["trips"],
    p["tri_lanes"] / max(1, p["tri_phases"])))
T = p["trips"]
print("per trip: finish %.2f pop %.2f (lanes/pop %.1f) slow-slab %.3f refill %.3f tri %.3f" % (
    p["finish_trips"] / T, p["pop_trips"] / T, p["pop_lanes"] / max(1, p["pop_trips"]), p["slow_slab_trips"] / T,
    p["refills"] / T, p["tri_phases"] / T))
print("refill: %.0f cycles each, %.0f cycles per wave per launch; launch %.1f us" % (
    p["_11"] / max(1, p["refills"]), p["_11"] / N / waves, st.ms_extend / N * 1e3))
print("units: nodes %.1fM tests %.1fM  | ms trace %.3f" % ((st.ext_nodes + st.any_nodes) / N / 1e6, (st.ext_tests + st.any_tests) / N / 1e6, st.ms_extend / N))
