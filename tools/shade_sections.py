"""k_shade section attribution, run on the GPU with a -DMCPT_DIAG_SHADE build:

  bash tools/build_variant.sh diagshade -DMCPT_DIAG_SHADE
  MCPT_LIB=$PWD/mc-path-tracer_amd/libmcpt_diagshade.so python tools/shade_sections.py [--config 2]

Renders one frame of the bench's workload and prints, per k_shade section, the wave entries (waves
with at least one lane in the section) and the active lanes, per frame (kernels.hip SD_*)."""
import argparse
import ctypes as C
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mc-path-tracer_amd"))
sys.path.insert(0, REPO)

NAMES = ["waves", "valid", "logic", "nee", "generate", "continue", "background"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import bench
    import mcpt

    rc = mcpt.CONFIGS[a.config]
    pt, _, _ = bench.make_tracer(0, argparse.Namespace(config=a.config), rc, rc.spp)
    pt.set_path_slots(bench.BENCH_SLOTS[a.config])
    pt.resize(rc.width, rc.height)
    lib = mcpt.lib()
    f = lib.mcpt_debug_shade_sections
    f.restype = C.c_int
    f.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.c_int, C.c_int]
    buf = (C.c_uint64 * 32)()
    pt.clear()
    f(pt.h, buf, 32, 1)  # reset
    st = pt.render()
    n = f(pt.h, buf, 32, 1)
    if n <= 0:
        sys.exit("not a -DMCPT_DIAG_SHADE build")
    out = {"config": a.config, "iterations": st.iterations, "rays": st.rays, "sections": {}}
    for i, nm in enumerate(NAMES):
        w, l = int(buf[2 * i]), int(buf[2 * i + 1])
        out["sections"][nm] = {"wave_entries": w, "lanes": l, "lanes_per_entry": round(l / max(1, w), 2)}
    print(json.dumps(out, indent=1))
    if a.out:
        json.dump(out, open(a.out, "w"), indent=1)
    pt.close()


if __name__ == "__main__":
    main()
