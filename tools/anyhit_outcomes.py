"""Outcomes of the any-hit rays k_trace traverses (round 6): how many of them end occluded -- the
share an occluder cache with more coverage could still take -- against those that reach the sky,
which only a traversal can prove.  One config-2 frame with the counting k_trace build (work
counters), the bench's layout.  Usage: python tools/anyhit_outcomes.py [--config 2]"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mc-path-tracer_amd"))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    a = ap.parse_args()
    import bench
    import mcpt

    rc = mcpt.CONFIGS[a.config]
    pt, _, _ = bench.make_tracer(0, argparse.Namespace(config=a.config, slots=None), rc, rc.spp)
    pt.set_path_slots(bench.BENCH_SLOTS[a.config])
    pt.resize(rc.width, rc.height)
    pt.set_work_counters(True)
    pt.clear()
    st = pt.render()
    rcnt = pt.ray_counts()
    trav = rcnt["any_hit_traversed"]
    out = {"config": a.config, "any_hit_rays": rcnt["any_hit"], "resolved_by_cache": rcnt["any_hit_occluder_cache"],
           "traversed": trav, "traversed_occluded": int(st.any_hits),
           "traversed_occluded_frac": round(st.any_hits / max(1, trav), 4),
           "any_pair_steps_per_traversed_ray": round(st.any_nodes / max(1, trav), 2)}
    print(json.dumps(out), flush=True)
    pt.close()


if __name__ == "__main__":
    main()
