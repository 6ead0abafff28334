# Round-5 experiment driver (CPU): boxes per ray of the product traversal model (oracle/trav_model.c, mode 2)
# on a config scene with and without MCPT_BVH_TREELET passes (commit history: the treelet pass itself).
import os, sys, time
import numpy as np
sys.path.insert(0, "/root/repo/mc-path-tracer_amd"); sys.path.insert(0, "/root/repo/oracle")
import mcpt, oracle_py as op

def rays(a, n, seed):
    rng = np.random.default_rng(seed)
    mn = a["bmin"][0]; mx = a["bmax"][0]
    o = (mn + (mx - mn) * rng.uniform(0.2, 0.8, (n, 3))).astype(np.float32)
    d = rng.normal(size=(n, 3)); d /= np.linalg.norm(d, axis=1, keepdims=True)
    pt, nrm, tri = op.trace_closest(a, o, d.astype(np.float32), nthreads=8)
    k = tri >= 0
    p = pt[k, :3] + nrm[k, :3] * 1e-3
    d2 = rng.normal(size=(k.sum(), 3)); d2 /= np.linalg.norm(d2, axis=1, keepdims=True)
    flip = (d2 * nrm[k, :3]).sum(1) < 0
    d2[flip] *= -1
    return np.concatenate([o, p]).astype(np.float32), np.concatenate([d, d2]).astype(np.float32)

cid = int(sys.argv[1]); passes = sys.argv[2:] or ["1"]
res = {}
for ps in ["0"] + passes:
    os.environ["MCPT_BVH_TREELET"] = ps
    t0 = time.time(); s = mcpt.build_config_scene(cid); tb = time.time() - t0
    a = s.arrays()
    if ps == "0":
        ro, rd = rays(a, 100000, 7)
    m = op.model_margins(a)
    tri, t, vis, boxes = op.model_trace(a, ro, rd, 2, m, nthreads=8)
    res[ps] = (tri, t, vis)
    print(f"C{cid} treelet passes {ps}: build {tb:.2f} s, nodes {len(a['nprims'])}, boxes/ray {boxes/len(ro):.2f}, P {m['p']:.4g}, contained {m['contained']}", flush=True)
    if ps != "0":
        same = np.array_equal(res["0"][0], tri) and np.array_equal(res["0"][1].view(np.uint32), t.view(np.uint32)) and np.array_equal(res["0"][2], vis)
        print("   results identical to the untouched tree:", same)
