"""HRDI light-table build: host (Scene.set_env_hdr, the serial restatement of
light_initialization_kernels.cu:3-112) against the device build at upload (env_build.hip), on
synthetic flat-RGBE maps of growing size; checks that both give the same tables.

  python tools/env_build_bench.py [--sizes 512x256,2048x1024,8192x4096] [--out gpurun_out/env_build.json]
"""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "mc-path-tracer_amd"))
import mcpt  # noqa: E402


def write_hdr(path, W, H, seed):
    rng = np.random.default_rng(seed)
    px = np.empty((H, W, 4), np.uint8)
    px[..., :3] = rng.integers(3, 256, (H, W, 3), dtype=np.uint8)  # R >= 3: never an RLE scanline marker
    px[..., 3] = rng.integers(118, 140, (H, W), dtype=np.uint8)
    with open(path, "wb") as f:
        f.write(b"#?RADIANCE\nFORMAT=32-bit_rle_rgbe\n\n-Y %d +X %d\n" % (H, W))
        f.write(px.tobytes())


def same(x, y):
    return bool(((x.view(np.uint32) == y.view(np.uint32)) | (np.isnan(x) & np.isnan(y))).all())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="512x256,2048x1024,8192x4096")
    ap.add_argument("--out", default="gpurun_out/env_build.json")
    args = ap.parse_args()
    rows = []
    pt = mcpt.PathTracer(0)
    with tempfile.TemporaryDirectory() as td:
        for k, sz in enumerate(args.sizes.split(",")):
            W, H = (int(v) for v in sz.split("x"))
            path = os.path.join(td, f"env{k}.hdr")
            write_hdr(path, W, H, k)
            s_host = mcpt.Scene()
            t0 = time.perf_counter()
            s_host.set_env_hdr(path, 1)
            t_host = time.perf_counter() - t0  # includes the file decode
            s_dev = mcpt.Scene()
            t0 = time.perf_counter()
            s_dev.set_env_hdr(path, 1, device_tables=True)
            t_decode = time.perf_counter() - t0
            for s in (s_host, s_dev):
                s.build()
            a = s_host.arrays()
            best = None
            for _ in range(3):
                t0 = time.perf_counter()
                pt.upload_scene(s_dev)
                t_up = time.perf_counter() - t0
                best = min(best or 1e9, pt.last_env_build_ms)
            t = pt.env_tables(W, H)
            ok = all(same(t[k2], a["env_" + k2]) for k2 in ("marginal_y", "conds_y", "pdf"))
            row = {"W": W, "H": H, "texels": W * H, "host_tables_s": round(t_host - t_decode, 4),
                   "hdr_decode_s": round(t_decode, 4), "device_build_ms": round(best, 3),
                   "device_upload_s": round(t_up, 4), "identical": ok, "guides": t["guides"]}
            print(json.dumps(row), flush=True)
            rows.append(row)
    pt.close()
    os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(rows, f, indent=1)
    assert all(r["identical"] for r in rows)


if __name__ == "__main__":
    main()
