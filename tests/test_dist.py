"""Multi-rank path on CPU (gloo, world_size 2): the tile partition and the frame-end gather to rank 0.

The rendering rank is played by the oracle (scalar C restatement of the reference kernels) so the
test runs without a GPU: every rank renders only its own tiles of the (tx + ty) mod N partition,
packs them as mcpt_film_pack_tiles does, sends them to rank 0 (mcpt/parallel.py, point-to-point
send / recv, the same calls the RCCL path makes), and rank 0's assembled film must equal the
one-process render bit for bit (the keyed RNG makes a pixel's result independent of its rank).
"""
import os
import socket
import subprocess
import sys

import numpy as np
import torch.multiprocessing as mp

from conftest import REPO
from mcpt import parallel


def test_partition_covers_every_tile_once():
    for W, H, world in [(1920, 1080, 1), (1920, 2160, 2), (1920, 8640, 8), (3840, 2160, 8), (300, 70, 3)]:
        seen = {}
        for r in range(world):
            for t in parallel.tiles_for_rank(r, world, W, H):
                assert t not in seen
                seen[t] = r
        nx, ny = parallel.tile_grid(W, H)
        assert len(seen) == nx * ny


def test_partition_balance_weak_scaling():
    """Each rank owns ~one 1080p frame of pixels when the frame is 1920 x 1080N."""
    for world in (2, 4, 8):
        W, H = 1920, 1080 * world
        counts = []
        for r in range(world):
            c = 0
            for tx, ty in parallel.tiles_for_rank(r, world, W, H):
                c += min(256, W - tx * 256) * min(256, H - ty * 256)
            counts.append(c)
        assert sum(counts) == W * H
        assert max(counts) / (W * H / world) < 1.12


def test_partition_balance_strong_scaling_config4():
    """bench.py --config 4 --scaling strong: the fixed 3840x2160 frame split over 2/4/8 ranks."""
    for world in (2, 4, 8):
        W, H = 3840, 2160
        counts = [sum(min(256, W - tx * 256) * min(256, H - ty * 256) for tx, ty in
                      parallel.tiles_for_rank(r, world, W, H)) for r in range(world)]
        assert sum(counts) == W * H and max(counts) / (W * H / world) < 1.15


def test_pack_unpack_roundtrip():
    rng = np.random.default_rng(0)
    W, H, T = 300, 170, 64
    Ld = rng.random((H, W, 3), dtype=np.float32)
    smp = rng.integers(0, 1 << 31, (H, W)).astype(np.uint32)
    tiles = parallel.tiles_for_rank(1, 3, W, H, T)
    L2, S2 = parallel.unpack(parallel.pack(Ld, smp, tiles, W, H, T), tiles, W, H, T)
    mask = np.zeros((H, W), bool)
    for tx, ty in tiles:
        mask[ty * T:(ty + 1) * T, tx * T:(tx + 1) * T] = True
    assert np.array_equal(L2[mask], Ld[mask]) and np.array_equal(S2[mask], smp[mask])
    assert not L2[~mask].any() and not S2[~mask].any()


W_, H_, T_, SPP_ = 300, 200, 64, 2


def _scene_and_camera():
    import mcpt

    s = mcpt.build_config_scene(2)
    rc = mcpt.CONFIGS[2]
    return s.arrays(), mcpt.config_camera(rc, W_, H_)


def _worker(rank, world, port, q):
    import torch
    import torch.distributed as dist

    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle_py

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        arrays, cam = _scene_and_camera()
        # this rank's partition only, rendered as a rank would (the oracle stands in for the GPU)
        Ld, smp, _ = oracle_py.render(arrays, cam, W_, H_, SPP_, 5, tile=T_, nthreads=2, part=(rank, world))
        tiles = parallel.tiles_for_rank(rank, world, W_, H_, T_)
        local = torch.from_numpy(parallel.pack(Ld, smp, tiles, W_, H_, T_))
        parts = parallel.gather_packed_to_root(local, rank, world, dist, W_, H_, T_)
        if rank == 0:
            L2 = S2 = None
            for r, p in enumerate(parts):
                L2, S2 = parallel.unpack(p.numpy(), parallel.tiles_for_rank(r, world, W_, H_, T_), W_, H_, T_, L2, S2)
            fL, fs, _ = oracle_py.render(arrays, cam, W_, H_, SPP_, 5, tile=T_, nthreads=4)
            q.put((bool(np.array_equal(L2.view(np.uint32), fL.view(np.uint32)) and np.array_equal(S2, fs)),
                   int(fs.sum()), int(S2.sum())))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_rendered_partition_gathered_to_root_gloo_world2():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    ok, n_full, n_gathered = q.get(timeout=240)
    for p in procs:
        p.join(60)
    assert n_full == (W_ - 1) * (H_ - 1) * SPP_  # every rendered pixel (last row / column never: :110)
    assert ok and n_gathered == n_full


def test_bench_gpus_flag_refuses_mismatched_world(tmp_path):
    """bench.py --gpus N under a launcher whose WORLD_SIZE differs exits non-zero before any GPU
    work (without a launcher it starts the N ranks itself)."""
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 2 and "WORLD_SIZE=1" in r.stderr


def _gather_worker(rank, world, port, q):
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        W, H, T = 300, 70, 256  # 2 x 1 tiles over 3 ranks: rank 2 owns none
        tiles = parallel.tiles_for_rank(rank, world, W, H, T)
        local = torch.full((len(tiles) * T * T, 4), float(rank + 1))
        parts = parallel.gather_packed_to_root(local, rank, world, dist, W, H, T)
        # a collective after the gather must see no stray point-to-point message
        x = torch.tensor([rank + 1.0])
        dist.all_reduce(x)
        dist.barrier()
        if rank == 0:
            q.put(([tuple(p.shape) for p in parts], [float(p[0, 0]) if len(p) else None for p in parts], float(x)))
    finally:
        dist.destroy_process_group()


def test_gather_with_an_empty_rank_gloo_world3():
    """More ranks than tiles: the rank without tiles sends nothing and rank 0 posts no receive for
    it (an unmatched send hangs RCCL or leaves a stray gloo message); a collective
    right after the gather completes with every rank's value."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_gather_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    shapes, firsts, total = q.get(timeout=120)
    for p in procs:
        p.join(60)
    assert shapes == [(65536, 4), (65536, 4), (0, 4)]
    assert firsts == [1.0, 2.0, None] and total == 6.0


def test_strong_split_slots():
    """The strong split (bench.py's N > 1 headline): path slots grow with the ranks so every GPU keeps
    the one-GPU run's paths in flight, bounded by spp, by 256 and by 2^31 paths of the rank's own
    (compact) path state, with an optional byte budget; one value for all ranks."""
    import bench

    T = bench.MULTI_TILE
    assert parallel.strong_slots(24, 1, 1920, 1080, 256, 256) == 24
    assert parallel.strong_slots(24, 2, 1920, 1080, 256, T) == 48
    assert parallel.strong_slots(24, 4, 1920, 1080, 256, T) == 96  # no longer capped by a whole-frame budget
    assert parallel.strong_slots(24, 8, 1920, 1080, 256, T) == 128  # spp / 2: a slot renders >= 2 samples
    for W, H, base, spp in ((1920, 1080, 24, 256), (3840, 2160, 16, 1024), (4096, 4096, 16, 4096)):
        for world in (2, 4, 8):
            s = parallel.strong_slots(base, world, W, H, spp, T)
            px = parallel.rank_path_pixels(world, W, H, T)
            assert base <= s <= min(base * world, 256) and s * px < 2 ** 31
            assert s * px * parallel.PATH_BYTES <= 40e9  # compact state: at most C5's 34 GB per GPU
    # no byte budget by default: C5 at N = 8 keeps 8 x 16 slots over its 1/8 of 4096^2
    assert parallel.strong_slots(16, 8, 4096, 4096, 4096, T) == 128
    assert parallel.strong_slots(16, 8, 4096, 4096, 4096, T, budget=16 << 30) < 128
    assert parallel.strong_slots(16, 8, 256, 256, 16, T) == 16  # spp bound: a slot renders at least one sample
    # the 2^31-path cap binds before base_slots: a 46341^2-pixel frame holds < 2 slots
    assert parallel.strong_slots(4, 1, 46341, 46341, 64, 256) == 1
    a = bench.parse(["--gpus", "8", "--no-gather"])
    assert a.no_gather and not a.no_strong and not a.no_weak and not a.no_verify_gather and a.scaling == "strong"


def test_rank_path_pixels_cover_the_partition():
    """The compact layout's per-rank path state: tiles x tile pixels of the rank's own tiles, edge
    overhang included; the ranks together hold every tile once (1/N of the full layout's state)."""
    for W, H, T in ((1920, 1080, 64), (3840, 2160, 64), (300, 70, 64)):
        nx, ny = parallel.tile_grid(W, H, T)
        for world in (1, 2, 3, 8):
            per = [len(parallel.tiles_for_rank(r, world, W, H, T)) * T * T for r in range(world)]
            assert sum(per) == nx * ny * T * T
            assert parallel.rank_path_pixels(world, W, H, T) == max(per)


def test_multi_gpu_tile_balances_pixels():
    """bench.py's multi-GPU partition uses 64 x 64 film tiles (MULTI_TILE): every rank's pixel
    count is within 2 % of the mean at N = 2 / 4 / 8 on the 1080p frame and on config 4's 4K frame
    (with 256 x 256 tiles a 1080p rank at N = 8 owns 5 tiles, one diagonal; the time spread the
    one-GPU rehearsal measured was 1.71x, profiles/partition_r04.json)."""
    import bench

    T = bench.MULTI_TILE
    for W, H in ((1920, 1080), (3840, 2160)):
        for world in (2, 4, 8):
            counts = [sum(min(T, W - tx * T) * min(T, H - ty * T) for tx, ty in
                          parallel.tiles_for_rank(r, world, W, H, T)) for r in range(world)]
            assert sum(counts) == W * H and max(counts) / (W * H / world) < 1.02
    assert bench.part_tile(1) == 256 and bench.part_tile(8) == T


class _FakeStats:
    def __init__(self, px):
        for k in ("extend_rays", "shadow_rays", "vis_rays", "iterations", "ms_shade", "ms_extend", "ext_nodes",
                  "ext_tests", "ext_hits", "any_nodes", "any_tests", "any_hits"):
            setattr(self, k, 0)
        self.extend_rays = px

    @property
    def rays(self):
        return self.extend_rays


class _FakeTracer:
    """The allocation rules of runtime.cpp: path state of slots x npx paths, npx = W x H (full
    layout) or the tile set's tiles x tile pixels (compact, mcpt_set_compact_paths); refused at >= 2^31
    paths; resize resets the tile set to every tile; set_path_slots keeps the tile set in the compact
    layout (re-sizes at the film size in the full one); set_tiles re-allocates in the compact layout.
    Plus a per-GPU memory cap (one MI355X: 288 GB) at ~234 B per path (state + queues)."""
    CAP = 288e9

    def __init__(self):
        self.W = self.H = self.T = 0
        self.slots = 1
        self.compact = False
        self.peak = 0.0
        self.ntiles = 0
        self.tiles = None

    def _alloc(self):
        if not self.W:
            return
        npx = self.ntiles * self.T * self.T if self.compact else self.W * self.H
        P = npx * self.slots
        assert P < 2 ** 31, f"film too large for the path slots: {npx} px x {self.slots}"
        assert P * 234 <= self.CAP, f"out of memory: {npx} px x {self.slots}"
        self.peak = max(self.peak, P * 234)

    def set_compact_paths(self, on=True):
        self.compact = bool(on)
        self._alloc()

    def set_path_slots(self, s):
        self.slots = s
        self._alloc()

    def resize(self, W, H, tw, th):
        self.W, self.H, self.T = W, H, tw
        nx, ny = parallel.tile_grid(W, H, tw)
        self.ntiles = nx * ny
        self.tiles = None
        self._alloc()

    def set_tiles(self, t):
        self.tiles = t
        nx, ny = parallel.tile_grid(self.W, self.H, self.T)
        self.ntiles = nx * ny if t is None else len(t)
        if self.compact:
            self._alloc()

    def clear(self):
        pass

    def render(self):
        import time
        time.sleep(0.002)  # a frame takes time (per-rank seconds are rounded to 0.1 ms)
        return _FakeStats(len(self.tiles or []))

    def occ_stats(self):
        return 0, True

    def ray_counts(self):
        return {}


class _FakeDist:
    def __init__(self, world):
        self.world = world

    def barrier(self):
        pass

    def all_gather(self, out, t):
        for o in out:
            o.copy_(t)

    def get_backend(self):
        return "gloo"


def test_split_layouts_fit_one_gpu():
    """bench.py N > 1: the headline split and the other one run back to back on every rank
    (strong then weak by default, and the reverse under --scaling weak).  Each layout allocates the
    film at one slot, then the rank's tiles (compact path state), then the slots, so no step asks for
    slots x the whole frame: the round-4 N = 4 rehearsal ran out of memory on a weak film with the
    strong split's slots.  Checked for N = 2 / 4 / 8 on configs 2, 4 and 5 with the allocator's rules;
    each rank's path state is its own tiles' (about 1/N of the frame)."""
    import argparse
    import types

    import torch

    import bench
    import mcpt

    fake_torch = types.SimpleNamespace(cuda=types.SimpleNamespace(synchronize=lambda: None), tensor=torch.tensor,
                                       zeros_like=torch.zeros_like, float64=torch.float64)
    for cid in (2, 4, 5):
        rc = mcpt.CONFIGS[cid]
        for world in (2, 4, 8):
            for order in (("strong", "weak"), ("weak", "strong")):
                pt = _FakeTracer()
                for rank in (0, world - 1):
                    for kind in order:
                        args = argparse.Namespace(slots=None, config=cid, steps=1, warmup=0)
                        run = bench.run_split(pt, rc, rank, world, _FakeDist(world), "gloo", kind, rc.spp, args,
                                              fake_torch)
                        lay = run["layout"]
                        assert pt.compact and pt.slots == lay["slots"] and [pt.W, pt.H] == lay["frame"]
                        assert lay["path_pixels_rank"] == len(pt.tiles) * pt.T * pt.T
                        assert lay["path_pixels_rank"] <= 1.1 * lay["frame"][0] * lay["frame"][1] / world + 4 * 64 * 64
                assert pt.peak <= _FakeTracer.CAP
