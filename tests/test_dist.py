"""Multi-rank path on CPU (gloo, world_size 2): tile partition and the film gather/unpack."""
import os
import socket

import numpy as np
import torch.multiprocessing as mp

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


def fake_film(W, H):
    rng = np.random.default_rng(0)
    return rng.random((H, W, 3), dtype=np.float32), rng.integers(0, 300, (H, W)).astype(np.uint32)


def pack(Ld, samples, tiles, W, H, tile=256):
    out = np.zeros((len(tiles) * tile * tile, 4), np.float32)
    for k, (tx, ty) in enumerate(tiles):
        blk = np.zeros((tile, tile, 4), np.float32)
        x0, y0 = tx * tile, ty * tile
        w, h = min(tile, W - x0), min(tile, H - y0)
        blk[:h, :w, :3] = Ld[y0:y0 + h, x0:x0 + w]
        blk[:h, :w, 3] = samples[y0:y0 + h, x0:x0 + w].view(np.float32)
        out[k * tile * tile:(k + 1) * tile * tile] = blk.reshape(-1, 4)
    return out


def _worker(rank, world, port, q):
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    W, H = 700, 530
    Ld, smp = fake_film(W, H)
    tiles = parallel.tiles_for_rank(rank, world, W, H)
    local = torch.from_numpy(pack(Ld, smp, tiles, W, H))
    parts = parallel.gather_packed(local, rank, world, dist)
    if rank == 0:
        L2 = S2 = None
        for r, p in enumerate(parts):
            L2, S2 = parallel.unpack(p.numpy(), parallel.tiles_for_rank(r, world, W, H), W, H, 256, L2, S2)
        q.put(bool(np.array_equal(L2, Ld) and np.array_equal(S2, smp)))
    dist.barrier()
    dist.destroy_process_group()


def test_gather_roundtrip_gloo_world2():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    ok = q.get(timeout=120)
    for p in procs:
        p.join(60)
    assert ok
