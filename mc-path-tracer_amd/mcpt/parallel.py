"""Multi-GPU frame tiling and the film gather.

Tiles are independent (keyed RNG: a pixel's result does not depend on who renders it), so the
only collective is one gather of the per-rank tile pixels at frame end: every rank packs its
tiles' pixels into a contiguous 16 B/px buffer (Ld rgb f32 + samples u32, mcpt_film_pack_tiles)
and one all_gather over RCCL/xGMI (torch.distributed, backend "nccl") brings them to every rank;
rank 0 scatters them into the full film.  No exchange happens while rendering.
"""
from __future__ import annotations

import numpy as np


def tile_grid(W, H, tile=256):
    return (W + tile - 1) // tile, (H + tile - 1) // tile


def tiles_for_rank(rank, world, W, H, tile=256):
    """Interleaved assignment: tile (tx, ty) -> rank (tx + ty) mod world (balances sky vs geometry
    and spreads the partial right/bottom tiles over ranks)."""
    nx, ny = tile_grid(W, H, tile)
    return [(tx, ty) for ty in range(ny) for tx in range(nx) if (tx + ty) % world == rank]


def unpack(packed: np.ndarray, tiles, W, H, tile=256, Ld=None, samples=None):
    """Scatter a rank's packed tile pixels ([n,4] float32, .w = samples bits) into a full film."""
    if Ld is None:
        Ld = np.zeros((H, W, 3), np.float32)
        samples = np.zeros((H, W), np.uint32)
    px = tile * tile
    for k, (tx, ty) in enumerate(tiles):
        blk = packed[k * px:(k + 1) * px].reshape(tile, tile, 4)
        x0, y0 = tx * tile, ty * tile
        w, h = min(tile, W - x0), min(tile, H - y0)
        Ld[y0:y0 + h, x0:x0 + w] = blk[:h, :w, :3]
        samples[y0:y0 + h, x0:x0 + w] = blk[:h, :w, 3].view(np.uint32)
    return Ld, samples


def gather_packed(local: "torch.Tensor", rank, world, dist):
    """all_gather of variable-length [n,4] float32 tensors (padded to the max); returns the list
    of per-rank tensors (trimmed).  Works with nccl (device tensors) and gloo (CPU tensors)."""
    import torch

    n = torch.tensor([local.shape[0]], dtype=torch.int64, device=local.device)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n)
    sizes = [int(s.item()) for s in sizes]
    mx = max(sizes)
    buf = torch.zeros((mx, 4), dtype=local.dtype, device=local.device)
    buf[: local.shape[0]] = local
    outs = [torch.zeros_like(buf) for _ in range(world)]
    dist.all_gather(outs, buf)
    return [o[:s] for o, s in zip(outs, sizes)]


def gather_film(pt, rank, world, tile=256):
    """Gather the film of a tiled multi-GPU render onto every rank; returns (Ld, samples) on rank 0."""
    import ctypes as C

    import torch
    import torch.distributed as dist

    from . import lib, _check

    n = C.c_uint32()
    _check(lib().mcpt_film_pack_tiles(pt.h, None, C.byref(n)), pt.h)
    local = torch.empty((n.value, 4), dtype=torch.float32, device="cuda")
    _check(lib().mcpt_film_pack_tiles(pt.h, C.c_void_p(local.data_ptr()), C.byref(n)), pt.h)
    if dist.get_backend() != "nccl":  # gloo rehearsal: host-side collective
        torch.cuda.synchronize()
        local = local.cpu()
    parts = gather_packed(local, rank, world, dist)
    if rank != 0:
        return None
    Ld = samples = None
    for r, part in enumerate(parts):
        Ld, samples = unpack(part.cpu().numpy(), tiles_for_rank(r, world, pt.W, pt.H, tile), pt.W, pt.H, tile, Ld, samples)
    return Ld, samples
