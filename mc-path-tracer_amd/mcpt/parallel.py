"""Multi-GPU frame tiling and the frame-end film gather.

Tiles are independent (keyed RNG: a pixel's result does not depend on who renders it), so the
only collective is one gather of the per-rank tile pixels at frame end, to rank 0.  Every rank
packs its tiles' pixels into a contiguous 16 B/px buffer (Ld rgb f32 + samples u32 bits,
mcpt_film_pack_tiles) and sends it to rank 0 over RCCL (torch.distributed send/recv, backend
"nccl": point-to-point over xGMI, each peer on its own link to rank 0 -- no ring, no N-fold
all_gather payload).  Rank 0 receives every buffer into device memory and scatters it into its
device film with mcpt_film_unpack_tiles, so its film readers return the whole frame.  The film's
home stays device memory, as in the reference (Film.cu:121-172).  Buffer sizes follow from the
deterministic tile partition, so no size exchange is needed.  No exchange happens while rendering.
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


# Path state per path (126 B).  The strong split has no byte budget of its own
# since every rank holds only its tiles' state (compact layout): C5 at N = 8, the largest case, is
# 2.1 M pixels x 128 slots x 126 B = 34 GB of a GPU's 288 GB.
PATH_BYTES = 126


def rank_path_pixels(world, W, H, tile):
    """Pixels of path state the largest rank allocates in the compact layout (mcpt_set_compact_paths):
    its tiles x tile pixels, the overhang of edge tiles included."""
    return max(len(tiles_for_rank(r, world, W, H, tile)) for r in range(world)) * tile * tile


def strong_slots(base_slots, world, W, H, spp, tile, budget=None):
    """Path slots for a frame split over `world` ranks: every rank keeps the paths in flight of the
    one-GPU run (base_slots x W x H) over its 1/world of the pixels, so slots scale with world --
    bounded by spp / 2 (a slot renders >= 2 samples: config 2 at N = 8 ran 43.4 ms per rank frame at
    128 slots against 44.7 at 192, whose 1.3 samples per slot leave a long tail;
    profiles/partition_r05_c2_slots.json), by the ABI's 256 and by fewer than 2^31 paths of the
    rank's own path state (compact layout: its tiles only); `budget` (bytes of path state per GPU)
    caps them further when given.  Not below base_slots unless the 2^31-path cap or the budget binds
    (then the cap).  `tile` is the partition's tile edge (tiles_for_rank's): no default, so the
    slots are sized for the partition the caller renders.  One value for every rank: the slot count
    sets the film's summation order, so the gathered frame then equals a one-rank frame rendered
    with the same slots bit for bit."""
    px = rank_path_pixels(world, W, H, tile) if world > 1 else W * H
    cap = max(1, ((1 << 31) - 1) // px)
    if budget is not None:
        cap = max(1, min(cap, budget // (PATH_BYTES * px)))
    return int(max(1, min(max(base_slots, min(base_slots * world, max(1, spp // 2), 256)), cap)))  # 1..256


def pack(Ld: np.ndarray, samples: np.ndarray, tiles, W, H, tile=256) -> np.ndarray:
    """Host restatement of mcpt_film_pack_tiles: a film's tile pixels as [n, 4] float32 (.w =
    samples bits), tile by tile, rows of tile_w pixels; pixels past the frame edge are zero."""
    out = np.zeros((len(tiles) * tile * tile, 4), np.float32)
    for k, (tx, ty) in enumerate(tiles):
        blk = np.zeros((tile, tile, 4), np.float32)
        x0, y0 = tx * tile, ty * tile
        w, h = min(tile, W - x0), min(tile, H - y0)
        blk[:h, :w, :3] = Ld[y0:y0 + h, x0:x0 + w]
        blk[:h, :w, 3] = np.ascontiguousarray(samples[y0:y0 + h, x0:x0 + w], np.uint32).view(np.float32)
        out[k * tile * tile:(k + 1) * tile * tile] = blk.reshape(-1, 4)
    return out


def unpack(packed: np.ndarray, tiles, W, H, tile=256, Ld=None, samples=None):
    """Scatter a rank's packed tile pixels ([n,4] float32, .w = samples bits) into a host film."""
    if Ld is None:
        Ld = np.zeros((H, W, 3), np.float32)
        samples = np.zeros((H, W), np.uint32)
    px = tile * tile
    for k, (tx, ty) in enumerate(tiles):
        blk = packed[k * px:(k + 1) * px].reshape(tile, tile, 4)
        x0, y0 = tx * tile, ty * tile
        w, h = min(tile, W - x0), min(tile, H - y0)
        Ld[y0:y0 + h, x0:x0 + w] = blk[:h, :w, :3]
        samples[y0:y0 + h, x0:x0 + w] = np.ascontiguousarray(blk[:h, :w, 3]).view(np.uint32)
    return Ld, samples


def gather_packed_to_root(local, rank, world, dist, W, H, tile=256):
    """Send every rank's packed [n, 4] float32 tensor to rank 0 (point-to-point send / recv,
    nccl with device tensors or gloo with host tensors).  Rank 0 gets the list of per-rank
    tensors (its own first) on local's device; the other ranks get None.  Sizes come from the
    tile partition (tiles_for_rank), which every rank computes identically."""
    import torch

    if rank != 0:
        # a rank with no tiles (fewer tiles than ranks) sends nothing, as rank 0 posts no receive for
        # it: an unmatched send would hang RCCL or leave a stray gloo message for a later collective
        if local.shape[0]:
            dist.send(local.contiguous(), dst=0)
        return None
    parts = [local]
    for r in range(1, world):
        n = len(tiles_for_rank(r, world, W, H, tile)) * tile * tile
        buf = torch.empty((n, 4), dtype=local.dtype, device=local.device)
        if n:
            dist.recv(buf, src=r)
        parts.append(buf)
    return parts


def gather_film_to_root(pt, rank, world, tile=256):
    """Frame-end gather of a tiled multi-GPU render into rank 0's device film: pack on every rank,
    send to rank 0 (RCCL over xGMI), scatter there with mcpt_film_unpack_tiles.  Afterwards
    pt.film() / write_png() on rank 0 return the whole frame."""
    import ctypes as C

    import torch
    import torch.distributed as dist

    from . import _check, lib

    n = C.c_uint32()
    _check(lib().mcpt_film_pack_tiles(pt.h, None, C.byref(n)), pt.h)
    local = torch.empty((n.value, 4), dtype=torch.float32, device="cuda")
    _check(lib().mcpt_film_pack_tiles(pt.h, C.c_void_p(local.data_ptr()), C.byref(n)), pt.h)
    host = dist.get_backend() != "nccl"  # gloo rehearsal: host-side point-to-point
    if host:
        local = local.cpu()
    parts = gather_packed_to_root(local, rank, world, dist, pt.W, pt.H, tile)
    if rank != 0:
        return None
    for r, part in enumerate(parts[1:], start=1):
        rt = tiles_for_rank(r, world, pt.W, pt.H, tile)
        if not rt:
            continue
        dev = part.cuda() if host else part
        xy = np.ascontiguousarray(rt, np.uint32).reshape(-1, 2)
        torch.cuda.synchronize()  # the received buffer is complete before the library's stream reads it
        _check(lib().mcpt_film_unpack_tiles(pt.h, C.c_void_p(dev.data_ptr()), xy.ctypes.data_as(C.POINTER(C.c_uint32)),
                                            len(rt)), pt.h)
    return True
