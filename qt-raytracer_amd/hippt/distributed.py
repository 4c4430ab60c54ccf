"""One-process-per-GPU row split.

Pixels are independent and the RNG seed depends only on the global (x, y, frame), so each
rank renders its own rows with no data-path collective.  Two splits: contiguous row bands
(row_band) and interleaved rows (rank r renders rows r, r+N, r+2N, ...: interleaved_rows).
Bands of a scene differ in cost by up to 1.6x (sky vs. walls), so the N-GPU step time — the
slowest rank — favours interleaving.  The only exchanges are the (untimed) host gather of the
ARGB rows for output and the max-over-ranks of the timed interval.
"""
from __future__ import annotations

import numpy as np


def row_band(rank: int, world: int, height: int):
    """Rows [floor(r*H/N), floor((r+1)*H/N)) — the same split libhippt uses across devices."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} of {world}")
    return (rank * height) // world, ((rank + 1) * height) // world


def interleaved_rows(rank: int, world: int, height: int) -> np.ndarray:
    """Rows rank, rank+N, ... < H — libhippt's hipptSetRowInterleave(rank, N)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} of {world}")
    return np.arange(rank, height, world)


def env_rank():
    import os
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0")),
            int(os.environ.get("WORLD_SIZE", "1")))


def max_over_ranks(value: float, dist=None) -> float:
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return float(value)
    import torch
    t = torch.tensor([float(value)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(value: int, dist=None) -> int:
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return int(value)
    import torch
    t = torch.tensor([int(value)], dtype=torch.int64)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return int(t.item())


def gather_bands(band: np.ndarray, height: int, dist=None) -> np.ndarray:
    """Assembles full-height images from per-rank row bands (every rank gets the image).

    band: (rows, W, ...) of this rank's row_band.  Works for any dtype via a byte view.
    """
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return band
    import torch
    world, rank = dist.get_world_size(), dist.get_rank()
    width_shape = band.shape[1:]
    row_bytes = int(np.prod(width_shape, dtype=np.int64)) * band.dtype.itemsize
    max_rows = max(row_band(r, world, height)[1] - row_band(r, world, height)[0] for r in range(world))
    buf = np.zeros((max_rows, row_bytes), np.uint8)
    raw = np.ascontiguousarray(band).view(np.uint8).reshape(band.shape[0], row_bytes)
    buf[: band.shape[0]] = raw
    outs = [torch.zeros((max_rows, row_bytes), dtype=torch.uint8) for _ in range(world)]
    dist.all_gather(outs, torch.from_numpy(buf))
    full = np.zeros((height, row_bytes), np.uint8)
    for r in range(world):
        y0, y1 = row_band(r, world, height)
        full[y0:y1] = outs[r].numpy()[: y1 - y0]
    del rank
    return full.view(band.dtype).reshape((height,) + width_shape)


def gather_interleaved(rows: np.ndarray, height: int, dist=None) -> np.ndarray:
    """Full-height images from per-rank interleaved rows (rows: (len(interleaved_rows), W, ...))."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return rows
    import torch
    world = dist.get_world_size()
    width_shape = rows.shape[1:]
    row_bytes = int(np.prod(width_shape, dtype=np.int64)) * rows.dtype.itemsize
    max_rows = -(-height // world)
    buf = np.zeros((max_rows, row_bytes), np.uint8)
    buf[: rows.shape[0]] = np.ascontiguousarray(rows).view(np.uint8).reshape(rows.shape[0], row_bytes)
    outs = [torch.zeros((max_rows, row_bytes), dtype=torch.uint8) for _ in range(world)]
    dist.all_gather(outs, torch.from_numpy(buf))
    full = np.zeros((height, row_bytes), np.uint8)
    for r in range(world):
        idx = interleaved_rows(r, world, height)
        full[idx] = outs[r].numpy()[: len(idx)]
    return full.view(rows.dtype).reshape((height,) + width_shape)


def gather_floats(values, dist=None) -> list:
    """Every rank's tuple of floats (e.g. its kernel ms and wall time per step), on every rank:
    [rank 0's values, rank 1's, ...].  Bench bookkeeping only, after the timed region."""
    vals = [float(v) for v in values]
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return [vals]
    import torch
    t = torch.tensor(vals, dtype=torch.float64)
    outs = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(outs, t)
    return [o.tolist() for o in outs]
