"""Row-stripe partition of a frame across ranks and the gather that reassembles it.

Stripe s (rows [s*stripe, (s+1)*stripe)) belongs to rank s % world, which interleaves cheap
(sky) and expensive (geometry) rows across GPUs.  Every rank renders its rows packed in
order into a buffer padded to `max_rows(...)` rows (fp32 RGB, or RGBA8 quantised on the device:
4 instead of 12 bytes per pixel on the wire), one gather to rank 0 (`gather_to_root`: RCCL over
xGMI on the GPU box, gloo in the CPU tests; SURVEY §8(e)'s ncclGather) concatenates the buffers
there, and `assemble` un-permutes them.
The RNG is keyed by the GLOBAL pixel index (curand_init(seed, pixel, 0), main.cu:268), so
the assembled frame is bit-identical to a single-GPU render.
"""
from __future__ import annotations

import numpy as np


def stripe_rows(height: int, stripe: int, world: int, rank: int) -> np.ndarray:
    r = np.arange(height)
    return r[(r // stripe) % world == rank].astype(np.int32)


def max_rows(height: int, stripe: int, world: int) -> int:
    stripes = (height + stripe - 1) // stripe
    return ((stripes + world - 1) // world) * stripe


def gather_to_root(local, world: int, rank: int, out=None):
    """Gather every rank's padded stripe buffer (a flat tensor, same shape on every rank) into
    `out` on rank 0 -- shape (world * local.numel(),), allocated if None -- and return it there
    (None on the other ranks).  One collective per frame; only rank 0 receives (the frame is
    written by rank 0), unlike an all-gather that would send every frame to every rank."""
    import torch
    import torch.distributed as dist
    if rank == 0:
        if out is None:
            out = torch.empty((world * local.numel(),), dtype=local.dtype, device=local.device)
        dist.gather(local, list(out.view(world, -1).unbind(0)), dst=0)
        return out
    dist.gather(local, None, dst=0)
    return None


def assemble(gathered, height: int, width: int, stripe: int, world: int, channels: int = 3):
    """gathered: array/tensor of shape (world, max_rows, width, channels) -> (height, width, channels).
    channels = 3 for fp32 RGB frames, 4 for device-quantised RGBA8 frames (PT_OUT_RGBA8)."""
    mr = max_rows(height, stripe, world)
    g = gathered.reshape(world, mr, width, channels)
    try:  # torch tensor
        import torch
        if isinstance(g, torch.Tensor):
            img = torch.empty((height, width, channels), dtype=g.dtype, device=g.device)
            for r in range(world):
                rows = torch.as_tensor(stripe_rows(height, stripe, world, r), device=g.device, dtype=torch.long)
                img[rows] = g[r, : len(rows)]
            return img
    except ImportError:
        pass
    img = np.empty((height, width, channels), dtype=g.dtype)
    for r in range(world):
        rows = stripe_rows(height, stripe, world, r)
        img[rows] = g[r, : len(rows)]
    return img
