"""Ray-parallel multi-GPU rendering.

Each ray's output depends only on the (replicated) point table, the MLP
weights and the ray itself (qpiw.py:442-528 threads are per sample; the
aggregator and composite are per ray), so the path shards by rays with no
exchange until the rendered tiles are assembled.  Pixels are dealt in
interleaved 16x16 tiles, round robin over ranks and rotated per frame so the
object-centred load balances; one all-gather over RCCL (xGMI) assembles the
frame on every rank.  One process per GPU, torch.distributed "nccl" (= RCCL
on ROCm); the same code runs on "gloo" for the CPU tests.
"""
from __future__ import annotations

import numpy as np
import torch

TILE = 16


def tile_owner(H: int, W: int, world: int, frame: int = 0) -> np.ndarray:
    """[H*W] rank owning each pixel (row-major pixel order)."""
    ty, tx = np.meshgrid(np.arange(H) // TILE, np.arange(W) // TILE, indexing="ij")
    tiles_x = (W + TILE - 1) // TILE
    return ((ty * tiles_x + tx + frame) % world).reshape(-1)


class TileShard:
    """This rank's share of a frame and the bookkeeping to reassemble it."""

    def __init__(self, H: int, W: int, rank: int, world: int, frame: int = 0, device=None):
        own = tile_owner(H, W, world, frame)
        self.H, self.W, self.rank, self.world = H, W, rank, world
        self.counts = np.bincount(own, minlength=world)
        self.max_count = int(self.counts.max())
        self.pixels = [np.nonzero(own == r)[0] for r in range(world)]
        self.idx = torch.from_numpy(self.pixels[rank]).to(device) if device is not None else \
            torch.from_numpy(self.pixels[rank])

    def select(self, per_pixel: torch.Tensor) -> torch.Tensor:
        """Rows of a [H*W, ...] tensor owned by this rank."""
        return per_pixel.index_select(0, self.idx.to(per_pixel.device)).contiguous()

    def assemble(self, local: torch.Tensor, group=None) -> torch.Tensor:
        """All-gather every rank's [count_r, C] rows into the full [H*W, C] frame."""
        import torch.distributed as dist
        C = local.shape[1]
        pad = local
        if local.shape[0] < self.max_count:
            pad = torch.cat([local, local.new_zeros((self.max_count - local.shape[0], C))])
        backend = dist.get_backend(group)
        if backend == "nccl":
            buf = torch.empty((self.world * self.max_count, C), dtype=local.dtype, device=local.device)
            dist.all_gather_into_tensor(buf, pad.contiguous(), group=group)
            parts = buf.view(self.world, self.max_count, C)
        else:
            lst = [torch.empty_like(pad) for _ in range(self.world)]
            dist.all_gather(lst, pad.contiguous(), group=group)
            parts = torch.stack(lst)
        out = torch.empty((self.H * self.W, C), dtype=local.dtype, device=local.device)
        for r in range(self.world):
            n = int(self.counts[r])
            out[torch.from_numpy(self.pixels[r]).to(local.device)] = parts[r, :n]
        return out
