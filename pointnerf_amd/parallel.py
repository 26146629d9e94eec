"""Ray-parallel multi-GPU rendering.

Each ray's output depends only on the (replicated) point table, the MLP
weights and the ray itself (qpiw.py:442-528 threads are per sample; the
aggregator and composite are per ray), so the path shards by rays with no
exchange until the rendered tiles are assembled.  Two ray batchings:
  * TileShard: one frame split over the ranks, one all-gather assembles it on
    every rank.  Layout "bands" (default): N horizontal bands of whole pixel
    rows, band b of frame f on rank (b + f) mod N, so over the N frames of a
    step every rank renders every band once (the same pixel count and, up to
    the per-frame view change, the same work) while its rays stay as
    spatially coherent as a whole frame's (neighbouring rays share neighbour
    points in L2).  Layout "tiles16": interleaved 16x16 tiles dealt round
    robin (finer balance, 1/N of the spatial coherence);
  * FrameShard: each rank renders whole frames (frame f on rank f mod N);
    one all-gather per step gives every rank the step's N frames.  One render
    call per rank per frame, so no per-call overhead grows with N.
One process per GPU, torch.distributed "nccl" (= RCCL on ROCm); the same code
runs on "gloo" for the CPU tests.
"""
from __future__ import annotations

import numpy as np
import torch

TILE = 16


def tile_owner(H: int, W: int, world: int, frame: int = 0, layout: str = "bands") -> np.ndarray:
    """[H*W] rank owning each pixel (row-major pixel order)."""
    if layout == "bands":
        band = (np.arange(H) * world) // H                    # H rows in `world` near-equal bands
        return np.repeat((band + frame) % world, W)
    if layout != "tiles16":
        raise ValueError(f"layout {layout!r}: 'bands' or 'tiles16'")
    ty, tx = np.meshgrid(np.arange(H) // TILE, np.arange(W) // TILE, indexing="ij")
    tiles_x = (W + TILE - 1) // TILE
    return ((ty * tiles_x + tx + frame) % world).reshape(-1)


class TileShard:
    """This rank's share of a frame and the bookkeeping to reassemble it."""

    def __init__(self, H: int, W: int, rank: int, world: int, frame: int = 0, device=None, layout: str = "bands"):
        own = tile_owner(H, W, world, frame, layout)
        self.H, self.W, self.rank, self.world, self.layout = H, W, rank, world, layout
        self.counts = np.bincount(own, minlength=world)
        self.max_count = int(self.counts.max())
        self.pixels = [np.nonzero(own == r)[0] for r in range(world)]
        # pixel -> row of the gathered [world * max_count] buffer (rank r's j-th pixel)
        src = np.empty(H * W, dtype=np.int64)
        for r in range(world):
            src[self.pixels[r]] = r * self.max_count + np.arange(self.pixels[r].size)
        self.idx = torch.from_numpy(self.pixels[rank])
        self.src = torch.from_numpy(src)
        if device is not None:
            self.idx, self.src = self.idx.to(device), self.src.to(device)

    def select(self, per_pixel: torch.Tensor) -> torch.Tensor:
        """Rows of a [H*W, ...] tensor owned by this rank."""
        return per_pixel.index_select(0, self.idx.to(per_pixel.device)).contiguous()

    def assemble(self, local: torch.Tensor, group=None) -> torch.Tensor:
        """All-gather every rank's [count_r, C] rows into the full [H*W, C] frame."""
        return self.assemble_async(local, group).wait()

    def assemble_async(self, local: torch.Tensor, group=None) -> "_Gather":
        """Start the all-gather and return a handle whose wait() yields the
        [H*W, C] frame.  On RCCL the collective runs on its own stream, so the
        caller can render the next ray batch while the tiles travel over xGMI."""
        import torch.distributed as dist
        C = local.shape[1]
        pad = local.new_zeros((self.max_count, C))
        pad[: local.shape[0]] = local
        if dist.get_backend(group) == "nccl":
            buf = torch.empty((self.world * self.max_count, C), dtype=local.dtype, device=local.device)
            work = dist.all_gather_into_tensor(buf, pad, group=group, async_op=True)
            return _Gather(self, work, buf, None)
        lst = [torch.empty_like(pad) for _ in range(self.world)]
        work = dist.all_gather(lst, pad, group=group, async_op=True)
        return _Gather(self, work, None, lst)


class _Gather:
    def __init__(self, shard, work, buf, parts):
        self.shard, self.work, self.buf, self.parts = shard, work, buf, parts

    def wait(self) -> torch.Tensor:
        self.work.wait()
        buf = self.buf if self.buf is not None else torch.cat(self.parts)
        return buf.index_select(0, self.shard.src.to(buf.device))


class StepShard:
    """A rank's shares of the N frames of one step rendered as ONE ray batch
    (NeuralPointsRayMarching.render_rays with ray_cam: one query / aggregate /
    composite launch for all N partial frames) and assembled with ONE
    all-gather: rank r's rows are its share of frame 0, then of frame 1, ...;
    wait() returns the N full frames [H*W, C] in step order."""

    def __init__(self, shards: list, device=None):
        self.shards = shards
        self.world = shards[0].world
        rank = shards[0].rank
        # per frame: rows of every rank's share, padded per rank to the step's max
        per_rank = np.array([[sh.counts[r] for sh in shards] for r in range(self.world)])   # [world, frames]
        self.sizes = per_rank[rank].tolist()
        self.max_count = int(per_rank.sum(1).max())
        offs = np.concatenate([np.zeros((self.world, 1), np.int64), np.cumsum(per_rank, 1)], 1)
        self.src = []
        for f, sh in enumerate(shards):
            src = np.empty(sh.H * sh.W, dtype=np.int64)
            for r in range(self.world):
                src[sh.pixels[r]] = r * self.max_count + offs[r, f] + np.arange(sh.pixels[r].size)
            self.src.append(torch.from_numpy(src).to(device) if device is not None else torch.from_numpy(src))
        idx = np.concatenate([sh.pixels[rank] for sh in shards])
        self.idx = torch.from_numpy(idx).to(device) if device is not None else torch.from_numpy(idx)
        cam = np.repeat(np.arange(len(shards), dtype=np.int32), self.sizes)
        self.ray_cam = torch.from_numpy(cam).to(device) if device is not None else torch.from_numpy(cam)

    def select(self, per_frame: list) -> torch.Tensor:
        """This rank's rays of the step: rows of each frame's [H*W, ...] tensor
        (per_frame[f]) it owns, concatenated in frame order."""
        return torch.cat([t.index_select(0, sh.idx.to(t.device)) for t, sh in zip(per_frame, self.shards)])

    def assemble_async(self, local: torch.Tensor, group=None) -> "_StepGather":
        import torch.distributed as dist
        C = local.shape[1]
        pad = local.new_zeros((self.max_count, C))
        pad[: local.shape[0]] = local
        if dist.get_backend(group) == "nccl":
            buf = torch.empty((self.world * self.max_count, C), dtype=local.dtype, device=local.device)
            work = dist.all_gather_into_tensor(buf, pad, group=group, async_op=True)
            return _StepGather(self, work, buf, None)
        lst = [torch.empty_like(pad) for _ in range(self.world)]
        work = dist.all_gather(lst, pad, group=group, async_op=True)
        return _StepGather(self, work, None, lst)


class _StepGather:
    def __init__(self, step, work, buf, parts):
        self.step, self.work, self.buf, self.parts = step, work, buf, parts

    def wait(self) -> list:
        self.work.wait()
        buf = self.buf if self.buf is not None else torch.cat(self.parts)
        return [buf.index_select(0, src.to(buf.device)) for src in self.step.src]


class FrameShard:
    """Whole-frame ray batches: rank r renders frames r, r + N, r + 2N, ...;
    assemble_async all-gathers one [P, C] frame from every rank into the
    step's [N, P, C] stack (frame r of the step from rank r)."""

    def __init__(self, rank: int, world: int):
        self.rank, self.world = rank, world

    def frame_of(self, step: int) -> int:
        return step * self.world + self.rank

    def assemble_async(self, local: torch.Tensor, group=None) -> "_FrameGather":
        import torch.distributed as dist
        local = local.contiguous()
        if dist.get_backend(group) == "nccl":
            buf = torch.empty((self.world,) + tuple(local.shape), dtype=local.dtype, device=local.device)
            work = dist.all_gather_into_tensor(buf, local, group=group, async_op=True)
            return _FrameGather(work, buf, None)
        lst = [torch.empty_like(local) for _ in range(self.world)]
        work = dist.all_gather(lst, local, group=group, async_op=True)
        return _FrameGather(work, None, lst)


class _FrameGather:
    def __init__(self, work, buf, parts):
        self.work, self.buf, self.parts = work, buf, parts

    def wait(self) -> torch.Tensor:
        self.work.wait()
        return self.buf if self.buf is not None else torch.stack(self.parts)


class GradReducer:
    """The data-parallel finetune step's gradient reduction.

    The reference wraps its whole net -- aggregator MLP and the neural point
    table as nn.Parameters -- in DistributedDataParallel (base_model.py:61-71,
    train_ddp.py:803-804), i.e. a mean all-reduce of every gradient.  Here the
    same mean is built for this path's sparsity: the MLP gradients (~0.5 MB) go
    as ONE flat all_reduce; the point table's gradients (N x 39 floats, 312 MB
    at 2 M points, zero outside the rows the rank's batch touched) go as the
    touched rows only -- an all-gather of (row ids, rows) and an index_add on
    every rank -- so the bytes on xGMI scale with the batch, not the table.
    After reduce() every rank holds the same gradients: the mean over ranks,
    equal (up to summation order) to one process stepping the union batch
    with a loss averaged per rank."""

    def __init__(self, dense_params, point_params, group=None, host_group=None):
        """Collective when the process group is not gloo: EVERY rank of the default
        group must construct its reducer, in the same order relative to other
        group creations -- it creates the gloo group that carries the host-side
        row counts (dist.new_group is a collective over the default group),
        whether or not this rank's reducer has point parameters, unless
        ``host_group`` (a gloo group over the same ranks as ``group``) is
        passed."""
        self.dense = [p for p in dense_params if p.requires_grad]
        self.points = [p for p in point_params if p is not None and p.requires_grad]
        self.group = group
        self._host_group = host_group   # gloo group for host-side integers (no device sync)
        if host_group is None:
            import torch.distributed as dist
            if dist.is_initialized() and dist.get_backend(group) != "gloo":
                ranks = None if group is None else dist.get_process_group_ranks(group)
                self._host_group = dist.new_group(ranks=ranks, backend="gloo")
        # point tables as [rows, channels] (the reference keeps them [1, N, C])
        if self.points:
            n = self.points[0].numel() // self.points[0].shape[-1]
            for p in self.points:
                if p.numel() // p.shape[-1] != n:
                    raise ValueError("GradReducer: point parameters must share their row count")

    @staticmethod
    def _grad(p):
        if p.grad is None:
            p.grad = torch.zeros_like(p)
        return p.grad

    def _all_gather(self, t):
        import torch.distributed as dist
        world = dist.get_world_size(self.group)
        if dist.get_backend(self.group) == "nccl":
            buf = torch.empty((world,) + tuple(t.shape), dtype=t.dtype, device=t.device)
            dist.all_gather_into_tensor(buf, t.contiguous(), group=self.group)
            return buf
        lst = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(lst, t.contiguous(), group=self.group)
        return torch.stack(lst)

    def _max_over_ranks(self, v: int) -> int:
        """max of a host integer over the ranks, on the CPU (gloo): the padding
        size of the row all-gather without a device -> host copy."""
        import torch.distributed as dist
        gloo = dist.get_backend(self.group) == "gloo"
        g = self.group if gloo else self._host_group
        if not gloo and g is None:
            raise RuntimeError("GradReducer: no gloo group for the host counts (construct it after "
                               "init_process_group, or pass host_group)")
        t = torch.tensor([int(v)], dtype=torch.int64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=g)
        return int(t.item())

    def reduce(self, touched: torch.Tensor | None = None, count: int | None = None):
        """touched: this rank's point rows with a (possibly) non-zero gradient
        (any integer dtype); None = every row (dense).  With ``count`` (host
        int = touched.numel()) the rows must be unique, -1 entries ignored --
        what render_rays_train's last_train_aux["touched_rows"] holds -- and the
        reduction never reads a device value on the host (the padding size is a
        max over ranks of the host counts, on gloo); without it duplicates are
        allowed (torch.unique, one sync)."""
        import torch.distributed as dist
        world = dist.get_world_size(self.group)
        if world == 1:
            return
        if self.dense:
            flat = torch.cat([self._grad(p).reshape(-1) for p in self.dense])
            dist.all_reduce(flat, group=self.group)
            flat.div_(world)
            o = 0
            for p in self.dense:
                k = p.numel()
                p.grad.copy_(flat[o:o + k].view_as(p))
                o += k
        if not self.points:
            return
        dev = self.points[0].device
        n = self.points[0].numel() // self.points[0].shape[-1]
        if touched is None:
            rows = torch.arange(n, device=dev)
            count = n
        elif count is None:
            rows = torch.unique(touched.to(device=dev, dtype=torch.int64))
            count = rows.numel()
        else:
            rows = touched.to(device=dev, dtype=torch.int64).reshape(-1)
            if rows.numel() != count:
                raise ValueError(f"GradReducer.reduce: count {count} != touched.numel() {rows.numel()}")
        widths = [p.shape[-1] for p in self.points]
        mx = self._max_over_ranks(count)
        ids = torch.full((mx,), -1, dtype=torch.int64, device=dev)
        ids[:count] = rows
        vals = torch.zeros((mx, sum(widths)), dtype=self.points[0].dtype, device=dev)
        if count:
            # -1 entries gather row 0 and are zeroed (where, not a product: row 0 may hold
            # inf / NaN, which a 0 * x would spread to every rank)
            src = rows.clamp(min=0)
            g = torch.cat([self._grad(p).reshape(n, -1)[src] for p in self.points], 1)
            vals[:count] = torch.where((rows >= 0)[:, None], g, torch.zeros((), dtype=g.dtype, device=dev))
        all_ids = self._all_gather(ids)      # [world, mx]
        all_vals = self._all_gather(vals)    # [world, mx, D]
        sel = all_ids.reshape(-1).clamp(min=0)
        v = all_vals.reshape(-1, sum(widths)).div_(world)
        o = 0
        for p, w in zip(self.points, widths):
            g = self._grad(p).reshape(n, w)
            g.zero_()
            g.index_add_(0, sel, v[:, o:o + w])
            o += w
