"""Neural point cloud + the fused render module (the north-star hot path).

``NeuralPoints`` mirrors the parameter table of
models/neural_points/neural_points.py:11-331 (same parameter names, so the
``neural_points.*`` keys of a reference checkpoint load into it) and its
14-tuple ``forward`` (neural_points.py:782-812) for API compatibility.

``NeuralPointsRayMarching`` mirrors
models/neural_points_volumetric_model.py:230-389 (forward(**input) -> dict with
coarse_raycolor / coarse_point_opacity / coarse_is_background / coarse_mask /
queried_shading / ray_mask).  Its forward is the fused MI355X path:
    pnr_query  (grid-resident march + layered KNN, device-side compaction)
 -> pnr_aggregate_fwd (gather + weights + PE + MFMA MLP + K-sum + colour MLP)
 -> pnr_composite_fwd (ray_dist + alpha composite + fill_invalid)
with one small device->host read of the sample counts per ray batch (to size
the feature buffer) and no ``raypos[R,400,3]`` / ``[R,SR,K,38]`` intermediates.
"""
from __future__ import annotations

import gc

import torch
import torch.nn as nn

from . import _lib as L
from .aggregator import PointAggregator
from .querier import QueryBuffers, lighting_fast_querier


class NeuralPoints(nn.Module):
    """Point table of neural_points.NeuralPoints (world-coordinate querier)."""

    def __init__(self, opt, device, xyz=None, embedding=None, color=None, dirs=None, conf=None,
                 Rw2c=None, emb_dtype=torch.float32):
        """emb_dtype torch.bfloat16 stores points_embeding in bf16 (SURVEY config
        c5: 104 B per point instead of 168; the bf16 render path reads it
        directly, the fp32 paths from an fp32 copy; training needs fp32)."""
        super().__init__()
        if emb_dtype not in (torch.float32, torch.bfloat16):
            raise L.PnrError(f"emb_dtype {emb_dtype}: float32 or bfloat16")
        self.emb_dtype = emb_dtype
        self._emb32 = (None, None)
        self.opt = opt
        self.device = torch.device(device)
        self.xyz = nn.Parameter(torch.zeros((0, 3), device=self.device), requires_grad=False)
        self.points_embeding = nn.Parameter(torch.zeros((1, 0, 32), device=self.device))
        self.points_conf = None
        self.points_dir = None
        self.points_color = None
        self.Rw2c = torch.eye(3, device=self.device)
        if xyz is not None:
            self.set_points(xyz, embedding, color, dirs, conf, Rw2c)
        self.querier = lighting_fast_querier(self.device, opt)

    def set_points(self, xyz, embedding, color=None, dirs=None, conf=None, Rw2c=None):
        """set_points (neural_points.py:480-546) with point_*_mode '1'; xyz is
        trainable with --xyz_grad 1 (neural_points.py:270: the HIP backward's
        pnr_aggregate_bwd_xyz, render_rays_train only)."""
        dev = self.device
        self.xyz = nn.Parameter(xyz.to(dev).float().reshape(-1, 3).contiguous(),
                                requires_grad=getattr(self.opt, "xyz_grad", 0) > 0)
        self.points_embeding = nn.Parameter(embedding.to(dev).to(self.emb_dtype).reshape(1, -1, 32).contiguous())
        self.points_color = None if color is None else nn.Parameter(color.to(dev).float().reshape(1, -1, 3).contiguous())
        self.points_dir = None if dirs is None else nn.Parameter(dirs.to(dev).float().reshape(1, -1, 3).contiguous())
        self.points_conf = None if conf is None else nn.Parameter(conf.to(dev).float().reshape(1, -1, 1).contiguous())
        # [3,3] uniform, or [N,3,3] per point (neural_points.py:289, 799; pnr_points.rw2c)
        self.Rw2c = torch.eye(3, device=dev) if Rw2c is None else Rw2c.to(dev).float().contiguous()
        if self.Rw2c.dim() == 3 and self.Rw2c.shape != (self.xyz.shape[0], 3, 3):
            raise L.PnrError(f"per-point Rw2c must be [N,3,3], got {tuple(self.Rw2c.shape)}")

    def embedding_fp32(self) -> torch.Tensor:
        """points_embeding as fp32 [N,32] (the table itself, or a copy of the bf16
        table cached on its storage and version)."""
        e = self.points_embeding.detach().reshape(-1, 32)
        if e.dtype == torch.float32:
            return e.contiguous()
        key = (e.data_ptr(), self.points_embeding._version, e.shape[0])
        if self._emb32[0] != key:
            self._emb32 = (key, e.float().contiguous())
        return self._emb32[1]

    def tables(self, campos=None, camrot=None, bf16: bool = False) -> tuple[L.Points, tuple]:
        """pnr_points of the table; bf16 (the bf16 aggregate) passes a bf16
        embedding table as emb_bf16 instead of an fp32 one."""
        e = self.points_embeding.detach().reshape(-1, 32)
        use_b = bf16 and e.dtype == torch.bfloat16
        keep = (self.xyz.detach().contiguous(), None if use_b else self.embedding_fp32(),
                None if self.points_color is None else self.points_color.detach().reshape(-1, 3).contiguous(),
                None if self.points_dir is None else self.points_dir.detach().reshape(-1, 3).contiguous(),
                None if self.points_conf is None else self.points_conf.detach().reshape(-1).contiguous(),
                e.contiguous() if use_b else None)
        p = L.Points(keep[0].shape[0], keep[0].data_ptr(), None, L.ptr(keep[1]), L.ptr(keep[2]), L.ptr(keep[3]),
                     L.ptr(keep[4]), L.ptr(campos), L.ptr(camrot))
        p.emb_bf16 = L.ptr(keep[5])
        rw = self.rw2c_table()
        p.rw2c = L.ptr(rw)
        return p, keep + (rw,)

    def rw2c_table(self):
        """The per-point Rw2c as the kernels read it ([N,9] fp32), or None for a
        uniform Rw2c (that one goes through the aggregator's pnr_mlp.rw2c)."""
        rw = self.Rw2c
        if rw is None or rw.dim() == 2:
            return None
        if rw.shape[0] != self.xyz.shape[0]:
            raise L.PnrError(f"per-point Rw2c has {rw.shape[0]} rows, the cloud {self.xyz.shape[0]} points")
        return rw.detach().reshape(-1, 9).float().contiguous()

    def bytes_per_point(self) -> int:
        """HBM bytes of one point's parameters (168 fp32, 104 with a bf16 embedding)."""
        b = 12 + 32 * self.points_embeding.element_size()
        for t, c in ((self.points_color, 3), (self.points_dir, 3), (self.points_conf, 1)):
            if t is not None:
                b += c * t.element_size()
        return b

    def w2pers(self, point_xyz, camrotc2w, campos):
        """neural_points.py:687-693."""
        point_xyz_shift = point_xyz[None, ...] - campos[:, None, :]
        xyz = torch.sum(camrotc2w[:, None, :, :] * point_xyz_shift[:, :, :, None], dim=-2)
        return torch.stack([xyz[:, :, 0] / xyz[:, :, 2], xyz[:, :, 1] / xyz[:, :, 2], xyz[:, :, 2]], dim=-1)

    def forward(self, inputs):
        """neural_points.py:782-812: query + gather, returns the 14-tuple the
        reference PointAggregator consumes (API path; the fused renderer does
        the gather inside pnr_aggregate_fwd instead)."""
        camrotc2w, campos = inputs["camrotc2w"], inputs["campos"]
        near, far = inputs["near"], inputs["far"]
        pers = self.w2pers(self.xyz, camrotc2w, campos)
        (sample_pidx, sample_loc, sample_loc_w, sample_ray_dirs, ray_mask, vsize, ranges) = \
            self.querier.query_points(inputs.get("pixel_idx"), pers, self.xyz[None, ...], None,
                                      inputs.get("h"), inputs.get("w"), inputs.get("intrinsic"),
                                      torch.min(near).item(), torch.max(far).item(), inputs["raydir"],
                                      campos, camrotc2w)
        mask = sample_pidx >= 0
        B, R, SR, K = sample_pidx.shape
        idx = torch.clamp(sample_pidx, min=0).view(-1).long()
        cat = torch.cat([self.xyz[None, ...], pers, self.points_embeding.float()], dim=-1)
        g = torch.index_select(cat, 1, idx).view(B, R, SR, K, cat.shape[-1])

        def sel(t, c):
            return None if t is None else torch.index_select(t, 1, idx).view(B, R, SR, K, c)

        rw = self.Rw2c if self.Rw2c.dim() == 2 else torch.index_select(self.Rw2c, 0, idx).view(B, R, SR, K, 3, 3)
        return (sel(self.points_color, 3), rw, sel(self.points_dir, 3), sel(self.points_conf, 1),
                g[..., 6:], g[..., 3:6], g[..., :3], mask, sample_loc, sample_loc_w, sample_ray_dirs,
                ray_mask, vsize, 0)


class _RenderState:
    """Device buffers one render stream reuses: the query buffers and the
    aggregate scratch (whose head holds P1, see pnr_points.p1_ready)."""

    def __init__(self):
        self.bufs = None
        self.scratch = None
        self.scratch_key = None
        self.side = None   # fp32h2: the side stream P1 runs on
        self.feat = None   # decoded features [rows, 129], reused by every call on this stream
        self.feat_h = None   # bf16 precision: the same as bf16 rows [rows, L.FEAT_H_PITCH] (uint16)

    def feat_rows(self, rows: int, dev) -> torch.Tensor:
        """[rows, 129] view of the persistent feature buffer.  The calls of one
        stream use it in stream order (a call's composite reads it before the
        next call's aggregate writes it), so it is allocated once and grown by
        1.5x: a multi-GB allocation inside a frame stalls the launch queue
        (c5: 20 GB per frame)."""
        rows = max(int(rows), 1)
        if self.feat is None or self.feat.shape[0] < rows or self.feat.device != dev:
            old = 0 if self.feat is None else self.feat.shape[0]
            self.feat = None
            self.feat = torch.empty((max(rows, int(1.5 * old)), 129), dtype=torch.float32, device=dev)
        return self.feat[:rows]

    def feat_h_rows(self, rows: int, dev) -> torch.Tensor:
        """feat_rows for pnr_aggregate_fwd_bf16_hf's bf16 feature rows."""
        rows = max(int(rows), 1)
        if self.feat_h is None or self.feat_h.shape[0] < rows or self.feat_h.device != dev:
            old = 0 if self.feat_h is None else self.feat_h.shape[0]
            self.feat_h = None
            self.feat_h = torch.empty((max(rows, int(1.5 * old)), L.FEAT_H_PITCH), dtype=torch.int16, device=dev)
        return self.feat_h[:rows]


def _counts_dict(c):
    """The 8 query counters (pnr_query_bufs.counts) as QueryBuffers.read_counts() returns them."""
    n_cand = (int(c[6]) & 0xffffffff) | (int(c[7]) << 32)
    return dict(S_filled=c[0], S_valid=c[1], R_hit=c[2], R_valid=c[3], n_pairs=c[4], n_cand=n_cand)


# The default is fp32h2, the measured headline path (fp32-accurate: the same
# render tolerance as fp32, tests/test_gpu_x3.py; an activation beyond f16's range
# re-renders the call on fp32x3).
# fp32: the reference's arithmetic on v_mfma_f32_32x32x2_f32.  fp32x3: the same
# fp32 GEMMs as exact 3-way bf16 splits on v_mfma_f32_32x32x16_bf16 (six cross
# products, fp32-accurate; pnr_aggregate_fwd_x3).  fp32h2: the same GEMMs as 2-way
# f16 splits on v_mfma_f32_32x32x16_f16 (three products, fp32-accurate;
# pnr_aggregate_fwd_h2).  bf16: bf16 operands (config c5).
PRECISIONS = ("fp32", "fp32x3", "fp32h2", "bf16")


class _ZeroOneConfLoss(torch.autograd.Function):
    """NeuralPointsRayMarching.zero_one_conf_loss on libpnr: the per-point entry
    counts of the query's neighbour lists (pnr_point_counts), then one fused
    reduction (pnr_zero_one_loss_fwd) and one backward kernel -- the same value
    and gradient as torch's clamp / log / mean over the gathered [1, R'', SR, K]
    conf_coefficient, in three launches and without host reads."""

    @staticmethod
    def forward(ctx, conf, bufs, SR, K, eps):
        dev = conf.device
        N = conf.numel()
        c = conf.detach().float().contiguous()
        counts = torch.zeros(N, dtype=torch.float32, device=dev)
        L.check(L.lib().pnr_point_counts(L.ptr(bufs.pidx), L.ptr(bufs.counts), K, bufs.pidx.numel() // K,
                                         L.ptr(counts), L.stream_ptr(dev)), "pnr_point_counts")
        part = torch.empty(1024, dtype=torch.float32, device=dev)
        out = torch.empty(3, dtype=torch.float32, device=dev)
        L.check(L.lib().pnr_zero_one_loss_fwd(L.ptr(c), L.ptr(counts), N, L.c_void_p(bufs.counts.data_ptr() + 12),
                                              SR * K, eps, L.ptr(part), L.ptr(out), L.stream_ptr(dev)),
                "pnr_zero_one_loss_fwd")
        ctx.save_for_backward(c, counts, out)
        ctx.eps = eps
        return out[0].clone()

    @staticmethod
    def backward(ctx, g):
        c, counts, out = ctx.saved_tensors
        d = torch.empty_like(c)
        g = g.reshape(1).float().contiguous()
        L.check(L.lib().pnr_zero_one_loss_bwd(L.ptr(c), L.ptr(counts), c.numel(), ctx.eps, L.ptr(out), L.ptr(g),
                                              L.ptr(d), L.stream_ptr(c.device)), "pnr_zero_one_loss_bwd")
        return d, None, None, None, None


# device bytes a training batch reserves per sample slot: the forward's kept activations
# (train.Saved: 8 pairs x (h1..h4, PE_5, extras, masks, weights) + the sample's colour
# rows) and the backward's dz1..dz4 rows (train.AggregateFn.backward)
TRAIN_BYTES_PER_SAMPLE = 8 * (4 * 1024 + 256 + 128 + 128 + 16) + 2660 + 8 * (4 * 1024 + 4) + 1024


class _TrainAux(dict):
    """render_rays_train's last_train_aux: keys whose values need the batch's
    host counts are computed when first read (so that the forward itself never
    waits for the GPU); ``"k" in aux`` is true for them without computing."""

    def __init__(self):
        super().__init__()
        self._lazy = {}

    def lazy(self, keys, fn):
        for k in keys:
            self._lazy[k] = fn

    def __contains__(self, k):
        return dict.__contains__(self, k) or k in self._lazy

    def __missing__(self, k):
        fn = self._lazy.get(k)
        if fn is None:
            raise KeyError(k)
        vals = fn()
        for kk in list(self._lazy):
            if self._lazy[kk] is fn:
                del self._lazy[kk]
        self.update(vals)
        return dict.__getitem__(self, k)

    def get(self, k, default=None):
        return self[k] if k in self else default


class NeuralPointsRayMarching(nn.Module):
    """neural_points_volumetric_model.NeuralPointsRayMarching, fused HIP path."""

    def __init__(self, opt, neural_points: NeuralPoints, aggregator: PointAggregator | None = None,
                 chunk_rays: int | None = None, precision: str = "fp32h2"):
        super().__init__()
        if precision not in PRECISIONS:
            raise L.PnrError(f"precision {precision!r}: one of {PRECISIONS}")
        self.precision = precision
        # render_rays_train's per-pair forward: "fp32x3" (split-bf16 MFMA,
        # fp32-accurate, the default) or "fp32" (native fp32 MFMA)
        # training path: fp32h2 (forward chain and the weight / point-half gradient GEMMs on f16-split
        # MFMA, the measured default) / fp32x3 (split-bf16 MFMA) / fp32
        self.train_precision = "fp32h2"
        self.p1_side_stream = True        # fp32h2 sync-free calls: P1 beside the query (see _render_rays)
        self.p1_used_only = True          # bf16: P1 for the referenced points only (see _render_rays)
        # bf16: the aggregated features themselves in bf16 (pnr_aggregate_fwd_bf16_hf ->
        # pnr_composite_fwd_hf: half the feature bytes written and read)
        self.bf16_features = True
        self.p1_side_max_points_per_ray = 4.0
        self.keep_train_saved = False   # tests: last_train_aux["saved"] = the forward's kept activations
        # render_rays_train sizes its per-sample buffers for every slot of the batch while
        # R * SR * TRAIN_BYTES_PER_SAMPLE fits this many bytes (None: a quarter of the
        # device memory), else it reads the batch's valid-sample count (train_count_reads)
        self.train_memory_budget = None
        self.train_count_reads = 0
        self._h2_blocked_key = None   # weights whose activations left the f16 range (render_rays)
        self.h2_fallbacks = 0
        self.opt = opt
        self.neural_points = neural_points
        self.aggregator = aggregator if aggregator is not None else PointAggregator(opt).to(neural_points.device)
        self.chunk_rays = chunk_rays
        self._state = _RenderState()     # query buffers + aggregate scratch of the eager path
        self._pending = []               # render_rays(sync=False) calls awaiting finish()
        self._sv_per_ray = None          # largest valid samples per ray seen (feature-buffer sizing)
        self.overflow_rerenders = 0
        # fork's 2-D CNN after the composite (neural_points_volumetric_model.py:258-260, 343-344)
        self.neural_render_2d = None
        if getattr(opt, "neural_render", "none") == "cnn":
            from .neural_render import NeuralRenderer
            self.neural_render_2d = NeuralRenderer(input_dim=128).to(neural_points.device)
        self._last_counts = None
        self._train_conf_src = None   # query buffers of the last render_rays_train (zero_one_conf_loss)
        self._rw2c_key = None
        if getattr(opt, "which_render_func", "radiance") != "radiance" or \
                getattr(opt, "which_blend_func", "alpha") != "alpha" or \
                getattr(opt, "which_tonemap_func", "off") != "off":
            raise L.PnrError("libpnr implements radiance render, alpha blend and tone map 'off'")

    def _sync_rw2c(self):
        """The aggregator renders with NeuralPoints.Rw2c (neural_points.py:289;
        applied to view dirs, distances and point dirs at
        point_aggregators.py:506, 526, 566): copied into the aggregator's
        buffer whenever the points' Rw2c tensor (storage or version) changes."""
        rw = self.neural_points.Rw2c
        key = (rw.data_ptr(), rw._version, tuple(rw.shape))
        if key != self._rw2c_key:
            # per-point [N,3,3]: the kernels read it from pnr_points.rw2c
            # (NeuralPoints.tables), the uniform matrix stays the identity
            self.aggregator.set_rw2c(rw.detach() if rw.dim() == 2 else None)
            self._rw2c_key = key

    @torch.no_grad()
    def render_rays(self, campos, camrot, raydir, near, far, bg_color, force_grid=False, events=None,
                    reuse_p1=False, sync=True, ray_cam=None, query_stream=None):
        """Fused query -> aggregate -> composite for one ray batch [R,3].
        Returns ray_color [R,C], opacity [R,SR], is_bg [R], ray_mask [R] (int8).
        ``events``: optional list that receives (stage, start, end) HIP events
        recorded on the launch stream around each stage.
        ``reuse_p1``: the caller guarantees points_embeding and block1.0 are
        unchanged since the previous render_rays call (e.g. the other partial
        frames of one multi-GPU step), so block1.0's per-point half (P1, which
        does not depend on the camera) is taken from that call's scratch
        instead of recomputed.  The ray chunks of one call always share it.
        ``ray_cam`` (int32 [R], optional): camera index of each ray into
        campos [n_cams,3] / camrot [n_cams,3,3] -- several frames' rays
        rendered as one batch (``render_views``).

        ``sync=False``: no host synchronisation at all.  The decoded-feature
        buffer is sized from the largest valid-sample count per ray seen so far
        (x 1.25) instead of this batch's count, and the two checks a
        synchronous call makes -- the count fits, the fp32h2 activations stayed
        in range -- are deferred to ``finish()``, which re-renders a call that
        failed either of them into the same output tensors.  The outputs are
        valid once ``finish()`` returned.  The first call (no estimate yet)
        runs synchronously.

        ``query_stream`` (sync-free calls): run the call's query on this HIP
        stream instead of the launch stream, so it overlaps the previous call's
        aggregate (the query is memory-latency bound, the aggregate MFMA bound,
        and one query workgroup fits beside a k_pairs_h2 workgroup on a CU).  The
        aggregate waits for it; the query waits only for the launch-stream work
        that last read its buffers (two sets, alternating) and, when the points
        changed since the last such call (new storage or version, or
        ``force_grid``), for the whole launch stream.  The call's own copies of
        its inputs (contiguous rays, camera tables) are made on the query
        stream; the caller makes ``raydir`` / ``campos`` / ``camrot`` /
        ``ray_cam`` themselves ready on that stream.

        fp32h2: the f16 split holds activations below 65504 only.  Each call
        reads the launches' range flag once (a 4-byte read after the last
        chunk); if an activation left the f16 range, the call is rendered again
        on the fp32x3 path (bf16 split: same accuracy, fp32 range) and h2 stays
        off for these weights until they change (``h2_fallbacks`` counts it)."""
        self._sync_rw2c()
        if self._pending and (sync or self._sv_per_ray is None):
            # a synchronous call reads (and may clear) the shared range flag and the
            # counts: complete the pending sync-free calls first so none of their
            # checks is lost; their counts stay queued for the caller's next finish()
            done = self.finish()
            self._done = done + getattr(self, "_done", [])
        prec = self._precision_now()
        if not sync and self._sv_per_ray is not None:
            out, rec = self._render_rays(prec, campos, camrot, raydir, near, far, bg_color, force_grid, events,
                                         reuse_p1, self._state, capacity=self._capacity_per_ray(), ray_cam=ray_cam,
                                         query_stream=query_stream)
            rec["args"] = (campos, camrot, raydir, near, far, bg_color, force_grid, reuse_p1, ray_cam)
            rec["out"] = out
            # what a re-render in finish() must find unchanged (weights, grid)
            rec["h2_key"] = self.aggregator.h2_key()
            rec["grid_key"] = self.neural_points.querier.grid.key
            self._pending.append(rec)
            return out
        n_ev = len(events) if events is not None else 0
        out, _ = self._render_rays(prec, campos, camrot, raydir, near, far, bg_color, force_grid, events, reuse_p1,
                                   self._state, ray_cam=ray_cam)
        if prec == "fp32h2" and not self.aggregator.h2_range_ok():
            self._block_h2()
            if events is not None:
                del events[n_ev:]
            out, _ = self._render_rays("fp32x3", campos, camrot, raydir, near, far, bg_color, force_grid, events,
                                       False, self._state, ray_cam=ray_cam)
        return out

    def render_views(self, views, near, far, bg_color, force_grid=False, events=None, reuse_p1=False, sync=True):
        """Render several frames' ray batches -- views = [(campos [3], camrot
        [3,3], raydir [R_i,3]), ...], e.g. the N band shares one rank renders
        per multi-GPU step -- as ONE batch: one query, one aggregate and one
        composite launch over all of them (pnr_rays.ray_cam), so no per-call
        cost grows with the number of views.  Returns one (ray_color, opacity,
        is_bg, ray_mask) tuple per view (views of the batch outputs); last_counts
        / finish() report the batch."""
        dev = views[0][2].device
        campos = torch.stack([v[0].reshape(3).float() for v in views]).to(dev)
        camrot = torch.stack([v[1].reshape(3, 3).float() for v in views]).to(dev)
        sizes = [int(v[2].shape[0]) for v in views]
        raydir = torch.cat([v[2].reshape(-1, 3).float() for v in views]).contiguous()
        ray_cam = torch.repeat_interleave(torch.arange(len(views), dtype=torch.int32, device=dev),
                                          torch.tensor(sizes, device=dev), output_size=sum(sizes))
        out = self.render_rays(campos, camrot, raydir, near, far, bg_color, force_grid, events, reuse_p1, sync,
                               ray_cam=ray_cam)
        return [tuple(t.split(sizes)[i] for t in out) for i in range(len(views))]

    def _precision_now(self):
        prec = self.precision
        if prec == "fp32h2" and self._h2_blocked_key is not None:
            if self._h2_blocked_key == self.aggregator.h2_key():
                prec = "fp32x3"
            else:
                self._h2_blocked_key = None
        return prec

    def _block_h2(self):
        self.aggregator.h2_reset_range()
        self._h2_blocked_key = self.aggregator.h2_key()
        self.h2_fallbacks += 1

    def _capacity_per_ray(self):
        return self._sv_per_ray * 1.25

    def _observe(self, counts, rays):
        r = counts["S_valid"] / max(rays, 1)
        self._sv_per_ray = r if self._sv_per_ray is None else max(self._sv_per_ray, r)

    @torch.no_grad()
    def finish(self, upto=None):
        """Complete every ``render_rays(sync=False)`` call issued since the last
        finish() -- or only the oldest ``upto`` of them, so the caller can keep
        the next calls queued on the GPU while the host checks these: one host
        synchronisation (on the last completed call), then the deferred checks.
        A call whose valid samples overflowed its feature buffer, or (fp32h2) any
        call when an activation left the f16 range, is rendered again
        synchronously into its own output tensors (a raised range flag is shared
        by the calls still in flight, so then every pending call is completed and
        the later ones' counts are kept for the next finish()).  Returns the
        per-call sample counts (the ``last_counts`` dict of each call, in issue
        order)."""
        from .querier import release_deferred
        release_deferred()
        done = getattr(self, "_done", [])
        n_all = len(done) + len(self._pending)
        k = n_all if upto is None else min(int(upto), n_all)
        need = k - len(done)
        if need > 0:
            head = self._pending[:need]
            head[-1]["event"].synchronize()
            # the range flags as copied to pinned memory behind each call's event (a
            # .item() here would queue behind -- and wait for -- the later calls)
            if need < len(self._pending) and any(int(r["range_host"][0]) != 0 for r in head
                                                 if r.get("range_flag") is not None):
                head = self._pending
                head[-1]["event"].synchronize()
            self._pending = self._pending[len(head):]
            done = done + self._complete(head)
        self._done = done[k:]
        return done[:k]

    def _complete(self, pend):
        """finish()'s checks on calls whose last kernels have completed."""
        if not pend:
            return []
        # every fp32h2 call's own range flag (the packs -- and their flag -- are
        # rebuilt when the weights change between calls)
        flags = {}
        for r in pend:
            f = r.get("range_flag")
            if f is not None:
                bad = int(r["range_host"][0]) != 0   # this call's own copy (taken after its launches)
                prev = flags.get(f.data_ptr())
                flags[f.data_ptr()] = (f, bad or (prev is not None and prev[1]))
        range_bad = any(bad for _, bad in flags.values())
        if range_bad:
            cur = self.aggregator.h2_key()
            for f, bad in flags.values():
                if bad:
                    f.zero_()
            self.aggregator.h2_reset_range()
            if any(r["h2_key"] == cur for r in pend if r.get("range_flag") is not None):
                self._h2_blocked_key = cur
            self.h2_fallbacks += 1
        counts = []
        for rec in pend:
            tot = dict(S_filled=0, S_valid=0, R_hit=0, R_valid=0, n_pairs=0, n_cand=0)
            over = False
            for (cap, rays), h in zip(rec["caps"], rec["host"].tolist()):
                c = _counts_dict(h)
                self._observe(c, rays)
                over |= c["S_valid"] > cap
                for k in tot:
                    tot[k] += c[k]
            f = rec.get("range_flag")
            rec_bad = f is not None and flags[f.data_ptr()][1]
            if over or rec_bad:
                if rec["h2_key"] != self.aggregator.h2_key() or rec["grid_key"] != self.neural_points.querier.grid.key:
                    raise L.PnrError("a render_rays(sync=False) call must be re-rendered, but the weights or the "
                                     "points changed before finish(): call finish() before modifying the model")
                cp, cr, rd, near, far, bg, fg, reuse, rcam = rec["args"]
                prec = "fp32x3" if rec_bad else rec["precision"]
                out, _ = self._render_rays(prec, cp, cr, rd, near, far, bg, fg, None, False, self._state,
                                           ray_cam=rcam)
                for dst, src in zip(rec["out"], out):
                    dst.copy_(src)
                tot = dict(self.last_counts)
                self.overflow_rerenders += int(over)
            counts.append(tot)
        self.last_counts = counts[-1]
        return counts

    def _render_rays(self, precision, campos, camrot, raydir, near, far, bg_color, force_grid, events, reuse_p1,
                     state, capacity=None, keep=None, record=True, ray_cam=None, query_stream=None):
        """One render call.  capacity None: size the feature buffer from this
        batch's counts (one host sync per chunk); else capacity = valid samples
        per ray the feature buffer is sized for (no sync; the per-chunk counts
        are copied to pinned host memory behind an event, returned in the
        record for finish() / RenderGraph.check())."""
        opt = self.opt
        dev = raydir.device
        L.require_gpu(raydir)
        np_ = self.neural_points
        q = np_.querier
        if force_grid:
            q.grid.key = None
        R = raydir.shape[0]
        SR, K = opt.SR, opt.K
        C = self.aggregator.C          # 128 (fork) or 3 (upstream RGB head)
        f32 = dict(dtype=torch.float32, device=dev)
        ray_color = torch.empty((R, C), **f32)
        opacity = torch.empty((R, SR), **f32)
        is_bg = torch.empty((R,), **f32)
        ray_mask = torch.empty((R,), dtype=torch.int8, device=dev)
        bg = bg_color.to(dev).float().reshape(-1).contiguous() if bg_color is not None else None
        if bg is not None and bg.numel() != C:
            bg = bg.expand(C).contiguous() if bg.numel() == 1 else None
            if bg is None:
                raise L.PnrError(f"bg_color must have 1 or {C} channels")
        from .querier import camera_tables
        use_qs = query_stream is not None and capacity is not None
        launch = torch.cuda.current_stream(dev)
        if use_qs:
            # The query's inputs are made on query_stream itself (the caller makes
            # campos / camrot / raydir / ray_cam ready on the launch stream, but the
            # copies below are this call's own).  The points can change on the launch
            # stream (an optimizer step on xyz, a forced rebuild): the query stream
            # then waits for the launch stream before the grid build reads them.
            xkey = (np_.xyz.data_ptr(), np_.xyz._version)
            if force_grid or getattr(state, "q_xkey", None) != xkey:
                query_stream.wait_stream(launch)
            state.q_xkey = xkey
            with torch.cuda.stream(query_stream):
                campos, camrot = camera_tables(campos, camrot, ray_cam)
                if ray_cam is not None:
                    ray_cam = ray_cam.to(device=dev, dtype=torch.int32).contiguous()
                ev_cam = torch.cuda.Event()
                ev_cam.record(query_stream)
            # np_.tables and the aggregate read the camera tables on the launch stream
            # (the query stream's tail is the previous query, which the launch stream
            # already waited for: no overlap is lost)
            launch.wait_event(ev_cam)
            for t in (campos, camrot, ray_cam):
                if t is not None:
                    t.record_stream(launch)
        else:
            campos, camrot = camera_tables(campos, camrot, ray_cam)
            if ray_cam is not None:
                ray_cam = ray_cam.to(device=dev, dtype=torch.int32).contiguous()
        bf16 = precision == "bf16"
        mlp, _keepw = self.aggregator.packed_bf16() if bf16 else self.aggregator.packed()
        mlpx = mlph = _keepx = _keeph = None
        if precision == "fp32x3":
            mlpx, _keepx = self.aggregator.packed_x3()
        elif precision == "fp32h2":
            mlph, _keeph = self.aggregator.packed_h2()
        if keep is not None:   # RenderGraph: the captured launches point into these packs
            keep += [mlp, _keepw, mlpx, _keepx, mlph, _keeph]
        pts, _keepp = np_.tables(campos, camrot, bf16=bf16)
        totals = dict(S_filled=0, S_valid=0, R_hit=0, R_valid=0, n_pairs=0, n_cand=0)
        chunk = max(1, self.chunk_rays or R)
        n_chunks = max(1, -(-R // chunk))
        rec = None
        if capacity is not None:
            host = torch.empty((n_chunks, 8), dtype=torch.int32, pin_memory=True) if record else None
            dcounts = None if record else torch.empty((n_chunks, 8), dtype=torch.int32, device=dev)
            rec = dict(precision=precision, caps=[], host=host, dcounts=dcounts,
                       range_flag=_keeph["range_flag"] if _keeph is not None else None)

        def mark(stream=None):
            if events is None:
                return None
            e = torch.cuda.Event(enable_timing=True)
            e.record(stream)
            return e

        # fp32h2: block1.0's per-point half (P1) depends on the points and weights
        # only, so it runs on a side stream beside the query (which is latency
        # bound and leaves the MFMA pipes idle) instead of in front of k_pairs_h2;
        # the aggregate waits on its event.  Sync-free calls only (their feature
        # buffer, hence the scratch holding P1, is sized before the query), not
        # under graph capture.
        p1_side = None
        # (only while P1 is the smaller job: P1 costs ~0.5 us per point, the query
        # ~3.5 us per ray -- measured 0.99 vs 2.25 ms at 2 M points / 640 k rays; at
        # 10 M points / 1.25 M rays the 5.8 ms P1 outlasted the query and the overlap
        # gained nothing)
        if (precision == "fp32h2" and capacity is not None and keep is None and self.p1_side_stream
                and pts.n <= self.p1_side_max_points_per_ray * R):
            c0 = min(chunk, R)
            Sv0 = min(int(c0 * capacity) + 1024, c0 * SR)
            scr0, ready0 = self._agg_scratch(state, max(Sv0, 1), pts.n, dev, bf16, reuse_p1, precision)
            if not ready0:
                if getattr(state, "side", None) is None:
                    state.side = torch.cuda.Stream(device=dev)
                main = torch.cuda.current_stream(dev)
                ev_in = torch.cuda.Event()
                ev_in.record(main)
                side = state.side
                side.wait_event(ev_in)
                s0 = mark(side)
                L.check(L.lib().pnr_point_pre_h2(L.ctypes.byref(pts), L.ctypes.byref(mlph), L.ptr(scr0),
                                                 scr0.numel() * 4, L.c_void_p(side.cuda_stream)), "pnr_point_pre_h2")
                s1 = mark(side)
                ev_p1 = torch.cuda.Event()
                ev_p1.record(side)
                scr0.record_stream(side)
                p1_side = ev_p1
                if events is not None:
                    events.append(("p1", s0, s1))

        for ci, r0 in enumerate(range(0, R, chunk)):
            r1 = min(R, r0 + chunk)
            if use_qs:   # a non-contiguous raydir's copy belongs to the query stream too
                with torch.cuda.stream(query_stream):
                    rd = raydir[r0:r1].contiguous()
                rd.record_stream(launch)
            else:
                rd = raydir[r0:r1].contiguous()
            rc = None if ray_cam is None else ray_cam[r0:r1]
            slot = None
            if use_qs:
                # the query on its own stream, two buffer sets in turn; each set is
                # reused after the launch-stream work that read it (its event)
                if getattr(state, "qring", None) is None:
                    state.qring, state.qfree, state.qslot = [None, None], [None, None], 1
                slot = state.qslot = state.qslot ^ 1
                if state.qfree[slot] is not None:
                    query_stream.wait_event(state.qfree[slot])
                with torch.cuda.stream(query_stream):
                    e0 = mark()
                    bufs, hp, rays, qp = q.run(np_.xyz.detach(), rd, campos, camrot, near, far,
                                               bufs=state.qring[slot], ray_cam=rc)
                    e1 = mark()
                    ev_q = torch.cuda.Event()
                    ev_q.record(query_stream)
                state.qring[slot] = bufs
                torch.cuda.current_stream(dev).wait_event(ev_q)
            else:
                e0 = mark()
                bufs, hp, rays, qp = q.run(np_.xyz.detach(), rd, campos, camrot, near, far, bufs=state.bufs,
                                           ray_cam=rc)
                e1 = mark()
                state.bufs = bufs
            if capacity is None:
                cnt = bufs.read_counts()
                for k in totals:
                    totals[k] += cnt[k]
                self._observe(cnt, r1 - r0)
                Sv = cnt["S_valid"]
            else:
                Sv = min(int((r1 - r0) * capacity) + 1024, (r1 - r0) * SR)
                rec["caps"].append((Sv, r1 - r0))
            hf = bf16 and C == 128 and self.bf16_features
            feat = state.feat_h_rows(Sv, dev) if hf else state.feat_rows(Sv, dev)
            s = L.Samples(bufs.valid_list.data_ptr(), bufs.counts.data_ptr() + 4, Sv, bufs.pidx.data_ptr(),
                          bufs.sample_w.data_ptr(), bufs.sample_p.data_ptr(), rd.data_ptr(),
                          bufs.fill_rs.data_ptr(), SR, K, L.ptr(rc))
            e2 = mark()
            # bf16 (config c5: 20 M points, a frame references a fraction of them): block1.0's
            # point half only for the points this batch's neighbour lists reference
            # (pnr_used_points, device list and count), written at their own rows of the P1
            # table (pnr_points.used without used_map) -- no indirection in the pairs kernel
            scratch, ready = self._agg_scratch(state, max(Sv, 1), pts.n, dev, bf16, reuse_p1 or r0 > 0, precision)
            # (a reuse_p1 call after a used-only one finds the table partial (key
            # cleared): it computes its own used rows, not the whole table)
            used_only = (bf16 and self.p1_used_only and n_chunks == 1 and keep is None and not ready)
            if used_only:
                pts.used = L.ptr(self._used_points(state, bufs, K, pts.n))
                pts.n_used, pts.used_map = pts.n, None
                pts.n_used_dev = bufs.counts.data_ptr() + 5 * 4
                ready, state.scratch_key = False, None   # the table holds this batch's rows only
            if p1_side is not None:   # P1 written into this same scratch by the side stream
                torch.cuda.current_stream(dev).wait_event(p1_side)
                ready = True
            pts.p1_ready = int(ready)
            if bf16:
                fn = L.lib().pnr_aggregate_fwd_bf16_hf if hf else L.lib().pnr_aggregate_fwd_bf16
                L.check(fn(L.ctypes.byref(pts), L.ctypes.byref(s), L.ctypes.byref(mlp), L.ptr(feat), None, None,
                           L.ptr(scratch), scratch.numel() * 4, L.stream_ptr(dev)),
                        "pnr_aggregate_fwd_bf16")
            elif precision == "fp32x3":
                L.check(L.lib().pnr_aggregate_fwd_x3(L.ctypes.byref(pts), L.ctypes.byref(s), L.ctypes.byref(mlp),
                                                     L.ctypes.byref(mlpx), L.ptr(feat), None, None, L.ptr(scratch),
                                                     scratch.numel() * 4, L.stream_ptr(dev)),
                        "pnr_aggregate_fwd_x3")
            elif precision == "fp32h2":
                L.check(L.lib().pnr_aggregate_fwd_h2(L.ctypes.byref(pts), L.ctypes.byref(s), L.ctypes.byref(mlp),
                                                     L.ctypes.byref(mlph), L.ptr(feat), None, None, L.ptr(scratch),
                                                     scratch.numel() * 4, L.stream_ptr(dev)),
                        "pnr_aggregate_fwd_h2")
            else:
                L.check(L.lib().pnr_aggregate_fwd(L.ctypes.byref(pts), L.ctypes.byref(s), L.ctypes.byref(mlp),
                                                  L.ptr(feat), None, None, L.ptr(scratch), scratch.numel() * 4,
                                                  L.stream_ptr(dev)),
                        "pnr_aggregate_fwd")
            if C == 3:   # upstream colour head: [alpha, rgb] rows
                feat = self.aggregator.apply_rgb_head(feat, n_dev=bufs.counts[1:2], n=Sv)
            e3 = mark()
            cp = L.CompositeParams(float(opt.vsize[2]), int(opt.raydist_mode_unit), C, L.ptr(bg), max(Sv, 1))
            comp = L.lib().pnr_composite_fwd_hf if hf else L.lib().pnr_composite_fwd
            L.check(comp(L.ctypes.byref(rays), L.ctypes.byref(qp), L.ctypes.byref(bufs.c), L.ctypes.byref(cp),
                         L.ptr(feat), L.ptr(ray_color[r0:r1]), L.ptr(opacity[r0:r1]), L.ptr(is_bg[r0:r1]),
                         L.ptr(ray_mask[r0:r1]), L.stream_ptr(dev)),
                    "pnr_composite_fwd")
            if rec is not None:
                if record:
                    rec["host"][ci].copy_(bufs.counts, non_blocking=True)
                else:
                    rec["dcounts"][ci].copy_(bufs.counts)
            if slot is not None:   # the launch stream's last reader of this query-buffer set
                ev_free = torch.cuda.Event()
                ev_free.record(torch.cuda.current_stream(dev))
                state.qfree[slot] = ev_free
            if events is not None:
                e4 = mark()
                events += [("query", e0, e1), ("aggregate", e2, e3), ("composite", e3, e4)]
        if rec is not None:
            if record:
                if rec["range_flag"] is not None:
                    # the fp32h2 range flag as it stands after this call's launches, to
                    # pinned memory behind the call's event: finish() reads it without
                    # a stream sync (which would wait for the calls queued after it)
                    rec["range_host"] = torch.empty(1, dtype=torch.int32, pin_memory=True)
                    rec["range_host"].copy_(rec["range_flag"], non_blocking=True)
                rec["event"] = torch.cuda.Event()
                rec["event"].record()
        else:
            self.last_counts = totals
        return (ray_color, opacity, is_bg, ray_mask), rec

    @staticmethod
    def _used_points(state, bufs, K, n_points):
        """pnr_used_points of a query (count into bufs.counts[5]) on buffers kept in
        the render state: the device list of referenced point rows."""
        dev = bufs.pidx.device
        if getattr(state, "used_n", None) != n_points:
            i32 = dict(dtype=torch.int32, device=dev)
            nb = L.c_size_t(0)
            L.check(L.lib().pnr_used_points_scratch_bytes(n_points, L.ctypes.byref(nb)),
                    "pnr_used_points_scratch_bytes")
            state.used_bufs = tuple(torch.empty(n_points, **i32) for _ in range(3)) + (
                torch.empty(max(int(nb.value), 16), dtype=torch.uint8, device=dev),)
            state.used_n = n_points
        flags, used_map, used, scr = state.used_bufs
        cap = bufs.pidx.numel() // K
        L.check(L.lib().pnr_used_points(L.ptr(bufs.pidx), L.ptr(bufs.counts), K, cap, n_points, L.ptr(flags),
                                        L.ptr(used_map), L.ptr(used), L.c_void_p(bufs.counts.data_ptr() + 20),
                                        L.ptr(scr), scr.numel(), L.stream_ptr(dev)), "pnr_used_points")
        return used

    def _agg_scratch(self, state, n_max, n_points, dev, bf16, reuse, precision="fp32"):
        """Persistent aggregate scratch (P1 lives at its start, see
        pnr_points.p1_ready) -> (tensor, P1 already valid).  The P1 is valid
        when reuse is requested and the embedding storage, block1.0 and the
        precision match the call that wrote it."""
        emb = self.neural_points.points_embeding
        b1 = self.aggregator.block1[0]
        # fp32h2 computes P1 on f16-split MFMA (k_point_pre_h2), the other fp32 paths on fp32 MFMA
        key = (bf16, precision == "fp32h2", n_points, emb.data_ptr(), emb._version, b1.weight.data_ptr(),
               b1.weight._version, b1.bias.data_ptr(), b1.bias._version)
        need = (L.aggregate_scratch_bf16 if bf16 else L.aggregate_scratch)
        nb = L.c_size_t(0)
        fn = L.lib().pnr_aggregate_scratch_bytes_bf16 if bf16 else L.lib().pnr_aggregate_scratch_bytes
        L.check(fn(int(n_max), int(n_points), L.ctypes.byref(nb)), "aggregate scratch bytes")
        buf = state.scratch
        if buf is None or buf.device != dev or buf.numel() * 4 < int(nb.value):
            # headroom (n_max varies per batch) and geometric growth: no allocation per frame
            rows = max(int(n_max * 1.5) + 1024, int(1.5 * getattr(state, "scratch_rows", 0)))
            state.scratch = buf = None
            buf = need(rows, n_points, dev)
            state.scratch_rows = rows
            state.scratch = buf
            state.scratch_key = None
        ready = reuse and state.scratch_key == key
        state.scratch_key = key
        return buf, ready

    @property
    def last_counts(self):
        """Sample counts of the last render call (dict); a training call leaves a
        pending CountsHandle that is read here, when first asked for."""
        c = self._last_counts
        if c is not None and not isinstance(c, dict):
            c = self._last_counts = c.get()
        return c

    @last_counts.setter
    def last_counts(self, v):
        self._last_counts = v

    def render_rays_train(self, campos, camrot, raydir, near, far, bg_color):
        """Differentiable render of one training ray batch [R,3] (SURVEY 8(a)
        a17): same query / aggregate / composite as render_rays, with autograd
        through pnr_aggregate_fwd_train -> pnr_aggregate_bwd_pairs and
        pnr_composite_fwd -> pnr_composite_bwd (train.py).  Returns ray_color
        [R,C] (requires grad w.r.t. points_embeding / color / dir / conf and the
        aggregator parameters), opacity [R,SR], is_bg [R], ray_mask [R]."""
        from .train import AggregateFn, AggSpec, CompositeFn, CompositeSpec, agg_params
        if self.neural_points.points_embeding.dtype != torch.float32:
            raise L.PnrError("training needs an fp32 points_embeding (NeuralPoints(emb_dtype=torch.float32))")
        self._sync_rw2c()
        opt = self.opt
        dev = raydir.device
        L.require_gpu(raydir)
        np_ = self.neural_points
        q = np_.querier
        R = raydir.shape[0]
        SR, K = opt.SR, opt.K
        C = self.aggregator.C
        bg = bg_color.to(dev).float().reshape(-1).contiguous() if bg_color is not None else None
        if bg is not None and bg.numel() == 1:
            bg = bg.expand(C).contiguous()
        campos = campos.reshape(3).float().contiguous()
        camrot = camrot.reshape(3, 3).float().contiguous()
        rd = raydir.float().contiguous()
        xyz = np_.xyz.detach().contiguous()
        bufs, hp, rays, qp = q.run(xyz, rd, campos, camrot, near, far, bufs=None)
        # block1.0's point half only for the points this batch references (device
        # list and count).  No host read here: the kernels take the device counts
        # (samples: counts[1], used points: counts[5]) with capacity-sized
        # buffers, and the counts travel to pinned memory behind an event that the
        # backward (or last_counts) waits on -- the forward never drains the GPU.
        from .train import used_points_device
        used_buf, used_map = used_points_device(bufs, K, xyz.shape[0])
        counts = bufs.read_counts_async()
        self.last_counts = counts
        # saved activations (train.Saved) and the backward's dz rows are sized by the
        # sample capacity: every slot of the batch (R * SR, no host read) while that
        # fits the memory budget, else this batch's valid-sample count (one host read)
        S_cap = R * SR
        if S_cap * TRAIN_BYTES_PER_SAMPLE > self._train_budget(dev):
            S_cap = max(int(bufs.read_counts()["S_valid"]), 1)
            self.train_count_reads += 1
        s = L.Samples(bufs.valid_list.data_ptr(), bufs.counts.data_ptr() + 4, S_cap, bufs.pidx.data_ptr(),
                      bufs.sample_w.data_ptr(), bufs.sample_p.data_ptr(), rd.data_ptr(),
                      bufs.fill_rs.data_ptr(), SR, K)
        n = xyz.shape[0]

        def tab(t, c):
            return None if t is None else t.reshape(n, c)

        used = (used_buf, used_map, bufs.counts[5:6])
        if self.train_precision not in ("fp32", "fp32x3", "fp32h2"):
            raise L.PnrError(f"train_precision {self.train_precision!r}: 'fp32h2', 'fp32x3' or 'fp32'")
        spec = AggSpec(self.aggregator, s, S_cap, dict(xyz=xyz, campos=campos, camrot=camrot, rw2c=np_.rw2c_table()),
                       keep=(bufs, rd),
                       used=used, x3=self.train_precision == "fp32x3", h2=self.train_precision == "fp32h2",
                       counts=counts)
        spec.keep_saved = self.keep_train_saved
        feat = AggregateFn.apply(spec, np_.points_embeding.reshape(n, 32), tab(np_.points_color, 3),
                                 tab(np_.points_dir, 3), tab(np_.points_conf, 1),
                                 np_.xyz if np_.xyz.requires_grad else None, *agg_params(self.aggregator))
        if spec.h2_fallback:
            self.h2_fallbacks += 1
        if C == 3:
            feat = self.aggregator.apply_rgb_head(feat, n_dev=bufs.counts[1:2], n=S_cap)
        cp = L.CompositeParams(float(opt.vsize[2]), int(opt.raydist_mode_unit), C, None)
        cspec = CompositeSpec(rays, qp, bufs, cp, R, SR, C, keep=(campos, camrot, rd, hp), counts=counts)
        # bg: differentiable (the fork optimises bg_color, mvs_points_volumetric_model.py:92-94)
        out = CompositeFn.apply(cspec, feat, bg)
        self._train_conf_src = bufs
        aux = _TrainAux()
        # rows of the point table this batch can give a gradient: the referenced
        # points, and point 0 (empty slots gather it in conf_coefficient) --
        # parallel.GradReducer reduces only these across ranks
        # (unique: pnr_used_points lists each referenced point once, ascending; the
        # appended point 0 is dropped (-1) when it is already referenced).  Read
        # when asked for (the used count is a host value).

        def touched():
            nu = counts.get()["n_used"]
            u = used_buf[:nu].long()
            zero = torch.zeros(1, dtype=torch.long, device=dev)
            if nu:
                zero = torch.where(u[:1] == 0, zero - 1, zero)
            return {"touched_rows": torch.cat([u, zero]), "touched_count": nu + 1}

        aux.lazy(("touched_rows", "touched_count"), touched)
        if self.keep_train_saved:
            aux["saved"] = spec.saved
        if np_.points_conf is not None or self.wants_aux():
            op = out[1]
            aux.lazy(("weight", "blend_weight", "sample_pidx", "conf_coefficient"),
                     lambda: self._march_aux(rays, qp, bufs, R, counts.get()["R_valid"], xyz, op))
        self.last_train_aux = aux
        return out

    def _train_budget(self, dev) -> int:
        """Bytes of per-sample training buffers a sync-free forward may reserve:
        train_memory_budget, or (None) a quarter of the device's memory."""
        if self.train_memory_budget is not None:
            return int(self.train_memory_budget)
        if getattr(self, "_budget_dev", None) is None:
            self._budget_dev = torch.cuda.get_device_properties(dev).total_memory // 4
        return self._budget_dev

    def wants_aux(self) -> bool:
        """The reference aggregator returns weight / conf_coefficient (and the
        module puts them with blend_weight into its output,
        neural_points_volumetric_model.py:335-338) unless no loss reads them
        (point_aggregators.py:814-815)."""
        o = self.opt
        return (getattr(o, "sparse_loss_weight", 0) > 0 or "conf_coefficient" in getattr(o, "zero_one_loss_items", ())
                or getattr(o, "prob", 0) != 0)

    def _march_aux(self, rays, qp, bufs, R, Rv, xyz, opacity):
        """weight [1,R'',SR,K] (detached: the aggregator's normalised weight),
        blend_weight [1,R'',SR,1] (detached), conf_coefficient [1,R'',SR,K]
        (gradiant_clamp of the gathered conf: straight-through gradient to
        points_conf, point_aggregators.py:724-726, 810-813; empty slots gather
        point 0 as torch.clamp(pidx, 0) does; 1 without a conf table) and
        sample_pidx, in pnr_query_compact's row order -- the reference's
        [1, R'', SR, ...] tensors of the same rays."""
        opt, np_ = self.opt, self.neural_points
        SR, K = opt.SR, opt.K
        dev = opacity.device
        f32 = dict(dtype=torch.float32, device=dev)
        pidx = torch.empty((1, Rv, SR, K), dtype=torch.int32, device=dev)
        scratch3 = [torch.empty((1, Rv, SR, 3), **f32) for _ in range(3)]
        rmask = torch.empty((1, R), dtype=torch.int8, device=dev)
        L.check(L.lib().pnr_query_compact(L.ctypes.byref(rays), L.ctypes.byref(qp), L.ctypes.byref(bufs.c), Rv,
                                          L.ptr(pidx), L.ptr(scratch3[0]), L.ptr(scratch3[1]),
                                          L.ptr(scratch3[2]), L.ptr(rmask), L.stream_ptr(dev)),
                "pnr_query_compact")
        weight = torch.empty((1, Rv, SR, K), **f32)
        blend = torch.empty((1, Rv, SR, 1), **f32)
        op = opacity.detach().contiguous()
        L.check(L.lib().pnr_march_aux(L.ctypes.byref(rays), L.ctypes.byref(qp), L.ctypes.byref(bufs.c),
                                      L.ptr(xyz), L.ptr(op), Rv, L.ptr(weight), L.ptr(blend), L.stream_ptr(dev)),
                "pnr_march_aux")
        aux = {"weight": weight, "blend_weight": blend, "sample_pidx": pidx, "conf_coefficient": 1}
        if np_.points_conf is not None:
            cf = np_.points_conf.reshape(-1)[pidx.clamp(min=0).long()]
            aux["conf_coefficient"] = cf - (cf - torch.clamp(cf, 1e-4, 1.0)).detach()
        return aux

    @torch.no_grad()
    def eval_aux(self, campos, camrot, raydir, near, far, opacity):
        """forward()'s weight / blend_weight / conf_coefficient for an
        evaluation render (render_rays keeps no per-pair state): the batch's
        query again, then pnr_query_compact + pnr_march_aux on the rendered
        opacity.  conf_coefficient carries no graph here (no_grad render)."""
        np_ = self.neural_points
        dev = raydir.device
        from .querier import camera_tables
        cp, cr = camera_tables(campos, camrot, None)
        xyz = np_.xyz.detach().contiguous()
        bufs, hp, rays, qp = np_.querier.run(xyz, raydir.float().contiguous(), cp, cr, near, far, bufs=None)
        cnt = bufs.read_counts()
        return self._march_aux(rays, qp, bufs, raydir.shape[0], cnt["R_valid"], xyz, opacity)

    def zero_one_conf_loss(self, zero_epsilon: float = 1e-3):
        """zero_one_loss(conf_coefficient) of the last render_rays_train, computed
        per point: every entry of conf_coefficient is a function of one point's
        conf, so the mean over the [1, R'', SR, K] entries equals
        sum_p count_p f(conf_p) / entries (count_p = entries gathering point p,
        point 0 also collecting the empty slots) -- same value and gradient
        without the gather's scatter-add backward.  The counts come from the
        query's own neighbour lists on the device (the R'' rays' filled samples
        hold every non-negative entry of sample_pidx; the other
        R'' * SR * K - sum_p count_p entries are empty slots, gathered as point 0):
        no host read of R'' and no compaction."""
        bufs = self._train_conf_src
        conf = self.neural_points.points_conf.reshape(-1)
        return _ZeroOneConfLoss.apply(conf, bufs, self.opt.SR, self.opt.K, float(zero_epsilon))

    @staticmethod
    def zero_one_loss(val, zero_epsilon: float = 1e-3):
        """base_rendering_model.py:630-641: mean(log(v) + log(1 - v)), v clamped
        to [eps, 1 - eps]."""
        v = torch.clamp(val, zero_epsilon, 1 - zero_epsilon)
        return torch.mean(torch.log(v) + torch.log(1 - v))

    def forward(self, campos, raydir, gt_image=None, bg_color=None, camrotc2w=None, pixel_idx=None,
                near=None, far=None, focal=None, h=None, w=None, intrinsic=None, **kargs):
        """neural_points_volumetric_model.py:272-352 (+ fill_invalid :354-389);
        B = 1.  With opt.neural_render == "cnn" the fork's 2-D decoder
        (NeuralRenderer, :343-344) adds final_coarse_raycolor (needs h, w)."""
        if raydir.dim() == 3 and raydir.shape[0] != 1:
            raise L.PnrError("batch size B > 1 is not supported (the reference uses B = 1)")
        near_v = float(torch.min(near).item()) if torch.is_tensor(near) else float(near)
        far_v = float(torch.max(far).item()) if torch.is_tensor(far) else float(far)
        if "bg_ray" in kargs:
            bg_color = None
        # training loop (model(...) then loss.backward(), as run/train_ft.py does):
        # differentiable path; evaluation / no_grad: the fused forward
        train = torch.is_grad_enabled() and self.training and (
            any(p.requires_grad for p in self.parameters()) or (torch.is_tensor(bg_color) and bg_color.requires_grad))
        if train:
            color, opacity, is_bg, ray_mask = self.render_rays_train(campos, camrotc2w, raydir.reshape(-1, 3),
                                                                     near_v, far_v, bg_color)
            aux = self.last_train_aux if self.wants_aux() else None
        else:
            color, opacity, is_bg, ray_mask = self.render_rays(campos, camrotc2w, raydir.reshape(-1, 3),
                                                               near_v, far_v, bg_color)
            aux = self.eval_aux(campos, camrotc2w, raydir.reshape(-1, 3), near_v, far_v, opacity) \
                if self.wants_aux() else None
        R = color.shape[0]
        mask_f = ray_mask.float().view(1, R, 1)
        out = dict(coarse_raycolor=color.view(1, R, -1), coarse_point_opacity=opacity.view(1, R, -1),
                   coarse_is_background=is_bg.view(1, R, 1), ray_mask=ray_mask.view(1, R))
        out["coarse_mask"] = 1 - out["coarse_is_background"]
        out["queried_shading"] = (1 - mask_f).repeat(1, 1, 3)
        if aux is not None:   # neural_points_volumetric_model.py:335-338
            out["weight"] = aux["weight"]
            out["blend_weight"] = aux["blend_weight"]
            out["conf_coefficient"] = aux["conf_coefficient"]
        if self.neural_render_2d is not None:
            img_h = int(h.item()) if torch.is_tensor(h) else int(h)
            img_w = int(w.item()) if torch.is_tensor(w) else int(w)
            out["final_coarse_raycolor"] = self.neural_render_2d(
                out["coarse_raycolor"].reshape(1, img_h, img_w, -1)).reshape(1, -1, 3)
        return out


class RenderGraph:
    """One ray batch's full render (query -> aggregate -> composite) captured
    in a HIP graph and replayed without any host work beyond the launch:
    SURVEY 8(f) rank 2 (the reference syncs at qpiw.py:656, 716 and
    neural_points.py:786).  The graph owns its query buffers, aggregate
    scratch and outputs; the camera and ray directions are static input
    tensors that ``replay`` refreshes in place.  Capture requires an already
    built grid and fixed weights (the launches point at the current grid
    tables and weight packs; rebuild the graph after either changes).

    The feature buffer is sized from an eager render of the same batch
    (valid samples x ``margin``); ``check()`` reads the replay's counts and
    the fp32h2 range flag (one host sync) and returns False when the replay
    overflowed that size or an activation left the f16 range -- then render
    that frame with ``render_rays`` instead."""

    def __init__(self, model: NeuralPointsRayMarching, campos, camrot, raydir, near, far, bg_color,
                 margin: float = 1.25):
        L.require_gpu(raydir)
        self.model = model
        dev = raydir.device
        self.campos = campos.reshape(3).float().to(dev).clone()
        self.camrot = camrot.reshape(3, 3).float().to(dev).clone()
        self.raydir = raydir.reshape(-1, 3).float().contiguous().clone()
        self.near, self.far = near, far
        self.bg = None if bg_color is None else bg_color.to(dev).float().reshape(-1).contiguous().clone()
        model._sync_rw2c()
        self.precision = model._precision_now()
        R = self.raydir.shape[0]
        chunk = max(1, model.chunk_rays or R)
        self.state = _RenderState()
        # eager render: builds nothing new (grid must exist), sizes the buffers
        model._render_rays(self.precision, self.campos, self.camrot, self.raydir, near, far, self.bg, False, None,
                           False, self.state)
        self.eager_counts = dict(model.last_counts)
        cap = margin * max(self.eager_counts["S_valid"], 1) / max(min(chunk, R), 1)
        self.keep = []
        stream = torch.cuda.Stream(dev)
        stream.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(stream):   # warm-up on a side stream (allocations, packs)
            model._render_rays(self.precision, self.campos, self.camrot, self.raydir, near, far, self.bg, False,
                               None, False, self.state, capacity=cap, record=False)
        torch.cuda.current_stream(dev).wait_stream(stream)
        torch.cuda.synchronize(dev)
        # Nothing may issue a capture-illegal HIP call (hipFree, an event or stream
        # sync) while the graph records -- from this thread, or from a finaliser
        # the garbage collector runs at some allocation inside the capture (the
        # GPUTEST_r04 failure).  Collect dead cycles now, keep the collector off
        # during the capture, and have GridHandle finalisers defer their frees
        # (querier._DEFERRED); other threads' calls cannot invalidate a
        # thread-local capture.
        from . import querier as Q
        gc.collect()
        Q.release_deferred()
        gc_was_on = gc.isenabled()
        gc.disable()
        Q._CAPTURES[0] += 1
        try:
            self.graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph, capture_error_mode="thread_local"):
                self.out, self.rec = model._render_rays(self.precision, self.campos, self.camrot, self.raydir, near,
                                                        far, self.bg, False, None, False, self.state, capacity=cap,
                                                        keep=self.keep, record=False)
        finally:
            Q._CAPTURES[0] -= 1
            if gc_was_on:
                gc.enable()
        Q.release_deferred()
        self.capacity = cap

    def replay(self, campos=None, camrot=None, raydir=None):
        """Render the batch again (new camera / rays copied into the static
        inputs first); returns (ray_color, opacity, is_bg, ray_mask), tensors the
        graph owns and overwrites on the next replay."""
        if campos is not None:
            self.campos.copy_(campos.reshape(3))
        if camrot is not None:
            self.camrot.copy_(camrot.reshape(3, 3))
        if raydir is not None:
            self.raydir.copy_(raydir.reshape(-1, 3))
        self.graph.replay()
        return self.out

    def check(self) -> bool:
        """True when the last replay's outputs are valid: every chunk's valid
        samples fit the captured feature buffer and (fp32h2) no activation left
        the f16 range.  Synchronises."""
        ok = True
        for (cap, rays), h in zip(self.rec["caps"], self.rec["dcounts"].cpu().tolist()):
            c = _counts_dict(h)
            self.last_counts = c
            ok &= c["S_valid"] <= cap
        if self.precision == "fp32h2" and not self.model.aggregator.h2_range_ok():
            self.model.aggregator.h2_reset_range()
            ok = False
        return ok
