"""Autograd through the HIP path (the per-scene finetune step).

``AggregateFn`` and ``CompositeFn`` are torch.autograd.Functions whose forward
runs ``pnr_aggregate_fwd_train`` (native-fp32 MFMA) or ``pnr_aggregate_fwd_train_x3``
(the per-pair chain on the fp32x3 split-bf16 MFMA kernel, the training default)
/ ``pnr_composite_fwd`` and whose backward runs

  colour branch backward      weight gradients on pnr_gemm_tn_x3, the dX products
                              (n x 128 x 128, LeakyReLU derivative fused) and block1.0's
                              point-half dX1 = dP1 W1[:, :224] on pnr_gemm_nn
  pnr_aggregate_bwd_pairs     fused per-pair dX chain on MFMA (k_pairs_bwd; with
  (_x3)                       train_precision fp32x3 its three dX GEMMs on split-bf16
                              MFMA, fp32-accurate): alpha
                              branch + K-sum backward, block3.2^T / block3.0^T /
                              block1.2^T, LeakyReLU masks, weight / conf / colour /
                              dir gradients, scatter-add of dz1 into the per-point
                              block1.0 partial (the gather's index_add)
  weight gradients            dW = dZ^T X over all pairs: pnr_gemm_tn_x3 (split-K,
                              fp32-accurate bf16x3 MFMA, deterministic reduction)
  pnr_point_pe3(_bwd)         block1.0's point half: dW1[:, :224] = dP1^T X1,
                              d emb = PE_3 backward of dP1 W1[:, :224]
  pnr_composite_bwd           reverse scans of the alpha composite

matching the autograd of point_aggregators.py:729-816 / 488-646,
gradiant_clamp (:724-726), the gather (neural_points.py:788-799) and
ray_march (diff_ray_marching.py:509-555).  Gradients are produced for
points_embeding, points_color, points_dir, points_conf and every aggregator
parameter; xyz gradients (xyz_grad) through pnr_aggregate_bwd_xyz.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib as L
from .aggregator import frag_pack, frag_pack_x3

# x3 backward: the block3.0 extras' colour / dir gradients per point inside
# pnr_pairs_to_points_ex (True, the product).  False hands them to
# pnr_aggregate_bwd_pairs_x3 (k_extras_bwd) -- DESIGN.md section 10.
X3_POINT_EXTRAS = True
# fp32h2 training: the backward's three dX GEMMs (k_pairs_bwd) on split-f16 MFMA
# as well (False: on fp32x3, the round-5 product) -- DESIGN.md section 10.
BWD_H2 = True
# fp32h2 training with a used-point list (the renderer's training forward): the
# whole backward through the aggregator as one native call
# (pnr_aggregate_bwd_step_h2) instead of the Python sequence below -- the same
# kernels, ~60 fewer host-side calls per step.
NATIVE_BWD = True

_PARAM_NAMES = ("block1.0.weight", "block1.0.bias", "block1.2.weight", "block1.2.bias",
                "block3.0.weight", "block3.0.bias", "block3.2.weight", "block3.2.bias",
                "alpha_branch.0.weight", "alpha_branch.0.bias",
                "color_branch.0.weight", "color_branch.0.bias", "color_branch.2.weight",
                "color_branch.2.bias", "color_branch.4.weight", "color_branch.4.bias")


def agg_params(agg) -> list:
    d = dict(agg.named_parameters())
    return [d[n] for n in _PARAM_NAMES]


BWD_H2_PAD = 3   # k_pairs_bwd<2> loads 3 k-steps ahead (kX3D)


def packed_bwd(agg, x3: bool = False, h2: bool = False):
    """Transposed fragment packs for the backward GEMMs: (pnr_mlp_bwd, None, keep)
    with native-fp32 packs, (pnr_mlp_bwd with w3e only, pnr_mlp_bwd_x3, keep)
    with split-bf16 packs (frag_pack_x3) for pnr_aggregate_bwd_pairs_x3, or (same,
    pnr_mlp_bwd_h2, keep) with the split-f16 packs of pnr_pack_bwd_h2 (one launch,
    shifts picked on the device) for pnr_aggregate_bwd_pairs_h2."""
    with torch.no_grad():
        W3 = agg.block3[0].weight
        t = dict(w3e=W3[:, 256:263].float().contiguous())
        if h2:
            dev = W3.device
            w4, w2 = agg.block3[2].weight.float().contiguous(), agg.block1[2].weight.float().contiguous()
            w3 = W3.float()
            if w3.stride(1) != 1:
                w3 = w3.contiguous()
            per = (16 + BWD_H2_PAD) * 2048
            t["packs"] = torch.empty(3 * per * 2, dtype=torch.int32, device=dev)   # 3 x per x 8 B
            t["scale"] = torch.empty(4, dtype=torch.float32, device=dev)
            L.check(L.lib().pnr_pack_bwd_h2(L.ptr(w4), L.ptr(w3), w3.stride(0), L.ptr(w2), BWD_H2_PAD,
                                            L.ptr(t["scale"]), L.ptr(t["packs"]), t["packs"].numel() * 4,
                                            L.stream_ptr(dev)), "pnr_pack_bwd_h2")
            t.update(w4=w4, w3=w3, w2=w2)
            base = t["packs"].data_ptr()
            m = L.MlpBwd(None, None, None, t["w3e"].data_ptr())
            return m, L.MlpBwdH2(base, base + per * 8, base + 2 * per * 8, t["scale"].data_ptr()), t
        mats = dict(w4t=agg.block3[2].weight.t(), w3t=W3[:, :256].t(), w2t=agg.block1[2].weight.t())
        if x3:
            t.update({k + "x": frag_pack_x3(v) for k, v in mats.items()})
        else:
            t.update({k: frag_pack(v) for k, v in mats.items()})
    if x3:
        m = L.MlpBwd(None, None, None, t["w3e"].data_ptr())
        return m, L.MlpBwdX3(*(t[k].data_ptr() for k in ("w4tx", "w3tx", "w2tx"))), t
    return L.MlpBwd(*(t[k].data_ptr() for k in ("w4t", "w3t", "w2t", "w3e"))), None, t


class Saved:
    """Device activations kept by pnr_aggregate_fwd_train (pnr_agg_saved)."""

    def __init__(self, n_max: int, device, n_dev=None, n_x1: int = 0):
        n = max(int(n_max), 1)
        f = dict(dtype=torch.float32, device=device)
        P = n * 8
        self.t = dict(h1=torch.empty((P, 256), **f), h2=torch.empty((P, 256), **f),
                      h3=torch.empty((P, 256), **f), h4=torch.empty((P, 256), **f),
                      pe5=torch.empty((P, 64), **f), x3e=torch.empty((P, 32), **f), pa=torch.empty(P, **f),
                      wt=torch.empty(P, **f), wn=torch.empty(P, **f),
                      prow=torch.empty(P, dtype=torch.int32, device=device),
                      hid=_rows_zeroed((n, 256), n_dev, device), vpe=torch.empty((n, 24), **f),
                      hc1=torch.empty((n, 128), **f), hc2=torch.empty((n, 128), **f),
                      hc3=torch.empty((n, 128), **f), vmask=torch.empty(n, dtype=torch.int32, device=device),
                      mask=torch.empty((P, 64), dtype=torch.int16, device=device),
                      dz_absmax=torch.zeros(6, dtype=torch.int32, device=device),   # |dz1..dz4|, |dpa|, |d_p1|
                      # [emb, PE_3(emb)] of the used points (fp32h2 forward's k_point_pre_h2; ABI 23)
                      x1=torch.empty((int(n_x1), 224), **f) if n_x1 else None)
        self.c = L.AggSaved(*(L.ptr(self.t[k]) for k, _ in L.AggSaved._fields_))

    def absmax(self, i: int):
        """[1] int32 view: float bits of max |dz_{i+1}| (i < 4), |dpa| (4), |d_p1| (5)."""
        return self.t["dz_absmax"][i:i + 1]

    def __getitem__(self, k):
        return self.t[k]


def _rows_zeroed(shape, n_dev, device):
    """fp32 [rows, cols] whose first *n_dev rows are zero (pnr_zero_rows: the
    device-counted part of a capacity-sized buffer, no host read), or all rows
    zero when n_dev is None / 0.  Rows past the count are never read."""
    if not n_dev:
        return torch.zeros(shape, dtype=torch.float32, device=device)
    t = torch.empty(shape, dtype=torch.float32, device=device)
    L.check(L.lib().pnr_zero_rows(L.ptr(t), t.shape[1] * 4, L.c_void_p(n_dev), t.shape[0], L.stream_ptr(device)),
            "pnr_zero_rows")
    return t


def used_points_device(bufs, K: int, n_points: int):
    """pnr_used_points on a query's buffers, count into bufs.counts[5] (read with
    the other counts by the caller's one read_counts()): (used [N] buffer,
    used_map [N]) -- slice used[:n_used] after the read."""
    dev = bufs.pidx.device
    i32 = dict(dtype=torch.int32, device=dev)
    flags, used_map, used = (torch.empty(n_points, **i32) for _ in range(3))
    nb = L.c_size_t(0)
    L.check(L.lib().pnr_used_points_scratch_bytes(n_points, L.ctypes.byref(nb)), "pnr_used_points_scratch_bytes")
    scratch = torch.empty(max(int(nb.value), 16), dtype=torch.uint8, device=dev)
    cap = bufs.pidx.numel() // K
    L.check(L.lib().pnr_used_points(L.ptr(bufs.pidx), L.ptr(bufs.counts), K, cap, n_points, L.ptr(flags),
                                    L.ptr(used_map), L.ptr(used), L.c_void_p(bufs.counts.data_ptr() + 20),
                                    L.ptr(scratch), scratch.numel(), L.stream_ptr(dev)), "pnr_used_points")
    return used, used_map


def used_points(pidx: torch.Tensor, n_points: int):
    """(used, used_map): sorted point rows referenced by a query's sample_pidx
    and the inverse map (-1 = unreferenced) -- pnr_points.used / used_map."""
    ids = pidx[pidx >= 0]
    used = torch.unique(ids).to(torch.int32)
    used_map = torch.full((n_points,), -1, dtype=torch.int32, device=pidx.device)
    used_map[used.long()] = torch.arange(used.numel(), dtype=torch.int32, device=pidx.device)
    return used, used_map


class AggSpec:
    """Non-tensor description of one aggregate call (structs + keep-alive)."""

    def __init__(self, agg, samples: L.Samples, n: int, pts_extra: dict, pair_mask=None, keep=(), used=None,
                 x3: bool = False, h2: bool = False, counts=None):
        self.agg, self.samples, self.n = agg, samples, int(n)
        self.counts = counts            # querier.CountsHandle: n / used are then capacities, the true
                                        # counts on the device (read by the backward, never the forward)
        self.h2 = bool(h2)              # forward per-pair chain on pnr_aggregate_fwd_train_h2 (fp32h2, f16 MFMA)
        self.x3 = bool(x3) or self.h2   # per-pair chain on pnr_aggregate_fwd_train_x3 (fp32x3 split MFMA);
                                        # the backward's dX chain on fp32x3 with either forward
        self.h2_fallback = False        # an earlier h2 forward's range flag was found raised (that call ran
                                        # its native-fp32 fallback on the device)
        self.used = used                # optional (used[int32], used_map[int32][, n_used device count])
        self.pts_extra = pts_extra      # xyz / pers / campos / camrot pointers (no grad)
        self.pair_mask = pair_mask
        self.keep = keep


class AggregateFn(torch.autograd.Function):
    """feat[n_max, 129] = aggregate(point tables, MLP); differentiable in emb,
    color, dir, conf, the 16 aggregator parameters and -- when xyz is given
    (--xyz_grad 1; the fused renderer path) -- the point positions."""

    @staticmethod
    def forward(ctx, spec: AggSpec, emb, color, dirs, conf, xyz, *params):
        dev = emb.device
        agg = spec.agg
        s = spec.samples
        n_max = int(s.n_max)
        N = emb.shape[0]
        tabs = [emb.detach().contiguous(), None if color is None else color.detach().contiguous(),
                None if dirs is None else dirs.detach().contiguous(),
                None if conf is None else conf.detach().reshape(-1).contiguous()]
        pe = spec.pts_extra
        pts = L.Points(N, pe["xyz"].data_ptr(), L.ptr(pe.get("pers")), tabs[0].data_ptr(), L.ptr(tabs[1]),
                       L.ptr(tabs[2]), L.ptr(tabs[3]), L.ptr(pe.get("campos")), L.ptr(pe.get("camrot")))
        pts.rw2c = L.ptr(pe.get("rw2c"))   # per-point Rw2c [N,9] or None
        n_p1 = N
        if spec.used is not None:
            used, used_map = spec.used[:2]
            pts.used, pts.n_used, pts.used_map = used.data_ptr(), used.numel(), used_map.data_ptr()
            if len(spec.used) > 2:   # device count: used.numel() is the capacity
                pts.n_used_dev = spec.used[2].data_ptr()
            n_p1 = used.numel()
        run_h2 = spec.pair_mask is None and spec.h2
        if run_h2:
            # an earlier step's raised flag (its fallback already ran): shifts re-picked now
            spec.h2_fallback = agg.h2_train_poll()
        # every pack of the step in one launch (the optimizer changed the weights)
        agg.packed_train(h2=run_h2)
        mlp, keepw = agg.packed()
        # fp32h2 with a used-point list: the forward also keeps block1.0's point-half inputs
        sv = Saved(n_max, dev, n_dev=s.n_dev, n_x1=n_p1 if (run_h2 and spec.used is not None) else 0)
        feat = _rows_zeroed((max(n_max, 1), 129), s.n_dev, dev)
        scratch = L.aggregate_scratch(max(n_max, 1), max(n_p1, 1), dev)
        keepx = None
        run_x3 = spec.pair_mask is None and spec.x3
        if run_h2:
            wh, keepx = agg.packed_h2_train()
            L.check(L.lib().pnr_aggregate_fwd_train_h2_guarded(
                ctypes.byref(pts), ctypes.byref(s), ctypes.byref(mlp), ctypes.byref(wh), ctypes.byref(sv.c),
                L.ptr(feat), None, None, L.ptr(scratch), scratch.numel() * 4, L.stream_ptr(dev)),
                "pnr_aggregate_fwd_train_h2_guarded")
            agg.h2_train_launched()
        elif run_x3:
            wx, keepx = agg.packed_x3()
            L.check(L.lib().pnr_aggregate_fwd_train_x3(ctypes.byref(pts), ctypes.byref(s), ctypes.byref(mlp),
                                                       ctypes.byref(wx), ctypes.byref(sv.c), L.ptr(feat), None, None,
                                                       L.ptr(scratch), scratch.numel() * 4, L.stream_ptr(dev)),
                    "pnr_aggregate_fwd_train_x3")
        elif spec.pair_mask is None:
            L.check(L.lib().pnr_aggregate_fwd_train(ctypes.byref(pts), ctypes.byref(s), ctypes.byref(mlp),
                                                    ctypes.byref(sv.c), L.ptr(feat), None, None, L.ptr(scratch),
                                                    scratch.numel() * 4, L.stream_ptr(dev)),
                    "pnr_aggregate_fwd_train")
        else:
            L.check(L.lib().pnr_aggregate_fwd_train_masked(ctypes.byref(pts), ctypes.byref(s), ctypes.byref(mlp),
                                                           L.ptr(spec.pair_mask), ctypes.byref(sv.c), L.ptr(feat),
                                                           None, None, L.ptr(scratch), scratch.numel() * 4,
                                                           L.stream_ptr(dev)),
                    "pnr_aggregate_fwd_train_masked")
        ctx.spec, ctx.sv, ctx.pts, ctx.tabs, ctx.mlp, ctx.keepw = spec, sv, pts, tabs, mlp, (keepw, keepx)
        if getattr(spec, "keep_saved", False):
            spec.saved = sv                 # tests: the kept activations of this forward
        ctx.has = (color is not None, dirs is not None, conf is not None)
        ctx.xyz_shape = None if xyz is None else xyz.shape
        ctx.shapes = (emb.shape, None if conf is None else conf.shape)
        ctx.save_for_backward(*params)
        return feat

    @staticmethod
    def backward(ctx, d_feat):
        spec, sv = ctx.spec, ctx.sv
        agg = spec.agg
        params = ctx.saved_tensors
        P = dict(zip(_PARAM_NAMES, params))
        dev = d_feat.device
        n = spec.n
        used_list = None if spec.used is None else spec.used[0]
        if spec.counts is not None:   # the forward ran on device counts: read them now (no drain)
            cnt = spec.counts.get()
            n = cnt["S_valid"]
            if used_list is not None:
                used_list = used_list[:cnt["n_used"]]
        n_max = n
        N = ctx.tabs[0].shape[0]
        slope = float(agg.neg_slope)
        d_feat = d_feat.contiguous()
        xyz_grad = ctx.xyz_shape is not None and ctx.needs_input_grad[5]
        if (NATIVE_BWD and spec.h2 and BWD_H2 and X3_POINT_EXTRAS and used_list is not None and not xyz_grad
                and spec.pair_mask is None):
            return _native_bwd_h2(ctx, spec, d_feat, n, used_list.numel(), params)
        f32 = dict(dtype=torch.float32, device=dev)
        grads = {}
        # ---- colour branch (color_branch.{0,2,4}: 280 -> 128 -> 128 -> 128, LeakyReLU each)
        hc1, hc2, hc3 = sv["hc1"][:n], sv["hc2"][:n], sv["hc3"][:n]
        # weight gradients dW = dZ^T X on pnr_gemm_tn_x3 (bias = column sums); the
        # dX = dZ W products with the LeakyReLU derivative fused on pnr_gemm_nn.
        # fp32h2: both on the f16-split kernels (pnr_gemm_*_h2), dZ's scale from one
        # pnr_absmax pass per layer (the colour batch is ~30 k rows)
        hg = L.H2Gemm(dev) if spec.h2 else None

        def amax(t):
            return hg.absmax(t) if hg is not None and t.shape[0] > 0 else None

        # dz = lrelu'(hc3) (d_feat[:, 1:] * vmask) and its max |.| in one pass
        dz = torch.empty((n, 128), **f32)
        am = hg.words[1:2] if hg is not None and n > 0 else None
        L.check(L.lib().pnr_color_dz(L.ptr(d_feat), d_feat.stride(0), L.ptr(sv["vmask"]), L.ptr(hc3), hc3.stride(0),
                                     n, 128, slope, L.ptr(dz), L.ptr(am), L.stream_ptr(dev)), "pnr_color_dz")
        grads["color_branch.4.weight"], grads["color_branch.4.bias"] = L.gemm_tn(
            dz, hc2.contiguous(), colsum=True, h2=hg, a_absmax=am)
        dz = L.gemm_nn(dz, P["color_branch.4.weight"], act=hc2, slope=slope, h2=hg, a_absmax=am)
        am = amax(dz)
        grads["color_branch.2.weight"], grads["color_branch.2.bias"] = L.gemm_tn(
            dz, hc1.contiguous(), colsum=True, h2=hg, a_absmax=am)
        dz = L.gemm_nn(dz, P["color_branch.2.weight"], act=hc1, slope=slope, h2=hg, a_absmax=am)
        am = amax(dz)
        gC0 = torch.empty((128, 280), **f32)
        gC0[:, :256], grads["color_branch.0.bias"] = L.gemm_tn(dz, sv["hid"][:n], colsum=True, h2=hg, a_absmax=am)
        vpe32 = torch.zeros((n, 32), **f32)
        vpe32[:, :24] = sv["vpe"][:n]
        gC0[:, 256:] = L.gemm_tn(dz, vpe32, h2=hg, a_absmax=am)[:, :24]
        grads["color_branch.0.weight"] = gC0
        d_hid = torch.empty((max(n_max, 1), 256), **f32)   # rows [0, n) written by the gemm_nn below
        L.gemm_nn(dz, P["color_branch.0.weight"][:, :256], out=d_hid[:n], h2=hg, a_absmax=am)
        # ---- per-pair chain on MFMA
        Pn = max(n_max, 1) * 8
        dz1, dz2, dz3, dz4 = (torch.empty((Pn, 256), **f32) for _ in range(4))
        dpa = torch.empty(Pn, **f32)
        used = used_list
        n_p1 = N if used is None else used.numel()
        # pnr_pairs_to_points writes the row of every point some pair references: every
        # row of a used-point list, only some of the whole table's
        d_p1 = (torch.empty if used is not None else torch.zeros)((max(n_p1, 1), 256), **f32)
        has_c, has_d, has_f = ctx.has
        d_color = torch.zeros((N, 3), **f32) if has_c else None
        d_dir = torch.zeros((N, 3), **f32) if has_d else None
        d_conf = torch.zeros(N, **f32) if has_f else None
        # fp32h2: the dX chain on split-f16 MFMA too (pnr_aggregate_bwd_pairs_h2)
        bwd_h2 = spec.h2 and BWD_H2
        wb, wbx, _keepb = packed_bwd(agg, x3=spec.x3 and not bwd_h2, h2=bwd_h2)
        point_extras = wbx is not None and (has_c or has_d) and X3_POINT_EXTRAS
        if point_extras:
            # the block3.0 extras' colour / dir gradients: per point inside
            # pnr_pairs_to_points_ex below (no float atomics), not in the pairs pass
            w3e_rm = _keepb["w3e"]
            wb.w3e = None
        # d_p1 = NULL: the per-point sums of dz1 come from pnr_pairs_to_points below
        # (pairs sorted by point: no atomics, deterministic) instead of the kernel's atomics
        bufs = (L.ptr(d_feat), L.ptr(d_hid), L.ptr(dz1), L.ptr(dz2), L.ptr(dz3), L.ptr(dz4), L.ptr(dpa),
                None, L.ptr(d_color), L.ptr(d_dir), L.ptr(d_conf), L.stream_ptr(dev))
        if bwd_h2:
            L.check(L.lib().pnr_aggregate_bwd_pairs_h2(ctypes.byref(ctx.pts), ctypes.byref(spec.samples),
                                                       ctypes.byref(ctx.mlp), ctypes.byref(wb), ctypes.byref(wbx),
                                                       ctypes.byref(sv.c), *bufs), "pnr_aggregate_bwd_pairs_h2")
        elif wbx is not None:
            L.check(L.lib().pnr_aggregate_bwd_pairs_x3(ctypes.byref(ctx.pts), ctypes.byref(spec.samples),
                                                       ctypes.byref(ctx.mlp), ctypes.byref(wb), ctypes.byref(wbx),
                                                       ctypes.byref(sv.c), *bufs), "pnr_aggregate_bwd_pairs_x3")
        else:
            L.check(L.lib().pnr_aggregate_bwd_pairs(ctypes.byref(ctx.pts), ctypes.byref(spec.samples),
                                                    ctypes.byref(ctx.mlp), ctypes.byref(wb), ctypes.byref(sv.c),
                                                    *bufs), "pnr_aggregate_bwd_pairs")
        m = n * 8
        # weight gradients on f16 MFMA (pnr_gemm_tn_h2, hg above) with the fp32h2
        # forward; fp32x3 keeps the bf16x3 GEMMs
        used_map = None if spec.used is None else spec.used[1]
        # the pairs grouped by point in pair order (torch.sort(prow, stable=True) natively)
        prow_sorted, pair_of = L.group_pairs(sv["prow"][:m], used_map, n_p1 if used_map is not None else N)
        if point_extras:
            g_pair = torch.empty((max(m, 1), 8), **f32)
            L.check(L.lib().pnr_aggregate_bwd_extras_rows(ctypes.byref(ctx.pts), ctypes.byref(spec.samples),
                                                          ctypes.byref(ctx.mlp), ctypes.byref(sv.c), L.ptr(w3e_rm),
                                                          L.ptr(dz3), L.ptr(g_pair), L.stream_ptr(dev)),
                    "pnr_aggregate_bwd_extras_rows")
            rw_pp = ctx.pts.rw2c or None
            rw_u = ctx.mlp.rw2c or None
            L.check(L.lib().pnr_pairs_to_points_ex(L.ptr(prow_sorted), L.ptr(pair_of), m, L.ptr(dz1), L.ptr(used_map),
                                                   L.ptr(d_p1), L.ptr(sv.absmax(5)), L.ptr(g_pair),
                                                   L.c_void_p(rw_u), L.c_void_p(rw_pp), L.ptr(d_color),
                                                   L.ptr(d_dir), L.stream_ptr(dev)),
                    "pnr_pairs_to_points_ex")
        else:
            L.check(L.lib().pnr_pairs_to_points(L.ptr(prow_sorted), L.ptr(pair_of), m, L.ptr(dz1), L.ptr(used_map),
                                                L.ptr(d_p1), L.ptr(sv.absmax(5)), L.stream_ptr(dev)),
                    "pnr_pairs_to_points")
        dz1, dz2, dz3, dz4, dpa = dz1[:m], dz2[:m], dz3[:m], dz4[:m], dpa[:m]
        h1, h2, h3, h4 = sv["h1"][:m], sv["h2"][:m], sv["h3"][:m], sv["h4"][:m]
        # dW = dZ^T X over all pairs: split-K MFMA GEMM (pnr_gemm_tn), bias = column sums
        # A operands' scales: the maxima k_pairs_bwd / pnr_pairs_to_points wrote (no extra pass)
        amx = sv.absmax
        grads["block3.2.weight"], grads["block3.2.bias"] = L.gemm_tn(dz4, h3, colsum=True, h2=hg, a_absmax=amx(3))
        gW3 = torch.empty((256, 263), **f32)
        gW3[:, :256], grads["block3.0.bias"] = L.gemm_tn(dz3, h2, colsum=True, h2=hg, a_absmax=amx(2))
        gW3[:, 256:] = L.gemm_tn(dz3, sv["x3e"][:m], h2=hg, a_absmax=amx(2))[:, :7]
        grads["block3.0.weight"] = gW3
        grads["block1.2.weight"], grads["block1.2.bias"] = L.gemm_tn(dz2, h1, colsum=True, h2=hg, a_absmax=amx(1))
        dpa32 = torch.zeros((m, 32), **f32)      # M padded to one 32-row MFMA tile
        dpa32[:, 0] = dpa
        grads["alpha_branch.0.weight"] = L.gemm_tn(dpa32, h4, h2=hg, a_absmax=amx(4))[:1]
        grads["alpha_branch.0.bias"] = dpa.sum(0, keepdim=True)
        # ---- block1.0: pair half from dz1 / PE_5, point half from dP1 / X1
        emb = ctx.tabs[0]
        d_p1 = d_p1[:n_p1]
        x1 = torch.empty((max(n_p1, 1), 224), **f32)[:n_p1]
        if sv["x1"] is not None and used is not None:
            x1 = sv["x1"][:n_p1]   # the forward's rows (k_point_pre_h2)
        elif used is None:
            L.check(L.lib().pnr_point_pe3(L.ptr(emb), n_p1, L.ptr(x1), L.stream_ptr(dev)), "pnr_point_pe3")
        else:   # PE_3 of the used rows, read through the list (no gathered copy)
            L.check(L.lib().pnr_point_pe3_rows(L.ptr(emb), L.ptr(used), n_p1, L.ptr(x1), L.stream_ptr(dev)),
                    "pnr_point_pe3_rows")
        gW1 = torch.empty((256, 284), **f32)
        am_p1 = amx(5)
        gW1[:, :224], grads["block1.0.bias"] = L.gemm_tn(d_p1, x1, colsum=True, h2=hg, a_absmax=am_p1)   # sum_p dP1 = sum_pairs dz1
        gW1[:, 224:] = L.gemm_tn(dz1, sv["pe5"][:m], h2=hg, a_absmax=amx(0))[:, :60]
        grads["block1.0.weight"] = gW1
        dx1 = L.gemm_nn(d_p1, P["block1.0.weight"][:, :224], h2=hg, a_absmax=am_p1)
        d_emb = torch.zeros((N, 32), **f32)
        if used is None:
            L.check(L.lib().pnr_point_pe3_bwd(L.ptr(emb), L.ptr(dx1), n_p1, L.ptr(d_emb), L.stream_ptr(dev)),
                    "pnr_point_pe3_bwd")
        else:   # straight into the used rows of the full gradient (no index_copy)
            L.check(L.lib().pnr_point_pe3_bwd_rows(L.ptr(emb), L.ptr(used), L.ptr(dx1), n_p1, L.ptr(d_emb),
                                                   L.stream_ptr(dev)), "pnr_point_pe3_bwd_rows")
        emb_shape, conf_shape = ctx.shapes
        d_xyz = None
        if ctx.xyz_shape is not None and ctx.needs_input_grad[5]:
            # d PE_5 = dz1 . W1[:, 224:284], then the distance / weight / w2pers chain per pair
            w1pe = torch.zeros((256, 64), **f32)          # N padded to the GEMM's 32-column tiles
            w1pe[:, :60] = P["block1.0.weight"][:, 224:284]
            d_pe = L.gemm_nn(dz1, w1pe)
            d_xyz = torch.zeros((N, 3), **f32)
            L.check(L.lib().pnr_aggregate_bwd_xyz(ctypes.byref(ctx.pts), ctypes.byref(spec.samples),
                                                  ctypes.byref(ctx.mlp), ctypes.byref(sv.c), L.ptr(d_feat),
                                                  L.ptr(d_hid), L.ptr(d_pe), L.ptr(d_xyz), L.stream_ptr(dev)),
                    "pnr_aggregate_bwd_xyz")
            d_xyz = d_xyz.view(ctx.xyz_shape)
        out = [None, d_emb.view(emb_shape), d_color, d_dir, None if d_conf is None else d_conf.view(conf_shape), d_xyz]
        out += [grads[k] for k in _PARAM_NAMES]
        return tuple(out)


def _native_bwd_h2(ctx, spec, d_feat, n: int, n_used: int, params) -> tuple:
    """AggregateFn.backward for fp32h2 through pnr_aggregate_bwd_step_h2: every
    gradient in one host call (outputs allocated here, written by the step)."""
    dev = d_feat.device
    N = ctx.tabs[0].shape[0]
    f32 = dict(dtype=torch.float32, device=dev)
    prm, out = L.AggParams(), L.AggGrads()
    grads = []
    for i, p in enumerate(params):
        if p.dtype != torch.float32 or not p.is_contiguous():
            raise L.PnrError(f"native backward: parameter {_PARAM_NAMES[i]} must be contiguous fp32")
        prm.p[i] = p.data_ptr()
        grads.append(torch.empty(p.shape, **f32))
        out.g[i] = grads[-1].data_ptr()
    has_c, has_d, has_f = ctx.has
    d_emb = torch.empty((N, 32), **f32)
    d_color = torch.empty((N, 3), **f32) if has_c else None
    d_dir = torch.empty((N, 3), **f32) if has_d else None
    d_conf = torch.empty(N, **f32) if has_f else None
    out.d_emb, out.d_color, out.d_dir, out.d_conf = (None if t is None else t.data_ptr()
                                                     for t in (d_emb, d_color, d_dir, d_conf))
    nb = L.c_size_t(0)
    L.check(L.lib().pnr_aggregate_bwd_step_h2_scratch_bytes(n, n_used, ctypes.byref(nb)),
            "pnr_aggregate_bwd_step_h2_scratch_bytes")
    scratch = torch.empty(max(int(nb.value), 256), dtype=torch.uint8, device=dev)
    L.check(L.lib().pnr_aggregate_bwd_step_h2(ctypes.byref(ctx.pts), ctypes.byref(spec.samples),
                                              ctypes.byref(ctx.mlp), ctypes.byref(prm), ctypes.byref(ctx.sv.c),
                                              L.ptr(d_feat), n, n_used, ctypes.byref(out), L.ptr(scratch),
                                              scratch.numel(), L.stream_ptr(dev)), "pnr_aggregate_bwd_step_h2")
    emb_shape, conf_shape = ctx.shapes
    return (None, d_emb.view(emb_shape), d_color, d_dir, None if d_conf is None else d_conf.view(conf_shape),
            None, *grads)


class RgbHeadFn(torch.autograd.Function):
    """[n, 4] = [feat[:, 0], raw2out_color(feat[:, 1:] W^T + b)] -- the upstream
    colour head (point_aggregators.py:343, 269-273, 637-638) on pnr_rgb_head_fwd,
    backward on pnr_rgb_head_bwd (d feat, d W, d b)."""

    @staticmethod
    def forward(ctx, feat, weight, bias, act_super, n_dev, n):
        dev = feat.device
        f = feat.detach().contiguous()
        w, b = weight.detach().float().contiguous(), bias.detach().float().contiguous()
        out = torch.zeros((max(f.shape[0], 1), 4), dtype=torch.float32, device=dev)[:f.shape[0]]
        L.check(L.lib().pnr_rgb_head_fwd(L.ptr(f), f.stride(0), L.ptr(n_dev), int(n), L.ptr(w), L.ptr(b),
                                         int(act_super), L.ptr(out), L.stream_ptr(dev)), "pnr_rgb_head_fwd")
        ctx.f, ctx.w, ctx.b, ctx.act, ctx.n_dev, ctx.n = f, w, b, int(act_super), n_dev, int(n)
        return out

    @staticmethod
    def backward(ctx, d_out):
        dev = d_out.device
        d_out = d_out.contiguous()
        d_feat = torch.zeros_like(ctx.f)
        d_wb = torch.empty((3, 129), dtype=torch.float32, device=dev)
        partials = torch.empty((L.HEAD_BWD_BLOCKS, 3, 129), dtype=torch.float32, device=dev)
        L.check(L.lib().pnr_rgb_head_bwd(L.ptr(d_out), L.ptr(ctx.f), ctx.f.stride(0), L.ptr(ctx.n_dev), ctx.n,
                                         L.ptr(ctx.w), L.ptr(ctx.b), ctx.act, L.ptr(d_feat), L.ptr(d_wb),
                                         L.ptr(partials), L.stream_ptr(dev)), "pnr_rgb_head_bwd")
        return d_feat, d_wb[:, :128].contiguous(), d_wb[:, 128].contiguous(), None, None, None


class CompositeSpec:
    def __init__(self, rays, qp, bufs, cp, R, SR, C, keep=(), counts=None):
        self.rays, self.qp, self.bufs, self.cp = rays, qp, bufs, cp
        self.R, self.SR, self.C = R, SR, C
        self.keep = keep
        self.counts = counts   # set: feat is capacity-sized, its rows counted on the device (counts[1])


class CompositeFn(torch.autograd.Function):
    """ray_color[R, C] = composite(feat[S_valid, C+1], bg[C]); opacity / is_bg /
    mask are returned as non-differentiable outputs.  bg (optional) is the
    learned background colour (mvs_points_volumetric_model.py:92-94): its
    gradient is sum_r is_bg[r] d ray_color[r] -- bg_T for a hit ray (the
    ray_march term, diff_ray_marching.py:544-546), 1 for a background ray
    (fill_invalid, neural_points_volumetric_model.py:373-375) -- on
    pnr_weighted_colsum."""

    @staticmethod
    def forward(ctx, spec: CompositeSpec, feat, bg=None):
        dev = feat.device
        f32 = dict(dtype=torch.float32, device=dev)
        R, SR, C = spec.R, spec.SR, spec.C
        ray_color = torch.empty((R, C), **f32)
        opacity = torch.empty((R, SR), **f32)
        is_bg = torch.empty((R,), **f32)
        ray_mask = torch.empty((R,), dtype=torch.int8, device=dev)
        feat_c = feat.detach().contiguous()
        bg_c = None if bg is None else bg.detach().float().reshape(-1).contiguous()
        spec.cp.bg_color = L.ptr(bg_c)
        L.check(L.lib().pnr_composite_fwd(ctypes.byref(spec.rays), ctypes.byref(spec.qp), ctypes.byref(spec.bufs.c),
                                          ctypes.byref(spec.cp), L.ptr(feat_c), L.ptr(ray_color), L.ptr(opacity),
                                          L.ptr(is_bg), L.ptr(ray_mask), L.stream_ptr(dev)),
                "pnr_composite_fwd")
        ctx.spec, ctx.feat, ctx.bg, ctx.is_bg = spec, feat_c, bg_c, is_bg
        ctx.mark_non_differentiable(opacity, is_bg, ray_mask)
        return ray_color, opacity, is_bg, ray_mask

    @staticmethod
    def backward(ctx, d_color, _d_op, _d_bg, _d_mask):
        spec = ctx.spec
        dev = ctx.feat.device
        if spec.counts is not None and ctx.feat.dim() == 2:   # zero only the device-counted rows
            d_feat = _rows_zeroed(tuple(ctx.feat.shape), spec.bufs.counts.data_ptr() + 4, dev)
        else:
            d_feat = torch.zeros_like(ctx.feat)
        if d_color is None:
            return None, d_feat, None
        d_color = d_color.contiguous()
        spec.cp.bg_color = L.ptr(ctx.bg)
        L.check(L.lib().pnr_composite_bwd(ctypes.byref(spec.rays), ctypes.byref(spec.qp), ctypes.byref(spec.bufs.c),
                                          ctypes.byref(spec.cp), L.ptr(ctx.feat), L.ptr(d_color), L.ptr(d_feat),
                                          L.stream_ptr(dev)),
                "pnr_composite_bwd")
        d_bg = None
        if ctx.bg is not None and ctx.needs_input_grad[2]:
            d_bg = L.weighted_colsum(ctx.is_bg, d_color)
        return None, d_feat, d_bg


def ray_march_bwd(ray_dist, ray_valid, feat, bg, d_color):
    """d feat of pnr_ray_march_fwd (dense mirror) for a given d ray_color."""
    NR, SR, CF = feat.shape
    d_feat = torch.zeros_like(feat)
    L.check(L.lib().pnr_ray_march_bwd(L.ptr(ray_dist), L.ptr(ray_valid), L.ptr(feat), L.ptr(bg), NR, SR, CF - 1,
                                      L.ptr(d_color.contiguous()), L.ptr(d_feat), L.stream_ptr(feat.device)),
            "pnr_ray_march_bwd")
    return d_feat
