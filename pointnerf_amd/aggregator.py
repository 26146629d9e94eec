"""PointAggregator drop-in on libpnr.so.

Same module tree and ``state_dict`` names as
models/aggregators/point_aggregators.py:12-348 for the lego configuration
(viewmlp, agg_intrp_order 2, linear kernel, agg_dist_pers 20): ``block1.{0,2}``,
``block3.{0,2}``, ``alpha_branch.0``, ``color_branch.{0,2,4}``, so reference
checkpoints load with ``load_state_dict(strict=False)`` as in
mvs_points_volumetric_model.py:320-335.  ``forward`` keeps the 13-argument
signature of point_aggregators.py:729 and runs the fused HIP kernel; the
renderer uses ``packed()`` + ``pnr_aggregate_fwd`` directly on query buffers.
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn as nn

from . import _lib as L

SUPPORTED = dict(which_agg_model="viewmlp", agg_intrp_order=2, agg_distance_kernel="linear",
                 agg_dist_pers=20, point_features_dim=32, num_feat_freqs=3, dist_xyz_freq=5,
                 num_viewdir_freqs=4, shading_feature_num=256, shading_feature_mlp_layer1=2,
                 shading_feature_mlp_layer2=0, shading_feature_mlp_layer3=2,
                 shading_alpha_mlp_layer=1, shading_color_mlp_layer=4,
                 apply_pnt_mask=1, agg_weight_norm=1)
# C_out: 128 = the fork (colour head cut, point_aggregators.py:343, 637-638);
# 3 = upstream (Linear(128, 3) + raw2out_color restored, rgb_head.hip)
COLOR_CHANNELS = (128, 3)


def check_supported(opt):
    bad = {k: (getattr(opt, k, v), v) for k, v in SUPPORTED.items() if getattr(opt, k, v) != v}
    if getattr(opt, "shading_color_channel_num", 128) not in COLOR_CHANNELS:
        bad["shading_color_channel_num"] = (opt.shading_color_channel_num, COLOR_CHANNELS)
    if getattr(opt, "dist_xyz_deno", 0.0) != 0.0:
        bad["dist_xyz_deno"] = (opt.dist_xyz_deno, 0.0)
    for k in ("agg_feat_xyz_mode", "agg_alpha_xyz_mode", "agg_color_xyz_mode"):
        if getattr(opt, k, "None") != "None":
            bad[k] = (getattr(opt, k), "None")
    if bad:
        raise L.PnrError(f"aggregator configuration not implemented by libpnr: {bad}")


def _xavier_(lin: nn.Linear, gain: float):
    # models/helpers/networks.py:71-122: uniform(+-gain*sqrt(2/(in+out))*sqrt(3)), bias 0
    std = gain * math.sqrt(2.0 / (lin.in_features + lin.out_features))
    with torch.no_grad():
        lin.weight.uniform_(-std * math.sqrt(3.0), std * math.sqrt(3.0))
        lin.bias.zero_()


def _init_seq(seq: nn.Sequential):
    # networks.py:163-172 init_seq
    mods = list(seq)
    for a, b in zip(mods[:-1], mods[1:]):
        if isinstance(a, nn.Linear):
            if isinstance(b, nn.LeakyReLU):
                _xavier_(a, nn.init.calculate_gain("leaky_relu", b.negative_slope))
            elif isinstance(b, nn.ReLU):
                _xavier_(a, nn.init.calculate_gain("relu"))
            else:
                _xavier_(a, 1.0)
    if isinstance(mods[-1], nn.Linear):
        _xavier_(mods[-1], 1.0)


PREFETCH_PAD = 8   # kPackPad in aggregate.hip: zero k-steps appended for the weight prefetch


def _pack_device(kind: int, W: torch.Tensor, bias: torch.Tensor | None, pad: int) -> torch.Tensor:
    """pnr_pack_weights: the pack of a CUDA weight (any strides) in one launch."""
    out_f, kin = W.shape
    assert out_f % 32 == 0
    cols = kin + (1 if bias is not None else 0)
    W = W.detach().float()
    b = None if bias is None else bias.detach().float().contiguous()
    if kind == 0:
        n = ((cols + 1) // 2 + pad) * (out_f // 32) * 64
        out = torch.empty(n, dtype=torch.float32, device=W.device)
    else:
        n = ((cols + 15) // 16 + pad) * (out_f // 32) * 64 * 3 * 8
        out = torch.empty(n, dtype=torch.bfloat16, device=W.device)
    L.check(L.lib().pnr_pack_weights(kind, W.data_ptr(), W.stride(0), W.stride(1), out_f, kin, L.ptr(b), pad,
                                     out.data_ptr(), out.numel() * out.element_size(), L.stream_ptr(W.device)),
            "pnr_pack_weights")
    return out


def _pack_h2_device(W: torch.Tensor, bias: torch.Tensor | None, shift: int, flag: torch.Tensor) -> torch.Tensor:
    """pnr_pack_weights_h2: frag_pack_h2(W, bias, shift)[0] of a CUDA weight in one
    launch (no host sync); flag (int32[1], device) raised when the shift is too small."""
    out_f, kin = W.shape
    assert out_f % 32 == 0
    cols = kin + (1 if bias is not None else 0)
    W = W.detach().float()
    b = None if bias is None else bias.detach().float().contiguous()
    n = ((cols + 15) // 16 + H2_PAD) * (out_f // 32) * 64 * 2 * 8
    out = torch.empty(n, dtype=torch.float16, device=W.device)
    L.check(L.lib().pnr_pack_weights_h2(W.data_ptr(), W.stride(0), W.stride(1), out_f, kin, L.ptr(b), H2_PAD,
                                        int(shift), flag.data_ptr(), out.data_ptr(), out.numel() * 2,
                                        L.stream_ptr(W.device)), "pnr_pack_weights_h2")
    return out


def pack_h2_dev(W: torch.Tensor, bias: torch.Tensor | None, scale_out: torch.Tensor) -> torch.Tensor:
    """pnr_pack_weights_h2_dev: frag_pack_h2(W, bias)[0] of a CUDA weight with the
    shift picked on the device (no host sync); scale_out (float32[2], device) gets
    the layer scale 2^(s - 11) in [0] ([1]: scratch)."""
    out_f, kin = W.shape
    assert out_f % 32 == 0 and scale_out.numel() >= 2
    cols = kin + (1 if bias is not None else 0)
    W = W.detach().float()
    b = None if bias is None else bias.detach().float().contiguous()
    n = ((cols + 15) // 16 + H2_PAD) * (out_f // 32) * 64 * 2 * 8
    out = torch.empty(n, dtype=torch.float16, device=W.device)
    L.check(L.lib().pnr_pack_weights_h2_dev(W.data_ptr(), W.stride(0), W.stride(1), out_f, kin, L.ptr(b), H2_PAD,
                                            scale_out.data_ptr(), out.data_ptr(), out.numel() * 2,
                                            L.stream_ptr(W.device)), "pnr_pack_weights_h2_dev")
    return out


def frag_pack(W: torch.Tensor, bias: torch.Tensor | None = None) -> torch.Tensor:
    """[out, Kin] nn.Linear weight (out a multiple of 32) and bias -> MFMA
    A-operand fragments F[t][T][lane] = W'[32T + (lane & 31)][2t + (lane >> 5)]
    of W' = [W | bias | 0]: the bias rides in the GEMM as input column Kin
    (the kernel sets X^T row Kin to 1).  ceil((Kin+1)/2) k-steps plus
    PREFETCH_PAD zero ones.  CUDA weights are packed by pnr_pack_weights (one
    launch); this torch restatement packs host tensors (and is the test's check)."""
    if W.is_cuda:
        return _pack_device(0, W, bias, PREFETCH_PAD)
    out_f, kin = W.shape
    assert out_f % 32 == 0
    cols = kin + (1 if bias is not None else 0)
    nsteps = (cols + 1) // 2
    NT = out_f // 32
    tot = nsteps + PREFETCH_PAD
    Wp = torch.zeros((out_f, 2 * tot), dtype=torch.float32, device=W.device)
    Wp[:, :kin] = W.float()
    if bias is not None:
        Wp[:, kin] = bias.float()
    return Wp.view(NT, 32, tot, 2).permute(2, 0, 3, 1).contiguous().view(-1)


BF16_PAD = 6   # kBPad in aggregate_bf16.hip (mlp_layer_b loads up to 6 k-steps ahead)


def frag_pack_bf16(W: torch.Tensor, bias: torch.Tensor | None = None) -> torch.Tensor:
    """bf16 A-operand fragments of v_mfma_f32_32x32x16_bf16:
    F[t][T][lane][j] = W'[32T + (lane & 31)][16t + 8(lane >> 5) + j] of
    W' = [W | bias | 0], ceil((Kin+1)/16) k-steps plus BF16_PAD zero ones
    (round-to-nearest-even conversion)."""
    out_f, kin = W.shape
    assert out_f % 32 == 0
    cols = kin + (1 if bias is not None else 0)
    tot = (cols + 15) // 16 + BF16_PAD
    NT = out_f // 32
    Wp = torch.zeros((out_f, 16 * tot), dtype=torch.float32, device=W.device)
    Wp[:, :kin] = W.float()
    if bias is not None:
        Wp[:, kin] = bias.float()
    F = Wp.view(NT, 32, tot, 2, 8).permute(2, 0, 3, 1, 4).contiguous()   # [t][T][h][r][j]
    return F.view(-1).to(torch.bfloat16)


X3_PAD = 3   # zero k-steps after each split pack (kWD in aggregate_x3.hip: weights three steps ahead)


def split3_bf16(W: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """fp32 W -> bf16 (W0, W1, W2) with W == W0 + W1 + W2 exactly (each residual
    is exact in fp32; round-to-nearest-even at every step, like v_cvt_pk_bf16_f32)."""
    W = W.float()
    w0 = W.to(torch.bfloat16)
    r = W - w0.float()
    w1 = r.to(torch.bfloat16)
    w2 = (r - w1.float()).to(torch.bfloat16)
    return w0, w1, w2


def frag_pack_x3(W: torch.Tensor, bias: torch.Tensor | None = None) -> torch.Tensor:
    """Split-bf16 A-operand packs for pnr_aggregate_fwd_x3:
    F[t][T][plane][lane][j] = plane of W'[32T + (lane & 31)][16t + 8(lane >> 5) + j],
    W' = [W | bias | 0], ceil((Kin+1)/16) k-steps plus X3_PAD zero ones; planes
    from split3_bf16 (W' == plane0 + plane1 + plane2 exactly).  CUDA weights:
    pnr_pack_weights (bitwise the same planes, one launch)."""
    if W.is_cuda:
        return _pack_device(1, W, bias, X3_PAD)
    out_f, kin = W.shape
    assert out_f % 32 == 0
    cols = kin + (1 if bias is not None else 0)
    tot = (cols + 15) // 16 + X3_PAD
    NT = out_f // 32
    Wp = torch.zeros((out_f, 16 * tot), dtype=torch.float32, device=W.device)
    Wp[:, :kin] = W.float()
    if bias is not None:
        Wp[:, kin] = bias.float()
    Wp = Wp.view(out_f, tot, 2, 8)                                      # k = 16t + 8h + j
    planes = torch.stack(split3_bf16(Wp), 0)                            # [3][out][t][h][j]
    F = planes.view(3, NT, 32, tot, 2, 8).permute(3, 1, 0, 4, 2, 5).contiguous()   # [t][T][pl][h][r][j]
    return F.view(-1)


H2_PAD = 8        # >= the weight ring depth of k_pairs_h2 / k_color_h2 (WRing::kWD)
# fp32h2 training: the colour branch on k_color_h2<true> (f16-split MFMA, k_color<true>'s
# saves) instead of the fp32 training kernel
H2_TRAIN_COLOR = True
H2_WMAX = 16.0    # |W 2^-s| < 16, so 2^11 Wh (made in registers) stays inside f16


def split2_f16(W: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
    """fp32 W -> f16 (Wh, Wl) with W ~= Wh + 2^-11 Wl: Wh = f16(W), Wl =
    f16((W - Wh) 2^11), round-to-nearest-even (as splith in agg_common.h);
    |W - Wh - 2^-11 Wl| <= 2^-24 |W| in the f16 normal range."""
    W = W.float()
    wh = W.to(torch.float16)
    wl = ((W - wh.float()) * 2048.0).to(torch.float16)
    return wh, wl


def h2_shift(W: torch.Tensor, bias: torch.Tensor | None = None) -> int:
    """The s with H2_WMAX / 2 <= max|2^-s [W | bias]| < H2_WMAX (frag_pack_h2), s may be
    negative: a layer of small weights is scaled UP so its high halves stay in the f16
    normal range (2^-14) and the split keeps its 22 significant bits; s = 0 for an
    all-zero layer."""
    amax = float(W.abs().max()) if W.numel() else 0.0
    if bias is not None and bias.numel():
        amax = max(amax, float(bias.abs().max()))
    if not np.isfinite(amax):
        raise L.PnrError("frag_pack_h2: non-finite weight")
    if amax == 0.0:
        return 0
    s = 0
    while amax * 2.0 ** -s >= H2_WMAX:
        s += 1
    while s > -100 and amax * 2.0 ** -(s - 1) < H2_WMAX:
        s -= 1
    return s


def frag_pack_h2(W: torch.Tensor, bias: torch.Tensor | None = None,
                 shift: int | None = None) -> tuple[torch.Tensor, float]:
    """Split-f16 A-operand packs for pnr_aggregate_fwd_h2 -> (pack, layer scale):
    F[t][T][plane][lane][j] = plane of (2^-s W')[32T + (lane & 31)][16t + 8(lane >> 5) + j],
    W' = [W | bias | 0], ceil((Kin+1)/16) k-steps plus H2_PAD zero ones, planes
    (Wh, Wl) of split2_f16; s (h2_shift, may be negative) puts max|2^-s W'| in
    [H2_WMAX/2, H2_WMAX); scale = 2^(s - 11) (the kernel's accumulator factor)."""
    out_f, kin = W.shape
    assert out_f % 32 == 0
    cols = kin + (1 if bias is not None else 0)
    tot = (cols + 15) // 16 + H2_PAD
    NT = out_f // 32
    Wp = torch.zeros((out_f, 16 * tot), dtype=torch.float32, device=W.device)
    Wp[:, :kin] = W.float()
    if bias is not None:
        Wp[:, kin] = bias.float()
    s = h2_shift(Wp) if shift is None else int(shift)   # shift: one scale for the parts of a split layer
    if float(Wp.abs().max()) * 2.0 ** -s >= H2_WMAX:
        raise L.PnrError("frag_pack_h2: shift too small for the weights")
    Wp = (Wp * 2.0 ** -s).view(out_f, tot, 2, 8)                       # k = 16t + 8h + j
    planes = torch.stack(split2_f16(Wp), 0)                             # [2][out][t][h][j]
    F = planes.view(2, NT, 32, tot, 2, 8).permute(3, 1, 0, 4, 2, 5).contiguous()   # [t][T][pl][h][r][j]
    return F.view(-1), 2.0 ** (s - 11)


def frag_unpack(F: torch.Tensor, kin: int, out_f: int = 256) -> torch.Tensor:
    NT = out_f // 32
    tot = F.numel() // (NT * 64)
    return F.view(tot, NT, 2, 32).permute(1, 3, 0, 2).reshape(out_f, 2 * tot)[:, :kin]


class PointAggregator(nn.Module):
    """point_aggregators.PointAggregator (viewmlp, order 2) on libpnr.so."""

    def __init__(self, opt):
        super().__init__()
        check_supported(opt)
        self.opt = opt
        act = opt.act_type
        if act == "LeakyReLU":
            mk, self.neg_slope = (lambda: nn.LeakyReLU(inplace=True)), 0.01
        elif act == "ReLU":
            mk, self.neg_slope = (lambda: nn.ReLU(inplace=True)), 0.0
        else:
            raise L.PnrError(f"act_type {act} not implemented by libpnr")
        self.act_super = int(getattr(opt, "act_super", 1))
        # shapes of point_aggregators.py:276-348 for the lego flag set
        self.block1 = nn.Sequential(nn.Linear(284, 256), mk(), nn.Linear(256, 256), mk())
        self.block3 = nn.Sequential(nn.Linear(263, 256), mk(), nn.Linear(256, 256), mk())
        self.alpha_branch = nn.Sequential(nn.Linear(256, 1))
        self.C = int(getattr(opt, "shading_color_channel_num", 128))
        cb = [nn.Linear(280, 128), mk(), nn.Linear(128, 128), mk(), nn.Linear(128, 128), mk()]
        if self.C == 3:   # upstream colour head (point_aggregators.py:343): color_branch.6
            cb.append(nn.Linear(128, 3))
        self.color_branch = nn.Sequential(*cb)
        for s in (self.block1, self.block3, self.alpha_branch, self.color_branch):
            _init_seq(s)
        self._packed = None
        self._packed_key = None
        self.register_buffer("rw2c", torch.eye(3), persistent=False)
        # bf16 path: samples bucketed by filled neighbour slots (KT = 1/2/4/8 tiles; same
        # outputs as 16 x 8 tiles, fewer empty MFMA columns on sparse scenes)
        self.pair_buckets = True

    # ---------------------------------------------------------------- weights
    def _fp32_key(self):
        return tuple((p.data_ptr(), p._version) for p in self.parameters()) + (
            (self.rw2c.data_ptr(), self.rw2c._version),)

    def _fp32_specs(self) -> list:
        """(name, W, bias) of the native-fp32 packs of packed()."""
        b1, b3, cb = self.block1, self.block3, self.color_branch
        return [("w1af", b1[0].weight[:, :224], b1[0].bias), ("w1bf", b1[0].weight[:, 224:], None),
                ("w2f", b1[2].weight, b1[2].bias), ("w3f", b3[0].weight, b3[0].bias),
                ("w4f", b3[2].weight, b3[2].bias), ("wc1f", cb[0].weight, cb[0].bias),
                ("wc2f", cb[2].weight, cb[2].bias), ("wc3f", cb[4].weight, cb[4].bias)]

    def _set_packed(self, t: dict, key):
        b1, b3, cb = self.block1, self.block3, self.color_branch
        t.update(b2=b1[2].bias.float().contiguous(), b3=b3[0].bias.float().contiguous(),
                 b4=b3[2].bias.float().contiguous(), wa=self.alpha_branch[0].weight.float().reshape(-1).contiguous(),
                 ba=self.alpha_branch[0].bias.float().contiguous(), bc1=cb[0].bias.float().contiguous(),
                 bc2=cb[2].bias.float().contiguous(), bc3=cb[4].bias.float().contiguous(),
                 rw2c=self.rw2c.float().contiguous())
        m = L.Mlp()
        for k, v in t.items():
            setattr(m, k, v.data_ptr())
        m.neg_slope = float(self.neg_slope)
        m.act_super = self.act_super
        self._packed, self._packed_key = (m, t), key
        return self._packed

    def packed(self) -> tuple[L.Mlp, dict]:
        """Fragment-packed weights on the module's device, rebuilt only when a
        parameter changed (version counters)."""
        key = self._fp32_key()
        if self._packed is not None and key == self._packed_key:
            return self._packed
        with torch.no_grad():
            t = {k: frag_pack(W, b) for k, W, b in self._fp32_specs()}
            return self._set_packed(t, key)

    def packed_train(self, h2: bool) -> None:
        """The training forward's packs -- packed() and, for fp32h2,
        packed_h2_train() -- rebuilt in ONE pnr_pack_batch launch when the weights
        changed (every step: the optimizer moved them); bitwise the packs of the
        per-matrix calls.  Afterwards packed() / packed_h2_train() return them
        from their caches."""
        dev = self.block1[0].weight.device
        if dev.type != "cuda":
            return
        kf = self._fp32_key()
        need_f = self._packed is None or kf != self._packed_key
        kh = self.h2_key()
        need_h = h2 and (getattr(self, "_packedh2t", None) is None or kh != self._packedh2t_key)
        if not (need_f or need_h):
            return
        jobs, keep, outs_f, outs_h = [], [], {}, []
        with torch.no_grad():
            if need_f:
                for name, W, b in self._fp32_specs():
                    out_f, kin = W.shape
                    n = ((kin + (b is not None) + 1) // 2 + PREFETCH_PAD) * (out_f // 32) * 64
                    outs_f[name] = torch.empty(n, dtype=torch.float32, device=dev)
                    jobs.append((0, W, b, PREFETCH_PAD, 0, None, outs_f[name]))
            if need_h:
                mats = self._h2t_mats()
                flag = self._h2t_prepare(mats)
                for (W, b), sft in zip(mats, self._h2t_shifts):
                    out_f, kin = W.shape
                    n = ((kin + (b is not None) + 15) // 16 + H2_PAD) * (out_f // 32) * 64 * 2 * 8
                    outs_h.append(torch.empty(n, dtype=torch.float16, device=dev))
                    jobs.append((2, W, b, H2_PAD, sft, flag, outs_h[-1]))
            arr = (L.PackJob * len(jobs))()
            for q, (kind, W, b, pad, sft, flag, out) in enumerate(jobs):
                W = W.detach().float()
                b = None if b is None else b.detach().float().contiguous()
                keep += [W, b]
                arr[q] = L.PackJob(kind, W.data_ptr(), W.stride(0), W.stride(1), W.shape[0], W.shape[1], L.ptr(b),
                                   pad, sft, L.ptr(flag), out.data_ptr(), out.numel() * out.element_size())
            L.check(L.lib().pnr_pack_batch(arr, len(jobs), L.stream_ptr(dev)), "pnr_pack_batch")
            if need_f:
                self._set_packed(outs_f, kf)
            if need_h:
                self._set_packedh2t(outs_h, kh)

    def packed_bf16(self) -> tuple[L.MlpBf16, dict]:
        """bf16 fragment packs for pnr_aggregate_fwd_bf16 (cached like packed())."""
        ps = list(self.parameters())
        key = tuple((p.data_ptr(), p._version) for p in ps) + ((self.rw2c.data_ptr(), self.rw2c._version),
                                                                bool(self.pair_buckets))
        if getattr(self, "_packed16", None) is not None and key == self._packed16_key:
            return self._packed16
        with torch.no_grad():
            b1, b3, cb = self.block1, self.block3, self.color_branch
            t = dict(w1af=frag_pack_bf16(b1[0].weight[:, :224], b1[0].bias),
                     w1bf=frag_pack_bf16(b1[0].weight[:, 224:]),
                     w2f=frag_pack_bf16(b1[2].weight, b1[2].bias), w3f=frag_pack_bf16(b3[0].weight, b3[0].bias),
                     w4f=frag_pack_bf16(b3[2].weight, b3[2].bias),
                     wa=self.alpha_branch[0].weight.float().reshape(-1).contiguous(),
                     ba=self.alpha_branch[0].bias.float().contiguous(),
                     wc1f=frag_pack_bf16(cb[0].weight, cb[0].bias), wc2f=frag_pack_bf16(cb[2].weight, cb[2].bias),
                     wc3f=frag_pack_bf16(cb[4].weight, cb[4].bias), rw2c=self.rw2c.float().contiguous())
        m = L.MlpBf16()
        for k, v in t.items():
            setattr(m, k, v.data_ptr())
        m.neg_slope = float(self.neg_slope)
        m.act_super = self.act_super
        m.pair_buckets = int(self.pair_buckets)
        self._packed16, self._packed16_key = (m, t), key
        return self._packed16

    def packed_x3(self) -> tuple[L.MlpX3, dict]:
        """Split-bf16 packs of block1.0[:, 224:], block1.2, block3.0, block3.2
        for pnr_aggregate_fwd_x3 (used with packed(); cached like it)."""
        ps = list(self.parameters())
        key = tuple((p.data_ptr(), p._version) for p in ps)
        if getattr(self, "_packedx3", None) is not None and key == self._packedx3_key:
            return self._packedx3
        with torch.no_grad():
            b1, b3 = self.block1, self.block3
            t = dict(w1bx=frag_pack_x3(b1[0].weight[:, 224:]), w2x=frag_pack_x3(b1[2].weight, b1[2].bias),
                     w3x=frag_pack_x3(b3[0].weight, b3[0].bias), w4x=frag_pack_x3(b3[2].weight, b3[2].bias))
        m = L.MlpX3(*(t[k].data_ptr() for k in ("w1bx", "w2x", "w3x", "w4x")))
        self._packedx3, self._packedx3_key = (m, t), key
        return self._packedx3

    def packed_h2(self) -> tuple[L.MlpH2, dict]:
        """Split-f16 packs of block1.0[:, 224:], block1.2, block3.0, block3.2
        for pnr_aggregate_fwd_h2 (used with packed(); cached like it).  The
        dict holds the device range flag (`range_flag`, int32[1])."""
        key = self.h2_key()
        if getattr(self, "_packedh2", None) is not None and key == self._packedh2_key:
            return self._packedh2
        with torch.no_grad():
            b1, b3, cb = self.block1, self.block3, self.color_branch
            # block1.2 / block3.2 without the bias column: k_pairs_h2 starts their
            # accumulators at bias / scale (pnr_mlp b2 / b4)
            packs = [frag_pack_h2(b1[0].weight[:, 224:]), frag_pack_h2(b1[2].weight),
                     frag_pack_h2(b3[0].weight, b3[0].bias), frag_pack_h2(b3[2].weight)]
            # colour layer 1 in two 144-row halves sharing one scale (k_color_h2)
            s1 = h2_shift(cb[0].weight, cb[0].bias)
            cpacks = [frag_pack_h2(cb[0].weight[:, :144], shift=s1),
                      frag_pack_h2(cb[0].weight[:, 144:], cb[0].bias, shift=s1),
                      frag_pack_h2(cb[2].weight, cb[2].bias), frag_pack_h2(cb[4].weight, cb[4].bias)]
            # block1.0's per-point half (k_point_pre_h2)
            p1pack = frag_pack_h2(b1[0].weight[:, :224], b1[0].bias)
        flag = torch.zeros(1, dtype=torch.int32, device=b1[0].weight.device)
        t = dict(w1bh=packs[0][0], w2h=packs[1][0], w3h=packs[2][0], w4h=packs[3][0], range_flag=flag,
                 wc1a=cpacks[0][0], wc1b=cpacks[1][0], wc2h=cpacks[2][0], wc3h=cpacks[3][0], w1ah=p1pack[0])
        m = L.MlpH2(*(t[k].data_ptr() for k in ("w1bh", "w2h", "w3h", "w4h")),
                    (L.c_float * 4)(*(p[1] for p in packs)), flag.data_ptr(),
                    *(t[k].data_ptr() for k in ("wc1a", "wc1b", "wc2h", "wc3h")),
                    (L.c_float * 3)(cpacks[1][1], cpacks[2][1], cpacks[3][1]),
                    t["w1ah"].data_ptr(), p1pack[1])
        self._packedh2, self._packedh2_key = (m, t), key
        return self._packedh2

    def packed_h2_train(self) -> tuple[L.MlpH2, dict]:
        """fp32h2 packs of the per-pair chain (block1.0[:, 224:], block1.2,
        block3.0, block3.2) and of block1.0's point half (P1 on k_point_pre_h2)
        for pnr_aggregate_fwd_train_h2, packed on the device
        (pnr_pack_weights_h2: no host sync while the weights change every step)
        with shifts kept from the last h2_shift pick; `range_flag` is raised by
        the pack when a weight outgrew its shift and by the forward when an
        activation left the f16 range -- the guarded forward then runs its
        fp32 fallback on the device, and h2_train_poll() re-picks the shifts."""
        key = self.h2_key()
        if getattr(self, "_packedh2t", None) is not None and key == self._packedh2t_key:
            return self._packedh2t
        mats = self._h2t_mats()
        flag = self._h2t_prepare(mats)
        packs = [_pack_h2_device(W, b, s, flag) for (W, b), s in zip(mats, self._h2t_shifts)]
        return self._set_packedh2t(packs, key)

    def _h2t_mats(self) -> list:
        b1, b3, cb = self.block1, self.block3, self.color_branch
        mats = [(b1[0].weight[:, 224:], None), (b1[2].weight, None), (b3[0].weight, b3[0].bias), (b3[2].weight, None),
                (b1[0].weight[:, :224], b1[0].bias)]   # then: block1.0's point half (k_point_pre_h2)
        if H2_TRAIN_COLOR:   # the colour branch (k_color_h2<true>): layer 1 in two halves of one shift
            mats += [(cb[0].weight[:, :144], None), (cb[0].weight[:, 144:], cb[0].bias), (cb[2].weight, cb[2].bias),
                     (cb[4].weight, cb[4].bias)]
        return mats

    def _h2t_prepare(self, mats) -> torch.Tensor:
        """The training packs' shifts (picked on the host once, kept until a raised
        range flag) and their device flag."""
        if getattr(self, "_h2t_shifts", None) is None or len(self._h2t_shifts) != len(mats):
            with torch.no_grad():
                self._h2t_shifts = [h2_shift(W, b) for W, b in mats[:5]]
                if len(mats) > 5:
                    cb = self.color_branch
                    s1 = h2_shift(cb[0].weight, cb[0].bias)   # one scale for both halves of layer 1
                    self._h2t_shifts += [s1, s1] + [h2_shift(W, b) for W, b in mats[7:]]
            self._h2t_flag = torch.zeros(1, dtype=torch.int32, device=self.block1[0].weight.device)
        return self._h2t_flag

    def _set_packedh2t(self, packs: list, key):
        flag = self._h2t_flag
        t = dict(w1bh=packs[0], w2h=packs[1], w3h=packs[2], w4h=packs[3], w1ah=packs[4], range_flag=flag)
        sc = [2.0 ** (s - 11) for s in self._h2t_shifts]
        if len(packs) > 5:
            t.update(wc1a=packs[5], wc1b=packs[6], wc2h=packs[7], wc3h=packs[8])
            cp, cs = [t[k].data_ptr() for k in ("wc1a", "wc1b", "wc2h", "wc3h")], (sc[6], sc[7], sc[8])
        else:
            cp, cs = [None] * 4, (0.0, 0.0, 0.0)
        m = L.MlpH2(*(t[k].data_ptr() for k in ("w1bh", "w2h", "w3h", "w4h")),
                    (L.c_float * 4)(*sc[:4]), flag.data_ptr(), *cp, (L.c_float * 3)(*cs), t["w1ah"].data_ptr(), sc[4])
        self._packedh2t, self._packedh2t_key = (m, t), key
        return self._packedh2t

    def h2_train_reset(self):
        """After a raised training range flag: shifts re-picked at the next pack."""
        self._h2t_shifts = None
        self._packedh2t = None

    def h2_train_launched(self):
        """After a pnr_aggregate_fwd_train_h2_guarded launch: its range flag is
        copied to pinned host memory behind an event, read by a later
        h2_train_poll() -- the step itself never waits for it (the guarded
        forward already ran its fp32 fallback on the device when the flag was up)."""
        if getattr(self, "_h2t_host", None) is None:
            self._h2t_host = torch.zeros(1, dtype=torch.int32, pin_memory=True)
        self._h2t_host.copy_(self._h2t_flag, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self._h2t_pending = ev

    def h2_train_poll(self, wait: bool = False) -> bool:
        """True once per raised flag of an earlier guarded forward (that step ran
        on the fp32 fallback): the shifts are then re-picked at the next pack.
        Does not block unless `wait`."""
        ev = getattr(self, "_h2t_pending", None)
        if ev is None or not (wait or ev.query()):
            return False
        ev.synchronize()
        self._h2t_pending = None
        if int(self._h2t_host[0]) == 0:
            return False
        self.h2_train_reset()
        return True

    def h2_key(self):
        """Identity of the current weights (storage + version of every
        parameter), the key packed_h2() caches on."""
        return tuple((p.data_ptr(), p._version) for p in self.parameters())

    def h2_reset_range(self):
        """Clear the h2 range flag (after the caller has acted on it)."""
        pk = getattr(self, "_packedh2", None)
        if pk is not None:
            pk[1]["range_flag"].zero_()

    def h2_range_ok(self) -> bool:
        """False when a pnr_aggregate_fwd_h2 launch since the packs were built
        saw an activation outside the f16 range (its outputs are invalid).
        Reads a device flag (synchronises)."""
        pk = getattr(self, "_packedh2", None)
        return pk is None or int(pk[1]["range_flag"].item()) == 0

    def rgb_head(self):
        """(W [3,128], b [3]) of the upstream colour head color_branch.6 (C_out = 3)."""
        lin = self.color_branch[6]
        return lin.weight.detach().float().contiguous(), lin.bias.detach().float().contiguous()

    def apply_rgb_head(self, feat: torch.Tensor, n_dev=None, n: int | None = None) -> torch.Tensor:
        """[n, 129] decoded features -> [n, 4] = [alpha, raw2out_color(color_branch.6(f))]
        on pnr_rgb_head_fwd (point_aggregators.py:343, 269-273, 637-638), or
        through RgbHeadFn when gradients are wanted."""
        n = feat.shape[0] if n is None else int(n)
        if torch.is_grad_enabled() and (feat.requires_grad or self.color_branch[6].weight.requires_grad):
            from .train import RgbHeadFn
            lin = self.color_branch[6]
            return RgbHeadFn.apply(feat, lin.weight, lin.bias, self.act_super, n_dev, n)
        w, b = self.rgb_head()
        out = torch.empty((max(n, 1), 4), dtype=torch.float32, device=feat.device)[:n]
        L.check(L.lib().pnr_rgb_head_fwd(L.ptr(feat), feat.stride(0), L.ptr(n_dev), n, L.ptr(w), L.ptr(b),
                                         self.act_super, L.ptr(out), L.stream_ptr(feat.device)),
                "pnr_rgb_head_fwd")
        return out

    def set_rw2c(self, rw2c: torch.Tensor | None):
        """Uniform Rw2c of the point cloud (neural_points.py:289; eye by default)."""
        with torch.no_grad():
            self.rw2c.copy_(torch.eye(3) if rw2c is None else rw2c.reshape(3, 3))

    # ---------------------------------------------------------------- forward
    def forward(self, sampled_color, sampled_Rw2c, sampled_dir, sampled_conf, sampled_embedding,
                sampled_xyz_pers, sampled_xyz, sample_pnt_mask, sample_loc, sample_loc_w,
                sample_ray_dirs, vsize, grid_vox_sz):
        """point_aggregators.py:729-816 -> (features [B,R,SR,C+1], ray_valid
        [B,R,SR], weight, conf_coefficient)."""
        L.require_gpu(sample_loc_w)
        B, R, SR, K = sample_pnt_mask.shape
        # uniform [3,3] or gathered per pair [B,R,SR,K,3,3] (neural_points.py:799): the
        # per-pair table is pnr_points.rw2c of the pair-table launch
        rw_pairs = None
        if sampled_Rw2c is not None and sampled_Rw2c.dim() != 2:
            rw_pairs = sampled_Rw2c.detach().reshape(B * R * SR * K, 9).float().contiguous()
            self.set_rw2c(None)
        elif sampled_Rw2c is not None:
            self.set_rw2c(sampled_Rw2c.to(self.rw2c.device))
        rows = B * R * SR
        dev = sample_loc_w.device
        C = 128   # the decoded features; the upstream head (C_out = 3) is applied at the end
        ray_valid = torch.any(sample_pnt_mask, dim=-1)
        weight = torch.empty((rows, K), dtype=torch.float32, device=dev)
        conf = torch.empty((rows, K), dtype=torch.float32, device=dev)
        if rows == 0:
            out = torch.zeros((rows, self.C + 1), dtype=torch.float32, device=dev)
            return out.view(B, R, SR, self.C + 1), ray_valid, weight.view(B, R, SR, K), conf.view(B, R, SR, K)

        def flat(t, c):
            return None if t is None else t.reshape(-1, c).float().contiguous()

        keep = dict(xyz=flat(sampled_xyz, 3), pers=flat(sampled_xyz_pers, 3),
                    sw=flat(sample_loc_w, 3), sp=flat(sample_loc, 3), sd=flat(sample_ray_dirs, 3),
                    mask=sample_pnt_mask.reshape(-1).contiguous().view(torch.uint8))
        s = L.Samples(None, None, rows, None, keep["sw"].data_ptr(), keep["sp"].data_ptr(),
                      keep["sd"].data_ptr(), None, 1, K)
        diff = [t for t in (sampled_embedding, sampled_color, sampled_dir, sampled_conf) if t is not None]
        if torch.is_grad_enabled() and (any(t.requires_grad for t in diff) or
                                        any(p.requires_grad for p in self.parameters())):
            # training path: autograd through pnr_aggregate_fwd_train / _bwd_pairs (train.py)
            from .train import AggSpec, AggregateFn, agg_params
            spec = AggSpec(self, s, rows, dict(xyz=keep["xyz"], pers=keep["pers"], rw2c=rw_pairs),
                           pair_mask=keep["mask"], keep=(keep, rw_pairs))
            out = AggregateFn.apply(spec, sampled_embedding.reshape(-1, 32).float(),
                                    None if sampled_color is None else sampled_color.reshape(-1, 3).float(),
                                    None if sampled_dir is None else sampled_dir.reshape(-1, 3).float(),
                                    None if sampled_conf is None else sampled_conf.reshape(-1, 1).float(),
                                    None, *agg_params(self))
            out = out[:rows]
        else:
            out = torch.zeros((rows, C + 1), dtype=torch.float32, device=dev)
            keep.update(emb=flat(sampled_embedding, 32), color=flat(sampled_color, 3), dir=flat(sampled_dir, 3),
                        conf=flat(sampled_conf, 1))
            pts = L.Points(rows * K, keep["xyz"].data_ptr(), keep["pers"].data_ptr(), keep["emb"].data_ptr(),
                           L.ptr(keep["color"]), L.ptr(keep["dir"]), L.ptr(keep["conf"]), None, None)
            pts.rw2c = L.ptr(rw_pairs)
            mlp, _ = self.packed()
            scratch = L.aggregate_scratch(rows, rows * K, dev)
            L.check(L.lib().pnr_aggregate_fwd_masked(L.ctypes.byref(pts), L.ctypes.byref(s),
                                                     L.ctypes.byref(mlp), L.ptr(keep["mask"]), L.ptr(out),
                                                     L.ptr(weight), L.ptr(conf), L.ptr(scratch),
                                                     scratch.numel() * 4, L.stream_ptr(dev)),
                    "pnr_aggregate_fwd_masked")
        if out.requires_grad:
            # weight / conf_coefficient as the reference returns them (conf with the
            # straight-through clamp gradient, point_aggregators.py:724-726, 803-804)
            with torch.no_grad():
                m = sample_pnt_mask.reshape(rows, K).float()
                xyz3 = keep["xyz"].view(rows, K, 3) - keep["sw"].view(rows, 1, 3)
                w = m / torch.clamp(torch.linalg.norm(xyz3, dim=-1), min=1e-6)
                weight = w / torch.clamp(w.sum(-1, keepdim=True), min=1e-8)
            if sampled_conf is not None:
                cf = sampled_conf.reshape(rows, K).float()
                conf = cf - (cf - torch.clamp(cf, 1e-4, 1.0)).detach()
            else:
                conf = torch.ones((rows, K), dtype=torch.float32, device=dev)
        weight, conf = weight.view(B, R, SR, K), conf.view(B, R, SR, K)
        if self.C == 3:
            out = self.apply_rgb_head(out)
            out = out * ray_valid.reshape(-1, 1).to(out.dtype)   # output_placeholder zeros (:643-645)
        o = self.opt
        if (getattr(o, "sparse_loss_weight", 0) <= 0 and "conf_coefficient" not in getattr(o, "zero_one_loss_items", [])
                and getattr(o, "prob", 0) == 0):
            weight, conf = None, None
        return out.view(B, R, SR, self.C + 1), ray_valid, weight, conf
