"""The fork's 2-D neural renderer on libpnr.

``NeuralRenderer`` keeps the module tree and parameter names of
models/neural_render/neural_renderer.py:7-104 for the configuration the fork
builds, ``NeuralRenderer(input_dim=128)`` (neural_points_volumetric_model.py:258-260):
n_feat 128 (conv_in = identity), img_size 64 -> 2 blocks, rgb skips, no norm,
LeakyReLU(0.2), final sigmoid -- so ``neural_render_2d.*`` checkpoint keys load.
Forward runs ``pnr_neural_render_fwd_h2`` (``precision="fp32h2"``, the
default): three fused implicit-GEMM 3x3 convolutions on f16 MFMA with the
fp32h2 operand split (fp32 accuracy), or ``pnr_neural_render_fwd``
(``precision="fp32"``) on fp32 MFMA.  With autograd enabled ``NeuralRenderFn`` keeps the
forward's activations and its backward runs ``pnr_neural_render_bwd`` (data
gradients as flipped-weight convolutions on the same kernel, weight gradients
as implicit-GEMM reductions over the pixels, deterministic), the gradients of
the reference's torch autograd through neural_renderer.py:81-104.
(The torch-convolution restatement the tests check against is tests/nr_ref.py.)
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn

from . import _lib as L
from .aggregator import frag_pack, pack_h2_dev


class NeuralRenderer(nn.Module):
    def __init__(self, n_feat=128, input_dim=128, out_dim=3, final_actvn=True, min_feat=32, img_size=64,
                 use_rgb_skip=True, upsample_feat="nn", upsample_rgb="bilinear", use_norm=False):
        super().__init__()
        n_blocks = int(math.log2(img_size) - 4)
        if (n_feat, input_dim, out_dim, n_blocks, use_rgb_skip, use_norm, final_actvn) != (128, 128, 3, 2, True,
                                                                                            False, True):
            raise L.PnrError("libpnr implements NeuralRenderer(input_dim=128) as built by the fork only")
        self.final_actvn = final_actvn
        self.conv_layers = nn.ModuleList([nn.Conv2d(128, 64, 3, 1, 1), nn.Conv2d(64, 32, 3, 1, 1)])
        self.conv_rgb = nn.ModuleList([nn.Conv2d(128, 3, 3, 1, 1), nn.Conv2d(64, 3, 3, 1, 1),
                                       nn.Conv2d(32, 3, 3, 1, 1)])
        self._packed = None
        self._packed_key = None
        self.precision = "fp32h2"      # or "fp32": the convolutions on fp32 MFMA

    @staticmethod
    def _trunk(conv):
        """[cout, cin, 3, 3] trunk weights -> fragment-packed rows (k = (ky*3 + kx)*cin + ci), bias."""
        W = conv.weight.float()
        return frag_pack(W.permute(0, 2, 3, 1).reshape(W.shape[0], -1).contiguous()), conv.bias.float().contiguous()

    @staticmethod
    def _rgb(conv):
        """[3, cin, 3, 3] rgb weights -> row-major [3, 9 * cin] (same k order), bias [3]."""
        W = conv.weight.float()
        return W.permute(0, 2, 3, 1).reshape(3, -1).contiguous(), conv.bias.float().contiguous()

    def packed(self):
        ps = list(self.parameters())
        key = tuple((p.data_ptr(), p._version) for p in ps)
        if self._packed is not None and key == self._packed_key:
            return self._packed
        with torch.no_grad():
            wf0, b0 = self._trunk(self.conv_layers[0])
            wf1, b1 = self._trunk(self.conv_layers[1])
            r = [self._rgb(cv) for cv in self.conv_rgb]
        t = dict(wf0=wf0, b0=b0, wf1=wf1, b1=b1, wrgb0=r[0][0], brgb0=r[0][1], wrgb1=r[1][0], brgb1=r[1][1],
                 wrgb2=r[2][0], brgb2=r[2][1])
        w = L.NeuralRenderW(*(t[k].data_ptr() for k, _ in L.NeuralRenderW._fields_[:-1]), 0.2)
        self._packed, self._packed_key = (w, t), key
        return self._packed

    @staticmethod
    def _stack(trunk, rgb, rows):
        """A stage's stacked [trunk; rgb; 0] conv weights [rows, cin, 3, 3] and biases [rows]."""
        convs = ([trunk] if trunk is not None else []) + [rgb]
        W = torch.cat([cv.weight for cv in convs], 0).float()
        b = torch.cat([cv.bias for cv in convs], 0).float()
        Wp = torch.zeros((rows,) + tuple(W.shape[1:]), dtype=torch.float32, device=W.device)
        bp = torch.zeros(rows, dtype=torch.float32, device=W.device)
        Wp[: W.shape[0]] = W
        bp[: b.shape[0]] = b
        return Wp, bp

    @classmethod
    def _stack_t(cls, trunk, rgb, rows):
        """Data-gradient weights of a stage: the stacked [rows, cin, 3, 3] weights
        flipped and transposed to [cin, 9 * rows] (k = (ky'*3 + kx') * rows + j,
        value W[j, ci, 2 - ky', 2 - kx']) (pnr_neural_render_wt before packing)."""
        Wp, _ = cls._stack(trunk, rgb, rows)
        cin = Wp.shape[1]
        return Wp.flip(2, 3).permute(1, 2, 3, 0).reshape(cin, 9 * rows).contiguous()

    def _stages(self):
        return ((self.conv_layers[0], self.conv_rgb[0], 96), (self.conv_layers[1], self.conv_rgb[1], 64),
                (None, self.conv_rgb[2], 32))

    def _key(self, tag):
        return (tag,) + tuple((p.data_ptr(), p._version) for p in self.parameters())

    def packed_t(self):
        key = self._key("t")
        if getattr(self, "_packed_t", None) is not None and self._packed_t_key == key:
            return self._packed_t
        with torch.no_grad():
            t = {f"wt{i}": frag_pack(self._stack_t(*st)) for i, st in enumerate(self._stages())}
        self._packed_t = L.NeuralRenderWT(t["wt0"].data_ptr(), t["wt1"].data_ptr(), t["wt2"].data_ptr(), 0.2), t
        self._packed_t_key = key
        return self._packed_t

    def packed_h2(self):
        """fp32h2 forward packs: per stage the stacked rows (k = (ky*3 + kx)*cin + ci)
        packed on the device with a device-picked shift (pnr_pack_weights_h2_dev:
        no host sync, so a training step repacks freely), the scales in one
        device array, and the stacked biases."""
        key = self._key("h2")
        if self._packed is not None and key == self._packed_key:
            return self._packed
        dev = self.conv_rgb[0].weight.device
        t = {"ws": torch.zeros(6, dtype=torch.float32, device=dev)}
        with torch.no_grad():
            for i, st in enumerate(self._stages()):
                Wp, bp = self._stack(*st)
                t[f"wp{i}"] = pack_h2_dev(Wp.permute(0, 2, 3, 1).reshape(Wp.shape[0], -1).contiguous(), None,
                                          t["ws"][2 * i:2 * i + 2])
                t[f"b{i}"] = bp.contiguous()
        w = L.NeuralRenderH2W(t["wp0"].data_ptr(), t["wp1"].data_ptr(), t["wp2"].data_ptr(), t["ws"].data_ptr(),
                              t["b0"].data_ptr(), t["b1"].data_ptr(), t["b2"].data_ptr(), 0.2)
        self._packed, self._packed_key = (w, t), key
        return self._packed

    def packed_t_h2(self):
        key = self._key("th2")
        if getattr(self, "_packed_t", None) is not None and self._packed_t_key == key:
            return self._packed_t
        dev = self.conv_rgb[0].weight.device
        t = {"ws": torch.zeros(6, dtype=torch.float32, device=dev)}
        with torch.no_grad():
            for i, st in enumerate(self._stages()):
                t[f"wt{i}"] = pack_h2_dev(self._stack_t(*st), None, t["ws"][2 * i:2 * i + 2])
        self._packed_t = L.NeuralRenderH2WT(t["wt0"].data_ptr(), t["wt1"].data_ptr(), t["wt2"].data_ptr(),
                                            t["ws"].data_ptr(), 0.2), t
        self._packed_t_key = key
        return self._packed_t

    def _fwd(self, x):
        """pnr_neural_render_fwd -> (rgb [H*W, 3], x [H*W, 128], forward scratch)."""
        L.require_gpu(x)
        B, H, W, C = x.shape
        if B != 1 or C != 128:
            raise L.PnrError("NeuralRenderer expects [1, H, W, 128]")
        xc = x.reshape(H * W, 128).float().contiguous()
        out = torch.empty((H * W, 3), dtype=torch.float32, device=x.device)
        h2 = self.precision == "fp32h2"
        sfx = "_h2" if h2 else ""
        nb = L.c_size_t(0)
        L.check(getattr(L.lib(), f"pnr_neural_render{sfx}_scratch_bytes")(H, W, L.ctypes.byref(nb)),
                "pnr_neural_render_scratch_bytes")
        scratch = torch.empty(max(int(nb.value) // 4, 4), dtype=torch.float32, device=x.device)
        w, _keep = self.packed_h2() if h2 else self.packed()
        L.check(getattr(L.lib(), f"pnr_neural_render_fwd{sfx}")(
            L.ptr(xc), H, W, L.ctypes.byref(w), L.ptr(out), L.ptr(scratch), scratch.numel() * 4,
            L.stream_ptr(x.device)), "pnr_neural_render_fwd")
        return out, xc, scratch

    def forward(self, x):
        """x [1, H, W, 128] -> rgb [1, H, W, 3]."""
        if torch.is_grad_enabled() and (x.requires_grad or any(p.requires_grad for p in self.parameters())):
            return NeuralRenderFn.apply(x, self, *self.parameters())
        out, _, _ = self._fwd(x)
        return out.view(1, *x.shape[1:3], 3)


class NeuralRenderFn(torch.autograd.Function):
    """Autograd of NeuralRenderer on libpnr: forward pnr_neural_render_fwd (its
    net0 / net1 kept), backward pnr_neural_render_bwd -> d x and the gradients of
    conv_layers.{0,1} / conv_rgb.{0,1,2} weight and bias (parameters() order)."""

    @staticmethod
    def forward(ctx, x, mod, *params):
        out, xc, scratch = mod._fwd(x.detach())
        ctx.mod, ctx.shape, ctx.h2 = mod, x.shape, mod.precision == "fp32h2"
        ctx.save_for_backward(xc, scratch, out)
        return out.view(1, *x.shape[1:3], 3)

    @staticmethod
    def backward(ctx, d_out):
        xc, fscr, out = ctx.saved_tensors
        mod = ctx.mod
        _, H, W, _ = ctx.shape
        dev = xc.device
        f32 = dict(dtype=torch.float32, device=dev)
        d_out = d_out.reshape(H * W, 3).float().contiguous()
        wt, _keep = mod.packed_t_h2() if ctx.h2 else mod.packed_t()
        sfx = "_h2" if ctx.h2 else ""
        nb = L.c_size_t(0)
        L.check(getattr(L.lib(), f"pnr_neural_render_bwd{sfx}_scratch_bytes")(H, W, L.ctypes.byref(nb)),
                "pnr_neural_render_bwd_scratch_bytes")
        scratch = torch.empty(max(int(nb.value) // 4, 4), **f32)
        d_x = torch.empty((H * W, 128), **f32)
        dws = [torch.empty(M * 9 * cin + M, **f32) for M, cin in ((96, 128), (64, 64), (32, 32))]
        L.check(getattr(L.lib(), f"pnr_neural_render_bwd{sfx}")(L.ptr(xc), L.ptr(fscr), L.ptr(out), L.ptr(d_out), H, W,
                                              L.ctypes.byref(wt), L.ptr(d_x), *(L.ptr(d) for d in dws),
                                              L.ptr(scratch), scratch.numel() * 4, L.stream_ptr(dev)),
                "pnr_neural_render_bwd")

        def split(dw, M, cin, cout):
            w = dw[: M * 9 * cin].view(M, 3, 3, cin).permute(0, 3, 1, 2)
            b = dw[M * 9 * cin:]
            return (w[:cout], b[:cout]), (w[cout:cout + 3], b[cout:cout + 3])

        (gw0, gb0), (gr0, grb0) = split(dws[0], 96, 128, 64)
        (gw1, gb1), (gr1, grb1) = split(dws[1], 64, 64, 32)
        _, (gr2, grb2) = split(dws[2], 32, 32, 0)
        grads = {"conv_layers.0.weight": gw0, "conv_layers.0.bias": gb0, "conv_layers.1.weight": gw1,
                 "conv_layers.1.bias": gb1, "conv_rgb.0.weight": gr0, "conv_rgb.0.bias": grb0,
                 "conv_rgb.1.weight": gr1, "conv_rgb.1.bias": grb1, "conv_rgb.2.weight": gr2,
                 "conv_rgb.2.bias": grb2}
        pg = [grads[n].contiguous() for n, _ in mod.named_parameters()]
        return (d_x.view(ctx.shape), None, *pg)
