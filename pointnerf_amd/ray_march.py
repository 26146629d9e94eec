"""ray_march drop-in (models/rendering/diff_ray_marching.py:509-555) on libpnr.so.

Supports the render/blend pair the reference configures for every scene
script: ``radiance_render`` (diff_render_func.py:48-50, features[..., 1:])
and ``alpha_blend`` (diff_render_func.py:36-37).

Differentiable like the reference's (it is called inside the training step,
neural_points_volumetric_model.py:314): ``RayMarchFn`` runs the forward on
``pnr_ray_march_fwd`` and the backward on ``pnr_ray_march_bwd_ex`` (gradients of
every output: ray_color, opacity, acc_transmission, blend_weight,
background_transmission) plus ``pnr_weighted_colsum`` for d bg_color, which the
fork optimises (mvs_points_volumetric_model.py:92-94).
"""
from __future__ import annotations

import torch

from . import _lib as L


def radiance_render(ray_feature):
    """diff_render_func.py:48-50 (the fork keeps all C channels)."""
    return ray_feature[..., 1:]


def alpha_blend(opacity, acc_transmission):
    """diff_render_func.py:36-37."""
    return opacity * acc_transmission


def no_tone_map(color, gamma=2.2, exposure=1):
    """diff_render_func.py:61-63."""
    return color


def _march_fwd(rd, rv, rf, bg, NR, SR, C):
    dev = rf.device
    f32 = dict(dtype=torch.float32, device=dev)
    color = torch.empty((NR, C), **f32)
    opacity = torch.empty((NR, SR), **f32)
    acc_T = torch.empty((NR, SR), **f32)
    blend_w = torch.empty((NR, SR), **f32)
    bg_T = torch.empty((NR,), **f32)
    L.check(L.lib().pnr_ray_march_fwd(L.ptr(rd), L.ptr(rv), L.ptr(rf), L.ptr(bg), NR, SR, C,
                                      L.ptr(color), L.ptr(opacity), L.ptr(acc_T), L.ptr(blend_w),
                                      L.ptr(bg_T), L.stream_ptr(dev)), "pnr_ray_march_fwd")
    return color, opacity, acc_T, blend_w, bg_T


class RayMarchFn(torch.autograd.Function):
    """(ray_color [NR,C], opacity, acc_T, blend_w [NR,SR], bg_T [NR]) of the
    flattened inputs; differentiable in ray_dist, the features and bg."""

    @staticmethod
    def forward(ctx, rd, rv, rf, bg):
        NR, SR = rd.shape
        C = rf.shape[-1] - 1
        outs = _march_fwd(rd, rv, rf, bg, NR, SR, C)
        ctx.save_for_backward(rd, rv, rf, bg if bg is not None else torch.empty(0, device=rf.device), outs[4])
        ctx.has_bg = bg is not None
        return outs

    @staticmethod
    def backward(ctx, d_color, d_op, d_accT, d_blend, d_bgT):
        rd, rv, rf, bg, bg_T = ctx.saved_tensors
        bg = bg if ctx.has_bg else None
        NR, SR = rd.shape
        C = rf.shape[-1] - 1
        dev = rf.device
        if d_color is None:
            d_color = torch.zeros((NR, C), dtype=torch.float32, device=dev)

        def c(t):
            return None if t is None else t.float().contiguous()

        d_color, d_op, d_accT, d_blend, d_bgT = map(c, (d_color, d_op, d_accT, d_blend, d_bgT))
        d_feat = torch.empty_like(rf)
        d_dist = torch.empty_like(rd) if ctx.needs_input_grad[0] else None
        L.check(L.lib().pnr_ray_march_bwd_ex(L.ptr(rd), L.ptr(rv), L.ptr(rf), L.ptr(bg), NR, SR, C, L.ptr(d_color),
                                             L.ptr(d_op), L.ptr(d_accT), L.ptr(d_blend), L.ptr(d_bgT),
                                             L.ptr(d_feat), L.ptr(d_dist), L.stream_ptr(dev)), "pnr_ray_march_bwd_ex")
        d_bg = L.weighted_colsum(bg_T, d_color) if (ctx.has_bg and ctx.needs_input_grad[3]) else None
        return d_dist, None, d_feat, d_bg


def ray_march(ray_dist, ray_valid, ray_features, render_func=radiance_render, blend_func=alpha_blend,
              bg_color=None):
    """Returns the reference 7-tuple (ray_color, point_color, opacity,
    acc_transmission, blend_weight, background_transmission,
    background_blend_weight) for inputs [B,R,SR] / [B,R,SR,C+1]; autograd flows
    to ray_features, ray_dist and bg_color as in the reference."""
    if render_func is not radiance_render and getattr(render_func, "__name__", "") != "radiance_render":
        raise L.PnrError("only radiance_render is implemented by libpnr ray_march")
    if blend_func is not alpha_blend and getattr(blend_func, "__name__", "") != "alpha_blend":
        raise L.PnrError("only alpha_blend is implemented by libpnr ray_march")
    L.require_gpu(ray_features)
    B, R, SR = ray_dist.shape
    C = ray_features.shape[-1] - 1
    NR = B * R
    dev = ray_features.device
    rd = ray_dist.reshape(NR, SR).float().contiguous()
    rv = ray_valid.reshape(NR, SR).to(torch.uint8).contiguous()
    rf = ray_features.reshape(NR, SR, C + 1).float().contiguous()
    bg = None
    if bg_color is not None:
        bg = bg_color.to(dev).float().reshape(-1)
        if bg.numel() != C:
            raise L.PnrError(f"bg_color has {bg.numel()} channels, features have {C}")
        bg = bg.contiguous()
    if torch.is_grad_enabled() and (rd.requires_grad or rf.requires_grad or (bg is not None and bg.requires_grad)):
        color, opacity, acc_T, blend_w, bg_T = RayMarchFn.apply(rd, rv, rf, bg)
    else:
        color, opacity, acc_T, blend_w, bg_T = _march_fwd(rd, rv, rf, bg, NR, SR, C)
    bgT = bg_T.view(B, R, 1)
    # background_blend_weight = blend_func(1, background_transmission)
    return (color.view(B, R, C), ray_features[..., 1:], opacity.view(B, R, SR), acc_T.view(B, R, SR),
            blend_w.view(B, R, SR, 1), bgT, bgT)
