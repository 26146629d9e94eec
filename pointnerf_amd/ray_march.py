"""ray_march drop-in (models/rendering/diff_ray_marching.py:509-555) on libpnr.so.

Supports the render/blend pair the reference configures for every scene
script: ``radiance_render`` (diff_render_func.py:48-50, features[..., 1:])
and ``alpha_blend`` (diff_render_func.py:36-37).
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


def ray_march(ray_dist, ray_valid, ray_features, render_func=radiance_render, blend_func=alpha_blend,
              bg_color=None):
    """Returns the reference 7-tuple (ray_color, point_color, opacity,
    acc_transmission, blend_weight, background_transmission,
    background_blend_weight) for inputs [B,R,SR] / [B,R,SR,C+1]."""
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
        bg = bg_color.to(dev).float().reshape(-1).contiguous()
        if bg.numel() != C:
            raise L.PnrError(f"bg_color has {bg.numel()} channels, features have {C}")
    f32 = dict(dtype=torch.float32, device=dev)
    color = torch.empty((NR, C), **f32)
    opacity = torch.empty((NR, SR), **f32)
    acc_T = torch.empty((NR, SR), **f32)
    blend_w = torch.empty((NR, SR), **f32)
    bg_T = torch.empty((NR,), **f32)
    L.check(L.lib().pnr_ray_march_fwd(L.ptr(rd), L.ptr(rv), L.ptr(rf), L.ptr(bg), NR, SR, C,
                                      L.ptr(color), L.ptr(opacity), L.ptr(acc_T), L.ptr(blend_w),
                                      L.ptr(bg_T), L.stream_ptr(dev)), "pnr_ray_march_fwd")
    bgT = bg_T.view(B, R, 1)
    return (color.view(B, R, C), ray_features[..., 1:], opacity.view(B, R, SR), acc_T.view(B, R, SR),
            blend_w.view(B, R, SR, 1), bgT, bgT)
