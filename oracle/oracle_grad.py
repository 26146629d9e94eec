"""TEST INFRASTRUCTURE ONLY -- differentiable CPU restatement for the backward pass.

torch fp32 (CPU) restatement of the reference's forward for the lego
configuration, written so torch autograd yields the reference's gradients:
  * PointAggregator.forward + viewmlp (agg_intrp_order 2), incl. the
    straight-through gradiant_clamp of conf   point_aggregators.py:724-816, 488-646
  * ray_march + radiance_render + alpha_blend diff_ray_marching.py:509-555,
                                              diff_render_func.py:36-63
Pinned by tests/golden/aggregator_bwd.npz and raymarch_bwd.npz (gradients of
the reference's own modules, tests/golden/make_golden.py).  Only tests/ may
import this module: it checks libpnr's HIP backward, it is never the product.
"""
from __future__ import annotations

import torch

F = torch.float32


def positional_encoding(x: torch.Tensor, freqs: int, ori: bool = False) -> torch.Tensor:
    # networks.py:175-190: bands 2^f, no pi; interleaved sin/cos per (channel, band)
    bands = 2.0 ** torch.arange(freqs, dtype=x.dtype)
    pts = (x[..., None] * bands).reshape(x.shape[:-1] + (-1,))
    if ori:
        return torch.cat([x, torch.sin(pts), torch.cos(pts)], -1)
    return torch.stack([torch.sin(pts), torch.cos(pts)], -1).reshape(pts.shape[:-1] + (pts.shape[-1] * 2,))


def gradiant_clamp(conf: torch.Tensor, lo: float = 1e-4, hi: float = 1.0) -> torch.Tensor:
    # point_aggregators.py:724-726: forward clamp, identity gradient
    return conf - (conf - torch.clamp(conf, lo, hi)).detach()


def aggregate(params: dict, sampled_color, sampled_dir, sampled_conf, sampled_embedding, sampled_xyz_pers,
              sampled_xyz, sample_pnt_mask, sample_loc, sample_loc_w, sample_ray_dirs, rw2c=None,
              neg_slope: float = 0.01, act_super: int = 1, C: int = 128):
    """Inputs [R,SR,K,.] (B dropped), params name -> tensor (requires_grad as
    wanted).  Returns features [R,SR,C+1], ray_valid, weight, conf_coefficient.
    Evaluated in the dtype of sampled_embedding (fp32 = the reference; fp64 =
    the high-precision truth the fp32 errors are measured against)."""
    F = sampled_embedding.dtype
    mask = sample_pnt_mask.bool()
    R, SR, K = mask.shape
    ray_valid = mask.any(-1)
    sx, sxp, sl, slw = sampled_xyz, sampled_xyz_pers, sample_loc, sample_loc_w
    xd = sxp[..., 0] * sxp[..., 2] - (sl[..., 0] * sl[..., 2])[..., None]
    yd = sxp[..., 1] * sxp[..., 2] - (sl[..., 1] * sl[..., 2])[..., None]
    zd = sxp[..., 2] - sl[..., None, 2]
    dists = torch.cat([sx - slw[..., None, :], torch.stack([xd, yd, zd], -1)], -1)
    w = mask.to(F) / torch.clamp(torch.linalg.norm(dists[..., :3], dim=-1), min=1e-6)
    w = w / torch.clamp(w.sum(-1, keepdim=True), min=1e-8)
    confc = gradiant_clamp(sampled_conf[..., 0]) if sampled_conf is not None else torch.ones_like(w)
    wt = w * confc
    Rw = torch.eye(3, dtype=F) if rw2c is None else rw2c
    per_pair = Rw.dim() > 2   # [R,SR,K,3,3] gathered per pair (point_aggregators.py:492-496)

    def rot(x, Rm):           # x @ Rm^T per row
        if Rm.dim() == 2:
            return x @ Rm.t()
        return (x[:, None, :] @ Rm.transpose(-1, -2)).squeeze(-2)

    act = lambda x: torch.nn.functional.leaky_relu(x, neg_slope)  # noqa: E731
    lin = lambda x, n: x @ params[n + ".weight"].t() + params[n + ".bias"]  # noqa: E731
    pm = mask.reshape(-1)
    Rpair = Rw.reshape(-1, 3, 3)[pm] if per_pair else Rw
    Rray = Rw[:, :, 0].reshape(-1, 3, 3) if per_pair else Rw   # slot 0's matrix rotates the view dir
    vd = rot(sample_ray_dirs.reshape(-1, 3), Rray)
    vpe = positional_encoding(vd, 4, ori=True)
    ori_v, vpe = vpe[:, :3], vpe[:, 3:]
    vpe = vpe[ray_valid.reshape(-1)]
    d = dists.reshape(-1, 6)[pm]
    d = torch.cat([rot(d[:, :3], Rpair), d[:, 3:]], -1)
    d = positional_encoding(d, 5)
    e = sampled_embedding.reshape(-1, 32)[pm]
    x = torch.cat([e, positional_encoding(e, 3), d], -1)
    x = act(lin(x, "block1.0"))
    x = act(lin(x, "block1.2"))
    col = sampled_color.reshape(-1, 3)[pm]
    sdir = rot(sampled_dir.reshape(-1, 3)[pm], Rpair)
    ov = ori_v[:, None, :].expand(-1, K, -1).reshape(-1, 3)[pm]
    x = torch.cat([x, col, sdir - ov, (sdir * ov).sum(-1, keepdim=True)], -1)
    x = act(lin(x, "block3.0"))
    x = act(lin(x, "block3.2"))
    a = lin(x, "alpha_branch.0")
    a = torch.nn.functional.softplus(a - 1) if act_super else torch.relu(a)
    ah = torch.zeros((R * SR * K, 1), dtype=F).index_put((pm.nonzero()[:, 0],), a)
    wv = wt.reshape(R * SR, K, 1)
    rv = ray_valid.reshape(-1)
    alpha = (ah.view(R * SR, K, 1) * wv).sum(-2)[rv]
    fh = torch.zeros((R * SR * K, x.shape[-1]), dtype=F).index_put((pm.nonzero()[:, 0],), x)
    f = (fh.view(R * SR, K, -1) * wv).sum(-2)[rv]
    c = torch.cat([f, vpe], -1)
    for n in ("color_branch.0", "color_branch.2", "color_branch.4"):
        c = act(lin(c, n))
    if C == 3:   # upstream head: Linear(128, 3) + raw2out_color (point_aggregators.py:343, 269-273)
        c = torch.sigmoid(lin(c, "color_branch.6"))
        if act_super > 0:
            c = c * (1 + 2e-3) - 1e-3
    out = torch.zeros((R * SR, C + 1), dtype=F).index_put((rv.nonzero()[:, 0],), torch.cat([alpha, c], -1))
    return out.view(R, SR, C + 1), ray_valid, w, confc


def ray_march(ray_dist, ray_valid, ray_features, bg_color=None):
    """diff_ray_marching.py:509-555 with radiance_render / alpha_blend; inputs
    [NR,SR], [NR,SR], [NR,SR,C+1]; returns ray_color [NR,C] (+ bg)."""
    sigma = ray_features[..., 0] * ray_valid.to(ray_features.dtype)
    opacity = 1 - torch.exp(-sigma * ray_dist)
    acc = torch.cumprod(1.0 - opacity + 1e-10, dim=-1)
    T = torch.cat([torch.ones_like(acc[..., :1]), acc[..., :-1]], -1)
    bw = opacity * T
    color = (bw[..., None] * ray_features[..., 1:]).sum(-2)
    if bg_color is not None:
        color = color + bg_color[None, :] * acc[..., -1:]
    return color


def ray_march_full(ray_dist, ray_valid, ray_features, bg_color=None):
    """Every differentiable output of diff_ray_marching.py:509-555:
    (ray_color [NR,C], opacity, acc_transmission (exclusive), blend_weight
    [NR,SR], background_transmission [NR,1])."""
    sigma = ray_features[..., 0] * ray_valid.to(ray_features.dtype)
    opacity = 1 - torch.exp(-sigma * ray_dist)
    acc = torch.cumprod(1.0 - opacity + 1e-10, dim=-1)
    bgT = acc[..., -1:]
    T = torch.cat([torch.ones_like(acc[..., :1]), acc[..., :-1]], -1)
    bw = opacity * T
    color = (bw[..., None] * ray_features[..., 1:]).sum(-2)
    if bg_color is not None:
        color = color + bg_color[None, :] * bgT
    return color, opacity, T, bw, bgT
