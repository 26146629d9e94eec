"""Small seeded scenes shared by the parity tests (inputs only)."""
import numpy as np
import torch

from pointnerf_amd import synthetic as S
from pointnerf_amd.options import lego_opt


def scene(n_points=20000, H=64, W=64, theta=30.0, seed=0, default_conf=None, **opt_over):
    opt = lego_opt(**opt_over)
    pts = S.lego_like_points(n_points, seed=seed)
    emb, color, dirs, conf = S.point_features(n_points, seed=seed, default_conf=default_conf)
    campos, camrot = S.camera(theta, -30.0, 4.0)
    focal = S.lego_focal(800) * (H / 800.0)
    raydir = S.pixel_rays(H, W, focal, camrot)
    bg = torch.rand(128, generator=torch.Generator().manual_seed(seed + 1))
    return dict(opt=opt, xyz=pts, emb=emb.numpy(), color=color.numpy(), dir=dirs.numpy(),
                conf=conf.numpy(), campos=campos, camrot=camrot, raydir=raydir, bg=bg.numpy())


def oracle_points(sc):
    return dict(xyz=sc["xyz"], emb=sc["emb"], color=sc["color"], dir=sc["dir"], conf=sc["conf"])


def flag_scene(name, n_points=30000, H=48, W=None, view=1, seed=0, default_conf=None, cap=None, scatter=0.0,
               **opt_over):
    """A seeded scene of one reference flag set (pointnerf_amd.options.FLAGSETS:
    lego / ship / scene101 / truck) at a reduced resolution: the flag set's own
    camera model (synthetic.SCENE_INTRINSICS, focal scaled to W) and views.
    cap / scatter: synthetic.scene_points (cap < 0: an uncapped cloud that may
    overflow max_o / P)."""
    from pointnerf_amd.options import flagset_opt
    opt = flagset_opt(name, **opt_over)
    W0, H0, f0 = S.SCENE_INTRINSICS[name]
    if W is None:
        W = max(1, round(H * W0 / H0))
    if name == "lego":
        pts = S.lego_like_points(n_points, seed=seed)
    else:
        pts = S.scene_points(name, n_points, opt, seed=seed, cap=cap, scatter=scatter)
    if default_conf is None and getattr(opt, "default_conf", -1.0) > 0:
        default_conf = opt.default_conf
    emb, color, dirs, conf = S.point_features(n_points, seed=seed, default_conf=default_conf)
    campos, camrot = S.scene_camera(name, view)
    raydir = S.pixel_rays(H, W, f0 * W / W0, camrot)
    bg = torch.rand(128, generator=torch.Generator().manual_seed(seed + 1))
    return dict(opt=opt, xyz=pts, emb=emb.numpy(), color=color.numpy(), dir=dirs.numpy(),
                conf=conf.numpy(), campos=campos, camrot=camrot, raydir=raydir, bg=bg.numpy(),
                near=float(opt.near_plane), far=float(opt.far_plane), name=name)
