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
