"""Reference checkpoints and point-cloud edits.

``{epoch}_net_ray_marching.pth`` holds the state_dict of the reference's
NeuralPointsRayMarching (base_model.py:99-116 save_networks): the point table
under ``neural_points.*`` (neural_points.py:241-326: xyz [N,3],
points_embeding [1,N,32], points_conf [1,N,1], points_dir [1,N,3],
points_color [1,N,3], optional Rw2c / eulers) and the aggregator under
``aggregator.*`` (point_aggregators.py:276-348).  ``pointnerf_amd`` uses the same
module tree and parameter names, so the reference files load here and files
saved here load in the reference.  Loading never unpickles code:
``torch.load(..., weights_only=True)``.

``prune`` / ``grow_points`` mirror neural_points.py:350-401; the persistent
voxel grid is keyed on the xyz tensor (storage, version, shape), so the next
query rebuilds it after either edit -- the reference instead rebuilds it for
every 2304-ray chunk.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import _lib as L
from .aggregator import PointAggregator
from .renderer import NeuralPoints, NeuralPointsRayMarching

_POINT_KEYS = ("xyz", "points_embeding", "points_conf", "points_dir", "points_color")


def load_ray_marching(path: str, opt, device, epoch_is_best: bool = False) -> NeuralPointsRayMarching:
    """Build NeuralPointsRayMarching from a reference ``*_net_ray_marching.pth``.

    Mirrors mvs_points_volumetric_model.py:320-335: aggregator weights load with
    strict=False; for the "best" epoch with 0 < default_conf <= 1 the file has no
    points_conf and it is filled with default_conf."""
    sd = torch.load(path, map_location="cpu", weights_only=True)
    if not isinstance(sd, dict):
        raise L.PnrError(f"{path}: expected a state_dict, got {type(sd).__name__}")
    np_sd = {k[len("neural_points."):]: v for k, v in sd.items() if k.startswith("neural_points.")}
    if "xyz" not in np_sd or "points_embeding" not in np_sd:
        raise L.PnrError(f"{path}: no neural_points.xyz / neural_points.points_embeding")
    xyz = np_sd["xyz"].float().reshape(-1, 3)
    n = xyz.shape[0]
    conf = np_sd.get("points_conf")
    dc = float(getattr(opt, "default_conf", -1.0))
    if conf is None and epoch_is_best and 0.0 < dc <= 1.0:
        conf = torch.full((1, n, 1), dc)
    rw = np_sd.get("Rw2c")   # [3,3] uniform or [N,3,3] per point (neural_points.py:289, 799)
    points = NeuralPoints(opt, device, xyz, np_sd["points_embeding"], np_sd.get("points_color"),
                          np_sd.get("points_dir"), conf, Rw2c=rw)
    agg = PointAggregator(opt).to(device)
    agg_sd = {k[len("aggregator."):]: v for k, v in sd.items() if k.startswith("aggregator.")}
    missing, unexpected = agg.load_state_dict(agg_sd, strict=False)
    model = NeuralPointsRayMarching(opt, points, agg)
    model.load_report = dict(missing=list(missing), unexpected=list(unexpected))
    if rw is not None and rw.dim() == 2:
        agg.set_rw2c(rw)
    return model


def save_ray_marching(model: NeuralPointsRayMarching, path: str):
    """save_networks (base_model.py:99-116): the module's state_dict, CPU tensors."""
    sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    np_ = model.neural_points
    if np_.Rw2c is not None and (np_.Rw2c.dim() != 2 or not torch.equal(np_.Rw2c.cpu(), torch.eye(3))):
        sd["neural_points.Rw2c"] = np_.Rw2c.detach().cpu()
    torch.save(sd, path)


def _param(t, grad_flag):
    p = nn.Parameter(t.contiguous())
    p.requires_grad = bool(grad_flag)
    return p


def prune(points: NeuralPoints, thresh: float):
    """neural_points.py:350-373: keep points with conf >= thresh (a per-point
    Rw2c is kept for the surviving points, :370-372; xyz stays trainable with
    --xyz_grad 1, :353)."""
    if points.points_conf is None:
        raise L.PnrError("prune needs points_conf")
    o = points.opt
    mask = points.points_conf.detach()[0, :, 0] >= thresh
    with torch.no_grad():
        points.xyz = _param(points.xyz[mask, :], getattr(o, "xyz_grad", 0) > 0)
        points.points_embeding = _param(points.points_embeding[:, mask, :], getattr(o, "feat_grad", 1) > 0)
        points.points_conf = _param(points.points_conf[:, mask, :], getattr(o, "conf_grad", 1) > 0)
        if points.points_dir is not None:
            points.points_dir = _param(points.points_dir[:, mask, :], getattr(o, "dir_grad", 1) > 0)
        if points.points_color is not None:
            points.points_color = _param(points.points_color[:, mask, :], getattr(o, "color_grad", 1) > 0)
        if points.Rw2c is not None and points.Rw2c.dim() > 2:
            points.Rw2c = points.Rw2c[mask].contiguous()
    return int((~mask).sum())


def grow_points(points: NeuralPoints, add_xyz, add_embedding, add_color=None, add_dir=None, add_conf=None,
                add_Rw2c=None):
    """neural_points.py:376-401: append points (add_* are [M, C]; add_Rw2c
    [M,3,3] when the cloud carries a per-point Rw2c, :400-402)."""
    o = points.opt
    dev = points.xyz.device
    with torch.no_grad():
        points.xyz = _param(torch.cat([points.xyz, add_xyz.to(dev).float()], 0), getattr(o, "xyz_grad", 0) > 0)
        # keep the table's dtype (a bf16 table stays bf16: torch.cat would promote it)
        emb_t = points.points_embeding.dtype
        points.points_embeding = _param(torch.cat([points.points_embeding, add_embedding.to(dev).to(emb_t)[None]], 1),
                                        getattr(o, "feat_grad", 1) > 0)
        if points.points_conf is not None:
            points.points_conf = _param(torch.cat([points.points_conf, add_conf.to(dev).float()[None]], 1),
                                        getattr(o, "conf_grad", 1) > 0)
        if points.points_dir is not None:
            points.points_dir = _param(torch.cat([points.points_dir, add_dir.to(dev).float()[None]], 1),
                                       getattr(o, "dir_grad", 1) > 0)
        if points.points_color is not None:
            points.points_color = _param(torch.cat([points.points_color, add_color.to(dev).float()[None]], 1),
                                         getattr(o, "color_grad", 1) > 0)
        if points.Rw2c is not None and points.Rw2c.dim() > 2:
            if add_Rw2c is None:
                raise L.PnrError("grow_points: the cloud has a per-point Rw2c, add_Rw2c [M,3,3] is required")
            points.Rw2c = torch.cat([points.Rw2c, add_Rw2c.to(dev).float().reshape(-1, 3, 3)], 0).contiguous()
