"""The differentiable CPU restatement (oracle/oracle_grad.py) against the
reference's own autograd gradients (tests/golden/*_bwd.npz)."""
import os
import sys

import numpy as np
import torch

from oracle import oracle_grad as OG

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
from formula import formula_params  # noqa: E402


def load(name):
    return np.load(os.path.join(HERE, "golden", name), allow_pickle=False)


def test_aggregate_grads_match_reference():
    g = load("aggregator.npz")
    gb = load("aggregator_bwd.npz")
    params = {k: torch.from_numpy(v).requires_grad_(True) for k, v in formula_params().items()}
    t = {k: torch.from_numpy(np.ascontiguousarray(g[k][0])) for k in
         ("sampled_color", "sampled_dir", "sampled_conf", "sampled_embedding", "sampled_xyz_pers",
          "sampled_xyz", "sample_pnt_mask", "sample_loc", "sample_loc_w", "sample_ray_dirs")}
    for k in ("sampled_color", "sampled_dir", "sampled_conf", "sampled_embedding"):
        t[k].requires_grad_(True)
    out, _, _, _ = OG.aggregate(params, t["sampled_color"], t["sampled_dir"], t["sampled_conf"],
                                t["sampled_embedding"], t["sampled_xyz_pers"], t["sampled_xyz"],
                                t["sample_pnt_mask"], t["sample_loc"], t["sample_loc_w"], t["sample_ray_dirs"])
    np.testing.assert_allclose(out.detach().numpy(), gb["features"][0], atol=1e-6, rtol=1e-5)
    (out * torch.from_numpy(gb["g_feat"][0])).sum().backward()
    for k in ("sampled_color", "sampled_dir", "sampled_conf", "sampled_embedding"):
        ref = gb["g_" + k][0]
        np.testing.assert_allclose(t[k].grad.numpy(), ref, atol=1e-6 + 1e-5 * np.abs(ref).max(), rtol=1e-4,
                                   err_msg=k)
    for k, p in params.items():
        ref = gb["gp_" + k.replace(".", "_")]
        np.testing.assert_allclose(p.grad.numpy(), ref, atol=1e-6 + 1e-5 * np.abs(ref).max(), rtol=1e-4,
                                   err_msg=k)


def test_ray_march_grads_match_reference():
    g = load("raymarch.npz")
    gb = load("raymarch_bwd.npz")
    rf = torch.from_numpy(g["ray_features"][0]).requires_grad_(True)
    c = OG.ray_march(torch.from_numpy(g["ray_dist"][0]), torch.from_numpy(g["ray_valid"][0]), rf,
                     torch.from_numpy(g["bg_color"]))
    np.testing.assert_allclose(c.detach().numpy(), g["ray_color"][0], atol=2e-6, rtol=1e-5)
    (c * torch.from_numpy(gb["g_color"][0])).sum().backward()
    ref = gb["g_features"][0]
    np.testing.assert_allclose(rf.grad.numpy(), ref, atol=1e-6 + 1e-5 * np.abs(ref).max(), rtol=1e-4)


def test_aggregate_grads_per_pair_rw2c():
    # autograd of the reference's PointAggregator with a per-pair Rw2c (aggregator_rw2c.npz)
    g = load("aggregator_rw2c.npz")
    params = {k: torch.from_numpy(v) for k, v in formula_params(salt=0.3).items()}
    t = {k: torch.from_numpy(np.ascontiguousarray(g[k][0])) for k in
         ("sampled_color", "sampled_dir", "sampled_conf", "sampled_embedding", "sampled_xyz_pers",
          "sampled_xyz", "sample_pnt_mask", "sample_loc", "sample_loc_w", "sample_ray_dirs", "sampled_Rw2c")}
    for k in ("sampled_color", "sampled_dir", "sampled_conf", "sampled_embedding"):
        t[k].requires_grad_(True)
    out, _, _, _ = OG.aggregate(params, t["sampled_color"], t["sampled_dir"], t["sampled_conf"],
                                t["sampled_embedding"], t["sampled_xyz_pers"], t["sampled_xyz"],
                                t["sample_pnt_mask"], t["sample_loc"], t["sample_loc_w"], t["sample_ray_dirs"],
                                rw2c=t["sampled_Rw2c"])
    np.testing.assert_allclose(out.detach().numpy(), g["features"][0], atol=1e-6, rtol=1e-5)
    (out * torch.from_numpy(g["g_feat"][0])).sum().backward()
    for k in ("sampled_color", "sampled_dir", "sampled_conf", "sampled_embedding"):
        ref = g["g_" + k][0]
        np.testing.assert_allclose(t[k].grad.numpy(), ref, atol=1e-6 + 1e-5 * np.abs(ref).max(), rtol=1e-4,
                                   err_msg=k)


def test_ray_march_full_grads_match_reference():
    # gradients of ray_features, ray_dist and bg_color for a loss on every ray_march output
    g = load("raymarch_full_bwd.npz")
    rd = torch.from_numpy(g["ray_dist"][0]).requires_grad_(True)
    rf = torch.from_numpy(g["ray_features"][0]).requires_grad_(True)
    bg = torch.from_numpy(g["bg_color"]).requires_grad_(True)
    outs = OG.ray_march_full(rd, torch.from_numpy(g["ray_valid"][0]), rf, bg)
    names = ("g_color", "g_opacity", "g_acc", "g_blend", "g_bgT")
    loss = sum((o.reshape(g[n][0].shape) * torch.from_numpy(g[n][0])).sum() for o, n in zip(outs, names))
    loss.backward()
    for got, ref in ((rf.grad, g["d_features"][0]), (rd.grad, g["d_ray_dist"][0]), (bg.grad, g["d_bg"])):
        np.testing.assert_allclose(got.numpy(), ref, atol=1e-6 + 1e-5 * np.abs(ref).max(), rtol=1e-4)
