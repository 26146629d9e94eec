"""Generate the golden vectors in tests/golden/*.npz from the REFERENCE code.

Runs only in the authoring container, where the reference tree is mounted at
/root/reference (read-only).  It imports the reference's own Python modules
(ray generation, positional encoding, PointAggregator, ray_march) and records
their inputs/outputs; nothing from the reference is copied into the repo.
The fixtures are data only; tests load them with numpy (allow_pickle=False).

    python tests/golden/make_golden.py [--ref /root/reference]
"""
import argparse
import os
import sys
from types import SimpleNamespace

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from formula import formula_params  # noqa: E402


def lego_agg_opt():
    # dev_scripts/w_n360/lego.sh values + PointAggregator defaults
    # (point_aggregators.py:15-217); agg_axis_weight None takes the same branch
    # as lego's "1 1 1" without allocating on cuda (point_aggregators.py:247).
    return SimpleNamespace(
        act_type="LeakyReLU", point_hyper_dim=256, point_features_dim=32,
        agg_distance_kernel="linear", agg_dist_pers=20, agg_axis_weight=None,
        num_pos_freqs=10, num_viewdir_freqs=4, which_agg_model="viewmlp",
        dist_xyz_freq=5, agg_feat_xyz_mode="None", agg_alpha_xyz_mode="None",
        agg_color_xyz_mode="None", weight_feat_dim=8, weight_xyz_freq=2, sh_degree=4,
        num_feat_freqs=3, agg_intrp_order=2, shading_feature_mlp_layer0=1,
        shading_feature_mlp_layer1=2, shading_feature_mlp_layer2=0,
        shading_feature_mlp_layer3=2, shading_feature_num=256, point_color_mode="1",
        point_dir_mode="1", shading_alpha_mlp_layer=1, shading_color_mlp_layer=4,
        shading_color_channel_num=128, act_super=1, dist_xyz_deno=0.0, apply_pnt_mask=1,
        agg_weight_norm=1, sparse_loss_weight=0, zero_one_loss_items=["conf_coefficient"],
        prob=0, view_ori=0, sh_dist_func="sh_quadric", sh_act="sigmoid", modulator_concat=0,
        num_hyperfeat_freqs=0, feature_init_method="rand")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--only", choices=("all", "r04"), default="all",
                    help="r04: only the round-4 fixtures (per-pair Rw2c aggregator, full ray_march backward)")
    args = ap.parse_args()
    sys.path.insert(0, args.ref)
    if args.only == "r04":
        return round4()
    from models.helpers.networks import positional_encoding
    from models.rendering.diff_ray_marching import near_far_linear_ray_generation, ray_march
    from models.rendering.diff_render_func import alpha_blend, radiance_render
    from models.aggregators.point_aggregators import PointAggregator

    rng = np.random.default_rng(1234)
    torch.set_num_threads(1)

    # 1. ray generation (diff_ray_marching.py:349-393), eval (jitter 0) and train (jitter 0.3)
    campos = torch.tensor([[0.3, -3.6, 1.9]], dtype=torch.float32)
    raydir = torch.tensor(rng.normal(size=(1, 8, 3)) * 0.3 + np.array([0.0, 1.0, -0.5]), dtype=torch.float32)
    pos0, seg0, _, mid0 = near_far_linear_ray_generation(campos, raydir, 400, near=2.0, far=6.0, jitter=0.0)
    torch.manual_seed(7)
    pos1, seg1, _, mid1 = near_far_linear_ray_generation(campos, raydir, 400, near=2.0, far=6.0, jitter=0.3)
    torch.manual_seed(7)
    rand1 = torch.rand((1, 8, 400))
    np.savez_compressed(os.path.join(HERE, "raygen.npz"), campos=campos.numpy(), raydir=raydir.numpy(),
                        mid0=mid0.numpy(), pos0=pos0.numpy(), mid1=mid1.numpy(), pos1=pos1.numpy(),
                        rand1=rand1.numpy(), near=np.float32(2.0), far=np.float32(6.0))

    # 2. positional encoding (networks.py:175-190)
    x = torch.tensor(rng.uniform(-1.5, 1.5, size=(64, 6)), dtype=torch.float32)
    np.savez_compressed(os.path.join(HERE, "pe.npz"), x=x.numpy(),
                        pe5=positional_encoding(x, 5).numpy(),
                        pe3=positional_encoding(x[:, :3], 3).numpy(),
                        pe4ori=positional_encoding(x[:, :3], 4, ori=True).numpy())

    # 3. PointAggregator (lego config), formula weights, random gathered inputs
    agg = PointAggregator(lego_agg_opt())
    params = formula_params()
    sd = agg.state_dict()
    assert set(sd.keys()) == set(params.keys()), (sorted(sd.keys()), sorted(params.keys()))
    for k in sd:
        assert tuple(sd[k].shape) == params[k].shape, (k, sd[k].shape, params[k].shape)
    agg.load_state_dict({k: torch.from_numpy(v) for k, v in params.items()})
    R, SR, K = 6, 10, 8
    mask = rng.uniform(size=(1, R, SR, K)) < 0.7
    mask[0, 0, :, :] = False          # a ray with no neighbours at all
    mask[0, 1, 3, :] = False          # an empty sample
    mask[0, 2, :, 1:] = False         # single-neighbour samples
    sloc_w = rng.uniform(-0.5, 0.5, size=(1, R, SR, 3)).astype(np.float32)
    campos_a = np.array([0.2, -3.8, 1.7], np.float32)
    sxyz = (sloc_w[..., None, :] + rng.normal(scale=0.008, size=(1, R, SR, K, 3))).astype(np.float32)

    def pers(p):
        c = p - campos_a
        rot = np.array([[0.99, 0.1, 0.0], [0.0, 0.3, -0.95], [-0.1, 0.95, 0.3]], np.float32)
        xc = c @ rot
        return np.stack([xc[..., 0] / xc[..., 2], xc[..., 1] / xc[..., 2], xc[..., 2]], -1).astype(np.float32)

    inputs = dict(
        sampled_color=rng.normal(size=(1, R, SR, K, 3)).astype(np.float32),
        sampled_dir=rng.normal(size=(1, R, SR, K, 3)).astype(np.float32),
        sampled_conf=rng.uniform(-0.2, 1.3, size=(1, R, SR, K, 1)).astype(np.float32),
        sampled_embedding=rng.uniform(-0.5, 0.5, size=(1, R, SR, K, 32)).astype(np.float32),
        sampled_xyz_pers=pers(sxyz), sampled_xyz=sxyz, sample_pnt_mask=mask,
        sample_loc=pers(sloc_w), sample_loc_w=sloc_w,
        sample_ray_dirs=np.broadcast_to(rng.normal(size=(1, R, 1, 3)), (1, R, SR, 3)).astype(np.float32))
    t = {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in inputs.items()}
    with torch.no_grad():
        feats, ray_valid, weight, conf = agg(t["sampled_color"], torch.eye(3), t["sampled_dir"],
                                             t["sampled_conf"], t["sampled_embedding"],
                                             t["sampled_xyz_pers"], t["sampled_xyz"],
                                             t["sample_pnt_mask"], t["sample_loc"], t["sample_loc_w"],
                                             t["sample_ray_dirs"], [0.004, 0.004, 0.004], 0)
    np.savez_compressed(os.path.join(HERE, "aggregator.npz"), features=feats.numpy(),
                        ray_valid=ray_valid.numpy(), weight=weight.numpy(), conf_coefficient=conf.numpy(),
                        **{k: np.ascontiguousarray(v) for k, v in inputs.items()})

    # 3b. PointAggregator backward (autograd of the same forward): upstream gradient
    #     g_feat on the output, grads of the gathered inputs and of every parameter
    tg = {k: v.clone().requires_grad_(k in ("sampled_color", "sampled_dir", "sampled_conf",
                                             "sampled_embedding"))
          for k, v in t.items()}
    agg.zero_grad()
    feats_g, _, _, _ = agg(tg["sampled_color"], torch.eye(3), tg["sampled_dir"], tg["sampled_conf"],
                           tg["sampled_embedding"], tg["sampled_xyz_pers"], tg["sampled_xyz"],
                           tg["sample_pnt_mask"], tg["sample_loc"], tg["sample_loc_w"],
                           tg["sample_ray_dirs"], [0.004, 0.004, 0.004], 0)
    g_feat = torch.tensor(rng.normal(size=tuple(feats_g.shape)), dtype=torch.float32)
    (feats_g * g_feat).sum().backward()
    grads = {"g_" + k: tg[k].grad.numpy() for k in ("sampled_color", "sampled_dir", "sampled_conf",
                                                   "sampled_embedding")}
    grads.update({"gp_" + k.replace(".", "_"): p.grad.numpy() for k, p in agg.named_parameters()})
    np.savez_compressed(os.path.join(HERE, "aggregator_bwd.npz"), g_feat=g_feat.numpy(),
                        features=feats_g.detach().numpy(), **grads)

    # 4. ray_march + radiance_render + alpha_blend (diff_ray_marching.py:509-555)
    NR, SRm, C = 12, 24, 128
    rd = torch.tensor(rng.uniform(0.0, 0.01, size=(1, NR, SRm)), dtype=torch.float32)
    rv = torch.tensor(rng.uniform(size=(1, NR, SRm)) < 0.6)
    rf = torch.tensor(np.concatenate([rng.uniform(0, 300, size=(1, NR, SRm, 1)),
                                      rng.normal(size=(1, NR, SRm, C))], -1), dtype=torch.float32)
    bg = torch.tensor(rng.uniform(size=(C,)), dtype=torch.float32)
    out = ray_march(rd, rv, rf, radiance_render, alpha_blend, bg)
    names = ["ray_color", "point_color", "opacity", "acc_transmission", "blend_weight",
             "background_transmission", "background_blend_weight"]
    np.savez_compressed(os.path.join(HERE, "raymarch.npz"), ray_dist=rd.numpy(), ray_valid=rv.numpy(),
                        ray_features=rf.numpy(), bg_color=bg.numpy(),
                        **{n: (o.numpy() if torch.is_tensor(o) else np.asarray(o)) for n, o in zip(names, out)})
    # 4b. ray_march backward: upstream gradient on ray_color -> d ray_features
    rfg = rf.clone().requires_grad_(True)
    outg = ray_march(rd, rv, rfg, radiance_render, alpha_blend, bg)
    g_color = torch.tensor(rng.normal(size=tuple(outg[0].shape)), dtype=torch.float32)
    (outg[0] * g_color).sum().backward()
    np.savez_compressed(os.path.join(HERE, "raymarch_bwd.npz"), g_color=g_color.numpy(),
                        g_features=rfg.grad.numpy())
    print("golden vectors written to", HERE)


def round4():
    """Round-4 fixtures (separate seed, the earlier files stay as they are):
    aggregator_rw2c.npz -- PointAggregator.forward with a per-pair Rw2c
    [1,R,SR,K,3,3] (neural_points.py:799 gathers one per point;
    point_aggregators.py:492-496, 506, 526, 566) and the gradients of its gathered
    inputs; raymarch_full_bwd.npz -- ray_march's gradients of ray_features,
    ray_dist and bg_color for a loss on every output (ray_color, opacity,
    acc_transmission, blend_weight, background_transmission)."""
    from models.rendering.diff_ray_marching import ray_march
    from models.rendering.diff_render_func import alpha_blend, radiance_render
    from models.aggregators.point_aggregators import PointAggregator

    rng = np.random.default_rng(4040)
    torch.set_num_threads(1)
    agg = PointAggregator(lego_agg_opt())
    agg.load_state_dict({k: torch.from_numpy(v) for k, v in formula_params(salt=0.3).items()})
    R, SR, K = 5, 9, 8
    mask = rng.uniform(size=(1, R, SR, K)) < 0.75
    mask[0, 1, 2, :] = False
    mask[0, 3, :, 2:] = False
    for r in range(R):           # the KNN fills slots in order: empty slots trail
        for s_ in range(SR):
            n = int(mask[0, r, s_].sum())
            mask[0, r, s_] = False
            mask[0, r, s_, :n] = True
    sloc_w = rng.uniform(-0.5, 0.5, size=(1, R, SR, 3)).astype(np.float32)
    sxyz = (sloc_w[..., None, :] + rng.normal(scale=0.008, size=(1, R, SR, K, 3))).astype(np.float32)
    campos_a = np.array([0.2, -3.8, 1.7], np.float32)
    rot = np.array([[0.99, 0.1, 0.0], [0.0, 0.3, -0.95], [-0.1, 0.95, 0.3]], np.float32)

    def pers(p):
        xc = (p - campos_a) @ rot
        return np.stack([xc[..., 0] / xc[..., 2], xc[..., 1] / xc[..., 2], xc[..., 2]], -1).astype(np.float32)

    # random proper rotations per pair (QR of Gaussian matrices)
    q, rr = np.linalg.qr(rng.normal(size=(1, R, SR, K, 3, 3)))
    q = q * np.sign(np.diagonal(rr, axis1=-2, axis2=-1))[..., None, :]
    inputs = dict(
        sampled_color=rng.normal(size=(1, R, SR, K, 3)).astype(np.float32),
        sampled_dir=rng.normal(size=(1, R, SR, K, 3)).astype(np.float32),
        sampled_conf=rng.uniform(-0.2, 1.3, size=(1, R, SR, K, 1)).astype(np.float32),
        sampled_embedding=rng.uniform(-0.5, 0.5, size=(1, R, SR, K, 32)).astype(np.float32),
        sampled_xyz_pers=pers(sxyz), sampled_xyz=sxyz, sample_pnt_mask=mask,
        sample_loc=pers(sloc_w), sample_loc_w=sloc_w,
        sample_ray_dirs=np.broadcast_to(rng.normal(size=(1, R, 1, 3)), (1, R, SR, 3)).astype(np.float32),
        sampled_Rw2c=q.astype(np.float32))
    t = {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in inputs.items()}
    for k in ("sampled_color", "sampled_dir", "sampled_conf", "sampled_embedding"):
        t[k].requires_grad_(True)
    feats, ray_valid, weight, conf = agg(t["sampled_color"], t["sampled_Rw2c"], t["sampled_dir"], t["sampled_conf"],
                                         t["sampled_embedding"], t["sampled_xyz_pers"], t["sampled_xyz"],
                                         t["sample_pnt_mask"], t["sample_loc"], t["sample_loc_w"],
                                         t["sample_ray_dirs"], [0.004, 0.004, 0.004], 0)
    g_feat = torch.tensor(rng.normal(size=tuple(feats.shape)), dtype=torch.float32)
    (feats * g_feat).sum().backward()
    grads = {"g_" + k: t[k].grad.numpy() for k in ("sampled_color", "sampled_dir", "sampled_conf",
                                                  "sampled_embedding")}
    np.savez_compressed(os.path.join(HERE, "aggregator_rw2c.npz"), features=feats.detach().numpy(),
                        ray_valid=ray_valid.numpy(), weight=weight.detach().numpy(), g_feat=g_feat.numpy(),
                        **grads, **{k: np.ascontiguousarray(v) for k, v in inputs.items()})

    NR, SRm, C = 10, 20, 128
    rd = torch.tensor(rng.uniform(0.0, 0.01, size=(1, NR, SRm)), dtype=torch.float32, requires_grad=True)
    rv = torch.tensor(rng.uniform(size=(1, NR, SRm)) < 0.6)
    rf = torch.tensor(np.concatenate([rng.uniform(0, 300, size=(1, NR, SRm, 1)),
                                      rng.normal(size=(1, NR, SRm, C))], -1), dtype=torch.float32,
                      requires_grad=True)
    bg = torch.tensor(rng.uniform(size=(C,)), dtype=torch.float32, requires_grad=True)
    out = ray_march(rd, rv, rf, radiance_render, alpha_blend, bg)
    gs = [torch.tensor(rng.normal(size=tuple(out[i].shape)), dtype=torch.float32) for i in (0, 2, 3, 4, 5)]
    loss = sum((out[i] * g).sum() for i, g in zip((0, 2, 3, 4, 5), gs))
    loss.backward()
    np.savez_compressed(os.path.join(HERE, "raymarch_full_bwd.npz"), ray_dist=rd.detach().numpy(),
                        ray_valid=rv.numpy(), ray_features=rf.detach().numpy(), bg_color=bg.detach().numpy(),
                        g_color=gs[0].numpy(), g_opacity=gs[1].numpy(), g_acc=gs[2].numpy(),
                        g_blend=gs[3].numpy(), g_bgT=gs[4].numpy(), d_features=rf.grad.numpy(),
                        d_ray_dist=rd.grad.numpy(), d_bg=bg.grad.numpy())
    print("round-4 golden vectors written to", HERE)


if __name__ == "__main__":
    main()
