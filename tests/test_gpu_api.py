"""Reference-API seams on the HIP path: the upstream RGB head (C_out = 3), the
seam-2 chain NeuralPoints.forward -> PointAggregator.forward -> ray_march that
the reference's NeuralPointsRayMarching.forward runs
(neural_points_volumetric_model.py:288-318), a non-identity Rw2c, and the
module forward's training path.

Tolerance: the fp32 render tolerance of test_gpu_render.py (|d| <= 2e-4 +
1e-4 |ref|, PSNR >= 60 dB) against the oracle; the C_out = 3 head itself is a
restatement of commented-out reference lines (point_aggregators.py:343,
269-273, 637-638), so its parity is unpinned by reference outputs."""
import numpy as np
import pytest
import torch

from formula import LEGO_SHAPES, UPSTREAM_SHAPES, formula_params
from oracle import oracle as O
from oracle import oracle_grad as OG
from nr_ref import neural_render_torch
from scenes import oracle_points, scene

pytestmark = pytest.mark.gpu


def _model(sc, cuda, params, precision="fp32", Rw2c=None, train=False):
    from pointnerf_amd.aggregator import PointAggregator
    from pointnerf_amd.renderer import NeuralPoints, NeuralPointsRayMarching
    agg = PointAggregator(sc["opt"]).to(cuda)
    agg.load_state_dict({k: torch.from_numpy(v) for k, v in params.items()})
    np_ = NeuralPoints(sc["opt"], cuda, torch.from_numpy(sc["xyz"]), torch.from_numpy(sc["emb"]),
                       torch.from_numpy(sc["color"]), torch.from_numpy(sc["dir"]), torch.from_numpy(sc["conf"]),
                       Rw2c=None if Rw2c is None else torch.from_numpy(Rw2c))
    m = NeuralPointsRayMarching(sc["opt"], np_, agg.train() if train else agg.eval(), precision=precision)
    m.train_precision = "fp32x3"   # the strict oracle comparisons; fp32h2 (the default) has its own tests
    return m


def _inputs(sc, cuda):
    return dict(campos=torch.from_numpy(sc["campos"]).to(cuda)[None],
                raydir=torch.from_numpy(sc["raydir"]).to(cuda)[None],
                bg_color=torch.from_numpy(sc["bg"]).to(cuda),
                camrotc2w=torch.from_numpy(sc["camrot"]).to(cuda)[None],
                near=torch.tensor([[2.0]], device=cuda), far=torch.tensor([[6.0]], device=cuda))


def _psnr(a, b):
    mse = float(np.mean((np.asarray(a, np.float64) - np.asarray(b, np.float64)) ** 2))
    return 10 * np.log10(float(np.abs(b).max()) ** 2 / max(mse, 1e-30))


@pytest.mark.parametrize("precision", ["fp32", "fp32h2", "fp32x3"])
def test_rgb_head_render_vs_oracle(cuda, precision):
    """C_out = 3: ray colours are RGB (radiance_render [..., 1:4], bg 3 channels)."""
    sc = scene(30000, H=40, W=40, theta=120.0, default_conf=None, shading_color_channel_num=3)
    sc["bg"] = np.array([1.0, 1.0, 1.0], np.float32)          # bg_color "white"
    params = formula_params(UPSTREAM_SHAPES, salt=0.4)
    m = _model(sc, cuda, params, precision)
    with torch.no_grad():
        out = m(**_inputs(sc, cuda))
    ref = O.render(sc["opt"], oracle_points(sc), params, sc["campos"], sc["camrot"], sc["raydir"], sc["bg"])
    got = out["coarse_raycolor"][0].cpu().numpy()
    assert got.shape == (1600, 3)
    assert np.array_equal(out["ray_mask"][0].cpu().numpy(), ref["ray_mask"])
    assert ref["ray_mask"].sum() > 300
    np.testing.assert_allclose(got, ref["coarse_raycolor"], atol=2e-4, rtol=1e-4)
    np.testing.assert_allclose(out["coarse_point_opacity"][0].cpu().numpy(), ref["coarse_point_opacity"],
                               atol=2e-4, rtol=1e-4)
    assert _psnr(got, ref["coarse_raycolor"]) >= 60.0
    assert got.min() >= -1e-3 - 1e-6 and got[ref["ray_mask"] > 0].max() <= 1.0 + 1e-3 + 1e-6


def test_rgb_head_backward_vs_torch(cuda):
    from pointnerf_amd.train import RgbHeadFn
    g = torch.Generator().manual_seed(4)
    n = 5000
    feat = torch.randn((n, 129), generator=g)
    W = torch.randn((3, 128), generator=g) * 0.1
    b = torch.randn(3, generator=g) * 0.1
    d = torch.randn((n, 4), generator=g)
    x = [t.to(cuda).requires_grad_(True) for t in (feat, W, b)]
    out = RgbHeadFn.apply(x[0], x[1], x[2], 1, None, n)
    (out * d.to(cuda)).sum().backward()
    r = [t.double().requires_grad_(True) for t in (feat, W, b)]
    ref = torch.cat([r[0][:, :1], torch.sigmoid(r[0][:, 1:] @ r[1].t() + r[2]) * (1 + 2e-3) - 1e-3], 1)
    (ref * d.double()).sum().backward()
    np.testing.assert_allclose(out.detach().cpu().numpy(), ref.detach().numpy(), atol=1e-6, rtol=1e-5)
    for a, e, name in zip(x, r, ("feat", "W", "b")):
        np.testing.assert_allclose(a.grad.cpu().numpy(), e.grad.numpy(), atol=1e-4 * float(e.grad.abs().max()),
                                   rtol=1e-4, err_msg=name)
    # d W / d b: per-block partials summed in block order -> bitwise repeatable
    first = [t.grad.clone() for t in x]
    for t in x:
        t.grad = None
    out = RgbHeadFn.apply(x[0], x[1], x[2], 1, None, n)
    (out * d.to(cuda)).sum().backward()
    for a, f, name in zip(x, first, ("feat", "W", "b")):
        assert torch.equal(a.grad, f), f"rgb head d{name} not repeatable"


def test_rgb_head_train_grads_vs_oracle(cuda):
    """End to end in C_out = 3 mode: render_rays_train -> MSE-like loss ->
    gradients of the point tables and every MLP weight incl. color_branch.6
    vs torch autograd of the CPU oracle."""
    from test_gpu_backward import close
    sc = scene(20000, H=32, W=32, theta=60.0, default_conf=None, shading_color_channel_num=3)
    sc["bg"] = np.array([1.0, 1.0, 1.0], np.float32)
    params = formula_params(UPSTREAM_SHAPES, salt=0.3)
    m = _model(sc, cuda, params, train=True)
    cp, cr = torch.from_numpy(sc["campos"]).to(cuda), torch.from_numpy(sc["camrot"]).to(cuda)
    rd, bg = torch.from_numpy(sc["raydir"]).to(cuda), torch.from_numpy(sc["bg"]).to(cuda)
    color, _, _, ray_mask = m.render_rays_train(cp, cr, rd, 2.0, 6.0, bg)
    assert color.shape[1] == 3
    G = torch.randn(color.shape, generator=torch.Generator().manual_seed(5)).to(cuda)
    (color * G).sum().backward()
    opt = sc["opt"]
    q = O.query_points(opt, sc["xyz"], sc["campos"], sc["camrot"], sc["raydir"], near=2.0, far=6.0)
    tp = {k: torch.from_numpy(np.ascontiguousarray(sc[k])).double().requires_grad_(True)
          for k in ("emb", "color", "dir", "conf")}
    pp = {k: torch.from_numpy(v).double().requires_grad_(True) for k, v in params.items()}
    pidx = torch.from_numpy(q["sample_pidx"]).long()
    mask = pidx >= 0
    idx = pidx.clamp(min=0).reshape(-1)
    shp = tuple(pidx.shape)
    xyz = torch.from_numpy(sc["xyz"]).double()
    pers = torch.from_numpy(O.w2pers(sc["xyz"], sc["campos"], sc["camrot"])).double()
    gsel = lambda a, c: a.reshape(-1, c)[idx].reshape(shp + (c,))  # noqa: E731
    feats, rv, _, _ = OG.aggregate(pp, gsel(tp["color"], 3), gsel(tp["dir"], 3), gsel(tp["conf"], 1),
                                   gsel(tp["emb"], 32), gsel(pers, 3), gsel(xyz, 3), mask,
                                   torch.from_numpy(q["sample_loc"]).double(),
                                   torch.from_numpy(q["sample_loc_w"]).double(),
                                   torch.from_numpy(q["sample_ray_dirs"]).double(), C=3)
    rdist = torch.from_numpy(O.ray_dist(q["sample_loc"], rv.numpy(), opt.vsize[2], opt.raydist_mode_unit))
    c_ref = OG.ray_march(rdist.double(), rv, feats, torch.from_numpy(sc["bg"]).double())
    mk = torch.from_numpy(q["ray_mask"] > 0)
    assert np.array_equal(ray_mask.cpu().numpy(), q["ray_mask"])
    close(color[mk.to(cuda)], c_ref, "ray_color", rel=1e-4, scale=2e-5)
    (c_ref * G.cpu().double()[mk]).sum().backward()
    npts = m.neural_points
    close(npts.points_embeding.grad.reshape(-1, 32), tp["emb"].grad, "d points_embeding", scale=5e-5)
    close(npts.points_color.grad.reshape(-1, 3), tp["color"].grad, "d points_color", scale=5e-5)
    close(npts.points_conf.grad.reshape(-1, 1), tp["conf"].grad, "d points_conf", scale=5e-5)
    for k, p in m.aggregator.named_parameters():
        close(p.grad, pp[k].grad, "d " + k, scale=3e-4)


@pytest.mark.parametrize("C", [128, 3])
def test_seam2_neural_points_aggregator_ray_march_chain(cuda, C):
    """The reference forward as three seams (neural_points_volumetric_model.py:288-318):
    NeuralPoints.forward's 14-tuple -> PointAggregator.forward(13 args) -> ray_dist ->
    ray_march -- equals the fused render and the oracle."""
    from pointnerf_amd.ray_march import alpha_blend, radiance_render, ray_march
    sc = scene(20000, H=32, W=32, theta=250.0, default_conf=None, shading_color_channel_num=C)
    if C == 3:
        sc["bg"] = np.array([0.2, 0.5, 0.9], np.float32)
    params = formula_params(UPSTREAM_SHAPES if C == 3 else LEGO_SHAPES, salt=0.2)
    m = _model(sc, cuda, params)
    inp = _inputs(sc, cuda)
    with torch.no_grad():
        fused = m(**inp)
        t = m.neural_points({"pixel_idx": None, "camrotc2w": inp["camrotc2w"], "campos": inp["campos"],
                             "near": inp["near"], "far": inp["far"], "focal": None, "h": 32, "w": 32,
                             "intrinsic": None, "gt_image": None, "raydir": inp["raydir"]})
        assert len(t) == 14
        (s_color, s_Rw2c, s_dir, s_conf, s_emb, s_pers, s_xyz, s_mask, s_loc, s_loc_w, s_dirs, ray_mask,
         vsize, grid_vox_sz) = t
        feats, ray_valid, weight, conf = m.aggregator(s_color, s_Rw2c, s_dir, s_conf, s_emb, s_pers, s_xyz, s_mask,
                                                      s_loc, s_loc_w, s_dirs, vsize, grid_vox_sz)
        assert feats.shape[-1] == C + 1
        rd = torch.cummax(s_loc[..., 2], dim=-1)[0]
        rd = torch.cat([rd[..., 1:] - rd[..., :-1], torch.full(rd.shape[:2] + (1,), float(vsize[2]), device=cuda)],
                       -1)
        msk = ((rd < 1e-8) | (rd > 2 * float(vsize[2]))).float()
        rd = (rd * (1 - msk) + msk * float(vsize[2])) * ray_valid.float()
        color = ray_march(rd, ray_valid, feats, radiance_render, alpha_blend,
                          torch.from_numpy(sc["bg"]).to(cuda))[0]
    ref = O.render(sc["opt"], oracle_points(sc), params, sc["campos"], sc["camrot"], sc["raydir"], sc["bg"])
    mk = ref["ray_mask"] > 0
    assert np.array_equal(ray_mask[0].cpu().numpy(), ref["ray_mask"])
    np.testing.assert_allclose(color[0].cpu().numpy(), ref["coarse_raycolor"][mk], atol=2e-4, rtol=1e-4)
    np.testing.assert_allclose(color[0].cpu().numpy(), fused["coarse_raycolor"][0].cpu().numpy()[mk],
                               atol=2e-4, rtol=1e-4)


def test_non_identity_rw2c(cuda):
    """NeuralPoints(Rw2c=R) reaches the aggregator (view dirs, distances and point
    dirs are rotated, point_aggregators.py:506, 526, 566)."""
    sc = scene(20000, H=32, W=32, theta=10.0, default_conf=None)
    a = np.deg2rad(35.0)
    R = np.array([[np.cos(a), -np.sin(a), 0], [np.sin(a), np.cos(a), 0], [0, 0, 1]], np.float32)
    from pointnerf_amd.aggregator import PointAggregator
    torch.manual_seed(0)   # the aggregator's own xavier init (the closed-form weights barely see R)
    params = {k: v.detach().numpy() for k, v in PointAggregator(sc["opt"]).state_dict().items()}
    m = _model(sc, cuda, params, Rw2c=R)
    with torch.no_grad():
        out = m(**_inputs(sc, cuda))
    pts = dict(oracle_points(sc), Rw2c=R)
    ref = O.render(sc["opt"], pts, params, sc["campos"], sc["camrot"], sc["raydir"], sc["bg"])
    ref_id = O.render(sc["opt"], oracle_points(sc), params, sc["campos"], sc["camrot"], sc["raydir"], sc["bg"])
    got = out["coarse_raycolor"][0].cpu().numpy()
    np.testing.assert_allclose(got, ref["coarse_raycolor"], atol=2e-4, rtol=1e-4)
    assert np.abs(got - ref_id["coarse_raycolor"]).max() > 5e-4    # R matters beyond the tolerance


def test_module_forward_trains(cuda):
    """model(...) in training mode with grad enabled is differentiable (the
    reference's optimize_parameters loop), in eval / no_grad it is the fused path."""
    sc = scene(8000, H=24, W=24, theta=10.0, default_conf=None)
    m = _model(sc, cuda, formula_params(salt=0.7), train=True)
    m.train()
    out = m(**_inputs(sc, cuda))
    assert out["coarse_raycolor"].requires_grad
    out["coarse_raycolor"][..., :3].square().mean().backward()
    assert m.neural_points.points_embeding.grad is not None
    assert float(m.neural_points.points_embeding.grad.abs().sum()) > 0
    m.eval()
    with torch.no_grad():
        out2 = m(**_inputs(sc, cuda))
    assert not out2["coarse_raycolor"].requires_grad
    np.testing.assert_allclose(out2["coarse_raycolor"].cpu().numpy(), out["coarse_raycolor"].detach().cpu().numpy(),
                               atol=1e-5, rtol=1e-5)


def test_module_neural_render_cnn_trains(cuda):
    """opt.neural_render = "cnn" (neural_points_volumetric_model.py:258-260,
    343-344) in the training loop: final_coarse_raycolor is differentiable through
    NeuralRenderFn (pnr_neural_render_bwd) down to the point embeddings, the
    aggregator and the 2-D renderer's own parameters; the gradient reaching the
    composited feature image equals torch autograd of the fp64 restatement."""
    H = W = 24
    sc = scene(8000, H=H, W=W, theta=10.0, default_conf=None, neural_render="cnn")
    m = _model(sc, cuda, formula_params(salt=0.7), train=True)
    m.train()
    out = m(**_inputs(sc, cuda), h=H, w=W)
    final = out["final_coarse_raycolor"]
    assert final.shape == (1, H * W, 3) and final.requires_grad
    g = torch.randn(final.shape, device=cuda, generator=torch.Generator(device=cuda).manual_seed(3))
    (final * g).sum().backward()
    nr = m.neural_render_2d
    for n, p in nr.named_parameters():
        assert p.grad is not None and float(p.grad.abs().sum()) > 0, n
    assert float(m.neural_points.points_embeding.grad.abs().sum()) > 0
    assert float(m.aggregator.block1[0].weight.grad.abs().sum()) > 0
    # the 2-D renderer's input gradient vs torch autograd in fp64
    coarse = out["coarse_raycolor"].detach().reshape(1, H, W, -1)
    x1 = coarse.clone().requires_grad_(True)
    (nr(x1) * g.reshape(1, H, W, 3)).sum().backward()
    from pointnerf_amd.neural_render import NeuralRenderer
    nr64 = NeuralRenderer(input_dim=128)
    nr64.load_state_dict({k: v.detach().cpu() for k, v in nr.state_dict().items()})
    nr64 = nr64.double().to(cuda)
    x2 = coarse.double().requires_grad_(True)
    (neural_render_torch(nr64, x2) * g.double().reshape(1, H, W, 3)).sum().backward()
    err = float((x1.grad.double() - x2.grad).abs().max())
    assert err <= 2e-5 * max(float(x2.grad.abs().max()), 1e-3), err
