"""The training contract of the drop-in seams (VERDICT r03 "What's missing"):

* ``pointnerf_amd.ray_march`` is differentiable like the reference's
  (diff_ray_marching.py:509-555, called in training at
  neural_points_volumetric_model.py:314): gradients of ray_features, ray_dist and
  bg_color for a loss on every output, against the reference's own autograd
  (tests/golden/raymarch_full_bwd.npz);
* ``NeuralPointsRayMarching.forward`` puts weight / blend_weight (detached) and
  conf_coefficient (straight-through) into its output
  (neural_points_volumetric_model.py:335-338), which compute_losses reads
  (zero-one loss base_rendering_model.py:630-641, sparse loss :653-657);
* the learned background colour gets its gradient (mvs_points_volumetric_model.py:92-94)
  from the hit rays' bg_T term and the missed rays' fill_invalid rows (:373-375);
* a per-point Rw2c [N,3,3] (neural_points.py:799; point_aggregators.py:492-566)
  renders and trains.

A reference-style training step runs through the seams -- NeuralPoints.forward ->
PointAggregator.forward -> ray_march -> fill_invalid, and through the module's
forward -- with the MSE colour loss plus the zero-one and sparse losses read from
the output dict; every gradient (point tables, aggregator weights, bg_color) is
checked against torch autograd of the CPU restatement in float64
(oracle/oracle_grad.py, itself pinned to the reference's gradients).

Tolerances: renders |d| <= 2e-4 + 1e-4 |ref| (test_gpu_render.py's fp32 bound);
gradients |d| <= scale * max|ref| + 1e-4 |ref| with the scales of
test_gpu_backward.py (5e-5 for point tables, 3e-4 for MLP weights)."""
import os

import numpy as np
import pytest
import torch

from formula import formula_params
from oracle import oracle as O
from oracle import oracle_grad as OG
from scenes import oracle_points, scene
from test_gpu_backward import close

pytestmark = pytest.mark.gpu


def _rotations(n, seed):
    """n random proper rotations (QR of Gaussian matrices), float32 [n,3,3]."""
    rng = np.random.default_rng(seed)
    q, r = np.linalg.qr(rng.normal(size=(n, 3, 3)))
    q = q * np.sign(np.diagonal(r, axis1=-2, axis2=-1))[..., None, :]
    return q.astype(np.float32)


def _signed_perms(n, seed):
    """n random proper rotations among the 24 signed permutation matrices
    (float32 [n,3,3]): per-point Rw2c whose products are exact, so the GPU's
    rotated distances equal the oracle's bit for bit and no LeakyReLU kink flips
    between them -- the whole-step gradient tests then hold the element bound.
    General rotations are covered by the render and xyz-gradient tests."""
    import itertools
    mats = []
    for perm in itertools.permutations(range(3)):
        for signs in itertools.product((1.0, -1.0), repeat=3):
            m = np.zeros((3, 3))
            m[range(3), perm] = signs
            if np.linalg.det(m) > 0:
                mats.append(m)
    rng = np.random.default_rng(seed)
    return np.stack(mats)[rng.integers(0, len(mats), n)].astype(np.float32)


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


def _inputs(sc, cuda, bg=None):
    return dict(campos=torch.from_numpy(sc["campos"]).to(cuda)[None],
                raydir=torch.from_numpy(sc["raydir"]).to(cuda)[None],
                bg_color=torch.from_numpy(sc["bg"]).to(cuda) if bg is None else bg,
                camrotc2w=torch.from_numpy(sc["camrot"]).to(cuda)[None],
                near=torch.tensor([[2.0]], device=cuda), far=torch.tensor([[6.0]], device=cuda))


# ------------------------------------------------------------------ ray_march seam
def test_ray_march_dropin_full_backward_vs_reference_golden(golden_dir, cuda):
    from pointnerf_amd.ray_march import alpha_blend, radiance_render, ray_march
    g = np.load(os.path.join(golden_dir, "raymarch_full_bwd.npz"), allow_pickle=False)
    rd = torch.from_numpy(g["ray_dist"]).to(cuda).requires_grad_(True)
    rv = torch.from_numpy(g["ray_valid"]).to(cuda)
    rf = torch.from_numpy(g["ray_features"]).to(cuda).requires_grad_(True)
    bg = torch.from_numpy(g["bg_color"]).to(cuda).requires_grad_(True)
    out = ray_march(rd, rv, rf, radiance_render, alpha_blend, bg)
    assert all(out[i].requires_grad for i in (0, 2, 3, 4, 5))
    loss = sum((out[i] * torch.from_numpy(g[n]).to(cuda)).sum()
               for i, n in zip((0, 2, 3, 4, 5), ("g_color", "g_opacity", "g_acc", "g_blend", "g_bgT")))
    loss.backward()
    close(rf.grad, g["d_features"], "d ray_features", scale=2e-5)
    close(rd.grad, g["d_ray_dist"], "d ray_dist", scale=2e-5)
    close(bg.grad, g["d_bg"], "d bg_color", scale=2e-5)
    # no grad wanted -> plain forward, same values
    with torch.no_grad():
        out2 = ray_march(rd, rv, rf, radiance_render, alpha_blend, bg)
    for a, b in zip(out, out2):
        assert torch.equal(a.detach(), b)


def test_weighted_colsum_repeatable_and_exact(cuda):
    from pointnerf_amd import _lib as L
    gen = torch.Generator().manual_seed(2)
    for R, C in ((0, 128), (1, 3), (1000, 128), (123457, 128), (5000, 3)):
        w = torch.rand(R, generator=gen)
        x = torch.randn((R, C), generator=gen)
        got = L.weighted_colsum(w.to(cuda), x.to(cuda))
        ref = (w.double()[:, None] * x.double()).sum(0)
        np.testing.assert_allclose(got.cpu().numpy(), ref.numpy(), atol=1e-5 * max(R, 1) ** 0.5, rtol=1e-5)
        assert torch.equal(got, L.weighted_colsum(w.to(cuda), x.to(cuda)))


# ------------------------------------------------------------- per-point Rw2c
def test_aggregator_mirror_per_pair_rw2c_vs_reference_golden(golden_dir, cuda):
    """PointAggregator.forward with sampled_Rw2c [1,R,SR,K,3,3] -- features and the
    gathered inputs' gradients equal the reference's (aggregator_rw2c.npz)."""
    from pointnerf_amd.aggregator import PointAggregator
    from pointnerf_amd.options import lego_opt
    g = np.load(os.path.join(golden_dir, "aggregator_rw2c.npz"), allow_pickle=False)
    agg = PointAggregator(lego_opt()).to(cuda)
    agg.load_state_dict({k: torch.from_numpy(v) for k, v in formula_params(salt=0.3).items()})
    names = ("sampled_color", "sampled_Rw2c", "sampled_dir", "sampled_conf", "sampled_embedding", "sampled_xyz_pers",
             "sampled_xyz", "sample_pnt_mask", "sample_loc", "sample_loc_w", "sample_ray_dirs")
    t = {k: torch.from_numpy(np.ascontiguousarray(g[k])).to(cuda) for k in names}
    with torch.no_grad():
        f, rv, w, _ = agg(*(t[k] for k in names), [0.004] * 3, 0)
    assert np.array_equal(rv.cpu().numpy(), g["ray_valid"])
    close(f, g["features"], "features", scale=1e-5)
    close(w, g["weight"], "weight", scale=1e-6)
    for k in ("sampled_color", "sampled_dir", "sampled_conf", "sampled_embedding"):
        t[k].requires_grad_(True)
    f2, _, _, _ = agg(*(t[k] for k in names), [0.004] * 3, 0)
    close(f2, g["features"], "train features", scale=1e-5)
    (f2 * torch.from_numpy(g["g_feat"]).to(cuda)).sum().backward()
    for k in ("sampled_color", "sampled_dir", "sampled_conf", "sampled_embedding"):
        close(t[k].grad, g["g_" + k], "d " + k, scale=5e-5)


@pytest.mark.parametrize("precision", ["fp32", "fp32x3", "fp32h2", "bf16"])
def test_per_point_rw2c_render_vs_oracle(cuda, precision):
    sc = scene(20000, H=32, W=32, theta=80.0, default_conf=None)
    from pointnerf_amd.aggregator import PointAggregator
    torch.manual_seed(0)   # the aggregator's own init: the closed-form weights barely see the rotations
    params = {k: v.detach().numpy() for k, v in PointAggregator(sc["opt"]).state_dict().items()}
    Rpp = _rotations(sc["xyz"].shape[0], 11)
    m = _model(sc, cuda, params, precision=precision, Rw2c=Rpp)
    with torch.no_grad():
        out = m(**_inputs(sc, cuda))
    ref = O.render(sc["opt"], dict(oracle_points(sc), Rw2c=Rpp), params, sc["campos"], sc["camrot"],
                   sc["raydir"], sc["bg"])
    ref_id = O.render(sc["opt"], oracle_points(sc), params, sc["campos"], sc["camrot"], sc["raydir"], sc["bg"])
    got = out["coarse_raycolor"][0].cpu().numpy()
    assert np.array_equal(out["ray_mask"][0].cpu().numpy(), ref["ray_mask"])
    assert ref["ray_mask"].sum() > 100
    if precision == "bf16":
        mse = float(np.mean((got - ref["coarse_raycolor"]) ** 2))
        assert 10 * np.log10(float(np.abs(ref["coarse_raycolor"]).max()) ** 2 / mse) >= 40.0
    else:
        np.testing.assert_allclose(got, ref["coarse_raycolor"], atol=2e-4, rtol=1e-4)
    assert np.abs(ref["coarse_raycolor"] - ref_id["coarse_raycolor"]).max() > 5e-4   # the rotations matter


def test_per_point_rw2c_prune_grow(cuda):
    """prune / grow_points keep the per-point Rw2c row-aligned with the points
    (neural_points.py:370-372, 400-402); xyz keeps requires_grad with --xyz_grad 1
    (:353, :379)."""
    from pointnerf_amd.checkpoint import grow_points, prune
    sc = scene(3000, H=8, W=8, default_conf=None, xyz_grad=1)
    Rpp = _rotations(3000, 5)
    m = _model(sc, cuda, formula_params(salt=0.2), Rw2c=Rpp)
    np_ = m.neural_points
    assert np_.xyz.requires_grad
    keep = sc["conf"].reshape(-1) >= 0.5
    prune(np_, 0.5)
    assert np_.xyz.requires_grad and np_.Rw2c.shape == (int(keep.sum()), 3, 3)
    assert torch.equal(np_.Rw2c.cpu(), torch.from_numpy(Rpp[keep]))
    n0 = np_.xyz.shape[0]
    add = torch.rand((7, 3))
    grow_points(np_, add, torch.rand((7, 32)), torch.rand((7, 3)), torch.rand((7, 3)), torch.rand((7, 1)),
                add_Rw2c=torch.from_numpy(_rotations(7, 6)))
    assert np_.xyz.requires_grad and np_.xyz.shape[0] == n0 + 7 and np_.Rw2c.shape == (n0 + 7, 3, 3)
    with pytest.raises(Exception):
        grow_points(np_, add, torch.rand((7, 32)), torch.rand((7, 3)), torch.rand((7, 3)), torch.rand((7, 1)))


# --------------------------------------------------- reference-style training step
def _oracle_step(sc, params, q, loss_fn, Rpp=None, dt=torch.float64):
    """torch autograd of the CPU restatement (fp64: the truth; fp32: the
    reference's own arithmetic) for the same loss: gradients of emb / color /
    dir / conf, every aggregator tensor and bg_color."""
    opt = sc["opt"]
    tp = {k: torch.from_numpy(np.ascontiguousarray(sc[k])).to(dt).requires_grad_(True)
          for k in ("emb", "color", "dir", "conf")}
    pp = {k: torch.from_numpy(v).to(dt).requires_grad_(True) for k, v in params.items()}
    bg = torch.from_numpy(sc["bg"]).to(dt).requires_grad_(True)
    pidx = torch.from_numpy(q["sample_pidx"]).long()
    mask = pidx >= 0
    idx = pidx.clamp(min=0).reshape(-1)
    shp = tuple(pidx.shape)
    xyz = torch.from_numpy(sc["xyz"]).to(dt)
    pers = torch.from_numpy(O.w2pers(sc["xyz"], sc["campos"], sc["camrot"])).to(dt)
    gsel = lambda a, c: a.reshape(-1, c)[idx].reshape(shp + (c,))  # noqa: E731
    rw = None if Rpp is None else torch.from_numpy(Rpp).to(dt).reshape(-1, 9)[idx].reshape(shp + (3, 3))
    feats, rv, w, confc = OG.aggregate(pp, gsel(tp["color"], 3), gsel(tp["dir"], 3), gsel(tp["conf"], 1),
                                       gsel(tp["emb"], 32), gsel(pers, 3), gsel(xyz, 3), mask,
                                       torch.from_numpy(q["sample_loc"]).to(dt),
                                       torch.from_numpy(q["sample_loc_w"]).to(dt),
                                       torch.from_numpy(q["sample_ray_dirs"]).to(dt), rw2c=rw)
    rdist = torch.from_numpy(O.ray_dist(q["sample_loc"], rv.numpy(), opt.vsize[2], opt.raydist_mode_unit)).to(dt)
    color, opacity, T, bw, bgT = OG.ray_march_full(rdist, rv, feats, bg)
    mk = torch.from_numpy(q["ray_mask"] > 0)
    R = mk.numel()
    full = bg[None, :].expand(R, -1).clone()            # fill_invalid (neural_points_volumetric_model.py:373-375)
    full = full.index_put((mk.nonzero()[:, 0],), color)
    out = dict(coarse_raycolor=full[None], ray_mask=mk[None].to(torch.int8), weight=w[None].detach(),
               blend_weight=bw[None, ..., None].detach(), conf_coefficient=confc[None])
    loss_fn(out).backward()
    return tp, pp, bg, out


def _losses(gt):
    """compute_losses of base_rendering_model.py:533-660 for the fork's flags:
    ray-masked MSE, plain MSE over all rays (misses show bg_color), 1e-4 x the
    zero-one loss of conf_coefficient (:630-641) and a sparse loss on weight /
    conf_coefficient (:653-657, weight 1e-3 here so its terms are exercised)."""
    def loss(out):
        c = out["coarse_raycolor"][..., :3]
        m = (out["ray_mask"] > 0)[..., None].expand(-1, -1, 3)
        g = gt.to(c.dtype).to(c.device)
        masked = torch.nn.functional.mse_loss(torch.masked_select(c, m), torch.masked_select(g, m))
        plain = torch.nn.functional.mse_loss(c, g)
        v = torch.clamp(out["conf_coefficient"], 1e-3, 1 - 1e-3)
        zero_one = torch.mean(torch.log(v) + torch.log(1 - v))
        w = out["weight"]
        sparse = torch.sum(w * torch.abs(1 - torch.exp(-2 * out["conf_coefficient"]))) / (torch.sum(w) + 1e-6)
        return masked + plain + 1e-4 * zero_one + 1e-3 * sparse
    return loss


def _check_grads(m, bg, o64, o32, label):
    """Every gradient against the fp64 oracle: per element within the
    test_gpu_backward tolerance, or -- where LeakyReLU kinks flip -- the kink
    bound below.  A pre-activation within fp32 noise of 0 takes the other slope
    in one of the two runs (a rotated per-point distance rounds differently on
    the GPU, whose mat3 fuses multiply-adds, than on the CPU); the pairs of that
    neuron then move their rows' gradients by a fraction of their size.  Such
    flips are few and local: at most 1e-4 of a tensor's entries may leave the
    element bound, none by more than 1 % of its largest entry, and the tensor's
    relative L2 error stays <= 1e-3 -- or the tensor's largest error is no
    more than twice the fp32 oracle's own (the flips the CPU shares)."""
    npts = m.neural_points
    got = {"points_embeding": (npts.points_embeding.grad.reshape(-1, 32), "emb", 5e-5),
           "points_color": (npts.points_color.grad.reshape(-1, 3), "color", 5e-5),
           "points_dir": (npts.points_dir.grad.reshape(-1, 3), "dir", 5e-5),
           "points_conf": (npts.points_conf.grad.reshape(-1, 1), "conf", 5e-5)}
    pairs = [(label + " d " + n, g, o64[0][k].grad, o32[0][k].grad, s) for n, (g, k, s) in got.items()]
    pairs += [(label + " d " + k, p.grad, o64[1][k].grad, o32[1][k].grad, 3e-4) for k, p in m.aggregator.named_parameters()]
    pairs.append((label + " d bg_color", bg.grad, o64[2].grad, o32[2].grad, 5e-5))
    for name, g, r64, r32, scale in pairs:
        try:
            close(g, r64, name, scale=scale)
        except AssertionError:
            gd = g.detach().cpu().double().reshape(r64.shape)
            d = (gd - r64).abs()
            e = float(d.max())
            e32 = float((r32.double() - r64).abs().max())
            big = float(r64.abs().max())
            if e <= 2.0 * e32 + 1e-6 * big:
                continue
            n_out = int((d > scale * big + 1e-4 * r64.abs()).sum())
            rel2 = float(d.norm() / max(float(r64.norm()), 1e-300))
            assert n_out <= max(1, int(1e-4 * d.numel())) and e <= 1e-2 * big and rel2 <= 1e-3, \
                (name, n_out, d.numel(), e, e32, big, rel2)


@pytest.mark.parametrize("rw", ["eye", "per_point"])
def test_reference_step_through_module_forward(cuda, rw):
    """model(...) in training mode: the output dict carries weight / blend_weight /
    conf_coefficient, compute_losses-style loss, backward: every gradient incl.
    bg_color vs the fp64 oracle."""
    sc = scene(20000, H=32, W=32, theta=140.0, default_conf=None)
    params = formula_params(salt=0.35)
    Rpp = _signed_perms(sc["xyz"].shape[0], 3) if rw == "per_point" else None
    m = _model(sc, cuda, params, Rw2c=Rpp, train=True)
    m.train()
    bg = torch.from_numpy(sc["bg"]).to(cuda).requires_grad_(True)
    gt = torch.rand((1, 32 * 32, 3), generator=torch.Generator().manual_seed(9))
    out = m(**_inputs(sc, cuda, bg=bg))
    for k in ("weight", "blend_weight", "conf_coefficient"):
        assert k in out, k
    assert not out["weight"].requires_grad and not out["blend_weight"].requires_grad
    assert out["conf_coefficient"].requires_grad
    loss_fn = _losses(gt)
    loss_fn(out).backward()
    q = O.query_points(sc["opt"], sc["xyz"], sc["campos"], sc["camrot"], sc["raydir"], near=2.0, far=6.0)
    *o64, ref = _oracle_step(sc, params, q, loss_fn, Rpp)
    *o32, _ = _oracle_step(sc, params, q, loss_fn, Rpp, dt=torch.float32)
    assert np.array_equal(out["ray_mask"].cpu().numpy(), ref["ray_mask"].numpy())
    Rv = int(ref["weight"].shape[1])
    assert out["weight"].shape == (1, Rv, sc["opt"].SR, sc["opt"].K)
    close(out["weight"], ref["weight"], "weight", scale=1e-6)
    # blend weights: 1 - exp(-sigma dist) of small sigma dist carries ~1e-7 absolute fp32 error
    close(out["blend_weight"], ref["blend_weight"], "blend_weight", rel=1e-4,
          scale=1e-7 / max(float(ref["blend_weight"].abs().max()), 1e-30))
    close(out["conf_coefficient"], ref["conf_coefficient"], "conf_coefficient", scale=1e-7)
    close(out["coarse_raycolor"], ref["coarse_raycolor"], "coarse_raycolor", scale=2e-5)
    _check_grads(m, bg, o64, o32, "module")


@pytest.mark.parametrize("rw", ["eye", "per_point"])
def test_reference_step_through_seams(cuda, rw):
    """The reference forward as its seams (neural_points_volumetric_model.py:288-389):
    NeuralPoints.forward (14-tuple, torch gathers of the point parameters) ->
    PointAggregator.forward (weight, conf_coefficient returned) -> ray_dist ->
    pointnerf_amd.ray_march (differentiable, bg_color) -> fill_invalid -> the
    compute_losses terms -> backward; every gradient vs the fp64 oracle."""
    from pointnerf_amd.ray_march import alpha_blend, radiance_render, ray_march
    sc = scene(20000, H=32, W=32, theta=140.0, default_conf=None)
    params = formula_params(salt=0.35)
    Rpp = _signed_perms(sc["xyz"].shape[0], 3) if rw == "per_point" else None
    m = _model(sc, cuda, params, Rw2c=Rpp, train=True)
    bg = torch.from_numpy(sc["bg"]).to(cuda).requires_grad_(True)
    inp = _inputs(sc, cuda, bg=bg)
    t = m.neural_points({"pixel_idx": None, "camrotc2w": inp["camrotc2w"], "campos": inp["campos"],
                         "near": inp["near"], "far": inp["far"], "focal": None, "h": 32, "w": 32,
                         "intrinsic": None, "gt_image": None, "raydir": inp["raydir"]})
    (s_color, s_Rw2c, s_dir, s_conf, s_emb, s_pers, s_xyz, s_mask, s_loc, s_loc_w, s_dirs, ray_mask,
     vsize, grid_vox_sz) = t
    assert s_emb.requires_grad
    feats, ray_valid, weight, conf = m.aggregator(s_color, s_Rw2c, s_dir, s_conf, s_emb, s_pers, s_xyz, s_mask,
                                                  s_loc, s_loc_w, s_dirs, vsize, grid_vox_sz)
    rd = torch.cummax(s_loc[..., 2], dim=-1)[0]
    rd = torch.cat([rd[..., 1:] - rd[..., :-1], torch.full(rd.shape[:2] + (1,), float(vsize[2]), device=cuda)], -1)
    msk = ((rd < 1e-8) | (rd > 2 * float(vsize[2]))).float()
    rd = (rd * (1 - msk) + msk * float(vsize[2])) * ray_valid.float()
    color, _, opacity, acc_T, blend_weight, bgT, _ = ray_march(rd, ray_valid, feats, radiance_render, alpha_blend,
                                                               bg)
    R = ray_mask.shape[1]
    mk = ray_mask[0] > 0
    full = bg[None, :].expand(R, -1).clone().index_put((mk.nonzero()[:, 0],), color[0])
    out = dict(coarse_raycolor=full[None], ray_mask=ray_mask, weight=weight.detach(),
               blend_weight=blend_weight.detach(), conf_coefficient=conf)
    gt = torch.rand((1, R, 3), generator=torch.Generator().manual_seed(9))
    loss_fn = _losses(gt)
    loss_fn(out).backward()
    q = O.query_points(sc["opt"], sc["xyz"], sc["campos"], sc["camrot"], sc["raydir"], near=2.0, far=6.0)
    *o64, ref = _oracle_step(sc, params, q, loss_fn, Rpp)
    *o32, _ = _oracle_step(sc, params, q, loss_fn, Rpp, dt=torch.float32)
    assert np.array_equal(ray_mask.cpu().numpy(), ref["ray_mask"].numpy())
    close(full, ref["coarse_raycolor"][0], "coarse_raycolor", scale=2e-5)
    _check_grads(m, bg, o64, o32, "seams")


def test_eval_forward_carries_aux_outputs(cuda):
    """Evaluation forward (no_grad): the same keys (the reference's aggregator
    returns them whenever a loss reads them, point_aggregators.py:814-815), equal
    to the training forward's values; without those flags the keys are absent."""
    sc = scene(20000, H=24, W=24, theta=40.0, default_conf=None)
    params = formula_params(salt=0.5)
    m = _model(sc, cuda, params, train=True)
    with torch.no_grad():
        ev = m.eval()(**_inputs(sc, cuda))
    tr = m.train()(**_inputs(sc, cuda))
    for k in ("weight", "blend_weight", "conf_coefficient"):
        close(ev[k], tr[k], k, scale=1e-6)
    m.opt.zero_one_loss_items = []
    with torch.no_grad():
        ev2 = m.eval()(**_inputs(sc, cuda))
    assert "weight" not in ev2 and "conf_coefficient" not in ev2
