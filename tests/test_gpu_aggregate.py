"""libpnr aggregation (gather + weights + PE + MFMA MLP + K-sums + colour MLP)
vs the reference's golden vectors and vs the CPU oracle.
Tolerance (north_star "stated fp32 tolerance"): |d| <= 1e-4 + 1e-4*|ref|."""
import os

import numpy as np
import pytest
import torch

from formula import formula_params
from oracle import oracle as O
from scenes import oracle_points, scene

pytestmark = pytest.mark.gpu
ATOL, RTOL = 1e-4, 1e-4


def _agg_with(params, cuda, **over):
    from pointnerf_amd.aggregator import PointAggregator
    from pointnerf_amd.options import lego_opt
    agg = PointAggregator(lego_opt(**over)).to(cuda)
    agg.load_state_dict({k: torch.from_numpy(v) for k, v in params.items()})
    agg.eval()
    return agg


def test_state_dict_names_match_reference():
    from pointnerf_amd.aggregator import PointAggregator
    from pointnerf_amd.options import lego_opt
    from formula import LEGO_SHAPES
    sd = PointAggregator(lego_opt()).state_dict()
    want = {f"{n}.weight": s for n, s in LEGO_SHAPES.items()}
    want.update({f"{n}.bias": (s[0],) for n, s in LEGO_SHAPES.items()})
    assert {k: tuple(v.shape) for k, v in sd.items()} == want


def test_pointaggregator_forward_vs_reference_golden(golden_dir, cuda):
    g = np.load(os.path.join(golden_dir, "aggregator.npz"), allow_pickle=False)
    agg = _agg_with(formula_params(), cuda)
    t = {k: torch.from_numpy(np.ascontiguousarray(g[k])).to(cuda) for k in g.files}
    with torch.no_grad():
        f, rv, w, cc = agg(t["sampled_color"], torch.eye(3, device=cuda), t["sampled_dir"], t["sampled_conf"],
                           t["sampled_embedding"], t["sampled_xyz_pers"], t["sampled_xyz"], t["sample_pnt_mask"],
                           t["sample_loc"], t["sample_loc_w"], t["sample_ray_dirs"], [0.004] * 3, 0)
    assert torch.equal(rv.cpu(), torch.from_numpy(g["ray_valid"]))
    np.testing.assert_allclose(f.cpu().numpy(), g["features"], atol=ATOL, rtol=RTOL)
    np.testing.assert_allclose(w.cpu().numpy(), g["weight"], atol=1e-6, rtol=1e-5)
    np.testing.assert_allclose(cc.cpu().numpy(), g["conf_coefficient"], atol=1e-7, rtol=0)


def test_pointaggregator_random_weights_vs_oracle(cuda):
    # default (xavier) init, random inputs incl. K < 8 valid neighbours
    from pointnerf_amd.aggregator import PointAggregator
    from pointnerf_amd.options import lego_opt
    torch.manual_seed(0)
    agg = PointAggregator(lego_opt()).to(cuda).eval()
    params = {k: v.detach().cpu().numpy() for k, v in agg.state_dict().items()}
    rng = np.random.default_rng(5)
    R, SR, K = 9, 17, 8
    mask = rng.uniform(size=(1, R, SR, K)) < 0.55
    sw = rng.uniform(-0.5, 0.5, size=(1, R, SR, 3)).astype(np.float32)
    sx = (sw[..., None, :] + rng.normal(scale=0.01, size=(1, R, SR, K, 3))).astype(np.float32)
    cam, rot = np.array([0.1, -3.9, 1.5], np.float32), np.eye(3, dtype=np.float32)
    inp = dict(sampled_color=rng.normal(size=(1, R, SR, K, 3)), sampled_dir=rng.normal(size=(1, R, SR, K, 3)),
               sampled_conf=rng.uniform(size=(1, R, SR, K, 1)),
               sampled_embedding=rng.uniform(-0.5, 0.5, size=(1, R, SR, K, 32)),
               sampled_xyz_pers=O.w2pers(sx, cam, rot), sampled_xyz=sx, sample_loc=O.w2pers(sw, cam, rot),
               sample_loc_w=sw, sample_ray_dirs=np.broadcast_to(rng.normal(size=(1, R, 1, 3)), (1, R, SR, 3)))
    inp = {k: np.ascontiguousarray(v, dtype=np.float32) for k, v in inp.items()}
    t = {k: torch.from_numpy(v).to(cuda) for k, v in inp.items()}
    with torch.no_grad():
        f, rv, w, cc = agg(t["sampled_color"], None, t["sampled_dir"], t["sampled_conf"], t["sampled_embedding"],
                           t["sampled_xyz_pers"], t["sampled_xyz"], torch.from_numpy(mask).to(cuda),
                           t["sample_loc"], t["sample_loc_w"], t["sample_ray_dirs"], [0.004] * 3, 0)
    ref = O.aggregate(params, inp["sampled_color"][0], None, inp["sampled_dir"][0], inp["sampled_conf"][0],
                      inp["sampled_embedding"][0], inp["sampled_xyz_pers"][0], inp["sampled_xyz"][0], mask[0],
                      inp["sample_loc"][0], inp["sample_loc_w"][0], inp["sample_ray_dirs"][0])
    np.testing.assert_allclose(f.cpu().numpy()[0], ref[0], atol=ATOL, rtol=RTOL)
    assert np.array_equal(rv.cpu().numpy()[0], ref[1])


def test_fused_gather_aggregate_vs_oracle(cuda):
    # the renderer's fused path: point-table gather inside the kernel from pidx
    from pointnerf_amd import _lib as L
    from pointnerf_amd.renderer import NeuralPoints
    sc = scene(20000, H=40, W=40, default_conf=None)
    torch.manual_seed(1)
    agg = _agg_with(formula_params(salt=0.3), cuda)
    np_ = NeuralPoints(sc["opt"], cuda, torch.from_numpy(sc["xyz"]), torch.from_numpy(sc["emb"]),
                       torch.from_numpy(sc["color"]), torch.from_numpy(sc["dir"]), torch.from_numpy(sc["conf"]))
    rd = torch.from_numpy(sc["raydir"]).to(cuda)
    cp, cr = torch.from_numpy(sc["campos"]).to(cuda), torch.from_numpy(sc["camrot"]).to(cuda)
    bufs, hp, rays, qp = np_.querier.run(np_.xyz.detach(), rd, cp, cr, 2.0, 6.0)
    c = bufs.read_counts()
    Sv, SR, K = c["S_valid"], sc["opt"].SR, sc["opt"].K
    feat = torch.zeros((Sv, 129), device=cuda)
    mlp, _k = agg.packed()
    pts, _p = np_.tables(cp, cr)
    s = L.Samples(bufs.valid_list.data_ptr(), bufs.counts.data_ptr() + 4, Sv, bufs.pidx.data_ptr(),
                  bufs.sample_w.data_ptr(), bufs.sample_p.data_ptr(), rd.data_ptr(), bufs.fill_rs.data_ptr(), SR, K)
    scratch = L.aggregate_scratch(Sv, pts.n, cuda)
    L.check(L.lib().pnr_aggregate_fwd(L.ctypes.byref(pts), L.ctypes.byref(s), L.ctypes.byref(mlp), L.ptr(feat),
                                      None, None, L.ptr(scratch), scratch.numel() * 4, L.stream_ptr()),
            "aggregate")
    # oracle: reference query -> gather -> aggregate, then pick the valid samples in the same order
    q = O.query_points(sc["opt"], sc["xyz"], sc["campos"], sc["camrot"], sc["raydir"], near=2.0, far=6.0)
    gth = O.gather(oracle_points(sc), q["sample_pidx"], sc["campos"], sc["camrot"])
    ref, rv, _, _ = O.aggregate(formula_params(salt=0.3), gth["sampled_color"], None, gth["sampled_dir"],
                                gth["sampled_conf"], gth["sampled_embedding"], gth["sampled_xyz_pers"],
                                gth["sampled_xyz"], gth["sample_pnt_mask"], q["sample_loc"], q["sample_loc_w"],
                                q["sample_ray_dirs"])
    want = ref[rv]                      # valid samples in (ray, slot) order == valid_list order
    assert want.shape[0] == Sv
    np.testing.assert_allclose(feat.cpu().numpy(), want, atol=ATOL, rtol=RTOL)
