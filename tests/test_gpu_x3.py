"""fp32-accurate split aggregation vs the CPU oracle: pnr_aggregate_fwd_x3
(3-way bf16 split, six products) and pnr_aggregate_fwd_h2 (2-way f16 split,
three products).

Same tolerance as the fp32 path (north_star "stated fp32 tolerance"):
|d| <= 1e-4 + 1e-4*|ref| against the fp32 oracle, rendered colour within 2e-4
and PSNR >= 60 dB.  Accuracy claim: against the oracle evaluated in float64
(its F32 dtype switched to float64 for the MLP, PE and K-sums), the split path's
error is no larger than about that of the native fp32 MFMA path."""
import contextlib

import numpy as np
import pytest
import torch

from formula import formula_params
from oracle import oracle as O
from scenes import oracle_points, scene

pytestmark = pytest.mark.gpu
ATOL, RTOL = 1e-4, 1e-4


@contextlib.contextmanager
def _oracle_f64():
    old = O.F32
    O.F32 = np.float64
    try:
        yield
    finally:
        O.F32 = old


def _setup(sc, cuda, params=None, seed=0):
    from pointnerf_amd.aggregator import PointAggregator
    from pointnerf_amd.renderer import NeuralPoints
    torch.manual_seed(seed)
    agg = PointAggregator(sc["opt"]).to(cuda)
    if params is not None:
        agg.load_state_dict({k: torch.from_numpy(v) for k, v in params.items()})
    np_ = NeuralPoints(sc["opt"], cuda, torch.from_numpy(sc["xyz"]), torch.from_numpy(sc["emb"]),
                       torch.from_numpy(sc["color"]), torch.from_numpy(sc["dir"]), torch.from_numpy(sc["conf"]))
    return agg.eval(), np_


SPLITS = ["x3", "h2"]


def _both(agg, np_, sc, cuda, used=False, variant="x3", check_range=True, scratch_fill=None):
    """fp32 and split-path features on one query -> (f32 [Sv,129], split [Sv,129]);
    used: P1 only for the referenced points (the training-batch layout)."""
    from pointnerf_amd import _lib as L
    cp, cr = torch.from_numpy(sc["campos"]).to(cuda), torch.from_numpy(sc["camrot"]).to(cuda)
    rd = torch.from_numpy(sc["raydir"]).to(cuda).contiguous()
    bufs, hp, rays, qp = np_.querier.run(np_.xyz.detach(), rd, cp, cr, 2.0, 6.0)
    cnt = bufs.read_counts()
    Sv = cnt["S_valid"]
    s = L.Samples(bufs.valid_list.data_ptr(), bufs.counts.data_ptr() + 4, Sv, bufs.pidx.data_ptr(),
                  bufs.sample_w.data_ptr(), bufs.sample_p.data_ptr(), rd.data_ptr(), bufs.fill_rs.data_ptr(),
                  sc["opt"].SR, sc["opt"].K)
    pts, _keep = np_.tables(cp, cr)
    n_p1 = pts.n
    if used:
        from pointnerf_amd.train import used_points
        u = used_points(bufs.pidx[:cnt["S_filled"] * sc["opt"].K], pts.n)
        pts.used, pts.n_used, pts.used_map = u[0].data_ptr(), u[0].numel(), u[1].data_ptr()
        n_p1 = u[0].numel()
    mlp, _k1 = agg.packed()
    mlpx, _k2 = agg.packed_x3() if variant == "x3" else agg.packed_h2()
    outs = []
    for fn, extra in (("pnr_aggregate_fwd", ()), (f"pnr_aggregate_fwd_{variant}", (L.ctypes.byref(mlpx),))):
        f = torch.zeros((Sv, 129), device=cuda)
        scr = L.aggregate_scratch(Sv, n_p1, cuda)
        if scratch_fill is not None:
            scr.fill_(scratch_fill)
        L.check(getattr(L.lib(), fn)(L.ctypes.byref(pts), L.ctypes.byref(s), L.ctypes.byref(mlp), *extra, L.ptr(f),
                                     None, None, L.ptr(scr), scr.numel() * 4, L.stream_ptr(cuda)), fn)
        outs.append(f)
    torch.cuda.synchronize()
    if variant == "h2" and check_range:
        assert agg.h2_range_ok()
    _keep_used = u if used else None   # noqa: F841 (keeps the used tables alive until here)
    return outs[0].cpu().numpy(), outs[1].cpu().numpy()


def _oracle_features(sc, params, f64=False):
    """Oracle query + gather in fp32 (as the reference), then the aggregator in
    fp32 or, with f64, in float64 on the same fp32 inputs."""
    q = O.query_points(sc["opt"], sc["xyz"], sc["campos"], sc["camrot"], sc["raydir"], near=2.0, far=6.0)
    gth = O.gather(oracle_points(sc), q["sample_pidx"], sc["campos"], sc["camrot"])
    with _oracle_f64() if f64 else contextlib.nullcontext():
        if f64:
            params = {k: v.astype(np.float64) for k, v in params.items()}
        ref, rv, _, _ = O.aggregate(params, gth["sampled_color"], None, gth["sampled_dir"], gth["sampled_conf"],
                                    gth["sampled_embedding"], gth["sampled_xyz_pers"], gth["sampled_xyz"],
                                    gth["sample_pnt_mask"], q["sample_loc"], q["sample_loc_w"],
                                    q["sample_ray_dirs"])
    return np.asarray(ref)[rv]


@pytest.mark.parametrize("variant", SPLITS)
def test_x3_used_subset_equals_full(cuda, variant):
    """P1 for the referenced points only (pts.used, the training layout) gives
    bit-identical features to P1 for every point."""
    sc = scene(20000, H=40, W=40, default_conf=None)
    agg, np_ = _setup(sc, cuda, formula_params(salt=0.4))
    _, a = _both(agg, np_, sc, cuda, variant=variant)
    _, b = _both(agg, np_, sc, cuda, used=True, variant=variant)
    assert np.array_equal(a, b)


@pytest.mark.parametrize("variant", SPLITS)
@pytest.mark.parametrize("salt", [0.3, None])
def test_x3_features_vs_oracle_fp32_and_fp64(cuda, salt, variant):
    """salt 0.3: closed-form weights (tests/golden/formula.py); None: the
    aggregator's own random init (xavier, networks.py:163-172)."""
    sc = scene(20000, H=40, W=40, default_conf=None)
    agg, np_ = _setup(sc, cuda, None if salt is None else formula_params(salt=salt))
    params = {k: v.detach().cpu().numpy() for k, v in agg.state_dict().items()}
    f32, x3 = _both(agg, np_, sc, cuda, variant=variant)
    want = _oracle_features(sc, params)
    assert want.shape == x3.shape and want.shape[0] > 500
    np.testing.assert_allclose(x3, want, atol=ATOL, rtol=RTOL)
    want64 = _oracle_features(sc, params, f64=True)
    assert want64.dtype == np.float64 and want64.shape == x3.shape
    e32 = np.abs(f32.astype(np.float64) - want64)
    ex3 = np.abs(x3.astype(np.float64) - want64)
    scale = np.abs(want64).max()
    print(f"\nerr vs f64 (max, rms) / max|ref| {scale:.3g}: fp32 {e32.max():.3g} {np.sqrt((e32 ** 2).mean()):.3g}"
          f"  fp32{variant} {ex3.max():.3g} {np.sqrt((ex3 ** 2).mean()):.3g}")
    assert ex3.max() <= 2.0 * e32.max() + 1e-7 * scale
    assert np.sqrt((ex3 ** 2).mean()) <= 1.5 * np.sqrt((e32 ** 2).mean()) + 1e-8 * scale


@pytest.mark.parametrize("variant", SPLITS)
def test_x3_render_vs_oracle(cuda, variant):
    from pointnerf_amd.renderer import NeuralPointsRayMarching
    sc = scene(30000, H=48, W=48, theta=200.0, default_conf=None)
    params = formula_params(salt=0.1)
    agg, np_ = _setup(sc, cuda, params)
    m = NeuralPointsRayMarching(sc["opt"], np_, agg, precision="fp32" + variant)
    args = [torch.from_numpy(sc[k]).to(cuda) for k in ("campos", "camrot", "raydir")]
    with torch.no_grad():
        c, op, bg, mask = m.render_rays(*args, 2.0, 6.0, torch.from_numpy(sc["bg"]).to(cuda))
        c2 = m.render_rays(*args, 2.0, 6.0, torch.from_numpy(sc["bg"]).to(cuda))[0]
    assert torch.equal(c, c2)            # deterministic
    ref = O.render(sc["opt"], oracle_points(sc), params, sc["campos"], sc["camrot"], sc["raydir"], sc["bg"])
    assert np.array_equal(mask.cpu().numpy(), ref["ray_mask"])
    x, y = c.cpu().numpy(), ref["coarse_raycolor"]
    np.testing.assert_allclose(x, y, atol=2e-4, rtol=1e-4)
    psnr = 10 * np.log10(float(np.abs(y).max()) ** 2 / max(float(np.mean((x - y) ** 2)), 1e-30))
    assert psnr >= 60.0, psnr


@pytest.mark.parametrize("variant", ["h2"])
def test_h2_large_weights_prescaled(cuda, variant):
    """Weights far above the f16 range of 2^11 Wh are pre-scaled in the pack
    (scale = 2^(s-11)); features stay within the fp32 tolerance."""
    sc = scene(20000, H=32, W=32, default_conf=None)
    params = formula_params(salt=0.3)
    params = dict(params)
    for k in ("block1.2.weight", "block3.2.weight"):
        params[k] = params[k] * np.float32(64.0)   # |W| up to ~64x: s > 0 for those layers
    for k in ("block3.0.weight", "block3.0.bias"):
        params[k] = params[k] / np.float32(64.0)   # keep activations O(1)
    for k in ("color_branch.0.weight",):
        params[k] = params[k] / np.float32(64.0)
    params["color_branch.2.weight"] = params["color_branch.2.weight"] * np.float32(64.0)   # colour pack s > 0
    params["color_branch.4.weight"] = params["color_branch.4.weight"] / np.float32(64.0)
    agg, np_ = _setup(sc, cuda, params)
    f32, h2 = _both(agg, np_, sc, cuda, variant=variant)
    want = _oracle_features(sc, {k: v.detach().cpu().numpy() for k, v in agg.state_dict().items()})
    np.testing.assert_allclose(h2, want, atol=ATOL, rtol=RTOL)


def test_h2_range_flag_and_fallback(cuda):
    """An activation beyond the f16 range sets the launch's range flag; the
    renderer then renders the call again on fp32x3 (bf16 split: same accuracy,
    fp32 range) -- bit-identical to an fp32x3 render -- and keeps h2 off for
    those weights until they change."""
    from pointnerf_amd.renderer import NeuralPointsRayMarching
    sc = scene(20000, H=32, W=32, default_conf=None)
    agg, np_ = _setup(sc, cuda, formula_params(salt=0.3))
    m = NeuralPointsRayMarching(sc["opt"], np_, agg, precision="fp32h2")
    mx = NeuralPointsRayMarching(sc["opt"], np_, agg, precision="fp32x3")
    args = [torch.from_numpy(sc[k]).to(cuda) for k in ("campos", "camrot", "raydir")]
    bg = torch.from_numpy(sc["bg"]).to(cuda)
    with torch.no_grad():
        m.render_rays(*args, 2.0, 6.0, bg)
        assert agg.h2_range_ok() and m.h2_fallbacks == 0
        agg.block1[2].bias.fill_(1e6)            # block1.2 outputs ~1e6 > 65504 (repacked: new version)
        got = m.render_rays(*args, 2.0, 6.0, bg)
        assert m.h2_fallbacks == 1 and agg.h2_range_ok()   # flag consumed by the fallback
        want = mx.render_rays(*args, 2.0, 6.0, bg)
        for a, b in zip(got, want):
            assert torch.equal(a, b)
        again = m.render_rays(*args, 2.0, 6.0, bg)   # blocked weights: straight to fp32x3
        assert m.h2_fallbacks == 1 and agg.h2_range_ok()
        for a, b in zip(again, want):
            assert torch.equal(a, b)
        agg.block1[2].bias.fill_(0.0)            # new weights: h2 again, no trip
        m.render_rays(*args, 2.0, 6.0, bg)
        assert m.h2_fallbacks == 1 and m._h2_blocked_key is None and agg.h2_range_ok()


def test_h2_mixed_sync_and_async_calls_keep_range_check(cuda):
    """a synchronous render_rays issued while sync=False calls are
    pending completes them first, so a pending call whose activations left the
    f16 range is re-rendered on fp32x3 (none is returned invalid); re-rendering
    after the weights changed raises instead of silently using new weights."""
    from pointnerf_amd import _lib as L
    from pointnerf_amd.renderer import NeuralPointsRayMarching
    sc = scene(20000, H=32, W=32, default_conf=None)
    agg, np_ = _setup(sc, cuda, formula_params(salt=0.3))
    m = NeuralPointsRayMarching(sc["opt"], np_, agg, precision="fp32h2")
    mx = NeuralPointsRayMarching(sc["opt"], np_, agg, precision="fp32x3")
    args = [torch.from_numpy(sc[k]).to(cuda) for k in ("campos", "camrot", "raydir")]
    bg = torch.from_numpy(sc["bg"]).to(cuda)
    with torch.no_grad():
        m.render_rays(*args, 2.0, 6.0, bg)             # first call: synchronous, sizes the buffers
        agg.block1[2].bias.fill_(1e6)                   # every h2 launch now overflows
        pend = m.render_rays(*args, 2.0, 6.0, bg, sync=False)
        assert len(m._pending) == 1
        sync_out = m.render_rays(*args, 2.0, 6.0, bg)   # must finish the pending call first
        assert not m._pending and m.h2_fallbacks >= 1
        want = mx.render_rays(*args, 2.0, 6.0, bg)
        for a, b, c in zip(pend, sync_out, want):
            assert torch.equal(a, c) and torch.equal(b, c)
        # weights changed between an overflowing sync=False call and finish(): refuse
        agg.block1[2].bias.fill_(0.0)
        m.render_rays(*args, 2.0, 6.0, bg)              # h2 again (new weights)
        agg.block1[2].bias.fill_(1e6)
        m.render_rays(*args, 2.0, 6.0, bg, sync=False)
        agg.block1[2].bias.fill_(2e6)
        with pytest.raises(L.PnrError):
            m.finish()


@pytest.mark.parametrize("variant", ["h2"])
def test_h2_raw_launch_sets_range_flag(cuda, variant):
    """pnr_aggregate_fwd_h2 itself: out-of-range activation -> *range_flag = 1."""
    sc = scene(20000, H=32, W=32, default_conf=None)
    agg, np_ = _setup(sc, cuda, formula_params(salt=0.3))
    with torch.no_grad():
        agg.block1[2].bias.fill_(1e6)
    _both(agg, np_, sc, cuda, variant=variant, check_range=False)
    assert not agg.h2_range_ok()


def test_h2_colour_branch_overflow_sets_flag(cuda):
    """Overflow only inside the colour branch (k_color_h2): colour layer-1
    outputs ~1e6 leave the f16 range -> non-finite outputs -> range flag."""
    sc = scene(20000, H=32, W=32, default_conf=None)
    agg, np_ = _setup(sc, cuda, formula_params(salt=0.3))
    with torch.no_grad():
        agg.color_branch[0].bias.fill_(1e6)
    _both(agg, np_, sc, cuda, variant="h2", check_range=False)
    assert not agg.h2_range_ok()
    agg.h2_reset_range()
    with torch.no_grad():
        agg.color_branch[0].bias.fill_(0.0)
    _both(agg, np_, sc, cuda, variant="h2")   # asserts the flag stays clear


@pytest.mark.parametrize("variant", ["h2"])
def test_h2_stale_scratch_ignored(cuda, variant):
    """k_color_h2 copies the f16-split hid planes of whole 64-sample tiles; rows
    past n (and of samples without a neighbour) are never written by k_pairs_h2.
    Scratch full of NaN must change neither the features (bit for bit) nor the
    range flag (_both asserts it stays clear)."""
    sc = scene(20000, H=32, W=32, default_conf=None)
    agg, np_ = _setup(sc, cuda, formula_params(salt=0.3))
    _, poisoned = _both(agg, np_, sc, cuda, variant=variant, scratch_fill=float("nan"))
    _, clean = _both(agg, np_, sc, cuda, variant=variant, scratch_fill=0.0)
    assert poisoned.shape[0] % 64 != 0   # a partial last tile is exercised
    assert np.array_equal(poisoned, clean)
