"""bf16-MFMA aggregation (pnr_aggregate_fwd_bf16, SURVEY config c5) against the
fp32 path / CPU oracle.

Tolerance (bf16 operands, 8-bit mantissa, fp32 accumulation): decoded
features within 2 % relative RMS and |d| <= 5 % of the tensor's max; the
rendered image within 40 dB PSNR of the fp32 oracle.  The query is shared
with the fp32 path, so ray masks are identical."""
import numpy as np
import pytest
import torch

from formula import formula_params
from oracle import oracle as O
from scenes import oracle_points, scene

pytestmark = pytest.mark.gpu


def _setup(sc, cuda, params=None):
    from pointnerf_amd.aggregator import PointAggregator
    from pointnerf_amd.renderer import NeuralPoints
    agg = PointAggregator(sc["opt"]).to(cuda)
    if params is not None:
        agg.load_state_dict({k: torch.from_numpy(v) for k, v in params.items()})
    np_ = NeuralPoints(sc["opt"], cuda, torch.from_numpy(sc["xyz"]), torch.from_numpy(sc["emb"]),
                       torch.from_numpy(sc["color"]), torch.from_numpy(sc["dir"]), torch.from_numpy(sc["conf"]))
    return agg.eval(), np_


def _features(agg, np_, sc, cuda, used=False):
    """Both aggregate paths on one query; returns (fp32 feat, bf16 feat)."""
    from pointnerf_amd import _lib as L
    cp, cr = torch.from_numpy(sc["campos"]).to(cuda), torch.from_numpy(sc["camrot"]).to(cuda)
    rd = torch.from_numpy(sc["raydir"]).to(cuda).contiguous()
    bufs, hp, rays, qp = np_.querier.run(np_.xyz.detach(), rd, cp, cr, 2.0, 6.0)
    cnt = bufs.read_counts()
    Sv, K = cnt["S_valid"], sc["opt"].K
    s = L.Samples(bufs.valid_list.data_ptr(), bufs.counts.data_ptr() + 4, Sv, bufs.pidx.data_ptr(),
                  bufs.sample_w.data_ptr(), bufs.sample_p.data_ptr(), rd.data_ptr(), bufs.fill_rs.data_ptr(),
                  sc["opt"].SR, K)
    pts, keep = np_.tables(cp, cr)
    n_p1 = pts.n
    if used:
        from pointnerf_amd.train import used_points
        u = used_points(bufs.pidx[:cnt["S_filled"] * K], pts.n)
        pts.used, pts.n_used, pts.used_map = u[0].data_ptr(), u[0].numel(), u[1].data_ptr()
        n_p1 = u[0].numel()
    f32 = torch.zeros((Sv, 129), device=cuda)
    f16 = torch.zeros((Sv, 129), device=cuda)
    mlp, _k1 = agg.packed()
    sc32 = L.aggregate_scratch(Sv, n_p1, cuda)
    L.check(L.lib().pnr_aggregate_fwd(L.ctypes.byref(pts), L.ctypes.byref(s), L.ctypes.byref(mlp), L.ptr(f32),
                                      None, None, L.ptr(sc32), sc32.numel() * 4, L.stream_ptr(cuda)), "fp32")
    mlp16, _k2 = agg.packed_bf16()
    sc16 = L.aggregate_scratch_bf16(Sv, n_p1, cuda)
    L.check(L.lib().pnr_aggregate_fwd_bf16(L.ctypes.byref(pts), L.ctypes.byref(s), L.ctypes.byref(mlp16),
                                           L.ptr(f16), None, None, L.ptr(sc16), sc16.numel() * 4,
                                           L.stream_ptr(cuda)), "bf16")
    torch.cuda.synchronize()
    return f32.cpu().numpy(), f16.cpu().numpy(), Sv


@pytest.mark.parametrize("used", [False, True])
def test_bf16_features_vs_fp32(cuda, used):
    sc = scene(30000, H=48, W=48, theta=30.0)
    torch.manual_seed(0)
    agg, np_ = _setup(sc, cuda)          # random xavier weights (networks.py:163-172)
    a, b, Sv = _features(agg, np_, sc, cuda, used=used)
    assert Sv > 1000
    for name, sl in (("alpha", slice(0, 1)), ("color", slice(1, 129))):
        d = np.abs(a[:, sl] - b[:, sl])
        r = np.abs(a[:, sl])
        assert np.sqrt((d ** 2).mean() / (r ** 2).mean()) < 0.02, name
        assert d.max() <= 0.05 * r.max(), name


def test_bf16_render_vs_oracle(cuda):
    from pointnerf_amd.renderer import NeuralPointsRayMarching
    sc = scene(30000, H=48, W=48, theta=200.0)
    params = formula_params(salt=0.1)
    agg, np_ = _setup(sc, cuda, params)
    m = NeuralPointsRayMarching(sc["opt"], np_, agg, precision="bf16")
    with torch.no_grad():
        c, op, bg, mask = m.render_rays(torch.from_numpy(sc["campos"]).to(cuda),
                                        torch.from_numpy(sc["camrot"]).to(cuda),
                                        torch.from_numpy(sc["raydir"]).to(cuda), 2.0, 6.0,
                                        torch.from_numpy(sc["bg"]).to(cuda))
        c2, _, _, _ = m.render_rays(torch.from_numpy(sc["campos"]).to(cuda), torch.from_numpy(sc["camrot"]).to(cuda),
                                    torch.from_numpy(sc["raydir"]).to(cuda), 2.0, 6.0,
                                    torch.from_numpy(sc["bg"]).to(cuda))
    assert torch.equal(c, c2)            # deterministic
    ref = O.render(sc["opt"], oracle_points(sc), params, sc["campos"], sc["camrot"], sc["raydir"], sc["bg"])
    assert np.array_equal(mask.cpu().numpy(), ref["ray_mask"])
    x, y = c.cpu().numpy(), ref["coarse_raycolor"]
    psnr = 10 * np.log10(float(np.abs(y).max()) ** 2 / max(float(np.mean((x - y) ** 2)), 1e-30))
    assert psnr >= 40.0, psnr


@pytest.mark.parametrize("flags", ["truck", "lego"])
def test_bf16_pair_buckets_equal_unbucketed(cuda, flags):
    """pair_buckets (samples on KT = 1/2/4/8-slot tiles by their last filled
    neighbour slot, buckets.hip) computes the same numbers as the 16 x 8 tiles:
    features, out_weight and out_conf bitwise equal -- on a truck-flag scene
    (~2 neighbours per sample, every bucket populated) and a lego one."""
    from pointnerf_amd import _lib as L
    from scenes import flag_scene
    sc = flag_scene(flags, n_points=60000 if flags == "truck" else 30000, H=64, view=0)
    agg, np_ = _setup(sc, cuda, formula_params(salt=0.6))
    cp, cr = torch.from_numpy(sc["campos"]).to(cuda), torch.from_numpy(sc["camrot"]).to(cuda)
    rd = torch.from_numpy(sc["raydir"]).to(cuda).contiguous()
    bufs, hp, rays, qp = np_.querier.run(np_.xyz.detach(), rd, cp, cr, sc["near"], sc["far"])
    cnt = bufs.read_counts()
    Sv, K = cnt["S_valid"], sc["opt"].K
    assert Sv > 1000
    s = L.Samples(bufs.valid_list.data_ptr(), bufs.counts.data_ptr() + 4, Sv, bufs.pidx.data_ptr(),
                  bufs.sample_w.data_ptr(), bufs.sample_p.data_ptr(), rd.data_ptr(), bufs.fill_rs.data_ptr(),
                  sc["opt"].SR, K)
    pts, keep = np_.tables(cp, cr)
    outs = []
    for bk in (False, True):
        agg.pair_buckets = bk
        mlp16, _k = agg.packed_bf16()
        f = torch.full((Sv, 129), float("nan"), device=cuda)
        rows = bufs.pidx.numel() // K
        w = torch.full((rows, K), -1.0, device=cuda)
        c = torch.full((rows, K), -1.0, device=cuda)
        scr = L.aggregate_scratch_bf16(Sv, pts.n, cuda)
        L.check(L.lib().pnr_aggregate_fwd_bf16(L.ctypes.byref(pts), L.ctypes.byref(s), L.ctypes.byref(mlp16),
                                               L.ptr(f), L.ptr(w), L.ptr(c), L.ptr(scr), scr.numel() * 4,
                                               L.stream_ptr(cuda)), "bf16")
        outs.append((f, w, c))
    torch.cuda.synchronize()
    (f0, w0, c0), (f1, w1, c1) = outs
    assert torch.equal(torch.nan_to_num(f0, nan=7.0), torch.nan_to_num(f1, nan=7.0))
    assert torch.equal(w0, w1) and torch.equal(c0, c1)
    # the scene exercises the small buckets
    pidx = bufs.pidx[:cnt["S_filled"] * K].view(-1, K)
    need = ((pidx >= 0) * torch.arange(1, K + 1, device=cuda)).amax(1)
    if flags == "truck":
        assert int((need <= 1).sum()) > 100 and int(((need > 2) & (need <= 4)).sum()) > 100


@pytest.mark.parametrize("flags", ["truck", "lego"])
def test_bf16_p1_used_only_equals_all_points(cuda, flags):
    """P1 (block1.0's point half) computed only for the points the batch
    references (pnr_used_points; pnr_points.used without used_map: the table stays
    indexed by point row) renders bitwise like P1 for every point; repeated
    calls with other cameras never reuse the partial table."""
    from pointnerf_amd.renderer import NeuralPointsRayMarching
    from scenes import flag_scene
    sc = flag_scene(flags, n_points=60000 if flags == "truck" else 30000, H=64, view=0)
    sc2 = flag_scene(flags, n_points=60000 if flags == "truck" else 30000, H=64, view=1)
    agg, np_ = _setup(sc, cuda, formula_params(salt=0.6))
    m = NeuralPointsRayMarching(sc["opt"], np_, agg, precision="bf16")
    bg = torch.from_numpy(sc["bg"]).to(cuda)
    outs = {}
    for used_only in (False, True):
        m.p1_used_only = used_only
        for tag, s in (("a", sc), ("b", sc2), ("a2", sc)):
            o = m.render_rays(torch.from_numpy(s["campos"]).to(cuda), torch.from_numpy(s["camrot"]).to(cuda),
                              torch.from_numpy(s["raydir"]).to(cuda), s["near"], s["far"], bg)
            outs[(used_only, tag)] = [t.clone() for t in o]
    assert int(outs[(True, "a")][3].sum()) > 100
    for tag in ("a", "b", "a2"):
        for x, y in zip(outs[(False, tag)], outs[(True, tag)]):
            assert torch.equal(x, y), tag


@pytest.mark.parametrize("flags", ["truck", "lego"])
def test_bf16_render_variant_equals_general(cuda, flags):
    """k_pairs_b's render variant (no per-point Rw2c / used_map / ray_cam /
    out_weight / out_conf: those branches compiled out, aggregate_bf16.hip GEN)
    computes the features of the general-path variant a call with out_weight /
    out_conf runs, bucketed and unbucketed: the same samples written, alpha
    within 2^-20 of its maximum, at most 0.1 % of the features one bf16 input
    step apart (round 5 allowed 1 %: hipcc contracted different products into
    FMAs per instantiation; aggregate_bf16.hip is now compiled with
    -ffp-contract=off)."""
    from pointnerf_amd import _lib as L
    from scenes import flag_scene
    sc = flag_scene(flags, n_points=60000 if flags == "truck" else 30000, H=64, view=0)
    agg, np_ = _setup(sc, cuda, formula_params(salt=0.6))
    cp, cr = torch.from_numpy(sc["campos"]).to(cuda), torch.from_numpy(sc["camrot"]).to(cuda)
    rd = torch.from_numpy(sc["raydir"]).to(cuda).contiguous()
    bufs, hp, rays, qp = np_.querier.run(np_.xyz.detach(), rd, cp, cr, sc["near"], sc["far"])
    cnt = bufs.read_counts()
    Sv, K = cnt["S_valid"], sc["opt"].K
    assert Sv > 1000
    s = L.Samples(bufs.valid_list.data_ptr(), bufs.counts.data_ptr() + 4, Sv, bufs.pidx.data_ptr(),
                  bufs.sample_w.data_ptr(), bufs.sample_p.data_ptr(), rd.data_ptr(), bufs.fill_rs.data_ptr(),
                  sc["opt"].SR, K)
    pts, keep = np_.tables(cp, cr)
    rows = bufs.pidx.numel() // K
    for bk in (True, False):
        agg.pair_buckets = bk
        mlp16, _k = agg.packed_bf16()
        outs = []
        for general in (False, True):
            f = torch.full((Sv, 129), float("nan"), device=cuda)
            w = torch.empty((rows, K), device=cuda) if general else None
            c = torch.empty((rows, K), device=cuda) if general else None
            scr = L.aggregate_scratch_bf16(Sv, pts.n, cuda)
            L.check(L.lib().pnr_aggregate_fwd_bf16(L.ctypes.byref(pts), L.ctypes.byref(s), L.ctypes.byref(mlp16),
                                                   L.ptr(f), L.ptr(w) if general else None,
                                                   L.ptr(c) if general else None, L.ptr(scr), scr.numel() * 4,
                                                   L.stream_ptr(cuda)), "bf16")
            outs.append(f)
        torch.cuda.synchronize()
        assert torch.equal(torch.isnan(outs[0]), torch.isnan(outs[1])), bk   # same samples written
        a, b = torch.nan_to_num(outs[0], nan=7.0), torch.nan_to_num(outs[1], nan=7.0)
        # aggregate_bf16.hip is compiled without FMA contraction (Makefile): the two
        # instantiations no longer contract different products into FMAs (round 5:
        # up to 1.3e-3 of the entries differed).  A last-bit difference of the fp32
        # accumulators is left (alpha, fp32 from the block3.2 accumulators, shows it:
        # <= 2^-22 of its maximum); it flips the bf16 rounding of a later GEMM input in
        # a few entries (measured: truck none, lego 6.9e-5 of the entries, by one bf16
        # step of the input carried to the outputs of its sample)
        d = (a - b).abs()
        frac = float((d > 0).float().mean())
        rel = float(d.max()) / float(a.abs().max())
        print(f"buckets={bk}: differing {frac:.2e} of the entries, max |d| / max |f| = {rel:.2e}")
        assert float(d[:, 0].max()) <= 2.0 ** -20 * float(a[:, 0].abs().max()), (bk, float(d[:, 0].max()))
        assert rel <= 2.0 ** -7 and frac <= 1e-3, (bk, frac, rel)
        assert int(torch.isfinite(outs[0][:, 0]).sum()) > 1000


@pytest.mark.parametrize("flags", ["truck", "lego"])
def test_bf16_feature_rows_are_rounded_fp32_rows(cuda, flags):
    """pnr_aggregate_fwd_bf16_hf (ABI 20): the alpha of every written row equals
    pnr_aggregate_fwd_bf16's bitwise, each feature is the round-to-nearest-even
    bf16 of its fp32 feature, and the unwritten rows are the same."""
    from pointnerf_amd import _lib as L
    from scenes import flag_scene
    sc = flag_scene(flags, n_points=60000 if flags == "truck" else 30000, H=64, view=0)
    agg, np_ = _setup(sc, cuda, formula_params(salt=0.6))
    cp, cr = torch.from_numpy(sc["campos"]).to(cuda), torch.from_numpy(sc["camrot"]).to(cuda)
    rd = torch.from_numpy(sc["raydir"]).to(cuda).contiguous()
    bufs, hp, rays, qp = np_.querier.run(np_.xyz.detach(), rd, cp, cr, sc["near"], sc["far"])
    cnt = bufs.read_counts()
    Sv, K = cnt["S_valid"], sc["opt"].K
    s = L.Samples(bufs.valid_list.data_ptr(), bufs.counts.data_ptr() + 4, Sv, bufs.pidx.data_ptr(),
                  bufs.sample_w.data_ptr(), bufs.sample_p.data_ptr(), rd.data_ptr(), bufs.fill_rs.data_ptr(),
                  sc["opt"].SR, K)
    pts, keep = np_.tables(cp, cr)
    mlp16, _k = agg.packed_bf16()
    f = torch.full((Sv, 129), float("nan"), device=cuda)
    fh = torch.full((Sv, L.FEAT_H_PITCH), -1, dtype=torch.int16, device=cuda)
    for fn, out in ((L.lib().pnr_aggregate_fwd_bf16, f), (L.lib().pnr_aggregate_fwd_bf16_hf, fh)):
        scr = L.aggregate_scratch_bf16(Sv, pts.n, cuda)
        L.check(fn(L.ctypes.byref(pts), L.ctypes.byref(s), L.ctypes.byref(mlp16), L.ptr(out), None, None, L.ptr(scr),
                   scr.numel() * 4, L.stream_ptr(cuda)), "bf16")
    torch.cuda.synchronize()
    written = ~torch.isnan(f[:, 0])
    assert int(written.sum()) > 1000
    assert torch.equal(~torch.isnan(f[:, 1:]).any(1), written)
    alpha_h = fh[:, :2].contiguous().view(torch.float32)[:, 0]
    assert torch.equal(alpha_h[written], f[written, 0])
    assert bool((fh[~written, :2] == -1).all())   # rows the kernel skipped stay untouched
    want = f[written, 1:].to(torch.bfloat16).view(torch.int16)
    assert torch.equal(fh[written, 8:8 + 128], want)


def test_bf16_render_with_bf16_features(cuda):
    """The bf16 render path with bf16 feature rows (pnr_composite_fwd_hf) against
    the same path with fp32 rows: one feature rounding apart (<= 2^-8 relative
    per feature, blended in fp32)."""
    from pointnerf_amd.renderer import NeuralPointsRayMarching
    from scenes import flag_scene
    sc = flag_scene("truck", n_points=60000, H=64, view=0)
    agg, np_ = _setup(sc, cuda, formula_params(salt=0.6))
    m = NeuralPointsRayMarching(sc["opt"], np_, agg, precision="bf16")
    cp, cr = torch.from_numpy(sc["campos"]).to(cuda), torch.from_numpy(sc["camrot"]).to(cuda)
    rd = torch.from_numpy(sc["raydir"]).to(cuda).contiguous()
    bg = torch.rand(128, generator=torch.Generator().manual_seed(3)).to(cuda)
    outs = []
    for hf in (False, True):
        m.bf16_features = hf
        outs.append([t.clone() for t in m.render_rays(cp, cr, rd, sc["near"], sc["far"], bg)])
    (c0, o0, b0, k0), (c1, o1, b1, k1) = outs
    assert torch.equal(k0, k1) and torch.equal(o0, o1) and torch.equal(b0, b1)   # alpha path unchanged
    d = (c0 - c1).abs()
    assert float(d.max()) <= 2 ** -7 * float(c0.abs().max()), float(d.max())
