"""The five BASELINE configs and the reference flag sets on the HIP path.

BASELINE.json configs (SURVEY 8(d) "Configs as concrete inputs"):
  c1  lego, 50 k points, 100x100 (focal / 8)          -> full frame vs the oracle
  c2  lego, ~500 k points, 800x800 forward            -> full-size properties + oracle ray sample
  c3  ship flags (ship.sh), ~2 M points, fwd + bwd    -> finetune-batch gradients vs oracle_grad
  c4  scene101 flags (scene101.sh: vsize .008, SR 24, P 30, near .1, far 8)
  c5  truck flags (truck.sh: kernel 5 = three Chebyshev shells, vsize .002, near 0, SR 40)
The c4 / c5 flag sets run at oracle-coverable sizes (their full sizes are 8-GPU
configs); c5 also through the bf16 path.  Query results are bit-exact vs the
oracle (integer / index work); decoded features and renders within the fp32
tolerance of the other render tests: |d| <= 2e-4 + 1e-4 |ref| and PSNR(build
vs oracle) >= 60 dB (bf16: >= 40 dB)."""
import functools

import numpy as np
import pytest
import torch

from formula import formula_params
from oracle import oracle as O
from oracle import oracle_grad as OG
from scenes import flag_scene, oracle_points, scene

pytestmark = pytest.mark.gpu

# oracle-coverable point counts that still put 1-8 neighbours in most samples
DENSE = {"ship": 300_000, "scene101": 600_000, "truck": 400_000}
PRECISIONS = ["fp32", "fp32x3", "fp32h2"]


@functools.lru_cache(maxsize=None)
def _flag_scene(name, n, H, view=1):
    return flag_scene(name, n, H=H, view=view)


@functools.lru_cache(maxsize=None)
def _oracle_query(name, n, H, view=1):
    sc = _flag_scene(name, n, H, view)
    return O.query_points(sc["opt"], sc["xyz"], sc["campos"], sc["camrot"], sc["raydir"],
                          near=sc["near"], far=sc["far"])


def _model(sc, cuda, params, precision="fp32", train=False, emb_dtype=torch.float32):
    from pointnerf_amd.aggregator import PointAggregator
    from pointnerf_amd.renderer import NeuralPoints, NeuralPointsRayMarching
    agg = PointAggregator(sc["opt"]).to(cuda)
    agg.load_state_dict({k: torch.from_numpy(v) for k, v in params.items()})
    np_ = NeuralPoints(sc["opt"], cuda, torch.from_numpy(sc["xyz"]), torch.from_numpy(sc["emb"]),
                       torch.from_numpy(sc["color"]), torch.from_numpy(sc["dir"]), torch.from_numpy(sc["conf"]),
                       emb_dtype=emb_dtype)
    m = NeuralPointsRayMarching(sc["opt"], np_, agg.train() if train else agg.eval(), precision=precision)
    m.train_precision = "fp32x3"   # the strict oracle comparisons; fp32h2 (the default) has its own tests
    return m


def _render(m, sc, cuda, rd=None):
    rd = sc["raydir"] if rd is None else rd
    near = sc.get("near", 2.0)
    far = sc.get("far", 6.0)
    with torch.no_grad():
        out = m.render_rays(torch.from_numpy(sc["campos"]).to(cuda), torch.from_numpy(sc["camrot"]).to(cuda),
                            torch.from_numpy(np.ascontiguousarray(rd)).to(cuda), near, far,
                            torch.from_numpy(sc["bg"]).to(cuda))
    return [t.cpu() for t in out]


def _psnr(a, b):
    mse = float(np.mean((np.asarray(a, np.float64) - np.asarray(b, np.float64)) ** 2))
    peak = float(np.abs(b).max())
    return 10 * np.log10(peak ** 2 / max(mse, 1e-30))


def _check_render(got, ref, min_psnr=60.0, tol=True):
    assert np.array_equal(got[3].numpy(), ref["ray_mask"])
    if tol:
        np.testing.assert_allclose(got[0].numpy(), ref["coarse_raycolor"], atol=2e-4, rtol=1e-4)
        np.testing.assert_allclose(got[1].numpy(), ref["coarse_point_opacity"], atol=2e-4, rtol=1e-4)
        np.testing.assert_allclose(got[2].numpy(), ref["coarse_is_background"][:, 0], atol=2e-4, rtol=1e-4)
    m = ref["ray_mask"] > 0
    assert _psnr(got[0].numpy()[m], ref["coarse_raycolor"][m]) >= min_psnr


# ------------------------------------------------------------ c3/c4/c5 flag sets
@pytest.mark.parametrize("name", ["ship", "scene101", "truck"])
def test_flagset_grid_and_query_bit_exact(cuda, name):
    """Grid tables and every query output bit-identical to the oracle at the
    scene script's flags (truck: kernel_size 5 -> the generic layer loop of
    k_knn, qpiw.py:481-527, three shells with the per-layer break)."""
    from pointnerf_amd.querier import lighting_fast_querier
    sc = _flag_scene(name, DENSE[name], 48)
    ref = _oracle_query(name, DENSE[name], 48)
    q = lighting_fast_querier(cuda, sc["opt"])
    xyz = torch.from_numpy(sc["xyz"]).to(cuda)
    hp = q.grid.build(sc["opt"], xyz)
    g = ref["grid"]
    assert np.array_equal(hp["dims"], g["hp"]["dims"]) and np.array_equal(hp["shift"], g["hp"]["shift"])
    t = q.grid.export()
    assert np.array_equal(t["coor_2_occ"].cpu().numpy(), g["coor_2_occ"])
    bits = t["occ_bits"].cpu().numpy().view(np.uint32)
    occ = ((bits[:, None] >> np.arange(32, dtype=np.uint32)) & 1).reshape(-1)[: g["coor_occ"].size]
    assert np.array_equal(occ.astype(np.uint8), g["coor_occ"])
    assert np.array_equal(t["occ_numpnts"].cpu().numpy(), g["occ_numpnts"])
    assert np.array_equal(t["occ_2_pnts"].cpu().numpy(), g["occ_2_pnts"])
    assert q.grid.stats()["n_points_dropped"] == 0
    rd = torch.from_numpy(sc["raydir"]).to(cuda)
    out = q.query_points(None, None, xyz[None], None, 0, 0, None, sc["near"], sc["far"], rd[None],
                         torch.from_numpy(sc["campos"]).to(cuda)[None], torch.from_numpy(sc["camrot"]).to(cuda)[None])
    pidx, loc, loc_w, dirs, ray_mask = [x.cpu().numpy()[0] for x in out[:5]]
    assert ref["ray_mask"].sum() > 500, "scene must exercise the query"
    assert np.array_equal(ray_mask, ref["ray_mask"])
    assert np.array_equal(pidx, ref["sample_pidx"])            # same neighbours, same order
    assert np.array_equal(loc_w, ref["sample_loc_w"])
    assert np.array_equal(loc, ref["sample_loc"])
    assert np.array_equal(dirs, ref["sample_ray_dirs"])
    full = (ref["sample_pidx"] >= 0).sum(-1) == sc["opt"].K
    assert full.sum() > 500, "too few samples with K neighbours: the replacement rule is not exercised"


def test_truck_kernel5_reaches_the_third_shell(cuda):
    """The generic loop's outer shell (layer 2) really contributes neighbours:
    a kernel-3 query of the same truck scene finds fewer."""
    from pointnerf_amd.querier import lighting_fast_querier
    sc = _flag_scene("truck", DENSE["truck"], 48)
    ref5 = _oracle_query("truck", DENSE["truck"], 48)
    opt3 = type(sc["opt"])(**{**vars(sc["opt"]), "kernel_size": [3, 3, 3]})
    q = lighting_fast_querier(cuda, opt3)
    xyz = torch.from_numpy(sc["xyz"]).to(cuda)
    rd = torch.from_numpy(sc["raydir"]).to(cuda)
    out = q.query_points(None, None, xyz[None], None, 0, 0, None, sc["near"], sc["far"], rd[None],
                         torch.from_numpy(sc["campos"]).to(cuda)[None], torch.from_numpy(sc["camrot"]).to(cuda)[None])
    n3 = int((out[0] >= 0).sum())
    n5 = int((ref5["sample_pidx"] >= 0).sum())
    assert n5 > n3


@pytest.mark.parametrize("precision", PRECISIONS)
@pytest.mark.parametrize("name", ["ship", "scene101", "truck"])
def test_flagset_render_vs_oracle(cuda, name, precision):
    sc = _flag_scene(name, DENSE[name], 48)
    params = formula_params(salt=0.35)
    m = _model(sc, cuda, params, precision)
    got = _render(m, sc, cuda)
    ref = O.render(sc["opt"], oracle_points(sc), params, sc["campos"], sc["camrot"], sc["raydir"], sc["bg"],
                   q=_oracle_query(name, DENSE[name], 48))
    _check_render(got, ref)
    assert getattr(m, "h2_fallbacks", 0) == 0


@pytest.mark.parametrize("emb_dtype", [torch.float32, torch.bfloat16])
def test_c5_truck_bf16_vs_oracle(cuda, emb_dtype):
    """c5: bf16 point features (the embedding table itself stored in bf16:
    104 B per point) + bf16 MFMA MLP at truck flags -- same query (bit-exact
    ray mask), image within 40 dB PSNR of the fp32 oracle; the fp32 paths
    render a bf16 table from its fp32 copy."""
    sc = _flag_scene("truck", DENSE["truck"], 48)
    params = formula_params(salt=0.35)
    m = _model(sc, cuda, params, "bf16", emb_dtype=emb_dtype)
    assert m.neural_points.bytes_per_point() == (104 if emb_dtype == torch.bfloat16 else 168)
    got = _render(m, sc, cuda)
    ref = O.render(sc["opt"], oracle_points(sc), params, sc["campos"], sc["camrot"], sc["raydir"], sc["bg"],
                   q=_oracle_query("truck", DENSE["truck"], 48))
    _check_render(got, ref, min_psnr=40.0, tol=False)
    if emb_dtype == torch.bfloat16:   # fp32 path on the same bf16 table = the oracle on bf16-rounded embeddings
        m.precision = "fp32"
        got32 = _render(m, sc, cuda)
        pts = dict(oracle_points(sc), emb=torch.from_numpy(sc["emb"]).bfloat16().float().numpy())
        ref32 = O.render(sc["opt"], pts, params, sc["campos"], sc["camrot"], sc["raydir"], sc["bg"],
                         q=_oracle_query("truck", DENSE["truck"], 48))
        _check_render(got32, ref32)


# ------------------------------------------------------------------------- c1
@pytest.mark.parametrize("precision", ["fp32", "fp32h2"])
def test_c1_lego_50k_100x100_full_frame(cuda, precision):
    """c1: 50 k points, the full 100x100 frame (focal 1111.1 / 8) vs the oracle."""
    sc = scene(50_000, H=100, W=100, theta=30.0, default_conf=0.15)
    params = formula_params(salt=0.45)
    got = _render(_model(sc, cuda, params, precision), sc, cuda)
    ref = O.render(sc["opt"], oracle_points(sc), params, sc["campos"], sc["camrot"], sc["raydir"], sc["bg"])
    assert ref["ray_mask"].sum() > 2000
    _check_render(got, ref)


# ------------------------------------------------------------------------- c2
@functools.lru_cache(maxsize=None)
def _c2_scene():
    return scene(500_000, H=800, W=800, theta=-100.0, default_conf=0.15)


@pytest.mark.parametrize("precision", PRECISIONS)
def test_c2_lego_500k_800_properties_and_oracle_sample(cuda, precision):
    """c2: ~500 k points, 800x800: bitwise repeatable, ray-independent, and 256
    random rays of the frame vs the oracle (full cloud, full grid)."""
    sc = _c2_scene()
    params = formula_params(salt=0.65)
    m = _model(sc, cuda, params, precision)
    a = _render(m, sc, cuda)
    b = _render(m, sc, cuda)
    for x, y in zip(a, b):
        assert torch.equal(x, y)
    c = m.last_counts
    assert c["R_valid"] > 100_000 and c["n_pairs"] > 2_000_000, c
    rng = np.random.default_rng(11)
    sel = np.sort(rng.choice(800 * 800, size=2048, replace=False))
    sub = _render(m, sc, cuda, sc["raydir"][sel])
    for x, y in zip(sub, a):
        assert torch.equal(x, y[torch.from_numpy(sel)])
    few = sel[::8]
    ref = O.render(sc["opt"], oracle_points(sc), params, sc["campos"], sc["camrot"], sc["raydir"][few], sc["bg"])
    assert ref["ray_mask"].sum() > 60
    _check_render([t[torch.from_numpy(few)] for t in a], ref)


# ------------------------------------------------------------------------- c3
@pytest.mark.parametrize("train_precision", ["fp32x3", "fp32h2"])
def test_c3_ship_finetune_batch_grads_vs_oracle(cuda, train_precision):
    """c3: ship flags, ~2 M points, one finetune batch of 3 600 random rays of an
    800x800 frame (random_sample_size 60): forward + backward through the HIP
    kernels; ray colours and every point-table / MLP gradient vs torch autograd
    of the CPU oracle (tolerances of test_gpu_backward.py).

    fp32h2 (the training default) is held to a stated contract instead of the
    strict bound: its per-layer error (~10x fp32 rounding) puts a few more
    LeakyReLU pre-activations on the other side of 0 than fp32 does, and each
    such kink flip changes one (pair, neuron) term by a factor 0.2 / 1.  Per
    tensor: at most 1e-5 of the entries (>= 16) outside the strict fp32 bound,
    the whole tensor within 0.5 % of fp64 in relative L2 norm, and no entry more
    than 6 % of the tensor's largest entry away (measured on this batch, round 6:
    6 of 4.8 M point-table entries outside, max 4.8 % (points_color), L2 <= 0.39 %,
    every MLP weight gradient inside the strict bound; the kernels are
    deterministic, so the numbers repeat -- round 5 allowed 0.1 %, 1 % and 10 %;
    DESIGN.md section 10)."""
    from test_gpu_backward import close
    sc = flag_scene("ship", 2_000_000, H=800, view=3, default_conf=None)
    params = formula_params(salt=0.15)
    m = _model(sc, cuda, params, train=True)
    m.train_precision = train_precision
    rng = np.random.default_rng(5)
    sel = np.sort(rng.choice(800 * 800, size=3600, replace=False))
    rdn = np.ascontiguousarray(sc["raydir"][sel])
    campos, camrot = torch.from_numpy(sc["campos"]).to(cuda), torch.from_numpy(sc["camrot"]).to(cuda)
    bg = torch.from_numpy(sc["bg"]).to(cuda)
    color, _, _, ray_mask = m.render_rays_train(campos, camrot, torch.from_numpy(rdn).to(cuda), sc["near"],
                                                 sc["far"], bg)
    G = torch.randn(color.shape, generator=torch.Generator().manual_seed(9)).to(cuda)
    (color * G).sum().backward()
    opt = sc["opt"]
    q = O.query_points(opt, sc["xyz"], sc["campos"], sc["camrot"], rdn, near=sc["near"], far=sc["far"])
    assert np.array_equal(ray_mask.cpu().numpy(), q["ray_mask"])
    assert q["ray_mask"].sum() > 500
    # the oracle differentiates only the referenced point rows (same gradient, less CPU work),
    # once in fp32 (the reference's arithmetic) and once in fp64 (the truth both are measured on)
    pidx = torch.from_numpy(q["sample_pidx"]).long()
    used = torch.unique(pidx[pidx >= 0])
    remap = torch.full((sc["xyz"].shape[0],), -1, dtype=torch.long)
    remap[used] = torch.arange(used.numel())
    lp = torch.where(pidx >= 0, remap[pidx.clamp(min=0)], torch.zeros_like(pidx))
    mask = pidx >= 0
    sub = lambda a: np.ascontiguousarray(np.asarray(a)[used.numpy()])  # noqa: E731
    idx = lp.reshape(-1)
    shp = tuple(lp.shape)
    mk = torch.from_numpy(q["ray_mask"] > 0)

    def oracle(dt):
        tp = {k: torch.from_numpy(sub(sc[k])).to(dt).requires_grad_(True) for k in ("emb", "color", "dir", "conf")}
        pp = {k: torch.from_numpy(v).to(dt).requires_grad_(True) for k, v in params.items()}
        xyz = torch.from_numpy(sub(sc["xyz"])).to(dt)
        pers = torch.from_numpy(O.w2pers(sub(sc["xyz"]), sc["campos"], sc["camrot"])).to(dt)
        gsel = lambda a, c: a.reshape(-1, c)[idx].reshape(shp + (c,))  # noqa: E731
        feats, rv, _, _ = OG.aggregate(pp, gsel(tp["color"], 3), gsel(tp["dir"], 3), gsel(tp["conf"], 1),
                                       gsel(tp["emb"], 32), gsel(pers, 3), gsel(xyz, 3), mask,
                                       torch.from_numpy(q["sample_loc"]).to(dt),
                                       torch.from_numpy(q["sample_loc_w"]).to(dt),
                                       torch.from_numpy(q["sample_ray_dirs"]).to(dt))
        rdist = torch.from_numpy(O.ray_dist(q["sample_loc"], rv.numpy(), opt.vsize[2], opt.raydist_mode_unit))
        c_ref = OG.ray_march(rdist.to(dt), rv, feats, torch.from_numpy(sc["bg"]).to(dt))
        (c_ref * G.cpu().to(dt)[mk]).sum().backward()
        g = {"points_embeding": tp["emb"].grad, "points_color": tp["color"].grad, "points_dir": tp["dir"].grad,
             "points_conf": tp["conf"].grad}
        g.update({k: p.grad for k, p in pp.items()})
        return c_ref.detach(), g

    c32, g32 = oracle(torch.float32)
    c64, g64 = oracle(torch.float64)
    close(color[mk.to(cuda)], c32, "ray_color", rel=1e-4, scale=2e-5)
    npts = m.neural_points
    u = used.to(cuda)
    got = {"points_embeding": npts.points_embeding.grad.reshape(-1, 32)[u],
           "points_color": npts.points_color.grad.reshape(-1, 3)[u],
           "points_dir": npts.points_dir.grad.reshape(-1, 3)[u], "points_conf": npts.points_conf.grad.reshape(-1, 1)[u]}
    got.update({k: p.grad for k, p in m.aggregator.named_parameters()})
    # Tolerance: the batch's gradients are sums over ~1e5 (sample, neighbour) terms of
    # random sign (G ~ N(0,1)), so fp32 summation error is large relative to the
    # cancelled result; the HIP backward must be within 4x the error the reference's
    # own fp32 arithmetic makes (the CPU fp32 oracle vs fp64), + 1e-4 relative, + a
    # max|ref|-scaled term for LeakyReLU kinks (a pre-activation within fp32 noise of
    # 0 takes the other slope; 5e-5 point tables, 3e-4 MLP weights as in
    # test_gpu_backward.py).
    errs, contract = [], []
    for k, ref in g64.items():
        a = got[k].detach().cpu().double().numpy()
        r = ref.numpy()
        e32 = float(np.abs(g32[k].double().numpy() - r).max())
        kink = (5e-5 if k.startswith("points_") else 3e-4) * float(np.abs(r).max())
        bad = np.abs(a - r) > 4 * e32 + 1e-4 * np.abs(r) + kink
        if train_precision == "fp32h2":
            rel_l2 = float(np.linalg.norm(a - r) / max(np.linalg.norm(r), 1e-300))
            rel_max = float(np.abs(a - r).max() / np.abs(r).max())
            ok = bad.sum() <= max(16, 1e-5 * bad.size) and rel_l2 <= 5e-3 and rel_max <= 0.06
            contract.append((k, int(bad.sum()), bad.size, round(rel_max, 5), rel_l2))
            if not ok:
                errs.append(f"d {k}: {bad.sum()} / {bad.size} outside the fp32 bound, max |d| / max |ref| "
                            f"{rel_max:.3e}, |d| / |ref| {rel_l2:.3e}")
        elif bad.any():
            errs.append(f"d {k}: {bad.sum()} / {bad.size} outside, max |d| {np.abs(a - r).max():.3e} vs fp32-oracle "
                        f"error {e32:.3e}, max |ref| {np.abs(r).max():.3e}")
    untouched = torch.ones(npts.points_embeding.shape[1], dtype=torch.bool, device=cuda)
    untouched[u] = False
    assert float(npts.points_embeding.grad.reshape(-1, 32)[untouched].abs().max()) == 0.0
    if contract:
        print("fp32h2 gradient contract (tensor, entries outside the fp32 bound, size, max |d| / max |ref|):",
              contract)
    assert not errs, errs
