"""Host-side logic: weight packing, hyperparameters, flag set, synthetic data."""
import numpy as np
import torch

from oracle import oracle as O


def test_frag_pack_roundtrip_and_layout():
    from pointnerf_amd.aggregator import frag_pack, frag_unpack
    W, b = torch.randn(256, 263), torch.randn(256)
    F = frag_pack(W, b)
    assert F.numel() == (132 + 8) * 8 * 64          # 263 + bias = 132 k-steps, +8 prefetch padding
    assert torch.equal(frag_unpack(F, 264), torch.cat([W, b[:, None]], 1))
    Wc, bc = torch.randn(128, 280), torch.randn(128)
    assert torch.equal(frag_unpack(frag_pack(Wc, bc), 281, 128), torch.cat([Wc, bc[:, None]], 1))
    assert frag_pack(torch.randn(256, 284), torch.randn(256)).numel() == (143 + 8) * 8 * 64
    # F[t][T][lane] = W[32T + (lane & 31)][2t + (lane >> 5)]
    Fv = F.view(140, 8, 64)
    assert torch.all(Fv[132:] == 0)
    for t, T, lane in [(0, 0, 0), (5, 3, 17), (131, 7, 40), (77, 2, 63)]:
        k = 2 * t + (lane >> 5)
        want = W[32 * T + (lane & 31), k] if k < 263 else (b[32 * T + (lane & 31)] if k == 263 else 0.0)
        assert float(Fv[t, T, lane]) == float(want)


def test_hyperparameters_match_oracle():
    from pointnerf_amd.options import lego_opt
    from pointnerf_amd.querier import hyperparameters_from_bbox
    from pointnerf_amd import synthetic as S
    opt = lego_opt()
    for n, seed in [(5000, 0), (30000, 1)]:
        pts = S.lego_like_points(n, seed=seed)
        a = hyperparameters_from_bbox(opt, pts.min(0), pts.max(0))
        b = O.get_hyperparameters(O.lego_opt(), pts)
        for k in ("ranges", "shift", "vsize_s", "dims", "radius_limit2"):
            assert np.array_equal(a[k], b[k]), k
    # no ranges (ranges[0] >= ranges[3] disables clipping, qpiw.py:61-62)
    pts = np.random.default_rng(0).uniform(-0.3, 0.3, size=(1000, 3)).astype(np.float32)
    a = hyperparameters_from_bbox(lego_opt(ranges=[1, 1, 1, 0, 0, 0]), pts.min(0), pts.max(0))
    b = O.get_hyperparameters(O.lego_opt(ranges=[1, 1, 1, 0, 0, 0]), pts)
    assert np.array_equal(a["dims"], b["dims"]) and np.array_equal(a["shift"], b["shift"])


def test_lego_flags():
    from pointnerf_amd.options import lego_opt
    o = lego_opt()
    assert (o.SR, o.K, o.P, o.max_o, o.z_depth_dim) == (80, 8, 9, 830000, 400)
    assert o.vsize == [0.004] * 3 and o.vscale == [2, 2, 2] and o.kernel_size == [3, 3, 3]
    assert lego_opt(query_size=[0, 0, 0]).query_size == [3, 3, 3]   # neural_points.py:329


def test_tvals_mirror_equals_oracle():
    from pointnerf_amd.querier import ray_mid_t
    assert np.array_equal(ray_mid_t(2.0, 6.0, 400)[0].numpy(), O.ray_mid_t(2.0, 6.0, 400)[0])


def test_synthetic_points_respect_voxel_capacity():
    from pointnerf_amd import synthetic as S
    pts = S.lego_like_points(50000, seed=2)
    g = O.grid_build(O.lego_opt(), pts)
    assert g["occ_numpnts"].max() <= 8 < O.lego_opt().P
    assert g["n_occ"] < O.lego_opt().max_o
    campos, camrot = S.camera(0.0, -30.0, 4.0)
    # camera looks at the origin: the centre pixel ray passes near it
    d = S.pixel_rays(2, 2, 1000.0, camrot)[0]
    t = -np.dot(campos, d) / np.dot(d, d)
    assert np.linalg.norm(campos + t * d) < 0.05


def test_product_fails_loudly_without_gpu():
    import pytest
    from pointnerf_amd import _lib as L
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    with pytest.raises(L.PnrError):
        L.require_gpu()
    from pointnerf_amd.querier import lighting_fast_querier
    from pointnerf_amd.options import lego_opt
    with pytest.raises(L.PnrError):
        lighting_fast_querier(torch.device("cpu"), lego_opt())


def test_frag_pack_h2_split_exactness():
    """frag_pack_h2: Wh + 2^-11 Wl reproduces the pre-scaled weights within
    2^-24 relative (f16 normal range), scale = 2^(s-11) with 8 <= max|W' 2^-s| < 16
    (small layers scaled up, s < 0), and the zero padding steps are zero."""
    import torch
    from pointnerf_amd.aggregator import H2_PAD, frag_pack_h2, h2_shift
    g = torch.Generator().manual_seed(0)
    assert h2_shift(torch.zeros(4, 4)) == 0
    for mag in (1e-4, 0.1, 40.0):
        W = torch.randn(256, 60, generator=g) * mag
        b = torch.randn(256, generator=g) * mag
        F, scale = frag_pack_h2(W, b)
        s = round(np.log2(scale)) + 11
        amax = float(torch.cat([W, b[:, None]], 1).abs().max())
        assert 8 <= amax * 2.0 ** -s < 16
        if mag < 1:
            assert s < 0
        tot = (61 + 15) // 16 + H2_PAD
        P = F.view(tot, 8, 2, 2, 32, 8).float()            # [t][T][pl][h][r][j]
        rec = P[:, :, 0] + P[:, :, 1] / 2048.0               # [t][T][h][r][j]
        rec = rec.permute(1, 3, 0, 2, 4).reshape(256, 16 * tot)
        want = torch.cat([W, b[:, None]], 1) * 2.0 ** -s
        err = (rec[:, :61].double() - want.double()).abs()
        assert float((err - 2.0 ** -23 * want.double().abs()).max()) <= 2.0 ** -35
        assert float(rec[:, 61:].abs().max()) == 0.0


def test_flagsets_match_scene_scripts():
    """options.FLAGSETS = the values dev_scripts/{w_n360/ship, w_scannet_etf/scene101,
    w_tt_ft/truck}.sh pass (the BASELINE c3 / c4 / c5 scenes)."""
    from pointnerf_amd.options import flagset_opt
    s = flagset_opt("ship")
    assert (s.P, s.max_o, s.SR, s.kernel_size, s.vsize) == (10, 1500000, 80, [3, 3, 3], [0.004] * 3)
    assert s.ranges == [-1.277, -1.300, -0.550, 1.371, 1.349, 0.729]
    c = flagset_opt("scene101")
    assert (c.SR, c.P, c.max_o, c.near_plane, c.far_plane, c.vsize) == (24, 30, 2000000, 0.1, 8.0, [0.008] * 3)
    t = flagset_opt("truck")
    assert (t.kernel_size, t.query_size, t.vsize, t.SR, t.P, t.near_plane, t.far_plane) == \
        ([5, 5, 5], [3, 3, 3], [0.002] * 3, 40, 10, 0.0, 3.5)
    assert flagset_opt("lego").P == 9


def test_scene_points_cap_and_fixed_bbox():
    """Synthetic flag-set clouds never overflow P (the reference's reservoir on
    overflow has no reproducible result) and their grid is the one the cap used."""
    from pointnerf_amd import synthetic as S
    from pointnerf_amd.options import flagset_opt
    for name, n in [("ship", 20000), ("scene101", 40000), ("truck", 30000)]:
        o = flagset_opt(name)
        p = S.scene_points(name, n, o, seed=2)
        assert p.shape == (n, 3) and p.dtype == np.float32
        g = O.grid_build(o, p)
        assert g["occ_numpnts"].max() <= o.P - 1
        assert np.all(p >= np.asarray(o.ranges[:3], np.float32)) and np.all(p <= np.asarray(o.ranges[3:], np.float32))



def test_grid_handle_finaliser_defers_destroy():
    """GridHandle.__del__ issues no HIP call (a finaliser may run inside someone's
    graph capture, GPUTEST_r04): the handle lands on querier._DEFERRED and is
    destroyed at the next safe point (release_deferred)."""
    import ctypes
    import gc
    from pointnerf_amd import querier as Q
    h = Q.GridHandle.__new__(Q.GridHandle)
    h.h = ctypes.c_void_p(0x1234)      # never dereferenced: the test takes it back below
    h.self_ref = h                     # a reference cycle: freed by the collector, not by refcount
    n0 = len(Q._DEFERRED)
    del h
    gc.collect()
    assert len(Q._DEFERRED) == n0 + 1
    assert Q._DEFERRED.pop().value == 0x1234
    Q._CAPTURES[0] += 1                # a capture in progress: nothing is released
    try:
        Q._DEFERRED.append(ctypes.c_void_p(0x5678))
        assert Q.release_deferred() == 0 and len(Q._DEFERRED) == n0 + 1
    finally:
        Q._CAPTURES[0] -= 1
        Q._DEFERRED.pop()
