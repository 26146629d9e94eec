"""The CPU oracle against golden vectors produced by the reference's own code
(tests/golden/make_golden.py imports the reference modules)."""
import os

import numpy as np

from formula import formula_params
from oracle import oracle as O


def load(golden_dir, name):
    return np.load(os.path.join(golden_dir, name), allow_pickle=False)


def test_ray_generation_bit_exact(golden_dir):
    # near_far_linear_ray_generation, diff_ray_marching.py:349-393
    g = load(golden_dir, "raygen.npz")
    mid0 = O.ray_mid_t(2.0, 6.0, 400, R=8)
    assert np.array_equal(mid0, g["mid0"][0])
    assert np.array_equal(O.raypos(g["campos"][0], g["raydir"][0], mid0), g["pos0"][0])
    mid1 = O.ray_mid_t(2.0, 6.0, 400, R=8, jitter=0.3, rand=g["rand1"])
    assert np.array_equal(mid1, g["mid1"][0])
    assert np.array_equal(O.raypos(g["campos"][0], g["raydir"][0], mid1), g["pos1"][0])


def test_positional_encoding(golden_dir):
    # networks.py:175-190 (interleaved sin/cos; ori=True concat)
    g = load(golden_dir, "pe.npz")
    x = g["x"]
    np.testing.assert_allclose(O.positional_encoding(x, 5), g["pe5"], atol=2e-7, rtol=0)
    np.testing.assert_allclose(O.positional_encoding(x[:, :3], 3), g["pe3"], atol=2e-7, rtol=0)
    np.testing.assert_allclose(O.positional_encoding(x[:, :3], 4, ori=True), g["pe4ori"], atol=2e-7, rtol=0)


def test_aggregator(golden_dir):
    # PointAggregator.forward, lego config (point_aggregators.py:729-816)
    g = load(golden_dir, "aggregator.npz")
    f, rv, w, cc = O.aggregate(formula_params(), g["sampled_color"][0], None, g["sampled_dir"][0],
                               g["sampled_conf"][0], g["sampled_embedding"][0], g["sampled_xyz_pers"][0],
                               g["sampled_xyz"][0], g["sample_pnt_mask"][0], g["sample_loc"][0],
                               g["sample_loc_w"][0], g["sample_ray_dirs"][0])
    assert np.array_equal(rv, g["ray_valid"][0])
    np.testing.assert_allclose(f, g["features"][0], atol=1e-6, rtol=1e-5)
    np.testing.assert_allclose(w, g["weight"][0], atol=1e-6, rtol=1e-5)
    np.testing.assert_allclose(cc, g["conf_coefficient"][0], atol=1e-7, rtol=0)
    # the edge cases the fixture forces: an all-empty ray and an empty sample give zeros
    assert not rv[0].any() and np.all(f[0] == 0)
    assert not rv[1, 3] and np.all(f[1, 3] == 0)


def test_ray_march(golden_dir):
    # ray_march + radiance_render + alpha_blend, diff_ray_marching.py:509-555
    g = load(golden_dir, "raymarch.npz")
    c, pc, op, T, bw, bgT = O.ray_march(g["ray_dist"][0], g["ray_valid"][0], g["ray_features"][0], g["bg_color"])
    np.testing.assert_allclose(c, g["ray_color"][0], atol=2e-6, rtol=1e-5)
    # 1 - exp(-x): numpy and torch exp may differ by 1 ulp
    np.testing.assert_allclose(op, g["opacity"][0], atol=2.5e-7, rtol=0)
    np.testing.assert_allclose(T, g["acc_transmission"][0], atol=2e-7, rtol=1e-6)
    np.testing.assert_allclose(bw, g["blend_weight"][0], atol=2e-7, rtol=1e-6)
    np.testing.assert_allclose(bgT, g["background_transmission"][0], atol=2e-7, rtol=1e-6)


def test_aggregator_per_pair_rw2c(golden_dir):
    # PointAggregator.forward with a per-pair Rw2c [1,R,SR,K,3,3] (neural_points.py:799 gathers
    # a per-point table; point_aggregators.py:492-496, 506, 526, 566), from the reference itself
    g = load(golden_dir, "aggregator_rw2c.npz")
    f, rv, w, cc = O.aggregate(formula_params(salt=0.3), g["sampled_color"][0], g["sampled_Rw2c"][0],
                               g["sampled_dir"][0], g["sampled_conf"][0], g["sampled_embedding"][0],
                               g["sampled_xyz_pers"][0], g["sampled_xyz"][0], g["sample_pnt_mask"][0],
                               g["sample_loc"][0], g["sample_loc_w"][0], g["sample_ray_dirs"][0])
    assert np.array_equal(rv, g["ray_valid"][0])
    np.testing.assert_allclose(f, g["features"][0], atol=1e-6, rtol=1e-5)
    np.testing.assert_allclose(w, g["weight"][0], atol=1e-6, rtol=1e-5)
    # the rotation matters: the same inputs with the identity differ
    f_eye = O.aggregate(formula_params(salt=0.3), g["sampled_color"][0], None, g["sampled_dir"][0],
                        g["sampled_conf"][0], g["sampled_embedding"][0], g["sampled_xyz_pers"][0],
                        g["sampled_xyz"][0], g["sample_pnt_mask"][0], g["sample_loc"][0],
                        g["sample_loc_w"][0], g["sample_ray_dirs"][0])[0]
    assert np.abs(f_eye - g["features"][0]).max() > 1e-3
