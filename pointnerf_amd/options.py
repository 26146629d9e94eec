"""Flag set of the hot path, reusing the reference's flag names.

Values are the lego scene script (dev_scripts/w_n360/lego.sh) plus the defaults
it relies on (models/neural_points/neural_points.py:13-230,
models/aggregators/point_aggregators.py:15-217,
models/neural_points_volumetric_model.py:47-52).  ``query_size`` resolves to
``kernel_size`` as neural_points.py:329 does when it is left at (0, 0, 0).
"""
from types import SimpleNamespace

LEGO = dict(
    vsize=[0.004, 0.004, 0.004], vscale=[2, 2, 2], kernel_size=[3, 3, 3], query_size=[3, 3, 3],
    SR=80, K=8, P=9, NN=2, max_o=830000, radius_limit_scale=4.0, depth_limit_scale=0.0,
    ranges=[-0.638, -1.141, -0.346, 0.634, 1.149, 1.141], z_depth_dim=400, inverse=0, is_train=0,
    wcoord_query=1, gpu_maxthr=1024, xyz_grad=0,
    which_agg_model="viewmlp", agg_intrp_order=2, agg_dist_pers=20, agg_distance_kernel="linear",
    agg_axis_weight=[1.0, 1.0, 1.0], num_feat_freqs=3, dist_xyz_freq=5, dist_xyz_deno=0.0,
    point_features_dim=32, shading_feature_mlp_layer0=1, shading_feature_mlp_layer1=2,
    shading_feature_mlp_layer2=0, shading_feature_mlp_layer3=2, shading_alpha_mlp_layer=1,
    shading_color_mlp_layer=4, shading_feature_num=256, shading_color_channel_num=128,
    num_viewdir_freqs=4, num_pos_freqs=10, act_type="LeakyReLU", act_super=1,
    agg_feat_xyz_mode="None", agg_alpha_xyz_mode="None", agg_color_xyz_mode="None",
    apply_pnt_mask=1, agg_weight_norm=1, point_color_mode="1", point_dir_mode="1",
    point_conf_mode="1", default_conf=0.15, raydist_mode_unit=1, near_plane=2.0, far_plane=6.0,
    which_render_func="radiance", which_blend_func="alpha", which_tonemap_func="off",
    sparse_loss_weight=0, zero_one_loss_items=["conf_coefficient"], prob=0,
    # libpnr-specific: reproduce `voxel_idx > 0` of fill_occ2pnts (qpiw.py:372)
    slot0_drop=1,
)


# Per-scene overrides of the other BASELINE configs (the flag values each
# reference script passes; everything else as in lego.sh).
FLAGSETS = {
    "lego": {},
    # dev_scripts/w_n360/ship.sh (config c3)
    "ship": dict(ranges=[-1.277, -1.300, -0.550, 1.371, 1.349, 0.729], P=10, max_o=1500000),
    # dev_scripts/w_scannet_etf/scene101.sh (config c4)
    "scene101": dict(vsize=[0.008, 0.008, 0.008], ranges=[-10.0, -10.0, -10.0, 10.0, 10.0, 10.0], SR=24, P=30,
                     max_o=2000000, near_plane=0.1, far_plane=8.0, default_conf=-1.0),
    # dev_scripts/w_tt_ft/truck.sh (config c5): kernel 5 = three Chebyshev shells, query (dilation) 3
    "truck": dict(vsize=[0.002, 0.002, 0.002], kernel_size=[5, 5, 5], query_size=[3, 3, 3],
                  ranges=[-1.125, -0.598, -1.052, 0.795, 0.203, 1.029], SR=40, P=10, max_o=1600000,
                  near_plane=0.0, far_plane=3.5, default_conf=0.1),
}


def lego_opt(**over):
    o = dict(LEGO)
    o.update(over)
    if o["query_size"][0] == 0:
        o["query_size"] = list(o["kernel_size"])
    return SimpleNamespace(**o)


def flagset_opt(name: str, **over):
    """Flag set of one reference scene script (FLAGSETS) plus overrides."""
    if name not in FLAGSETS:
        raise KeyError(f"unknown flag set {name!r}: one of {sorted(FLAGSETS)}")
    o = dict(FLAGSETS[name])
    o.update(over)
    return lego_opt(**o)
