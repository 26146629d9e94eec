"""ctypes binding of libpnr.so (include/pnr.h).

The library is the only compute path of this package: if it is missing, or no
GPU is visible, every op raises -- there is no CPU fallback.  ``torch`` is
imported first so that libpnr.so binds to the HIP runtime torch already loaded
(both have soname libamdhip64.so.7): one runtime, shared streams and pointers.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (must be loaded before libpnr.so, see module doc)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PNR_LIB", os.path.join(_HERE, "libpnr.so"))

c_int, c_int8, c_int32, c_int64 = ctypes.c_int, ctypes.c_int8, ctypes.c_int32, ctypes.c_int64
c_float, c_size_t, c_void_p = ctypes.c_float, ctypes.c_size_t, ctypes.c_void_p
PNR_OK, PNR_EINVAL, PNR_EOVERFLOW, PNR_EHIP, PNR_ENOMEM = 0, 1, 2, 3, 4
ABI_VERSION = 23
FEAT_H_PITCH = 136   # PNR_FEAT_H_PITCH: uint16 per bf16 feature row (pnr_aggregate_fwd_bf16_hf)
HEAD_BWD_BLOCKS = 512   # PNR_HEAD_BWD_BLOCKS (include/pnr.h)


class PnrError(RuntimeError):
    pass


class GridParams(ctypes.Structure):
    _fields_ = [("shift", c_float * 3), ("vsize", c_float * 3), ("dims", c_int32 * 3),
                ("query_size", c_int32 * 3), ("max_o", c_int32), ("P", c_int32),
                ("slot0_drop", c_int32), ("seed", ctypes.c_uint64)]


class GridSpec(ctypes.Structure):
    _fields_ = [("ranges", c_float * 6), ("pad", c_float * 3), ("vsize", ctypes.c_double * 3),
                ("vscale", c_int32 * 3), ("vsize_s", c_float * 3), ("dims_max", c_int32 * 3),
                ("query_size", c_int32 * 3), ("max_o", c_int32), ("P", c_int32), ("slot0_drop", c_int32),
                ("seed", ctypes.c_uint64)]


class GridStats(ctypes.Structure):
    _fields_ = [("n_points_in_grid", c_int64), ("n_voxels", c_int64), ("n_voxels_kept", c_int64),
                ("n_points_dropped", c_int64), ("max_points_per_voxel", c_int32),
                ("dims", c_int32 * 3)]


class Rays(ctypes.Structure):
    _fields_ = [("campos_dev", c_void_p), ("camrot_dev", c_void_p), ("raydir_dev", c_void_p),
                ("tvals_dev", c_void_p), ("R", c_int64), ("D", c_int32), ("tvals_per_ray", c_int32),
                ("ray_cam", c_void_p)]


class QueryParams(ctypes.Structure):
    _fields_ = [("SR", c_int32), ("K", c_int32), ("kernel_size", c_int32 * 3),
                ("radius_limit2", c_float)]


class QueryBufs(ctypes.Structure):
    _fields_ = [("n_filled", c_void_p), ("slot_d", c_void_p), ("ray_off", c_void_p),
                ("fill_rs", c_void_p), ("pidx", c_void_p), ("valid_off", c_void_p),
                ("valid_list", c_void_p), ("vflag", c_void_p), ("ray_vcnt", c_void_p),
                ("ray_row", c_void_p), ("sample_w", c_void_p), ("sample_p", c_void_p),
                ("counts", c_void_p), ("scratch", c_void_p), ("scratch_bytes", c_size_t)]


class Mlp(ctypes.Structure):
    _fields_ = [("w1af", c_void_p), ("w1bf", c_void_p), ("w2f", c_void_p), ("b2", c_void_p),
                ("w3f", c_void_p), ("b3", c_void_p), ("w4f", c_void_p), ("b4", c_void_p),
                ("wa", c_void_p), ("ba", c_void_p), ("wc1f", c_void_p), ("bc1", c_void_p),
                ("wc2f", c_void_p), ("bc2", c_void_p), ("wc3f", c_void_p), ("bc3", c_void_p),
                ("rw2c", c_void_p), ("neg_slope", c_float), ("act_super", c_int32)]


class NeuralRenderW(ctypes.Structure):
    _fields_ = [(n, c_void_p) for n in ("wf0", "b0", "wf1", "b1", "wrgb0", "brgb0", "wrgb1", "brgb1", "wrgb2",
                                        "brgb2")] + [("neg_slope", c_float)]


class NeuralRenderWT(ctypes.Structure):
    _fields_ = [("wt0", c_void_p), ("wt1", c_void_p), ("wt2", c_void_p), ("neg_slope", c_float)]


class NeuralRenderH2W(ctypes.Structure):
    _fields_ = [("wp0", c_void_p), ("wp1", c_void_p), ("wp2", c_void_p), ("ws", c_void_p), ("b0", c_void_p),
                ("b1", c_void_p), ("b2", c_void_p), ("neg_slope", c_float)]


class NeuralRenderH2WT(ctypes.Structure):
    _fields_ = [("wt0", c_void_p), ("wt1", c_void_p), ("wt2", c_void_p), ("ws", c_void_p), ("neg_slope", c_float)]


class MlpBf16(ctypes.Structure):
    _fields_ = [("w1af", c_void_p), ("w1bf", c_void_p), ("w2f", c_void_p), ("w3f", c_void_p), ("w4f", c_void_p),
                ("wa", c_void_p), ("ba", c_void_p), ("wc1f", c_void_p), ("wc2f", c_void_p), ("wc3f", c_void_p),
                ("rw2c", c_void_p), ("neg_slope", c_float), ("act_super", c_int32), ("pair_buckets", c_int32)]


class Points(ctypes.Structure):
    _fields_ = [("n", c_int64), ("xyz", c_void_p), ("pers", c_void_p), ("emb", c_void_p), ("color", c_void_p),
                ("dir", c_void_p), ("conf", c_void_p), ("campos", c_void_p), ("camrot", c_void_p),
                ("used", c_void_p), ("n_used", c_int64), ("used_map", c_void_p),
                ("p1_ready", c_int32), ("emb_bf16", c_void_p), ("rw2c", c_void_p),
                ("n_used_dev", c_void_p)]


class Samples(ctypes.Structure):
    _fields_ = [("samp_list", c_void_p), ("n_dev", c_void_p), ("n_max", c_int64), ("pidx", c_void_p),
                ("sample_w", c_void_p), ("sample_p", c_void_p), ("dirs", c_void_p),
                ("dir_map", c_void_p), ("dir_div", c_int32), ("K", c_int32), ("ray_cam", c_void_p)]


class CompositeParams(ctypes.Structure):
    _fields_ = [("vsize_z", c_float), ("raydist_mode_unit", c_int32), ("C", c_int32),
                ("bg_color", c_void_p), ("feat_rows", c_int64)]


class AggSaved(ctypes.Structure):
    _fields_ = [(n, c_void_p) for n in ("h1", "h2", "h3", "h4", "pe5", "x3e", "pa", "wt", "wn", "prow", "hid",
                                        "vpe", "hc1", "hc2", "hc3", "vmask", "mask", "dz_absmax", "x1")]


class MlpX3(ctypes.Structure):
    _fields_ = [(n, c_void_p) for n in ("w1bx", "w2x", "w3x", "w4x")]


class MlpH2(ctypes.Structure):
    _fields_ = ([(n, c_void_p) for n in ("w1bh", "w2h", "w3h", "w4h")] + [("scale", c_float * 4),
                                                                        ("range_flag", c_void_p)] +
                [(n, c_void_p) for n in ("wc1a", "wc1b", "wc2h", "wc3h")] + [("cscale", c_float * 3)] +
                [("w1ah", c_void_p), ("scale1a", c_float)])


class MlpBwd(ctypes.Structure):
    _fields_ = [("w4t", c_void_p), ("w3t", c_void_p), ("w2t", c_void_p), ("w3e", c_void_p)]


class MlpBwdX3(ctypes.Structure):
    _fields_ = [("w4tx", c_void_p), ("w3tx", c_void_p), ("w2tx", c_void_p)]


class PackJob(ctypes.Structure):
    _fields_ = [("kind", c_int32), ("W", c_void_p), ("ld_row", c_int64), ("ld_col", c_int64), ("out_f", c_int32),
                ("kin", c_int32), ("bias", c_void_p), ("pad_steps", c_int32), ("shift", c_int32),
                ("range_flag", c_void_p), ("out", c_void_p), ("out_bytes", c_size_t)]


class AggParams(ctypes.Structure):
    _fields_ = [("p", c_void_p * 16)]


class AggGrads(ctypes.Structure):
    _fields_ = [("g", c_void_p * 16), ("d_emb", c_void_p), ("d_color", c_void_p), ("d_dir", c_void_p),
                ("d_conf", c_void_p)]


class MlpBwdH2(ctypes.Structure):
    _fields_ = [("w4th", c_void_p), ("w3th", c_void_p), ("w2th", c_void_p), ("scale", c_void_p)]


P = ctypes.POINTER
# name -> (restype, argtypes); exactly the functions include/pnr.h declares.
SIGNATURES = {
    "pnr_abi_version": (c_int, []),
    "pnr_clock_probe": (c_int, [c_void_p, c_int32, c_void_p]),
    "pnr_adam_step": (c_int, [c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, ctypes.c_double,
                              ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_double, c_int64, c_void_p]),
    "pnr_last_error": (ctypes.c_char_p, []),
    "pnr_create": (c_int, [c_int, P(c_void_p)]),
    "pnr_destroy": (c_int, [c_void_p]),
    "pnr_points_bbox": (c_int, [c_void_p, c_int64, c_void_p, c_void_p]),
    "pnr_grid_build": (c_int, [c_void_p, c_void_p, c_int64, P(GridParams), c_void_p]),
    "pnr_grid_stats_get": (c_int, [c_void_p, P(GridStats)]),
    "pnr_grid_build_dev": (c_int, [c_void_p, c_void_p, c_int64, P(GridSpec), c_void_p]),
    "pnr_grid_geometry": (c_int, [c_void_p, P(c_float), P(c_float), P(c_int32)]),
    "pnr_grid_bbox": (c_int, [c_void_p, P(c_float)]),
    "pnr_grid_export": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "pnr_query_scratch_bytes": (c_int, [c_int64, c_int32, P(c_size_t)]),
    "pnr_query": (c_int, [c_void_p, P(Rays), P(QueryParams), P(QueryBufs), c_void_p]),
    "pnr_query_compact": (c_int, [P(Rays), P(QueryParams), P(QueryBufs), c_int64, c_void_p, c_void_p,
                                  c_void_p, c_void_p, c_void_p, c_void_p]),
    "pnr_aggregate_scratch_bytes": (c_int, [c_int64, c_int64, P(c_size_t)]),
    "pnr_aggregate_fwd": (c_int, [P(Points), P(Samples), P(Mlp), c_void_p, c_void_p, c_void_p,
                                  c_void_p, c_size_t, c_void_p]),
    "pnr_aggregate_fwd_x3": (c_int, [P(Points), P(Samples), P(Mlp), P(MlpX3), c_void_p, c_void_p, c_void_p,
                                     c_void_p, c_size_t, c_void_p]),
    "pnr_point_pre_h2": (c_int, [P(Points), P(MlpH2), c_void_p, c_size_t, c_void_p]),
    "pnr_aggregate_fwd_h2": (c_int, [P(Points), P(Samples), P(Mlp), P(MlpH2), c_void_p, c_void_p, c_void_p,
                                     c_void_p, c_size_t, c_void_p]),
    "pnr_aggregate_fwd_masked": (c_int, [P(Points), P(Samples), P(Mlp), c_void_p, c_void_p,
                                         c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "pnr_aggregate_scratch_bytes_bf16": (c_int, [c_int64, c_int64, P(c_size_t)]),
    "pnr_aggregate_fwd_bf16": (c_int, [P(Points), P(Samples), P(MlpBf16), c_void_p, c_void_p, c_void_p,
                                       c_void_p, c_size_t, c_void_p]),
    "pnr_aggregate_fwd_bf16_hf": (c_int, [P(Points), P(Samples), P(MlpBf16), c_void_p, c_void_p, c_void_p,
                                          c_void_p, c_size_t, c_void_p]),
    "pnr_aggregate_fwd_train": (c_int, [P(Points), P(Samples), P(Mlp), P(AggSaved), c_void_p, c_void_p,
                                        c_void_p, c_void_p, c_size_t, c_void_p]),
    "pnr_aggregate_fwd_train_x3": (c_int, [P(Points), P(Samples), P(Mlp), P(MlpX3), P(AggSaved), c_void_p,
                                           c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "pnr_aggregate_fwd_train_h2": (c_int, [P(Points), P(Samples), P(Mlp), P(MlpH2), P(AggSaved), c_void_p,
                                           c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "pnr_aggregate_fwd_train_h2_guarded": (c_int, [P(Points), P(Samples), P(Mlp), P(MlpH2), P(AggSaved), c_void_p,
                                                   c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "pnr_aggregate_fwd_train_masked": (c_int, [P(Points), P(Samples), P(Mlp), c_void_p, P(AggSaved), c_void_p,
                                               c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "pnr_aggregate_bwd_pairs": (c_int, [P(Points), P(Samples), P(Mlp), P(MlpBwd), P(AggSaved), c_void_p,
                                        c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                        c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "pnr_aggregate_bwd_pairs_x3": (c_int, [P(Points), P(Samples), P(Mlp), P(MlpBwd), P(MlpBwdX3), P(AggSaved),
                                           c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                           c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "pnr_aggregate_bwd_pairs_h2": (c_int, [P(Points), P(Samples), P(Mlp), P(MlpBwd), P(MlpBwdH2), P(AggSaved),
                                           c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                           c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "pnr_color_dz": (c_int, [c_void_p, c_int64, c_void_p, c_void_p, c_int64, c_int64, c_int32, c_float, c_void_p,
                             c_void_p, c_void_p]),
    "pnr_group_pairs_scratch_bytes": (c_int, [c_int64, c_int64, P(c_size_t)]),
    "pnr_group_pairs": (c_int, [c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_size_t,
                                c_void_p]),
    "pnr_alpha_colsum_scratch_floats": (c_int, [P(c_int64)]),
    "pnr_alpha_colsum": (c_int, [c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_void_p]),
    "pnr_aggregate_bwd_step_h2_scratch_bytes": (c_int, [c_int64, c_int64, P(c_size_t)]),
    "pnr_aggregate_bwd_step_h2": (c_int, [P(Points), P(Samples), P(Mlp), P(AggParams), P(AggSaved), c_void_p,
                                          c_int64, c_int64, P(AggGrads), c_void_p, c_size_t, c_void_p]),
    "pnr_pack_batch": (c_int, [P(PackJob), c_int32, c_void_p]),
    "pnr_pack_bwd_h2": (c_int, [c_void_p, c_void_p, c_int64, c_void_p, c_int32, c_void_p, c_void_p, c_size_t,
                                c_void_p]),
    "pnr_aggregate_bwd_xyz": (c_int, [P(Points), P(Samples), P(Mlp), P(AggSaved), c_void_p, c_void_p, c_void_p,
                                      c_void_p, c_void_p]),
    "pnr_used_points_scratch_bytes": (c_int, [c_int64, P(c_size_t)]),
    "pnr_used_points": (c_int, [c_void_p, c_void_p, c_int32, c_int64, c_int64, c_void_p, c_void_p, c_void_p,
                                c_void_p, c_void_p, c_size_t, c_void_p]),
    "pnr_pairs_to_points": (c_int, [c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "pnr_pack_weights_h2": (c_int, [c_void_p, c_int64, c_int64, c_int32, c_int32, c_void_p, c_int32, c_int32,
                                    c_void_p, c_void_p, c_size_t, c_void_p]),
    "pnr_pack_weights_h2_dev": (c_int, [c_void_p, c_int64, c_int64, c_int32, c_int32, c_void_p, c_int32,
                                        c_void_p, c_void_p, c_size_t, c_void_p]),
    "pnr_pack_weights": (c_int, [c_int32, c_void_p, c_int64, c_int64, c_int32, c_int32, c_void_p, c_int32,
                                 c_void_p, c_size_t, c_void_p]),
    "pnr_gemm_tn_scratch_bytes": (c_int, [c_int64, c_int32, c_int32, P(c_size_t)]),
    "pnr_gemm_tn": (c_int, [c_void_p, c_int64, c_void_p, c_int64, c_int64, c_int32, c_int32, c_void_p, c_void_p,
                            c_void_p, c_size_t, c_void_p]),
    "pnr_gemm_tn_x3": (c_int, [c_void_p, c_int64, c_void_p, c_int64, c_int64, c_int32, c_int32, c_void_p, c_void_p,
                               c_void_p, c_size_t, c_void_p]),
    "pnr_gemm_nn": (c_int, [c_void_p, c_int64, c_void_p, c_int64, c_int64, c_int32, c_int32, c_void_p, c_int64,
                            c_float, c_void_p, c_int64, c_void_p]),
    "pnr_point_pe3": (c_int, [c_void_p, c_int64, c_void_p, c_void_p]),
    "pnr_point_pe3_bwd": (c_int, [c_void_p, c_void_p, c_int64, c_void_p, c_void_p]),
    "pnr_composite_bwd": (c_int, [P(Rays), P(QueryParams), P(QueryBufs), P(CompositeParams), c_void_p,
                                  c_void_p, c_void_p, c_void_p]),
    "pnr_ray_march_bwd": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int32, c_int32,
                                  c_void_p, c_void_p, c_void_p]),
    "pnr_ray_march_bwd_ex": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int32, c_int32,
                                     c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                     c_void_p]),
    "pnr_zero_rows": (c_int, [c_void_p, c_int64, c_void_p, c_int64, c_void_p]),
    "pnr_gemm_tn_h2": (c_int, [c_void_p, c_int64, c_void_p, c_int64, c_int64, c_int32, c_int32, c_void_p, c_void_p,
                               c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "pnr_gemm_nn_h2": (c_int, [c_void_p, c_int64, c_void_p, c_int64, c_int64, c_int32, c_int32, c_void_p, c_int64,
                               c_float, c_void_p, c_int64, c_void_p, c_void_p, c_void_p]),
    "pnr_aggregate_bwd_extras_rows": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                              c_void_p, c_void_p]),
    "pnr_pairs_to_points_ex": (c_int, [c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_void_p,
                                       c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "pnr_point_counts": (c_int, [c_void_p, c_void_p, c_int32, c_int64, c_void_p, c_void_p]),
    "pnr_point_pe3_rows": (c_int, [c_void_p, c_void_p, c_int64, c_void_p, c_void_p]),
    "pnr_point_pe3_bwd_rows": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_void_p]),
    "pnr_zero_one_loss_fwd": (c_int, [c_void_p, c_void_p, c_int64, c_void_p, c_int64, c_float, c_void_p, c_void_p,
                                      c_void_p]),
    "pnr_zero_one_loss_bwd": (c_int, [c_void_p, c_void_p, c_int64, c_float, c_void_p, c_void_p, c_void_p, c_void_p]),
    "pnr_absmax_scratch_floats": (c_int, [P(c_int64)]),
    "pnr_absmax": (c_int, [c_void_p, c_int64, c_void_p, c_void_p, c_void_p]),
    "pnr_weighted_colsum_scratch_floats": (c_int, [c_int32, P(c_int64)]),
    "pnr_weighted_colsum": (c_int, [c_void_p, c_void_p, c_int64, c_int32, c_void_p, c_void_p, c_void_p]),
    "pnr_march_aux": (c_int, [P(Rays), P(QueryParams), P(QueryBufs), c_void_p, c_void_p, c_int64, c_void_p,
                              c_void_p, c_void_p]),
    "pnr_composite_fwd": (c_int, [P(Rays), P(QueryParams), P(QueryBufs), P(CompositeParams),
                                  c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "pnr_composite_fwd_hf": (c_int, [P(Rays), P(QueryParams), P(QueryBufs), P(CompositeParams),
                                     c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "pnr_ray_march_fwd": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int32, c_int32,
                                  c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "pnr_neural_render_scratch_bytes": (c_int, [c_int32, c_int32, P(c_size_t)]),
    "pnr_neural_render_fwd": (c_int, [c_void_p, c_int32, c_int32, P(NeuralRenderW), c_void_p, c_void_p, c_size_t,
                                      c_void_p]),
    "pnr_neural_render_bwd_scratch_bytes": (c_int, [c_int32, c_int32, P(c_size_t)]),
    "pnr_neural_render_bwd": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int32, c_int32, P(NeuralRenderWT),
                                      c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "pnr_neural_render_h2_scratch_bytes": (c_int, [c_int32, c_int32, P(c_size_t)]),
    "pnr_neural_render_fwd_h2": (c_int, [c_void_p, c_int32, c_int32, P(NeuralRenderH2W), c_void_p, c_void_p,
                                         c_size_t, c_void_p]),
    "pnr_neural_render_bwd_h2_scratch_bytes": (c_int, [c_int32, c_int32, P(c_size_t)]),
    "pnr_neural_render_bwd_h2": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int32, c_int32,
                                         P(NeuralRenderH2WT), c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                         c_size_t, c_void_p]),
    "pnr_rgb_head_fwd": (c_int, [c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_void_p, c_int32, c_void_p,
                                 c_void_p]),
    "pnr_rgb_head_bwd": (c_int, [c_void_p, c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_void_p, c_int32,
                                 c_void_p, c_void_p, c_void_p, c_void_p]),
    "pnr_vox_closest_scratch_bytes": (c_int, [c_int64, P(c_size_t)]),
    "pnr_vox_closest": (c_int, [c_void_p, c_int64, c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                c_size_t, c_void_p]),
    "pnr_scan_scratch_bytes": (c_int, [c_int64, P(c_size_t)]),
    "pnr_exclusive_scan_i32": (c_int, [c_void_p, c_int64, c_void_p, c_void_p, c_int64, c_void_p, c_void_p,
                                       c_size_t, c_void_p]),
}

_lib = None


def lib():
    """Load libpnr.so once; raise loudly when it is absent."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise PnrError(f"libpnr.so not found at {LIB_PATH}: build it with "
                           "`python -c 'import __graft_entry__ as g; g.build()'` or `make`")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        if L.pnr_abi_version() != ABI_VERSION:
            raise PnrError(f"libpnr ABI {L.pnr_abi_version()} != expected {ABI_VERSION}")
        _lib = L
    return _lib


def check(rc: int, what: str):
    if rc != PNR_OK:
        msg = lib().pnr_last_error().decode(errors="replace")
        raise PnrError(f"{what} failed (status {rc}): {msg}")


def require_gpu(t: torch.Tensor | None = None):
    if not torch.cuda.is_available():
        raise PnrError("pointnerf_amd needs a ROCm GPU (torch.cuda.is_available() is False); "
                       "there is no CPU fallback")
    if t is not None and not t.is_cuda:
        raise PnrError("pointnerf_amd ops take device tensors; got a CPU tensor")


def ptr(t: torch.Tensor | None):
    return None if t is None else c_void_p(t.data_ptr())


def aggregate_scratch(n_max: int, n_points: int, device) -> torch.Tensor:
    """Device scratch for pnr_aggregate_fwd(_masked): per-point block1 partial
    products, K-summed features, masks."""
    nb = c_size_t(0)
    check(lib().pnr_aggregate_scratch_bytes(int(n_max), int(n_points), ctypes.byref(nb)),
          "pnr_aggregate_scratch_bytes")
    return torch.empty((int(nb.value) + 15) // 16 * 4, dtype=torch.float32, device=device)


class H2Gemm:
    """State shared by the pnr_gemm_tn_h2 calls of one backward: the range flag
    (zeroed here; raised -> those calls ran their x3 fallback on the device) and
    the pnr_absmax scratch."""

    def __init__(self, device):
        # [0]: the range flag; [1:]: pre-zeroed absmax words for fused producers
        self.words = torch.zeros(8, dtype=torch.int32, device=device)
        self.flag = self.words[:1]
        n = ctypes.c_int64(0)
        check(lib().pnr_absmax_scratch_floats(ctypes.byref(n)), "pnr_absmax_scratch_floats")
        self.part = torch.empty(int(n.value), dtype=torch.float32, device=device)

    def absmax(self, A: torch.Tensor) -> torch.Tensor:
        """[1] int32 holding the float bits of max |A| (device, no sync)."""
        out = torch.empty(1, dtype=torch.int32, device=A.device)
        a = A if A.is_contiguous() else A.contiguous()
        check(lib().pnr_absmax(ptr(a), a.numel(), ptr(self.part), ptr(out), stream_ptr(A.device)), "pnr_absmax")
        return out


def gemm_tn(A: torch.Tensor, B: torch.Tensor, colsum: bool = False, x3: bool = True, h2: H2Gemm | None = None,
            a_absmax: torch.Tensor | None = None):
    """C = A^T B (A [K,M], B [K,N], fp32 row-major with unit column stride) on
    pnr_gemm_tn_x3 (fp32-accurate on bf16 MFMA; x3=False: pnr_gemm_tn, native
    fp32 MFMA; h2: pnr_gemm_tn_h2, fp32-accurate on f16 MFMA with A's scale
    from a_absmax or a pnr_absmax pass); returns C [M,N] (and A's column sums
    when colsum)."""
    K, M = A.shape
    N = B.shape[1]
    assert B.shape[0] == K and A.stride(1) == 1 and B.stride(1) == 1
    nb = c_size_t(0)
    check(lib().pnr_gemm_tn_scratch_bytes(K, M, N, ctypes.byref(nb)), "pnr_gemm_tn_scratch_bytes")
    scratch = torch.empty(max(int(nb.value) // 4, 1), dtype=torch.float32, device=A.device)
    C = torch.empty((M, N), dtype=torch.float32, device=A.device)
    cs = torch.empty(M, dtype=torch.float32, device=A.device) if colsum else None
    if h2 is not None:
        am = a_absmax if a_absmax is not None else h2.absmax(A)
        check(lib().pnr_gemm_tn_h2(ptr(A), A.stride(0), ptr(B), B.stride(0), K, M, N, ptr(C), ptr(cs), ptr(am),
                                   ptr(h2.flag), ptr(scratch), scratch.numel() * 4, stream_ptr(A.device)),
              "pnr_gemm_tn_h2")
        return (C, cs) if colsum else C
    fn = lib().pnr_gemm_tn_x3 if x3 else lib().pnr_gemm_tn
    check(fn(ptr(A), A.stride(0), ptr(B), B.stride(0), K, M, N, ptr(C), ptr(cs), ptr(scratch),
             scratch.numel() * 4, stream_ptr(A.device)), "pnr_gemm_tn")
    return (C, cs) if colsum else C


def group_pairs(prow: torch.Tensor, key_map: torch.Tensor | None, n_keys: int):
    """(prow_sorted, pair_of) int32 [m]: the pairs grouped by point in pair order
    (pnr_group_pairs -- torch.sort(prow, stable=True) with the empty pairs last)."""
    m = prow.numel()
    dev = prow.device
    nb = c_size_t(0)
    check(lib().pnr_group_pairs_scratch_bytes(m, max(int(n_keys), 1), ctypes.byref(nb)),
          "pnr_group_pairs_scratch_bytes")
    scratch = torch.empty(max(int(nb.value), 16), dtype=torch.uint8, device=dev)
    ps, po = (torch.empty(max(m, 1), dtype=torch.int32, device=dev) for _ in range(2))
    check(lib().pnr_group_pairs(ptr(prow), m, ptr(key_map), max(int(n_keys), 1), ptr(ps), ptr(po), ptr(scratch),
                                scratch.numel(), stream_ptr(dev)), "pnr_group_pairs")
    return ps[:m], po[:m]


def gemm_nn(A: torch.Tensor, B: torch.Tensor, act: torch.Tensor | None = None, slope: float = 0.0,
            out: torch.Tensor | None = None, h2: "H2Gemm | None" = None, a_absmax: torch.Tensor | None = None):
    """C = A B (A [M,K], B [K,N], unit column strides) on pnr_gemm_nn (exact fp32
    products, fp32 MFMA) or, with h2, pnr_gemm_nn_h2 (fp32-accurate f16-split
    MFMA, A's scale from a_absmax or a pnr_absmax pass); with act: C *=
    where(act > 0, 1, slope) (the LeakyReLU derivative of the saved activation).
    out: optional [M,N] destination view."""
    M, K = A.shape
    N = B.shape[1]
    assert B.shape[0] == K and A.stride(1) == 1 and B.stride(1) == 1
    assert act is None or (act.shape == (M, N) and act.stride(1) == 1)
    C = torch.empty((M, N), dtype=torch.float32, device=A.device) if out is None else out
    assert C.shape == (M, N) and C.stride(1) == 1
    if h2 is not None:
        am = a_absmax if a_absmax is not None else h2.absmax(A)
        check(lib().pnr_gemm_nn_h2(ptr(A), A.stride(0), ptr(B), B.stride(0), M, K, N, ptr(act),
                                   act.stride(0) if act is not None else 0, float(slope), ptr(C), C.stride(0),
                                   ptr(am), ptr(h2.flag), stream_ptr(A.device)), "pnr_gemm_nn_h2")
        return C
    check(lib().pnr_gemm_nn(ptr(A), A.stride(0), ptr(B), B.stride(0), M, K, N, ptr(act),
                            act.stride(0) if act is not None else 0, float(slope), ptr(C), C.stride(0),
                            stream_ptr(A.device)), "pnr_gemm_nn")
    return C


def aggregate_scratch_bf16(n_max: int, n_points: int, device) -> torch.Tensor:
    nb = c_size_t(0)
    check(lib().pnr_aggregate_scratch_bytes_bf16(int(n_max), int(n_points), ctypes.byref(nb)),
          "pnr_aggregate_scratch_bytes_bf16")
    return torch.empty((int(nb.value) + 15) // 16 * 4, dtype=torch.float32, device=device)


def stream_ptr(device=None):
    return c_void_p(torch.cuda.current_stream(device).cuda_stream)


def weighted_colsum(w: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
    """out[c] = sum_r w[r] x[r, c] on pnr_weighted_colsum (deterministic): the
    background colour's gradient from d ray_color and is_bg / bg_T."""
    w = w.reshape(-1).float().contiguous()
    x = x.reshape(w.numel(), x.shape[-1]).float().contiguous()
    C = x.shape[1]
    n = ctypes.c_int64(0)
    check(lib().pnr_weighted_colsum_scratch_floats(C, ctypes.byref(n)), "pnr_weighted_colsum_scratch_floats")
    part = torch.empty(int(n.value), dtype=torch.float32, device=x.device)
    out = torch.empty(C, dtype=torch.float32, device=x.device)
    check(lib().pnr_weighted_colsum(ptr(w), ptr(x), w.numel(), C, ptr(out), ptr(part), stream_ptr(x.device)),
          "pnr_weighted_colsum")
    return out
