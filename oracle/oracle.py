"""TEST INFRASTRUCTURE ONLY -- CPU oracle of the Point-NeRF hot path.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module, and only as the checker / the CPU baseline.  The
product package ``pointnerf_amd`` never imports it.

A plain NumPy (fp32) restatement of the reference algorithm, plus ctypes access
to ``query_ref.c`` (the serial C restatement of the query kernels).  Every
function cites the reference lines it restates (paths relative to the
reference tree; ``qpiw.py`` = models/neural_points/query_point_indices_worldcoords.py).

Pinning (see DESIGN.md "Oracle"):
  * ray generation, positional encoding, PointAggregator (lego config) and
    ray_march are pinned by golden vectors produced by importing the
    reference's own Python modules (tests/golden/make_golden.py);
  * the query (CUDA text JIT-compiled by pycuda in the reference, unbuildable
    here) is pinned through the golden ray generation plus brute-force
    property tests -- "query parity pinned by restatement + properties".
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "liboracle_query.so")
_lib = None

F32 = np.float32


def _load():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            subprocess.check_call(["make", "-s", "-C", _HERE])
        lib = ctypes.CDLL(_LIB_PATH)
        P = ctypes.c_void_p
        lib.oracle_grid_build.restype = ctypes.c_int64
        lib.oracle_grid_build.argtypes = [P, ctypes.c_int64, P, P, P, P, ctypes.c_int, ctypes.c_int,
                                          ctypes.c_int, ctypes.c_uint64, P, P, P, P]
        lib.oracle_ray_march.restype = None
        lib.oracle_ray_march.argtypes = [P, P, ctypes.c_int64, P, ctypes.c_int, ctypes.c_int,
                                         ctypes.c_int, P, P, P, P, P, P]
        lib.oracle_set_threads.restype = None
        lib.oracle_set_threads.argtypes = [ctypes.c_int]
        lib.oracle_knn.restype = ctypes.c_int64
        lib.oracle_knn.argtypes = [P, P, ctypes.c_int64, P, P, P, P, ctypes.c_int, ctypes.c_int,
                                   ctypes.c_float, P, P, P, P]
        _lib = lib
    return _lib


def set_threads(n: int):
    """OpenMP threads of the C query's ray / sample loops (results do not depend on it)."""
    _load().oracle_set_threads(int(n))


def _p(a: np.ndarray):
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(ctypes.c_void_p)


# --------------------------------------------------------------------- options
def lego_opt(**over):
    """The lego flag set (dev_scripts/w_n360/lego.sh) + defaults it relies on
    (neural_points.py:13-230, point_aggregators.py:15-217)."""
    from types import SimpleNamespace
    o = dict(vsize=[0.004, 0.004, 0.004], vscale=[2, 2, 2], kernel_size=[3, 3, 3],
             query_size=[3, 3, 3], SR=80, K=8, P=9, NN=2, max_o=830000, radius_limit_scale=4.0,
             depth_limit_scale=0.0, ranges=[-0.638, -1.141, -0.346, 0.634, 1.149, 1.141],
             z_depth_dim=400, inverse=0, is_train=0, wcoord_query=1,
             agg_intrp_order=2, agg_dist_pers=20, agg_distance_kernel="linear",
             num_feat_freqs=3, dist_xyz_freq=5, dist_xyz_deno=0.0, point_features_dim=32,
             shading_feature_mlp_layer1=2, shading_feature_mlp_layer2=0,
             shading_feature_mlp_layer3=2, shading_alpha_mlp_layer=1,
             shading_color_mlp_layer=4, shading_feature_num=256, shading_color_channel_num=128,
             num_viewdir_freqs=4, num_pos_freqs=10, act_type="LeakyReLU", act_super=1,
             raydist_mode_unit=1, apply_pnt_mask=1, agg_weight_norm=1,
             point_color_mode="1", point_dir_mode="1", point_conf_mode="1",
             near_plane=2.0, far_plane=6.0, slot0_drop=1)
    o.update(over)
    return SimpleNamespace(**o)


# ------------------------------------------------------------- hyperparameters
def get_hyperparameters(opt, xyz):
    """qpiw.py:48-81 (same numpy/torch dtype promotions)."""
    xyz = np.asarray(xyz, dtype=F32).reshape(-1, 3)
    vsize_np = opt.vsize
    min_xyz, max_xyz = xyz.min(axis=0), xyz.max(axis=0)
    vscale_np = np.array(opt.vscale, dtype=np.int32)
    scaled_vsize_np = (vsize_np * vscale_np).astype(np.float32)
    ranges = opt.ranges
    if ranges is not None and ranges[0] >= ranges[3]:
        ranges = None
    if ranges is not None:
        min_xyz = np.maximum(min_xyz, np.asarray(ranges[:3], dtype=F32))
        max_xyz = np.minimum(max_xyz, np.asarray(ranges[3:], dtype=F32))
    pad = (scaled_vsize_np * opt.kernel_size / 2).astype(F32)
    min_xyz = (min_xyz - pad).astype(F32)
    max_xyz = (max_xyz + pad).astype(F32)
    ranges_np = np.concatenate([min_xyz, max_xyz]).astype(np.float32)
    vdim_np = (max_xyz - min_xyz) / vsize_np
    scaled_vdim_np = np.ceil(vdim_np / vscale_np).astype(np.int32)
    radius_limit_np = np.asarray(opt.radius_limit_scale * max(vsize_np[0], vsize_np[1])).astype(np.float32)
    return dict(ranges=ranges_np, shift=ranges_np[:3].copy(), vsize_s=scaled_vsize_np,
                dims=scaled_vdim_np, radius_limit=radius_limit_np,
                radius_limit2=np.float32(radius_limit_np ** 2), vsize=np.asarray(vsize_np))


# -------------------------------------------------------------- ray generation
def ray_mid_t(near, far, D, R=1, jitter=0.0, rand=None):
    """middle_point_ts of near_far_linear_ray_generation
    (models/rendering/diff_ray_marching.py:369-385); [R, D] float32.
    Evaluated with torch CPU ops so linspace/cumsum round like the reference."""
    import torch
    tvals = torch.linspace(0, 1, D + 1).view(1, -1)
    tvals = near * (1 - tvals) + far * tvals
    if rand is None:
        rand = torch.rand((1, R, D))
    else:
        rand = torch.as_tensor(rand, dtype=torch.float32).view(1, R, D)
    seg = (tvals[..., 1:] - tvals[..., :-1]) * (1 + jitter * (rand - 0.5))
    end = torch.cumsum(seg, dim=2)
    end = torch.cat([torch.zeros((1, R, 1)), end], dim=2)
    end = near + end
    mid = (end[:, :, :-1] + end[:, :, 1:]) / 2
    return mid[0].numpy().astype(F32)


def raypos(campos, raydir, mid_t):
    """diff_ray_marching.py:387: campos + raydir * t (fp32 mul, then add)."""
    campos = np.asarray(campos, F32)
    raydir = np.asarray(raydir, F32)
    t = np.asarray(mid_t, F32)
    if t.ndim == 1:
        t = np.broadcast_to(t, (raydir.shape[0], t.shape[0]))
    return (campos[None, None, :] + (raydir[:, None, :] * t[:, :, None]).astype(F32)).astype(F32)


def w2pers(p, campos, camrot):
    """qpiw.py:102-109 / neural_points.py:687-693: (x/z, y/z, z) of R^T (p - c)."""
    p = np.asarray(p, F32)
    s = (p - np.asarray(campos, F32)).astype(F32)
    R = np.asarray(camrot, F32)
    xc = [((s[..., 0] * R[0, j]).astype(F32) + (s[..., 1] * R[1, j]).astype(F32)).astype(F32)
          + (s[..., 2] * R[2, j]).astype(F32) for j in range(3)]
    xc = [x.astype(F32) for x in xc]
    return np.stack([xc[0] / xc[2], xc[1] / xc[2], xc[2]], axis=-1).astype(F32)


# ----------------------------------------------------------------------- query
def grid_build(opt, xyz, hp=None):
    """build_occ_vox (qpiw.py:546-611) via query_ref.c; max_o / P overflow keeps
    the seeded reservoir's uniform subsets (opt.grid_seed, query_ref.c)."""
    lib = _load()
    xyz = np.ascontiguousarray(np.asarray(xyz, F32).reshape(-1, 3))
    hp = hp or get_hyperparameters(opt, xyz)
    dims = np.ascontiguousarray(hp["dims"].astype(np.int32))
    gvol = int(np.prod(dims.astype(np.int64)))
    coor_2_occ = np.empty(gvol, np.int32)
    coor_occ = np.empty(gvol, np.uint8)
    occ_numpnts = np.empty(opt.max_o, np.int32)
    occ_2_pnts = np.empty(opt.max_o * opt.P, np.int32)
    qs = np.ascontiguousarray(np.asarray(opt.query_size, np.int32))
    shift = np.ascontiguousarray(hp["shift"].astype(F32))
    vs = np.ascontiguousarray(hp["vsize_s"].astype(F32))
    n_occ = lib.oracle_grid_build(_p(xyz), xyz.shape[0], _p(shift), _p(vs), _p(dims), _p(qs),
                                  opt.max_o, opt.P, int(getattr(opt, "slot0_drop", 1)),
                                  int(getattr(opt, "grid_seed", 0)),
                                  _p(coor_2_occ), _p(coor_occ), _p(occ_numpnts), _p(occ_2_pnts))
    return dict(hp=hp, coor_2_occ=coor_2_occ, coor_occ=coor_occ, occ_numpnts=occ_numpnts,
                occ_2_pnts=occ_2_pnts.reshape(opt.max_o, opt.P), n_occ=int(n_occ))


def query_points(opt, xyz, campos, camrot, raydir, mid_t=None, near=None, far=None, grid=None):
    """lighting_fast_querier.query_points (qpiw.py:84-99) +
    query_grid_point_index (qpiw.py:614-721), serial semantics.

    Returns the reference outputs (B = 1 dropped) plus internals:
      sample_pidx [R'',SR,K] int32, sample_loc [R'',SR,3], sample_loc_w [R'',SR,3],
      sample_ray_dirs [R'',SR,3], ray_mask [R] int8, n_filled [R], slot_d [R,SR].
    """
    lib = _load()
    xyz = np.ascontiguousarray(np.asarray(xyz, F32).reshape(-1, 3))
    raydir = np.ascontiguousarray(np.asarray(raydir, F32).reshape(-1, 3))
    campos = np.ascontiguousarray(np.asarray(campos, F32).reshape(3))
    camrot = np.asarray(camrot, F32).reshape(3, 3)
    grid = grid or grid_build(opt, xyz)
    hp = grid["hp"]
    R, SR, K, D = raydir.shape[0], opt.SR, opt.K, opt.z_depth_dim
    if mid_t is None:
        mid_t = ray_mid_t(near, far, D)[0]
    mid_t = np.ascontiguousarray(np.asarray(mid_t, F32))
    per_ray = 1 if mid_t.ndim == 2 else 0
    dims = np.ascontiguousarray(hp["dims"].astype(np.int32))
    shift = np.ascontiguousarray(hp["shift"].astype(F32))
    vs = np.ascontiguousarray(hp["vsize_s"].astype(F32))
    n_filled = np.zeros(R, np.int32)
    slot_d = np.full(R * SR, -1, np.int32)
    lib.oracle_ray_march(_p(campos), _p(raydir), R, _p(mid_t), per_ray, D, SR, _p(shift), _p(vs),
                         _p(dims), _p(grid["coor_occ"]), _p(n_filled), _p(slot_d))
    slot_d = slot_d.reshape(R, SR)
    # R' compaction and get_shadingloc (qpiw.py:655-677)
    rp = raypos(campos, raydir, mid_t)  # [R, D, 3]
    ray_hit = n_filled > 0
    sloc_w = np.zeros((R, SR, 3), F32)
    smask = np.zeros((R, SR), bool)
    for r in np.nonzero(ray_hit)[0]:
        n = n_filled[r]
        sloc_w[r, :n] = rp[r, slot_d[r, :n]]
        smask[r, :n] = True
    # query_neigh_along_ray_layered over filled samples
    flat = np.ascontiguousarray(sloc_w[smask])
    pidx_f = np.full((flat.shape[0], K), -1, np.int32)
    ks = np.ascontiguousarray(np.asarray(opt.kernel_size, np.int32))
    assert K <= 64, "oracle_knn keeps at most 64 neighbours"
    if flat.shape[0]:
        lib.oracle_knn(_p(xyz), _p(flat), flat.shape[0], _p(shift), _p(vs), _p(dims), _p(ks), K,
                       opt.P, float(hp["radius_limit2"]), _p(grid["coor_2_occ"]),
                       _p(grid["occ_numpnts"]), _p(np.ascontiguousarray(grid["occ_2_pnts"])),
                       _p(pidx_f))
    pidx = np.full((R, SR, K), -1, np.int32)
    pidx[smask] = pidx_f
    # R'' compaction (qpiw.py:715-719)
    ray_valid = np.any(pidx >= 0, axis=(1, 2))
    sample_pidx = pidx[ray_valid]
    sample_loc_w = sloc_w[ray_valid]
    sample_loc = w2pers(sample_loc_w, campos, camrot)
    sample_ray_dirs = np.broadcast_to(raydir[ray_valid][:, None, :], sample_loc.shape).astype(F32)
    return dict(sample_pidx=sample_pidx, sample_loc=sample_loc, sample_loc_w=sample_loc_w,
                sample_ray_dirs=np.ascontiguousarray(sample_ray_dirs),
                ray_mask=ray_valid.astype(np.int8), n_filled=n_filled, slot_d=slot_d,
                pidx_dense=pidx, grid=grid, mid_t=mid_t, vsize=np.asarray(opt.vsize),
                ranges=hp["ranges"])


def knn_bruteforce(xyz, loc, hp, opt, grid):
    """Independent statement of the searched-shell KNN used by the property
    tests: candidates = points stored in occupied voxels of Chebyshev shells
    <= the last shell the layered loop visits, within radius; result = the K
    smallest squared distances (as a set)."""
    xyz = np.asarray(xyz, F32)
    shift, vs, dims = hp["shift"], hp["vsize_s"], hp["dims"]
    f = np.floor((np.asarray(loc, F32) - shift) / vs).astype(np.int64)
    r2 = np.float32(hp["radius_limit2"])
    layers = (opt.kernel_size[0] + 1) // 2
    occ = grid["occ_2_pnts"]
    cnts = np.minimum(grid["occ_numpnts"], opt.P)
    out = []
    for s in range(f.shape[0]):
        found = []
        for layer in range(layers):
            for x in range(-layer, layer + 1):
                for y in range(-layer, layer + 1):
                    for z in range(-layer, layer + 1):
                        if max(abs(x), abs(y), abs(z)) != layer:
                            continue
                        c = f[s] + (x, y, z)
                        if np.any(c < 0) or np.any(c >= dims):
                            continue
                        slot = grid["coor_2_occ"][(c[0] * dims[1] + c[1]) * dims[2] + c[2]]
                        if slot < 0:
                            continue
                        for pi in occ[slot, :cnts[slot]]:
                            d = (xyz[pi] - loc[s]).astype(F32)
                            d2 = F32(F32(F32(d[0] * d[0]) + F32(d[1] * d[1])) + F32(d[2] * d[2]))
                            if r2 == 0 or d2 <= r2:
                                found.append((d2, int(pi)))
            if len(found) >= opt.K:
                break
        found.sort()
        out.append(found)
    return out


# --------------------------------------------------------- gather + aggregate
def positional_encoding(x, freqs, ori=False):
    """models/helpers/networks.py:175-190."""
    x = np.asarray(x, F32)
    bands = (2.0 ** np.arange(freqs)).astype(F32)
    pts = (x[..., None] * bands).reshape(x.shape[:-1] + (freqs * x.shape[-1],)).astype(F32)
    if ori:
        return np.concatenate([x, np.sin(pts), np.cos(pts)], axis=-1).astype(F32)
    return np.stack([np.sin(pts), np.cos(pts)], axis=-1).reshape(pts.shape[:-1] + (pts.shape[-1] * 2,)).astype(F32)


def gather(points, sample_pidx, campos, camrot):
    """NeuralPoints.forward (neural_points.py:782-812) for B = 1.  points: dict
    xyz[N,3], emb[N,32], color[N,3] | None, dir[N,3] | None, conf[N,1] | None."""
    xyz = np.asarray(points["xyz"], F32)
    pers = w2pers(xyz, campos, camrot)
    mask = sample_pidx >= 0
    idx = np.clip(sample_pidx, 0, None).reshape(-1)
    shp = sample_pidx.shape

    def g(a, c):
        return None if a is None else np.asarray(a, F32).reshape(-1, c)[idx].reshape(shp + (c,))

    rw = points.get("Rw2c")
    if rw is not None and np.asarray(rw).ndim > 2:   # per-point Rw2c (neural_points.py:799)
        rw = np.asarray(rw, F32).reshape(-1, 9)[idx].reshape(shp + (3, 3))
    return dict(sampled_color=g(points.get("color"), 3), sampled_dir=g(points.get("dir"), 3),
                sampled_conf=g(points.get("conf"), 1), sampled_embedding=g(points["emb"], 32),
                sampled_xyz_pers=g(pers, 3), sampled_xyz=g(xyz, 3), sample_pnt_mask=mask, sampled_Rw2c=rw)


def _lin(x, params, name):
    W = np.asarray(params[name + ".weight"], F32)
    b = np.asarray(params[name + ".bias"], F32)
    return (np.matmul(x.astype(F32), W.T).astype(F32) + b).astype(F32)


def _lrelu(x, s):
    return np.where(x > 0, x, x * F32(s)).astype(F32)


def _softplus(x):
    return np.where(x > 20, x, np.log1p(np.exp(np.minimum(x, 20)))).astype(F32)


def aggregate(params, sampled_color, sampled_Rw2c, sampled_dir, sampled_conf, sampled_embedding,
              sampled_xyz_pers, sampled_xyz, sample_pnt_mask, sample_loc, sample_loc_w,
              sample_ray_dirs, neg_slope=0.01, act_super=1, C=128):
    """PointAggregator.forward (point_aggregators.py:729-816) for the lego
    configuration: agg_dist_pers 20, linear kernel, weight norm, conf clamp,
    viewmlp agg_intrp_order 2 (:488-646), num_feat_freqs 3, dist_xyz_freq 5,
    num_viewdir_freqs 4, block1 x2, block3 x2, alpha x1, colour x3.
    Inputs [R,SR,K,.] (B = 1 dropped).  Returns features [R,SR,C+1],
    ray_valid [R,SR], weight [R,SR,K], conf_coefficient [R,SR,K]."""
    mask = np.asarray(sample_pnt_mask, bool)
    R, SR, K = mask.shape
    ray_valid = mask.any(-1)
    sx, sxp = np.asarray(sampled_xyz, F32), np.asarray(sampled_xyz_pers, F32)
    sl, slw = np.asarray(sample_loc, F32), np.asarray(sample_loc_w, F32)
    xdist = (sxp[..., 0] * sxp[..., 2]).astype(F32) - (sl[:, :, None, 0] * sl[:, :, None, 2]).astype(F32)
    ydist = (sxp[..., 1] * sxp[..., 2]).astype(F32) - (sl[:, :, None, 1] * sl[:, :, None, 2]).astype(F32)
    zdist = sxp[..., 2] - sl[:, :, None, 2]
    dists = np.concatenate([(sx - slw[..., None, :]).astype(F32),
                            np.stack([xdist, ydist, zdist], -1).astype(F32)], -1).astype(F32)
    # linear kernel (:421-429) + normalisation (:803-804)
    w = (1.0 / np.maximum(np.sqrt((dists[..., :3] ** 2).sum(-1)), F32(1e-6))).astype(F32)
    w = (mask * w).astype(F32)
    w = (w / np.maximum(w.sum(-1, keepdims=True), F32(1e-8))).astype(F32)
    conf = np.ones(mask.shape, F32) if sampled_conf is None else np.asarray(sampled_conf, F32)[..., 0]
    confc = np.clip(conf, F32(1e-4), F32(1)).astype(F32)
    wt = (w * confc).astype(F32)
    Rw = np.eye(3, dtype=F32) if sampled_Rw2c is None else np.asarray(sampled_Rw2c, F32)
    per_pair = Rw.ndim > 2   # [R,SR,K,3,3] gathered per pair (point_aggregators.py:492-496)

    def rot(x, Rm):          # x @ Rm^T per row (Rm [3,3] or one [3,3] per row)
        if Rm.ndim == 2:
            return (x @ Rm.T).astype(F32)
        return np.einsum("ni,nji->nj", x, Rm).astype(F32)

    out = np.zeros((R, SR, C + 1), F32)
    if not ray_valid.any():
        return out, ray_valid, w, confc
    pm = mask.reshape(-1)
    Rpair = Rw.reshape(-1, 3, 3)[pm] if per_pair else Rw
    Rray = Rw[:, :, 0].reshape(-1, 3, 3) if per_pair else Rw   # slot 0's matrix rotates the view dir
    vd = rot(np.asarray(sample_ray_dirs, F32).reshape(-1, 3), Rray)
    vpe = positional_encoding(vd, 4, ori=True)
    ori_v, vpe = vpe[:, :3], vpe[:, 3:]
    vpe = vpe[ray_valid.reshape(-1)]
    d = dists.reshape(-1, 6)[pm].copy()
    d[:, :3] = rot(d[:, :3], Rpair)
    d = positional_encoding(d, 5)
    e = np.asarray(sampled_embedding, F32).reshape(-1, 32)[pm]
    feat = np.concatenate([e, positional_encoding(e, 3), d], -1)
    feat = _lrelu(_lin(feat, params, "block1.0"), neg_slope)
    feat = _lrelu(_lin(feat, params, "block1.2"), neg_slope)
    col = np.asarray(sampled_color, F32).reshape(-1, 3)[pm]
    sdir = rot(np.asarray(sampled_dir, F32).reshape(-1, 3)[pm], Rpair)
    ov = np.repeat(ori_v[:, None, :], K, 1).reshape(-1, 3)[pm]
    feat = np.concatenate([feat, col, sdir - ov, (sdir * ov).sum(-1, keepdims=True)], -1).astype(F32)
    feat = _lrelu(_lin(feat, params, "block3.0"), neg_slope)
    feat = _lrelu(_lin(feat, params, "block3.2"), neg_slope)
    a = _lin(feat, params, "alpha_branch.0")
    a = _softplus(a - 1) if act_super else np.maximum(a, 0)
    ah = np.zeros((R * SR * K, 1), F32)
    ah[pm] = a
    wv = wt.reshape(R * SR, K, 1)
    alpha = (ah.reshape(R * SR, K, 1) * wv).sum(-2)[ray_valid.reshape(-1)]
    fh = np.zeros((R * SR * K, feat.shape[-1]), F32)
    fh[pm] = feat
    f = (fh.reshape(R * SR, K, -1) * wv).sum(-2)[ray_valid.reshape(-1)].astype(F32)
    c = np.concatenate([f, vpe], -1)
    for name in ("color_branch.0", "color_branch.2", "color_branch.4"):
        c = _lrelu(_lin(c, params, name), neg_slope)
    if C == 3:
        # upstream colour head, commented out in the fork: the final Linear(in, 3)
        # (point_aggregators.py:343) and raw2out_color (:269-273, :637): sigmoid,
        # then * (1 + 2e-3) - 1e-3 when act_super > 0 (parity unpinned: no
        # reference code path runs it)
        z = _lin(c, params, "color_branch.6").astype(np.float64)
        c = (1.0 / (1.0 + np.exp(-z))).astype(F32)
        if act_super > 0:
            c = (c * F32(1 + 2e-3) - F32(1e-3)).astype(F32)
    flat = out.reshape(-1, C + 1)
    flat[ray_valid.reshape(-1)] = np.concatenate([alpha, c], -1)
    return out, ray_valid, w, confc


# ------------------------------------------------------------------- composite
def ray_march(ray_dist, ray_valid, ray_features, bg_color=None):
    """ray_march + radiance_render + alpha_blend (diff_ray_marching.py:509-555,
    diff_render_func.py:36-50); inputs [R,SR,...] (B = 1 dropped)."""
    f = np.asarray(ray_features, F32)
    sigma = f[..., 0] * np.asarray(ray_valid, F32)
    opacity = (1 - np.exp(-sigma * np.asarray(ray_dist, F32))).astype(F32)
    T = np.cumprod((1.0 - opacity + F32(1e-10)).astype(F32), axis=-1, dtype=F32)
    bgT = T[:, -1:]
    T = np.concatenate([np.ones((T.shape[0], 1), F32), T[:, :-1]], -1)
    bw = (opacity * T)[..., None]
    color = (f[..., 1:] * bw).sum(-2).astype(F32)
    if bg_color is not None:
        color = (color + np.asarray(bg_color, F32).reshape(1, -1) * bgT).astype(F32)
    return color, f[..., 1:], opacity, T, bw, bgT


def ray_dist(sample_loc, ray_valid, vsize_z, unit=1):
    """NeuralPointsRayMarching.forward (neural_points_volumetric_model.py:293-301)."""
    z = np.maximum.accumulate(np.asarray(sample_loc, F32)[..., 2], axis=-1)
    d = np.concatenate([z[..., 1:] - z[..., :-1], np.full(z.shape[:-1] + (1,), F32(vsize_z))], -1).astype(F32)
    m = d < F32(1e-8)
    if unit:
        m = m | (d > F32(2 * vsize_z))
    m = m.astype(F32)
    d = (d * (1 - m) + m * F32(vsize_z)).astype(F32)
    return (d * np.asarray(ray_valid, F32)).astype(F32)


def render(opt, points, params, campos, camrot, raydir, bg_color, mid_t=None, q=None):
    """NeuralPointsRayMarching.forward + fill_invalid
    (neural_points_volumetric_model.py:272-389), eval mode, tone_map 'off'."""
    if q is None:
        q = query_points(opt, points["xyz"], campos, camrot, raydir, mid_t=mid_t,
                         near=opt.near_plane, far=opt.far_plane)
    g = gather(points, q["sample_pidx"], campos, camrot)
    neg = 0.01 if opt.act_type == "LeakyReLU" else 0.0
    feats, rv, w, cc = aggregate(params, g["sampled_color"], g["sampled_Rw2c"], g["sampled_dir"],
                                 g["sampled_conf"], g["sampled_embedding"], g["sampled_xyz_pers"],
                                 g["sampled_xyz"], g["sample_pnt_mask"], q["sample_loc"],
                                 q["sample_loc_w"], q["sample_ray_dirs"], neg_slope=neg,
                                 act_super=opt.act_super, C=opt.shading_color_channel_num)
    rd = ray_dist(q["sample_loc"], rv, opt.vsize[2], opt.raydist_mode_unit)
    color, _, opacity, T, bw, bgT = ray_march(rd, rv, feats, bg_color)
    R = q["ray_mask"].shape[0]
    C = opt.shading_color_channel_num
    mask = q["ray_mask"] > 0
    out_color = np.broadcast_to(np.asarray(bg_color, F32).reshape(1, C), (R, C)).copy()
    out_color[mask] = color
    out_op = np.zeros((R, opt.SR), F32)
    out_op[mask] = opacity
    is_bg = np.ones((R, 1), F32)
    is_bg[mask] = bgT
    qs = np.ones((R, 3), F32)
    qs[mask] = np.repeat((~rv.any(-1, keepdims=True)).astype(F32), 3, -1)
    return dict(coarse_raycolor=out_color, coarse_point_opacity=out_op, coarse_is_background=is_bg,
                coarse_mask=1 - is_bg, queried_shading=qs, ray_mask=q["ray_mask"],
                features=feats, ray_valid=rv, ray_dist=rd, query=q)
