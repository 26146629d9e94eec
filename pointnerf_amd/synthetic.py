"""Seeded synthetic scenes of the lego configuration (no datasets offline).

Points: surfaces (ellipsoid shells, box shells, a ground slab) inside the
lego ``ranges`` of dev_scripts/w_n360/lego.sh, capped at P-1 points per query
voxel so the voxel tables never overflow (reservoir sampling in the reference
has no reproducible result).  Features follow the reference initialisers:
embedding ~ U(-0.5, 0.5) (neural_points.py:292), colour/dir ~ N(0, 1),
conf = default_conf 0.15 (lego.sh).  Cameras: NeRF-synthetic orbit
(nerf_synth360_ft_dataset.py:45-72, radius 4, elevation -30 deg, focal
1111.111 at 800^2), converted to the OpenCV camrotc2w the renderer consumes;
ray directions as get_dtu_raydir with dir_norm 0 (data/data_utils.py:55-69).
"""
from __future__ import annotations

import math

import numpy as np
import torch


def _ellipsoid(rng, n, c, r):
    v = rng.normal(size=(n, 3))
    v /= np.linalg.norm(v, axis=1, keepdims=True)
    return c + v * r


def _box(rng, n, lo, hi):
    lo, hi = np.asarray(lo, float), np.asarray(hi, float)
    ext = hi - lo
    areas = np.array([ext[1] * ext[2], ext[0] * ext[2], ext[0] * ext[1]]) * 2
    face = rng.choice(3, size=n, p=areas / areas.sum())
    p = lo + rng.uniform(size=(n, 3)) * ext
    side = rng.integers(0, 2, size=n)
    p[np.arange(n), face] = np.where(side, hi[face], lo[face])
    return p


def lego_like_points(n_points: int, seed: int = 0, ranges=(-0.638, -1.141, -0.346, 0.634, 1.149, 1.141),
                     vsize=0.004, vscale=2, kernel=3, cap: int = 8) -> np.ndarray:
    """[n_points, 3] float32, <= cap points in every query voxel of the grid the
    querier will build (the bbox is clipped to ``ranges`` by a ground slab that
    spans them, so the grid origin does not depend on the sampling)."""
    rng = np.random.default_rng(seed)
    lo, hi = np.asarray(ranges[:3]), np.asarray(ranges[3:])
    ctr, half = (lo + hi) / 2, (hi - lo) / 2
    over = int(n_points * 1.6) + 1000
    shapes = [  # (weight, sampler)
        (0.22, lambda m: _ellipsoid(rng, m, ctr + [0, 0, 0.05], half * [0.85, 0.8, 0.75])),
        (0.14, lambda m: _ellipsoid(rng, m, ctr + [0.1, -0.3, 0.2], half * [0.45, 0.4, 0.5])),
        (0.14, lambda m: _ellipsoid(rng, m, ctr + [-0.15, 0.4, -0.1], half * [0.5, 0.35, 0.45])),
        (0.18, lambda m: _box(rng, m, ctr - half * [0.7, 0.6, 0.3], ctr + half * [0.6, 0.7, 0.2])),
        (0.12, lambda m: _box(rng, m, ctr - half * [0.3, 0.9, 0.8], ctr + half * [0.35, 0.2, 0.9])),
        (0.20, lambda m: np.stack([rng.uniform(lo[0] - 0.02, hi[0] + 0.02, m),
                                   rng.uniform(lo[1] - 0.02, hi[1] + 0.02, m),
                                   np.where(rng.uniform(size=m) < 0.5, lo[2] - 0.001, hi[2] + 0.001)], 1)),
    ]
    pts = np.concatenate([f(int(over * w)) for w, f in shapes]).astype(np.float32)
    # cap points per voxel of the querier's grid (qpiw.py:48-81 with the bbox clipped to ranges)
    vs = np.float32(vsize * vscale)
    shift = (np.asarray(lo, np.float32) - np.float32(vs * kernel / 2)).astype(np.float32)
    cell = np.floor((pts - shift) / vs).astype(np.int64)
    key = (cell[:, 0] * 4096 + cell[:, 1]) * 4096 + cell[:, 2]
    order = rng.permutation(len(pts))
    key_o = key[order]
    srt = np.argsort(key_o, kind="stable")
    ks = key_o[srt]
    first = np.r_[0, np.nonzero(np.diff(ks))[0] + 1]
    rank = np.arange(len(ks)) - np.repeat(first, np.diff(np.r_[first, len(ks)]))
    keep = order[srt[rank < cap]]
    if len(keep) < n_points:
        raise ValueError(f"only {len(keep)} points after the per-voxel cap; lower n_points")
    keep = rng.choice(keep, size=n_points, replace=False)
    return pts[np.sort(keep)]


def _ellipsoid_shell(rng, n, c, r):
    return _ellipsoid(rng, n, np.asarray(c, float), np.asarray(r, float))


def _disk(rng, n, c, radius, axis=2):
    """Uniform disk of the given radius, normal along `axis`, centred at c."""
    rho = radius * np.sqrt(rng.uniform(size=n))
    phi = rng.uniform(0, 2 * np.pi, size=n)
    p = np.repeat(np.asarray(c, float)[None], n, 0)
    a, b = [i for i in range(3) if i != axis]
    p[:, a] += rho * np.cos(phi)
    p[:, b] += rho * np.sin(phi)
    return p


def _plane(rng, n, lo, hi, axis, value):
    p = np.asarray(lo, float) + rng.uniform(size=(n, 3)) * (np.asarray(hi, float) - np.asarray(lo, float))
    p[:, axis] = value
    return p


# Surfaces of the non-lego flag sets, all inside the scene script's `ranges`
# (options.FLAGSETS): (weight, sampler(rng, m)).
SCENE_SHAPES = {
    # NeRF-synthetic ship: hull, deck, cabin, mast, water disk (ship.sh ranges)
    "ship": [
        (0.25, lambda r, m: _ellipsoid_shell(r, m, [0.05, 0.0, -0.15], [1.1, 0.45, 0.3])),
        (0.12, lambda r, m: _box(r, m, [-0.8, -0.35, 0.0], [0.7, 0.35, 0.15])),
        (0.10, lambda r, m: _box(r, m, [-0.3, -0.2, 0.15], [0.2, 0.2, 0.45])),
        (0.05, lambda r, m: _box(r, m, [0.3, -0.03, 0.15], [0.36, 0.03, 0.7])),
        (0.28, lambda r, m: _disk(r, m, [0.05, 0.02, -0.45], 1.3)),
        (0.10, lambda r, m: _ellipsoid_shell(r, m, [0.05, 0.0, -0.1], [0.95, 0.38, 0.22])),
        (0.10, lambda r, m: np.concatenate([_box(r, m // 3 + (i < m % 3), [x - 0.12, -0.3, 0.15],
                                                  [x + 0.12, 0.3, 0.3]) for i, x in enumerate([-0.6, 0.45, 0.7])])),
    ],
    # ScanNet-like room (z up, metres): floor / walls / ceiling, bed, table, cabinet, sofa
    "scene101": [
        (0.45, lambda r, m: _box(r, m, [-2.4, -2.0, 0.0], [2.6, 2.2, 2.7])),
        (0.15, lambda r, m: _box(r, m, [-2.2, -1.8, 0.0], [-0.6, 0.2, 0.5])),
        (0.10, lambda r, m: _box(r, m, [0.8, 0.5, 0.0], [1.8, 1.5, 0.75])),
        (0.12, lambda r, m: _box(r, m, [1.9, -1.9, 0.0], [2.5, -0.9, 1.8])),
        (0.18, lambda r, m: _ellipsoid_shell(r, m, [0.0, 1.6, 0.4], [0.9, 0.4, 0.4])),
    ],
    # Tanks&Temples-like truck (y down, normalised units): ground, cargo box, cab, wheels
    "truck": [
        (0.35, lambda r, m: _plane(r, m, [-1.1, 0.19, -1.04], [0.78, 0.19, 1.02], 1, 0.19)),
        (0.30, lambda r, m: _box(r, m, [-0.75, -0.45, -0.5], [0.45, 0.1, 0.85])),
        (0.15, lambda r, m: _box(r, m, [-0.6, -0.3, -0.95], [0.3, 0.1, -0.5])),
        (0.20, lambda r, m: np.concatenate([
            _ellipsoid_shell(r, m // 4 + (i < m % 4), [x, 0.1, z], [0.04, 0.09, 0.09])
            for i, (x, z) in enumerate([(-0.78, -0.7), (0.48, -0.7), (-0.78, 0.6), (0.48, 0.6)])])),
    ],
}


def scene_points(name: str, n_points: int, opt, seed: int = 0, cap: int | None = None,
                 scatter: float = 0.0) -> np.ndarray:
    """[n_points, 3] float32 surface samples of SCENE_SHAPES[name] inside opt.ranges,
    with <= cap (default P - 1) points in every voxel of the grid the querier
    builds for them (qpiw.py:48-81: the bbox of the returned points clipped to
    ranges): the six extreme points of the oversampled set are always kept, so
    the bbox -- hence the grid origin the cap was computed on -- is fixed.
    cap < 0: no cap (the cloud may overflow P and max_o: the reference's
    reservoir case); scatter: that fraction of the points spread uniformly over
    the ranges (stray MVS points, one per voxel -- what makes a real cloud
    occupy more voxels than max_o)."""
    from .querier import hyperparameters_from_bbox
    cap = int(opt.P) - 1 if cap is None else int(cap)
    if cap < 0:
        rng = np.random.default_rng(seed)
        lo, hi = np.asarray(opt.ranges[:3], np.float32), np.asarray(opt.ranges[3:], np.float32)
        n_sc = int(round(n_points * scatter))
        parts, need = [], n_points - n_sc
        while need > 0:   # surface samples, rejection-clipped to the ranges
            m = int(need * 1.1) + 1000
            p = np.concatenate([f(rng, max(1, int(m * w))) for w, f in SCENE_SHAPES[name]]).astype(np.float32)
            p = p[np.all((p >= lo) & (p <= hi), axis=1)][:need]
            parts.append(p)
            need -= len(p)
        parts.append((lo + rng.uniform(size=(n_sc, 3)) * (hi - lo)).astype(np.float32))
        pts = np.concatenate(parts)
        return pts[rng.permutation(len(pts))]
    for factor in (1.8, 3.0, 5.0, 8.0):   # oversample until the capped set holds n_points
        rng = np.random.default_rng(seed)
        over = int(n_points * factor) + 1000
        lo, hi = np.asarray(opt.ranges[:3], np.float32), np.asarray(opt.ranges[3:], np.float32)
        pts = np.concatenate([f(rng, int(over * w)) for w, f in SCENE_SHAPES[name]]).astype(np.float32)
        pts = pts[np.all((pts >= lo) & (pts <= hi), axis=1)]
        mn, mx = pts.min(0), pts.max(0)
        hp = hyperparameters_from_bbox(opt, mn, mx)
        cell = np.floor((pts - hp["shift"]) / hp["vsize_s"]).astype(np.int64)
        key = (cell[:, 0] * 8192 + cell[:, 1]) * 8192 + cell[:, 2]
        anchors = np.unique(np.concatenate([pts.argmin(0), pts.argmax(0)]))
        order = rng.permutation(len(pts))
        order = np.concatenate([anchors, order[~np.isin(order, anchors)]])   # anchors win their voxel
        key_o = key[order]
        srt = np.argsort(key_o, kind="stable")
        ks = key_o[srt]
        first = np.r_[0, np.nonzero(np.diff(ks))[0] + 1]
        rank = np.arange(len(ks)) - np.repeat(first, np.diff(np.r_[first, len(ks)]))
        keep = order[srt[rank < cap]]
        if len(keep) >= n_points:
            break
    else:
        raise ValueError(f"{name}: only {len(keep)} points after the per-voxel cap; lower n_points")
    rest = keep[~np.isin(keep, anchors)]
    keep = np.concatenate([anchors, rng.choice(rest, size=n_points - len(anchors), replace=False)])
    out = pts[np.sort(keep)]
    assert np.array_equal(out.min(0), mn) and np.array_equal(out.max(0), mx)
    return out


def look_at(campos, target, up) -> tuple[np.ndarray, np.ndarray]:
    """(campos[3], camrotc2w[3,3]) of a camera at campos looking at target, OpenCV
    axes (x right, y down, z forward) as the renderer consumes them."""
    c = np.asarray(campos, np.float64)
    z = np.asarray(target, np.float64) - c
    z /= np.linalg.norm(z)
    x = np.cross(z, np.asarray(up, np.float64))
    x /= np.linalg.norm(x)
    y = np.cross(z, x)
    return c.astype(np.float32), np.stack([x, y, z], 1).astype(np.float32)


def scene_camera(name: str, view: int = 0, n_views: int = 8):
    """(campos, camrotc2w) of view `view` of n_views for a flag set: the NeRF
    orbit for lego / ship, a pan inside the room for scene101, an orbit around
    the truck."""
    a = 2 * np.pi * view / n_views
    if name in ("lego", "ship"):
        return camera(-180.0 + 360.0 * view / n_views, -30.0, 4.0)
    if name == "scene101":
        return look_at([0.2, -0.4, 1.5], [0.2 + 2.0 * np.cos(a), -0.4 + 2.0 * np.sin(a), 0.9], [0, 0, 1])
    if name == "truck":
        ctr = np.array([-0.15, -0.15, 0.0])
        return look_at(ctr + [2.0 * np.cos(a), -0.6, 2.0 * np.sin(a)], ctr, [0, -1, 0])
    raise KeyError(name)


# (W, H, focal at that width) of each flag set's camera
SCENE_INTRINSICS = {"lego": (800, 800, 0.5 * 800 / math.tan(0.5 * 0.6911112070083618)),
                    "ship": (800, 800, 0.5 * 800 / math.tan(0.5 * 0.6911112070083618)),
                    "scene101": (1296, 968, 1170.0),     # ScanNet colour camera
                    "truck": (1920, 1080, 1160.0)}       # Tanks&Temples full resolution (~66 deg hfov)


def point_features(n: int, seed: int = 0, default_conf: float | None = 0.15):
    g = torch.Generator().manual_seed(seed)
    emb = torch.rand((n, 32), generator=g) - 0.5
    color = torch.randn((n, 3), generator=g)
    dirs = torch.randn((n, 3), generator=g)
    conf = torch.full((n, 1), default_conf) if default_conf is not None else torch.rand((n, 1), generator=g)
    return emb, color, dirs, conf


def pose_spherical(theta_deg: float, phi_deg: float, radius: float) -> np.ndarray:
    """Blender c2w of the NeRF-synthetic orbit (nerf_synth360_ft_dataset.py:45-72)."""
    t = np.eye(4)
    t[2, 3] = radius
    ph, th = math.radians(phi_deg), math.radians(theta_deg)
    rphi = np.array([[1, 0, 0, 0], [0, math.cos(ph), -math.sin(ph), 0], [0, math.sin(ph), math.cos(ph), 0],
                     [0, 0, 0, 1]])
    rth = np.array([[math.cos(th), 0, -math.sin(th), 0], [0, 1, 0, 0], [math.sin(th), 0, math.cos(th), 0],
                    [0, 0, 0, 1]])
    swap = np.array([[-1, 0, 0, 0], [0, 0, 1, 0], [0, 1, 0, 0], [0, 0, 0, 1]], float)
    return swap @ rth @ rphi @ t


def camera(theta_deg: float = 30.0, phi_deg: float = -30.0, radius: float = 4.0):
    """(campos[3], camrotc2w[3,3]) in the OpenCV convention used by the renderer."""
    c2w = pose_spherical(theta_deg, phi_deg, radius) @ np.diag([1.0, -1.0, -1.0, 1.0])
    return c2w[:3, 3].astype(np.float32), c2w[:3, :3].astype(np.float32)


def pixel_rays(H: int, W: int, focal: float, camrot: np.ndarray, pixels: np.ndarray | None = None):
    """get_dtu_raydir (data/data_utils.py:55-69), dir_norm 0: [R,3] float32."""
    if pixels is None:
        px, py = np.meshgrid(np.arange(W, dtype=np.float32), np.arange(H, dtype=np.float32))
        pixels = np.stack([px, py], -1).reshape(-1, 2)
    x = (pixels[:, 0] + 0.5 - W / 2) / focal
    y = (pixels[:, 1] + 0.5 - H / 2) / focal
    d = np.stack([x, y, np.ones_like(x)], -1)
    return (d @ camrot.astype(np.float64).T).astype(np.float32)


def lego_focal(H: int = 800) -> float:
    return 0.5 * H / math.tan(0.5 * 0.6911112070083618)
