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
