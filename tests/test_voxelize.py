"""Point-cloud init down-sampling (construct_vox_points_closest,
models/mvs/mvs_utils.py:537-561): the oracle restatement (CPU) and the HIP
pipeline pnr_vox_closest against it (GPU).  The cell / unique part is pinned by
torch.unique itself; torch_scatter is absent, so the reductions are checked
against their published semantics (parity unpinned)."""
import os
import sys

import numpy as np
import pytest
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle.voxelize import construct_vox_points_closest as oracle_vox  # noqa: E402


def _cloud(n, seed, lattice=False):
    rng = np.random.default_rng(seed)
    x = rng.normal(size=(n, 3)).astype(np.float32) * np.float32(0.6)
    if lattice:   # exact duplicates and equal residuals: exercises the tie rule
        x = (np.round(x * 8) / 8).astype(np.float32)
    return x


@pytest.mark.parametrize("lattice", [False, True])
def test_oracle_reductions_by_brute_force(lattice):
    x = _cloud(3000, 1, lattice)
    c, g, m, inv = oracle_vox(x, 24)
    assert np.array_equal(np.unique(g, axis=0), g)          # lexicographic, unique
    for v in range(0, len(g), 37):
        pts = np.nonzero(inv == v)[0]
        s = np.zeros(3, np.float32)
        for p in pts:                                         # scatter_add order
            s = (s + x[p]).astype(np.float32)
        assert np.array_equal(c[v], (s / np.float32(len(pts))).astype(np.float32))
        r = np.sqrt(((x[pts] - c[v]) ** 2).sum(1).astype(np.float32))
        assert m[v] == pts[np.argmin(r)]                      # argmin: first minimum


@pytest.mark.gpu
@pytest.mark.parametrize("lattice", [False, True])
@pytest.mark.parametrize("n,res", [(7, 8), (5000, 16), (60000, 128)])
def test_gpu_vox_closest_bit_exact(cuda, lattice, n, res):
    from pointnerf_amd.voxelize import construct_vox_points_closest
    x = _cloud(n, 2 + n, lattice)
    c, g, m, inv = oracle_vox(x, res)
    gc, gg, gm, ginv = construct_vox_points_closest(torch.from_numpy(x).to(cuda), res, return_inverse=True)
    assert np.array_equal(gg.cpu().numpy(), g)
    assert np.array_equal(ginv.cpu().numpy(), inv)
    assert np.array_equal(gc.cpu().numpy(), c)
    assert np.array_equal(gm.cpu().numpy(), m)


@pytest.mark.gpu
def test_gpu_vox_closest_2m_properties(cuda):
    """The 2M-point lego-like cloud at vox_res 800: the picked point of every
    voxel lies in that voxel, every point belongs to exactly one voxel, the
    voxel list is strictly increasing; deterministic across calls."""
    from pointnerf_amd import synthetic as S
    from pointnerf_amd.voxelize import construct_vox_points_closest
    x = torch.from_numpy(S.lego_like_points(2_000_000, seed=3)).to(cuda)
    c, g, m, inv = construct_vox_points_closest(x, 800, return_inverse=True)
    c2, g2, m2 = construct_vox_points_closest(x, 800)
    assert torch.equal(c, c2) and torch.equal(g, g2) and torch.equal(m, m2)
    assert torch.equal(inv[m], torch.arange(g.shape[0], device=cuda))
    key = (g[:, 0].long() << 42) | (g[:, 1].long() << 21) | g[:, 2].long()
    assert bool((key[1:] > key[:-1]).all())
    assert int(torch.bincount(inv, minlength=g.shape[0]).sum()) == x.shape[0]
