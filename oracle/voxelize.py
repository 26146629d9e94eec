"""TEST INFRASTRUCTURE ONLY (the checker of tests/, never the product path):
NumPy restatement of construct_vox_points_closest
(models/mvs/mvs_utils.py:537-561, space_min = None).

torch_scatter (scatter_mean / scatter_min) is absent from this image, so the
reductions are restated from its published semantics (torch_scatter 2.x:
scatter_sum then true_divide by the clamped count; scatter_min returns the
arg-min index): sums in ascending point order (the CPU scatter_add order),
arg-min ties to the smallest index.  The space / cell / unique part uses the
same torch ops as the reference (torch.unique(dim=0, return_inverse=True)),
so it is pinned by torch itself; the reductions are parity-unpinned.
"""
import numpy as np
import torch


def construct_vox_points_closest(xyz_val, vox_res):
    xyz_t = torch.as_tensor(np.asarray(xyz_val, dtype=np.float32))
    # mvs_utils.py:540-552 (torch ops, same fp32 rounding as the reference)
    xyz_min, xyz_max = torch.min(xyz_t, dim=-2)[0], torch.max(xyz_t, dim=-2)[0]
    space_edge = torch.max(xyz_max - xyz_min) * 1.05
    xyz_mid = (xyz_max + xyz_min) / 2
    space_min = xyz_mid - space_edge / 2
    construct_vox_sz = space_edge / vox_res
    xyz_shift = xyz_t - space_min[None, ...]
    sparse_grid_idx, inv_idx = torch.unique(torch.floor(xyz_shift / construct_vox_sz[None, ...]).to(torch.int32),
                                            dim=0, return_inverse=True)
    inv = inv_idx.numpy()
    xyz = xyz_t.numpy()
    m = sparse_grid_idx.shape[0]
    # scatter_mean: sequential fp32 sums in point order, / count
    s = np.zeros((m, 3), np.float32)
    np.add.at(s, inv, xyz)
    cnt = np.bincount(inv, minlength=m).astype(np.float32)
    centroid = (s / cnt[:, None]).astype(np.float32)
    # scatter_min of |xyz - centroid[inv]|: arg-min, ties to the smallest index
    d = (xyz - centroid[inv]).astype(np.float32)
    r = np.sqrt(((d[:, 0] * d[:, 0]) + (d[:, 1] * d[:, 1])) + (d[:, 2] * d[:, 2])).astype(np.float32)
    order = np.lexsort((np.arange(len(r)), r, inv))      # by voxel, then residual, then index
    first = np.ones(len(order), bool)
    first[1:] = inv[order[1:]] != inv[order[:-1]]
    min_idx = np.empty(m, np.int64)
    min_idx[inv[order[first]]] = order[first]
    return centroid, sparse_grid_idx.numpy(), min_idx, inv.astype(np.int64)
