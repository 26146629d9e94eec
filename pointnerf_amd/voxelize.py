"""Point-cloud initialisation on libpnr.so: voxel down-sampling to the point
closest to each voxel centroid.

Mirrors ``construct_vox_points_closest`` of models/mvs/mvs_utils.py:537-561
(same name, arguments and outputs), which the reference drivers use to turn
the MVS / lidar cloud into the initial neural points (train_ddp.py:135,
train_waymo_v1.py:145, 615): torch.unique of the voxel cells plus
torch_scatter's scatter_mean / scatter_min, here one HIP pipeline
(pnr_vox_closest: keys, stable radix sort, run scan, per-voxel reductions).
"""
from __future__ import annotations

import torch

from . import _lib as L


def construct_vox_points_closest(xyz_val: torch.Tensor, vox_res: int, partition_xyz=None, space_min=None,
                                 space_max=None, return_inverse: bool = False):
    """mvs_utils.py:537-561 with space_min = None (the form every reference
    caller uses) -> (xyz_centroid [M,3] fp32, sparse_grid_idx [M,3] int32,
    min_idx [M] int64) [, inv_idx [N] int64].  min_idx ties go to the smallest
    point index (torch_scatter's scatter_min leaves them to atomics)."""
    if partition_xyz is not None or space_min is not None or space_max is not None:
        raise L.PnrError("construct_vox_points_closest: only partition_xyz = space_min = space_max = None "
                         "(the reference drivers' call) is implemented by libpnr")
    L.require_gpu(xyz_val)
    xyz = xyz_val.reshape(-1, 3).float().contiguous()
    n = xyz.shape[0]
    if n == 0:
        raise L.PnrError("construct_vox_points_closest: empty point cloud")
    dev = xyz.device
    nb = L.c_size_t(0)
    L.check(L.lib().pnr_vox_closest_scratch_bytes(n, L.ctypes.byref(nb)), "pnr_vox_closest_scratch_bytes")
    scratch = torch.empty((int(nb.value) + 15) // 16 * 16, dtype=torch.uint8, device=dev)
    centroid = torch.empty((n, 3), dtype=torch.float32, device=dev)
    grid = torch.empty((n, 3), dtype=torch.int32, device=dev)
    min_idx = torch.empty(n, dtype=torch.int64, device=dev)
    inv = torch.empty(n, dtype=torch.int32, device=dev) if return_inverse else None
    counts = torch.zeros(2, dtype=torch.int32, device=dev)
    L.check(L.lib().pnr_vox_closest(L.ptr(xyz), n, int(vox_res), L.ptr(centroid), L.ptr(grid), L.ptr(min_idx),
                                    L.ptr(inv), L.ptr(counts), L.ptr(scratch), scratch.numel(), L.stream_ptr(dev)),
            "pnr_vox_closest")
    m, bad = counts.tolist()
    if bad:
        raise L.PnrError("construct_vox_points_closest: a voxel coordinate left +-2^20")
    out = (centroid[:m], grid[:m], min_idx[:m])
    return out + (inv.long(),) if return_inverse else out
