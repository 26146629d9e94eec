import os, sys
sys.path[:0] = [os.getcwd(), "tests"]
import numpy as np, torch
from oracle.voxelize import construct_vox_points_closest as oracle_vox
from pointnerf_amd.voxelize import construct_vox_points_closest
from test_voxelize import _cloud
x = _cloud(5000, 5002, False)
c, g, m, inv = oracle_vox(x, 16)
gc, gg, gm, ginv = construct_vox_points_closest(torch.from_numpy(x).cuda(), 16, return_inverse=True)
gc = gc.cpu().numpy()
bad = np.nonzero((gc != c).any(1))[0]
print("bad voxels", len(bad), "of", len(c))
for v in bad[:3]:
    pts = np.nonzero(inv == v)[0]
    s = np.zeros(3, np.float32)
    for p in pts: s = (s + x[p]).astype(np.float32)
    s64 = x[pts].astype(np.float64).sum(0)
    print(v, len(pts), c[v], gc[v], s / np.float32(len(pts)), s64 / len(pts))
