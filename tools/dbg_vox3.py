import os, sys
sys.path[:0] = [os.getcwd(), "tests"]
import numpy as np, torch
from oracle.voxelize import construct_vox_points_closest as oracle_vox
from pointnerf_amd.voxelize import construct_vox_points_closest
from test_voxelize import _cloud
x = _cloud(60000, 60002, False)
c, g, m, inv = oracle_vox(x, 128)
gc, gg, gm, ginv = construct_vox_points_closest(torch.from_numpy(x).cuda(), 128, return_inverse=True)
gm = gm.cpu().numpy()
bad = np.nonzero(gm != m)[0]
for v in bad[:4]:
    pts = np.nonzero(inv == v)[0]
    d = (x[pts] - c[v]).astype(np.float32)
    r2 = ((d[:, 0] * d[:, 0]) + (d[:, 1] * d[:, 1])) + (d[:, 2] * d[:, 2])
    print("v", v, "pts", pts.tolist(), "oracle", m[v], "gpu", gm[v])
    print("   r2", [float(t) for t in r2], "r", [float(t) for t in np.sqrt(r2)])
