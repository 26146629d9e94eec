import os, sys
sys.path[:0] = [os.getcwd(), "tests"]
import numpy as np, torch
from oracle.voxelize import construct_vox_points_closest as oracle_vox
from pointnerf_amd.voxelize import construct_vox_points_closest
from test_voxelize import _cloud
for n, res in [(7, 8), (7, 8), (5000, 16), (60000, 128), (5000, 16)]:
    for lat in (False, True):
        x = _cloud(n, 2 + n, lat)
        c, g, m, inv = oracle_vox(x, res)
        for rep in range(3):
            gc, gg, gm, ginv = construct_vox_points_closest(torch.from_numpy(x).cuda(), res, return_inverse=True)
            gc, gm, ginv = gc.cpu().numpy(), gm.cpu().numpy(), ginv.cpu().numpy()
            badc = np.nonzero((gc != c).any(1))[0]
            print(n, res, lat, rep, "grid", np.array_equal(gg.cpu().numpy(), g), "inv", np.array_equal(ginv, inv),
                  "cent bad", len(badc), "min bad", int((gm != m).sum()), flush=True)
            for v in badc[:2]:
                pts = np.nonzero(inv == v)[0]
                print("   v", v, len(pts), c[v], gc[v], (x[pts].astype(np.float64).sum(0) / len(pts)))
