"""Dev tool: time the sync-free voxel-grid build (pnr_grid_build_dev) of the
bench cloud (2M lego points) with HIP events, check its tables against the C
oracle at that size, and print one JSON line.  Run it under
`rocprofv3 --kernel-trace --stats` for the per-kernel split."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="headline")
    ap.add_argument("--points", type=int, default=None)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--no-oracle", action="store_true")
    a = ap.parse_args()
    import bench
    cfg = bench.CONFIGS[a.config]
    a.points = a.points or cfg["points"]
    from oracle import oracle as O
    dev = torch.device("cuda:0")
    opt, pts, feats, agg, model = bench.build_scene(
        argparse.Namespace(points=a.points, config=a.config, dtype=cfg["dtype"]), dev)
    q = model.neural_points.querier
    xyz = model.neural_points.xyz.detach().contiguous()
    ts = []
    for _ in range(a.reps):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        q.grid.build(opt, xyz, force=True)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    st = q.grid.stats()
    out = {"config": a.config, "points": a.points, "build_ms_median": round(float(np.median(ts)), 4),
           "build_ms": [round(x, 4) for x in ts], "n_voxels": int(st["n_voxels"]),
           "n_voxels_kept": int(st["n_voxels_kept"]), "n_points_dropped": int(st["n_points_dropped"])}
    if not a.no_oracle:
        g = O.grid_build(opt, pts)
        t = q.grid.export()
        out["oracle_n_occ"] = int(g["n_occ"])
        out["bit_exact"] = {k: bool(np.array_equal(t[k].cpu().numpy(), g[k]))
                            for k in ("coor_2_occ", "occ_numpnts", "occ_2_pnts")}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
