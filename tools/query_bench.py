"""Dev tool: time the query stage (march + layered KNN + compactions) of the
bench frame (800x800, 2M lego points, grid built once) with the libpnr.so named
by $PNR_LIB; prints one JSON line with the per-query time and the
SURVEY 8(d) KNN bytes."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="headline", help="bench.py config: headline / c4 / c5")
    ap.add_argument("--points", type=int, default=None)
    ap.add_argument("--hw", type=int, default=None)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    import bench
    cfg = bench.CONFIGS[a.config]
    a.points = a.points or cfg["points"]
    H, W = (a.hw, a.hw) if a.hw else (cfg["H"], cfg["W"])
    dev = torch.device("cuda:0")
    opt, pts, feats, agg, model = bench.build_scene(argparse.Namespace(points=a.points, config=a.config,
                                                                       dtype=cfg["dtype"]), dev)
    q = model.neural_points.querier
    xyz = model.neural_points.xyz.detach()
    res = []
    for ci, (campos, camrot, rd) in enumerate(bench.cameras(8, H, W, cfg["flags"])[:4]):
        cp, cr, rd = [torch.from_numpy(x).to(dev) for x in (campos, camrot, rd)]
        near, far = opt.near_plane, opt.far_plane
        bufs, hp, rays, qp = q.run(xyz, rd, cp, cr, near, far)
        torch.cuda.synchronize()
        ts = []
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            q.run(xyz, rd, cp, cr, near, far, bufs=bufs)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        c = bufs.read_counts()
        R = rd.shape[0]
        knn_b = c["S_filled"] * 27 * 8 + c["n_cand"] * 16
        q_b = knn_b + R * int(opt.z_depth_dim) * 4 + R * 16   # bench.stage_rooflines' query bytes
        pid = bufs.pidx[: c["S_filled"] * opt.K].to(torch.int64)
        res.append({"cam": ci, "query_ms": round(float(np.median(ts)), 4), "counts": c, "knn_bytes": knn_b, "query_bytes": q_b,
                    "frac_hbm": round(q_b / (float(np.median(ts)) * 1e-3) / 8e12, 4),
                    "pidx_checksum": int(pid.sum().item())})
    print(json.dumps({"lib": os.environ.get("PNR_LIB", "default"), "cams": res}))


if __name__ == "__main__":
    main()
