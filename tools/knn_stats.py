"""Dev tool: layer statistics of the generic KNN walk (c5's kernel 5) from the
tools/_var/libpnr_qstats.so variant (PNR_LIB): samples, samples reaching
layers 1 / 2, bitmap-word loads and rec_off lookups, per camera."""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c5")
    a = ap.parse_args()
    import bench
    from pointnerf_amd import _lib as L
    cfg = bench.CONFIGS[a.config]
    dev = torch.device("cuda:0")
    opt, pts, feats, agg, model = bench.build_scene(argparse.Namespace(points=cfg["points"], config=a.config,
                                                                       dtype=cfg["dtype"]), dev)
    q = model.neural_points.querier
    xyz = model.neural_points.xyz.detach()
    lib = L.lib()
    out = []
    for ci, (campos, camrot, rd) in enumerate(bench.cameras(8, cfg["H"], cfg["W"], cfg["flags"])[:2]):
        cp, cr, rd = [torch.from_numpy(x).to(dev) for x in (campos, camrot, rd)]
        q.run(xyz, rd, cp, cr, opt.near_plane, opt.far_plane)
        torch.cuda.synchronize()
        assert lib.pnr_dev_knn_stats_reset() == 0
        bufs, hp, rays, qp = q.run(xyz, rd, cp, cr, opt.near_plane, opt.far_plane)
        torch.cuda.synchronize()
        st = (ctypes.c_ulonglong * 8)()
        assert lib.pnr_dev_knn_stats(ctypes.cast(st, ctypes.c_void_p)) == 0
        c = bufs.read_counts()
        out.append({"cam": ci, "samples": st[0], "reach_l1": st[1], "reach_l2": st[2], "word_loads": st[3],
                    "rec_lookups": st[4], "n_cand": c["n_cand"], "S_filled": c["S_filled"]})
    print(json.dumps(out))


if __name__ == "__main__":
    main()
