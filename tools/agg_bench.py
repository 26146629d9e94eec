"""Dev tool: time the stages of one 800x800 frame render (2M points) with the
libpnr.so named by $PNR_LIB; prints one JSON line."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--points", type=int, default=2_000_000)
    ap.add_argument("--hw", type=int, default=800)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--precision", default="fp32")
    ap.add_argument("--config", default="headline", choices=("headline", "c4", "c5"))
    ap.add_argument("--p1-all", action="store_true", help="bf16: P1 for every point (not only the referenced)")
    a = ap.parse_args()
    import bench
    dev = torch.device("cuda:0")
    cfg = bench.CONFIGS[a.config]
    pts_n = a.points if a.config == "headline" else cfg["points"]
    H, W = (a.hw, a.hw) if a.config == "headline" else (cfg["H"], cfg["W"])
    ns = argparse.Namespace(points=pts_n, config=a.config, dtype=a.precision)
    opt, pts, feats, agg, model = bench.build_scene(ns, dev)
    model.precision = a.precision
    model.p1_used_only = not a.p1_all
    campos, camrot, rd = bench.cameras(1, H, W, cfg["flags"])[0]
    cp, cr, rd = [torch.from_numpy(x).to(dev) for x in (campos, camrot, rd)]
    bg = torch.rand(128, device=dev)
    near, far = opt.near_plane, opt.far_plane
    model.render_rays(cp, cr, rd, near, far, bg)
    per = {}
    for _ in range(a.reps):
        ev = []
        out = model.render_rays(cp, cr, rd, near, far, bg, events=ev)
        torch.cuda.synchronize()
        for n, s, e in ev:
            per.setdefault(n, []).append(s.elapsed_time(e))
    c = model.last_counts
    flops = c["n_pairs"] * 542720 + c["S_valid"] * 137216
    agg_ms = float(np.median(per["aggregate"]))
    print(json.dumps({"lib": os.environ.get("PNR_LIB", "default"),
                      "stages_ms": {k: round(float(np.median(v)), 3) for k, v in per.items()},
                      "agg_tflops": round(flops / agg_ms / 1e9, 2), "counts": c,
                      "checksum": float(out[0].double().sum().item())}))


if __name__ == "__main__":
    main()
