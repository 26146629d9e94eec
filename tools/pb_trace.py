"""Dev tool: phase timeline of k_pairs_b<KT> from the diagnostic build
(tools/_var/libpnr_pbtrace<KT>.so: -DPNR_PB_TRACE=KT, s_memtime stamps per phase
of the first 8 tiles of every wave of workgroups < 512).  Renders the c5 frame
twice and prints per-phase cycle medians over waves and tiles 1..6."""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

NAMES = ["prow+P1 issue", "gather", "B(gather)", "unpack", "L1.0b", "act1", "L1.2", "act2", "L3.0", "act3",
         "L3.2", "ksum+alpha parts", "B+alpha/PE", "colour L1+act", "colour L2+act", "colour L3+stage",
         "stores+B"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kt", type=int, default=1)
    a = ap.parse_args()
    os.environ.setdefault("PNR_LIB", os.path.join(ROOT, "tools", "_var", f"libpnr_pbtrace{a.kt}.so"))
    import bench
    dev = torch.device("cuda:0")
    cfg = bench.CONFIGS["c5"]
    ns = argparse.Namespace(points=cfg["points"], config="c5", dtype="bf16")
    opt, pts, feats, agg, model = bench.build_scene(ns, dev)
    model.precision = "bf16"
    campos, camrot, rd = bench.cameras(1, cfg["H"], cfg["W"], cfg["flags"])[0]
    cp, cr, rd = [torch.from_numpy(x).to(dev) for x in (campos, camrot, rd)]
    bg = torch.rand(128, device=dev)
    for _ in range(2):
        model.render_rays(cp, cr, rd, opt.near_plane, opt.far_plane, bg)
    torch.cuda.synchronize()
    lib = ctypes.CDLL(os.environ["PNR_LIB"])
    buf = np.zeros(512 * 4 * 8 * 20, dtype=np.uint64)
    assert lib.pnr_dev_pb_trace(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(buf.nbytes)) == 0
    t = buf.reshape(512, 4, 8, 20).astype(np.int64)
    st = t[:, :, 1:7, :18]
    ok = (st > 0).all(-1)
    d = np.diff(st, axis=-1)[ok]
    res = {"kt": a.kt, "tiles_used": int(ok.sum()),
           "phase_cycles_median": {NAMES[i]: float(np.median(d[:, i])) for i in range(17)}}
    tile = (t[:, :, 2:8, 0] - t[:, :, 1:7, 0])[ok & (t[:, :, 2:8, 0] > 0)]
    res["tile_cycles_median"] = float(np.median(tile)) if tile.size else None
    lay = [4, 6, 8, 10]
    res["pair_layers_frac"] = float(np.median(d[:, lay].sum(1) / d.sum(1)))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
