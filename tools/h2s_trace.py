"""Dev tool: phase timeline of k_pairs_h2s from the diagnostic build
(tools/_var/libpnr_trace.so, -DPNR_H2S_TRACE: s_memtime stamps per phase of the
first 8 tiles of every wave).  Renders one 800x800 frame (2M points) with
PNR_PAIRS_H2S=1 and prints per-phase cycle medians and the phase overlap of the
two workgroups that share a CU."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("PNR_LIB", os.path.join(ROOT, "tools", "_var", "libpnr_trace.so"))
os.environ.setdefault("PNR_PAIRS_H2S", "1")

NAMES = ["top", "gather+pe", "B0", "L1.0", "B2(act1)", "L1.2", "B4(act2)", "L3.0", "B6(act3)", "L3.2", "tail",
         "p1issue", "B7"]


def main():
    import bench
    dev = torch.device("cuda:0")
    ns = __import__("argparse").Namespace(points=2_000_000, config="headline", dtype="fp32h2")
    opt, pts, feats, agg, model = bench.build_scene(ns, dev)
    model.precision = "fp32h2"
    campos, camrot, rd = bench.cameras(1, 800, 800)[0]
    cp, cr, rd = [torch.from_numpy(x).to(dev) for x in (campos, camrot, rd)]
    bg = torch.rand(128, device=dev)
    model.render_rays(cp, cr, rd, 2.0, 6.0, bg)
    model.render_rays(cp, cr, rd, 2.0, 6.0, bg)
    torch.cuda.synchronize()
    lib = ctypes.CDLL(os.environ["PNR_LIB"])
    buf = np.zeros(512 * 4 * 8 * 16, dtype=np.uint64)
    assert lib.pnr_dev_h2s_trace(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(buf.nbytes)) == 0
    t = buf.reshape(512, 4, 8, 16).astype(np.int64)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    np.save(os.path.join(ROOT, "gpurun_out", "h2s_trace.npy"), t)
    hw = t[:, 0, 0, 14]
    xcc = t[:, 0, 0, 15]
    # phase durations (stamp i+1 - stamp i) of tiles 1..6, wave 0..3
    st = t[:, :, 1:7, :13]
    d = np.diff(st, axis=-1)
    res = {"phase_cycles_median": {NAMES[i + 1]: float(np.median(d[..., i])) for i in range(12)}}
    tile = t[:, :, 2:8, 0] - t[:, :, 1:7, 0]
    res["tile_cycles_median"] = float(np.median(tile))
    # CU partners: same xcc, same HW_ID bits except the wave slot
    cu = (xcc << 16) | ((hw >> 8) & 0xFF) | (((hw >> 13) & 0x7) << 8)
    groups = {}
    for b in range(512):
        groups.setdefault(int(cu[b]), []).append(b)
    res["wg_per_cu_hist"] = {str(k): int(v) for k, v in zip(*np.unique([len(g) for g in groups.values()], return_counts=True))}
    # overlap of the partners' MFMA phases (wave 0, layers = phases 3,5,7,9), tiles 1..6
    fr = []
    for g in groups.values():
        if len(g) != 2:
            continue
        a, b = g
        def layers(blk):
            s = t[blk, 0, 1:7]
            return [(s[i][j], s[i][j + 1]) for i in range(6) for j in (2, 4, 6, 8)]
        la, lb = layers(a), layers(b)
        lo = max(min(x[0] for x in la), min(x[0] for x in lb))
        hi = min(max(x[1] for x in la), max(x[1] for x in lb))
        if hi <= lo:
            continue
        grid = np.linspace(lo, hi, 2000)
        ina = np.zeros_like(grid, bool)
        inb = np.zeros_like(grid, bool)
        for x0, x1 in la:
            ina |= (grid >= x0) & (grid < x1)
        for x0, x1 in lb:
            inb |= (grid >= x0) & (grid < x1)
        fr.append([(ina & inb).mean(), (ina ^ inb).mean(), (~ina & ~inb).mean()])
    if fr:
        f = np.array(fr)
        res["partners_in_layers"] = {"both": float(f[:, 0].mean()), "one": float(f[:, 1].mean()),
                                     "none": float(f[:, 2].mean()), "pairs": len(fr)}
    print(json.dumps(res, indent=1, default=float))


if __name__ == "__main__":
    main()
