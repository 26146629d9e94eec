"""Dev tool: per-phase cycle stamps of k_pairs_x3 block 0 (build with
tools/build_variant.sh trace -DPNR_TRACE=1, run with PNR_LIB=tools/_ablate/trace/libpnr.so)."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import argparse
    import bench
    dev = torch.device("cuda:0")
    opt, pts, feats, agg, model = bench.build_scene(argparse.Namespace(points=2_000_000), dev)
    model.precision = os.environ.get("PNR_PREC", "fp32h2")
    campos, camrot, rd = bench.cameras(1, 800, 800)[0]
    cp, cr, rd = [torch.from_numpy(x).to(dev) for x in (campos, camrot, rd)]
    bg = torch.rand(128, device=dev)
    for _ in range(2):
        model.render_rays(cp, cr, rd, 2.0, 6.0, bg)
    torch.cuda.synchronize()
    from pointnerf_amd import _lib as L
    buf = (ctypes.c_ulonglong * (2 * 64 * 16))()
    fn = L.lib().pnr_debug_x3_trace
    fn.restype = ctypes.c_int
    assert fn(buf, 2 * 64 * 16) == 0
    t = np.frombuffer(buf, dtype=np.uint64).reshape(2, 64, 16).astype(np.int64)
    c = t[0, 8:60]
    names = ["layer1", "S1 wait", "P1 add+S1b", "store1", "S2 wait", "layer2", "S3 wait", "store2+S4", "layer3",
             "S5 wait", "store3+S6", "layer4", "tail", "S7 wait"]
    c = c[:, :15]
    d = np.diff(c, axis=1)
    tile = c[1:, 0] - c[:-1, 0]
    print("consumer wave 0, cycles per tile (median over tiles 8..59): total", int(np.median(tile)))
    for i, nme in enumerate(names):
        print(f"  {nme:14s} {int(np.median(d[:, i])):7d}")
    s15 = t[0, 8:60, 15] - t[0, 8:60, 3]
    print(f"  (store_act of store1 alone: {int(np.median(s15))})")
    blk = (ctypes.c_ulonglong * (1024 * 2))()
    assert L.lib().pnr_debug_x3_blocks(blk, 2048) == 0
    b = np.frombuffer(blk, dtype=np.uint64).reshape(1024, 2).astype(np.int64)
    b = b[b[:, 1] > 0]
    dur = (b[:, 1] - b[:, 0]) / 100.0   # wall clock: 100 MHz -> microseconds
    t0 = b[:, 0].min()
    print(f"blocks {len(b)}: loop us min {dur.min():.0f} median {np.median(dur):.0f} max {dur.max():.0f}; "
          f"start spread us {(b[:, 0].max() - t0) / 100:.0f}; end spread us {(b[:, 1].max() - b[:, 1].min()) / 100:.0f}")
    order = np.argsort(-dur)[:8]
    print("slowest blocks:", [(int(i), round(float(dur[i]))) for i in order])
    p = t[1, 8:60]
    pn = ["park+finalize", "S1..S2 wait", "gather", "S3 wait+fetch", "S4+pe1+S5"]
    dp = np.diff(p[:, :6], axis=1)
    print("producer wave 4")
    for i, nme in enumerate(pn):
        print(f"  {nme:14s} {int(np.median(dp[:, i])):7d}")


if __name__ == "__main__":
    main()
