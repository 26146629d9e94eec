"""Dev tool: time pnr_adam_step on the finetune step's parameter set (2 M points x
(32 + 3 + 3 + 1) floats + the aggregator MLP) with the libpnr named by PNR_LIB
(A/B of Adam variants).  Prints one JSON line: median ms per step and HBM GB/s
at 28 B per element."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from pointnerf_amd import _lib as L  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    shapes = [(2_000_000, 32), (2_000_000, 3), (2_000_000, 3), (2_000_000, 1), (256, 284), (256, 256), (256, 263),
              (256, 256), (128, 280), (128, 128), (128, 128)]
    g = torch.Generator(device=dev).manual_seed(0)
    ts = [[torch.randn(s, device=dev, generator=g) * 0.1 for _ in range(4)] for s in shapes]
    for t in ts:
        t[3].abs_()
    n = len(ts)
    P = L.c_void_p * n
    args = [P(*(t[i].data_ptr() for t in ts)) for i in range(4)]
    numel = (L.c_int64 * n)(*(t[0].numel() for t in ts))
    st = L.stream_ptr(dev)
    elems = sum(t[0].numel() for t in ts)

    def step(k):
        L.check(L.lib().pnr_adam_step(n, args[0], args[1], args[2], args[3], numel, 5e-4, 0.9, 0.999, 1e-8, 0.0, k,
                                      st), "pnr_adam_step")

    for k in range(1, 6):
        step(k)
    torch.cuda.synchronize()
    times = []
    for r in range(7):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for k in range(20):
            step(6 + 20 * r + k)
        e1.record()
        torch.cuda.synchronize()
        times.append(e0.elapsed_time(e1) / 20)
    ms = sorted(times)[len(times) // 2]
    chk = float(sum(t[0].double().sum() for t in ts))
    print(json.dumps({"lib": os.environ.get("PNR_LIB", "default"), "ms": round(ms, 4),
                      "GBps": round(28 * elems / ms / 1e6, 1), "elems": elems, "checksum": chk}))


if __name__ == "__main__":
    t0 = time.time()
    main()
