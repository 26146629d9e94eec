"""Dev tool: time pnr_gemm_tn_x3 (the training step's weight-gradient GEMM,
dW = dZ^T X) at the finetune shape (K = 236 000 pairs, M = N = 256) with the
libpnr.so named by $PNR_LIB; prints one JSON line (median / min of 20 timed
calls, events on the launch stream)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from pointnerf_amd import _lib as L
    dev = torch.device("cuda:0")
    K = int(os.environ.get("GEMM_K", "236000"))
    g = torch.Generator(device=dev).manual_seed(0)
    A = torch.randn(K, 256, device=dev, generator=g)
    B = torch.randn(K, 256, device=dev, generator=g)
    for _ in range(3):
        L.gemm_tn(A, B)
    torch.cuda.synchronize()
    ts = []
    for _ in range(20):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        C = L.gemm_tn(A, B)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts.sort()
    print(json.dumps({"lib": os.environ.get("PNR_LIB", "default"), "K": K, "ms_med": round(ts[10], 4),
                      "ms_min": round(ts[0], 4), "c_checksum": float(C.double().sum())}))


if __name__ == "__main__":
    main()
