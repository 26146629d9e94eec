"""Dev tool: time the training step's weight-gradient GEMM (dW = dZ^T X) with
the libpnr.so named by $PNR_LIB; prints one JSON line per shape (median / min
of 20 timed calls, events on the launch stream, and a hash of C and of the
column sums, so variant libraries can be compared bit for bit).
GEMM_MODE: x3 (default) or h2; GEMM_SHAPES: "K:M:N,..." (default the finetune
step's big product, 236 000 x 256 x 256)."""
import hashlib
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from pointnerf_amd import _lib as L
    dev = torch.device("cuda:0")
    mode = os.environ.get("GEMM_MODE", "x3")
    shapes = [tuple(int(x) for x in s.split(":")) for s in os.environ.get("GEMM_SHAPES", "236000:256:256").split(",")]
    for shp in shapes:
        K, M, N = shp[:3]
        big = len(shp) > 3 and shp[3] > 0   # a few rows of B past the h2 split's range: the x3 fallback
        g = torch.Generator(device=dev).manual_seed(K + M + N)
        A = torch.randn(K, M, device=dev, generator=g) * 1e-3
        B = torch.randn(K, N, device=dev, generator=g).relu_()
        if big:
            B[::997] *= 1e5
        h2 = L.H2Gemm(dev) if mode == "h2" else None

        def run():
            return L.gemm_tn(A, B, colsum=True, h2=h2)
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        ts = []
        for _ in range(20):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            C, cs = run()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        ts.sort()
        hc = hashlib.sha1(C.cpu().numpy().tobytes() + cs.cpu().numpy().tobytes()).hexdigest()[:16]
        print(json.dumps({"lib": os.environ.get("PNR_LIB", "default")[-24:], "mode": mode, "K": K, "M": M, "N": N, "big": big,
                          "flag": int(h2.flag.item()) if h2 is not None else None,
                          "ms_med": round(ts[10], 4), "ms_min": round(ts[0], 4), "hash": hc,
                          "c_checksum": float(C.double().sum())}))


if __name__ == "__main__":
    main()
