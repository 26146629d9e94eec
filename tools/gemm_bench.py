"""Dev tool: time pnr_gemm_tn vs pnr_gemm_tn_x3 at the training batch's shapes."""
import json, os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pointnerf_amd import _lib as L
dev = torch.device("cuda:0")
K = 236_000
res = {}
for (M, N) in [(256, 256), (256, 64), (256, 224)]:
    A = torch.randn((K, M), device=dev)
    B = torch.randn((K, N), device=dev)
    for x3 in (False, True):
        for _ in range(3):
            L.gemm_tn(A, B, colsum=True, x3=x3)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            L.gemm_tn(A, B, colsum=True, x3=x3)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 20
        res[f"{M}x{N}{'_x3' if x3 else ''}"] = {"ms": round(ms, 4), "tflops": round(2 * K * M * N / ms / 1e9, 1)}
print(json.dumps(res))
