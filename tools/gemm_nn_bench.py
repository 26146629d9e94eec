"""Dev tool: time pnr_gemm_nn vs torch.matmul (hipBLASLt) at the training step's dX shapes."""
import json, os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pointnerf_amd import _lib as L
dev = torch.device("cuda:0")
res = {}
for (M, K, N) in [(29906, 128, 128), (29906, 128, 256), (200000, 256, 224)]:
    A = torch.randn((M, K), device=dev)
    B = torch.randn((K, N + 32), device=dev)[:, :N]
    act = torch.randn((M, N), device=dev)
    for name, fn in (("pnr", lambda: L.gemm_nn(A, B, act=act, slope=0.2)),
                     ("torch", lambda: torch.where(act > 0, A @ B, (A @ B) * 0.2))):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 20
        res[f"{M}x{K}x{N}_{name}"] = {"ms": round(ms, 4), "tflops": round(2 * M * K * N / ms / 1e9, 1)}
print(json.dumps(res))
