"""Dev tool: time pnr_neural_render_fwd on an 800x800x128 feature image."""
import json, os, sys, time
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pointnerf_amd.neural_render import NeuralRenderer
dev = torch.device("cuda:0")
torch.manual_seed(0)
m = NeuralRenderer(input_dim=128).to(dev)
x = torch.randn((1, 800, 800, 128), device=dev)
with torch.no_grad():
    for _ in range(3):
        m(x)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        m(x)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 10
    t0 = time.perf_counter()
    for _ in range(3):
        m.forward_torch(x)
    torch.cuda.synchronize()
    ms_t = (time.perf_counter() - t0) / 3 * 1e3
flops = 800 * 800 * 2 * 9 * (128 * 64 + 128 * 3 + 64 * 32 + 64 * 3 + 32 * 3)
print(json.dumps({"ms_hip": round(ms, 3), "tflops": round(flops / ms / 1e9, 1), "ms_torch_miopen": round(ms_t, 3)}))
