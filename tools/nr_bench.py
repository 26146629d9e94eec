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

# forward + backward (training): NeuralRenderFn (pnr_neural_render_bwd) vs torch autograd (MIOpen)
g = torch.randn((1, 800, 800, 3), device=dev)
xg = x.clone().requires_grad_(True)


def step_hip():
    m.zero_grad(set_to_none=True)
    (m(xg) * g).sum().backward()


def step_torch():
    m.zero_grad(set_to_none=True)
    (m.forward_torch(xg) * g).sum().backward()


res = {}
for name, fn in (("hip", step_hip), ("torch_miopen", step_torch)):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        fn()
    e1.record()
    torch.cuda.synchronize()
    res["fwd_bwd_ms_" + name] = round(e0.elapsed_time(e1) / 5, 3)
res["fwd_bwd_tflops_hip"] = round(3 * flops / res["fwd_bwd_ms_hip"] / 1e9, 1)
print(json.dumps(res))
