"""Dev tool: time the 2-D neural renderer on an 800x800x128 feature image,
forward and forward + backward, per precision (fp32h2 / fp32) vs torch (MIOpen)."""
import json, os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pointnerf_amd.neural_render import NeuralRenderer
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from nr_ref import neural_render_torch  # noqa: E402
dev = torch.device("cuda:0")
torch.manual_seed(0)
m = NeuralRenderer(input_dim=128).to(dev)
x = torch.randn((1, 800, 800, 128), device=dev)
g = torch.randn((1, 800, 800, 3), device=dev)
xg = x.clone().requires_grad_(True)
flops = 800 * 800 * 2 * 9 * (128 * 64 + 128 * 3 + 64 * 32 + 64 * 3 + 32 * 3)


def timed(fn, n):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


def fwd():
    with torch.no_grad():
        m(x)


def step():
    m.zero_grad(set_to_none=True)
    (m(xg) * g).sum().backward()


def step_torch():
    m.zero_grad(set_to_none=True)
    (neural_render_torch(m, xg) * g).sum().backward()


res = {}
for prec in ("fp32h2", "fp32"):
    m.precision = prec
    res[f"fwd_ms_{prec}"] = round(timed(fwd, 10), 3)
    res[f"fwd_tflops_{prec}"] = round(flops / res[f"fwd_ms_{prec}"] / 1e9, 1)
    res[f"fwd_bwd_ms_{prec}"] = round(timed(step, 5), 3)
res["fwd_bwd_ms_torch_miopen"] = round(timed(step_torch, 5), 3)
print(json.dumps(res))
