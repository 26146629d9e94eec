"""Dev tool: bf16 render vs fp32 render and the CPU oracle on a small scene."""
import os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden"))
from formula import formula_params
from scenes import scene
from pointnerf_amd.aggregator import PointAggregator
from pointnerf_amd.renderer import NeuralPoints, NeuralPointsRayMarching
cuda = torch.device("cuda:0")
sc = scene(30000, H=48, W=48, theta=30.0)
params = formula_params(salt=0.1)
agg = PointAggregator(sc["opt"]).to(cuda)
torch.manual_seed(0)
agg = PointAggregator(sc["opt"]).to(cuda)
np_ = NeuralPoints(sc["opt"], cuda, torch.from_numpy(sc["xyz"]), torch.from_numpy(sc["emb"]),
                   torch.from_numpy(sc["color"]), torch.from_numpy(sc["dir"]), torch.from_numpy(sc["conf"]))
outs = {}
for prec in ("fp32", "bf16"):
    m = NeuralPointsRayMarching(sc["opt"], np_, agg.eval(), precision=prec)
    with torch.no_grad():
        outs[prec] = [t.cpu() for t in m.render_rays(torch.from_numpy(sc["campos"]).to(cuda),
                      torch.from_numpy(sc["camrot"]).to(cuda), torch.from_numpy(sc["raydir"]).to(cuda),
                      2.0, 6.0, torch.from_numpy(sc["bg"]).to(cuda))]
a, b = outs["fp32"][0].numpy(), outs["bf16"][0].numpy()
print("mask equal", torch.equal(outs["fp32"][3], outs["bf16"][3]))
d = np.abs(a - b)
print("color max|d|", d.max(), "mean", d.mean(), "max|ref|", np.abs(a).max())
mse = float(np.mean((a - b) ** 2)); peak = float(np.abs(a).max())
print("PSNR(bf16 vs fp32) dB", 10 * np.log10(peak ** 2 / mse))
op = np.abs(outs["fp32"][1].numpy() - outs["bf16"][1].numpy())
print("opacity max|d|", op.max())

# feature-level comparison (same query, both aggregate paths)
from pointnerf_amd import _lib as L
m = NeuralPointsRayMarching(sc["opt"], np_, agg.eval())
q = np_.querier
cp, cr = torch.from_numpy(sc["campos"]).to(cuda), torch.from_numpy(sc["camrot"]).to(cuda)
rd = torch.from_numpy(sc["raydir"]).to(cuda).contiguous()
bufs, hp, rays, qp = q.run(np_.xyz.detach(), rd, cp, cr, 2.0, 6.0)
cnt = bufs.read_counts(); Sv = cnt["S_valid"]
s = L.Samples(bufs.valid_list.data_ptr(), bufs.counts.data_ptr() + 4, Sv, bufs.pidx.data_ptr(),
              bufs.sample_w.data_ptr(), bufs.sample_p.data_ptr(), rd.data_ptr(), bufs.fill_rs.data_ptr(),
              sc["opt"].SR, sc["opt"].K)
pts, keep = np_.tables(cp, cr)
f32 = torch.zeros((Sv, 129), device=cuda); f16 = torch.zeros((Sv, 129), device=cuda)
mlp, _k1 = agg.packed(); sc32 = L.aggregate_scratch(Sv, pts.n, cuda)
L.check(L.lib().pnr_aggregate_fwd(L.ctypes.byref(pts), L.ctypes.byref(s), L.ctypes.byref(mlp), L.ptr(f32), None, None,
                                  L.ptr(sc32), sc32.numel() * 4, L.stream_ptr(cuda)), "fp32")
mlp16, _k2 = agg.packed_bf16(); sc16 = L.aggregate_scratch_bf16(Sv, pts.n, cuda)
L.check(L.lib().pnr_aggregate_fwd_bf16(L.ctypes.byref(pts), L.ctypes.byref(s), L.ctypes.byref(mlp16), L.ptr(f16),
                                       None, None, L.ptr(sc16), sc16.numel() * 4, L.stream_ptr(cuda)), "bf16")
torch.cuda.synchronize()
a, b = f32.cpu().numpy(), f16.cpu().numpy()
for name, sl in (("alpha", slice(0, 1)), ("color", slice(1, 129))):
    d = np.abs(a[:, sl] - b[:, sl]); r = np.abs(a[:, sl])
    print(name, "max|ref|", r.max(), "max|d|", d.max(), "rel rms", float(np.sqrt((d ** 2).mean() / (r ** 2).mean())))
