"""Dev timing: pnr_aggregate_fwd_h2 (wt / as pairs kernel) on one mid-size query."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests", "golden"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import torch
from formula import formula_params
from scenes import scene
from test_gpu_x3 import _setup
from pointnerf_amd import _lib as L
cuda = torch.device("cuda:0")
sc = scene(400000, H=400, W=400, default_conf=None)
agg, np_ = _setup(sc, cuda, formula_params(salt=0.4))
cp, cr = torch.from_numpy(sc["campos"]).to(cuda), torch.from_numpy(sc["camrot"]).to(cuda)
rd = torch.from_numpy(sc["raydir"]).to(cuda).contiguous()
bufs, hp, rays, qp = np_.querier.run(np_.xyz.detach(), rd, cp, cr, 2.0, 6.0)
cnt = bufs.read_counts()
Sv = cnt["S_valid"]
s = L.Samples(bufs.valid_list.data_ptr(), bufs.counts.data_ptr() + 4, Sv, bufs.pidx.data_ptr(),
              bufs.sample_w.data_ptr(), bufs.sample_p.data_ptr(), rd.data_ptr(), bufs.fill_rs.data_ptr(),
              sc["opt"].SR, sc["opt"].K)
pts, _keep = np_.tables(cp, cr)
mlp, _k1 = agg.packed()
f = torch.zeros((Sv, 129), device=cuda)
scr = L.aggregate_scratch(Sv, pts.n, cuda)
for kern in sys.argv[1:] or ["wt", "as"]:
    agg.pairs_kernel = kern
    mlpx, _k2 = agg.packed_h2()
    def run():
        L.check(L.lib().pnr_aggregate_fwd_h2(L.ctypes.byref(pts), L.ctypes.byref(s), L.ctypes.byref(mlp),
                                             L.ctypes.byref(mlpx), L.ptr(f), None, None, L.ptr(scr),
                                             scr.numel() * 4, L.stream_ptr(cuda)), "h2")
    for _ in range(3):
        run()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(10):
        run()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 10
    print(f"{kern}: samples {Sv} pairs-ish {Sv * 8} aggregate {ms:.3f} ms  ({Sv / ms / 1e3:.1f} Msamples/s)")
