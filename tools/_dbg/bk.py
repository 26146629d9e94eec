import sys, os
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests")); sys.path.insert(0, os.path.join(os.getcwd(), "tests", "golden"))
import numpy as np, torch
from formula import formula_params
from scenes import flag_scene
from pointnerf_amd import _lib as L
from pointnerf_amd.aggregator import PointAggregator
from pointnerf_amd.renderer import NeuralPoints
cuda = torch.device("cuda:0")
for flags in ("truck", "lego"):
    sc = flag_scene(flags, n_points=60000 if flags == "truck" else 30000, H=64, view=0)
    agg = PointAggregator(sc["opt"]).to(cuda)
    agg.load_state_dict({k: torch.from_numpy(v) for k, v in formula_params(salt=0.6).items()})
    np_ = NeuralPoints(sc["opt"], cuda, torch.from_numpy(sc["xyz"]), torch.from_numpy(sc["emb"]), torch.from_numpy(sc["color"]), torch.from_numpy(sc["dir"]), torch.from_numpy(sc["conf"]))
    cp, cr = torch.from_numpy(sc["campos"]).to(cuda), torch.from_numpy(sc["camrot"]).to(cuda)
    rd = torch.from_numpy(sc["raydir"]).to(cuda).contiguous()
    bufs, hp, rays, qp = np_.querier.run(np_.xyz.detach(), rd, cp, cr, sc["near"], sc["far"])
    cnt = bufs.read_counts(); Sv, K = cnt["S_valid"], sc["opt"].K
    s = L.Samples(bufs.valid_list.data_ptr(), bufs.counts.data_ptr() + 4, Sv, bufs.pidx.data_ptr(), bufs.sample_w.data_ptr(), bufs.sample_p.data_ptr(), rd.data_ptr(), bufs.fill_rs.data_ptr(), sc["opt"].SR, K)
    pts, keep = np_.tables(cp, cr)
    outs = []
    for rep, bk in ((0, False), (1, False), (2, True), (3, True)):
        agg.pair_buckets = bk
        mlp16, _k = agg.packed_bf16()
        f = torch.full((Sv, 129), float("nan"), device=cuda)
        scr = L.aggregate_scratch_bf16(Sv, pts.n, cuda)
        scr.fill_(rep + 1.5)
        L.check(L.lib().pnr_aggregate_fwd_bf16(L.ctypes.byref(pts), L.ctypes.byref(s), L.ctypes.byref(mlp16), L.ptr(f), None, None, L.ptr(scr), scr.numel() * 4, L.stream_ptr(cuda)), "bf16")
        torch.cuda.synchronize()
        outs.append(f.clone())
        if bk:
            # bucket list: scratch = P1 | hid | vmask | list | info
            nb = scr.view(torch.int32)
            off = (pts.n * 256 * 2 + Sv * 256 * 2) // 4 + ((Sv + 3) // 4) * 4
            lst = nb[off: off + Sv].cpu().numpy()
            info = nb[off + ((Sv + 3) // 4) * 4: off + ((Sv + 3) // 4) * 4 + 8].cpu().numpy()
            print(flags, "info", info, "sum", info[4:].sum(), "Sv", Sv, "perm ok", np.array_equal(np.sort(lst), np.arange(Sv)))
    for i in range(1, 4):
        d = (torch.nan_to_num(outs[0], nan=7.0) - torch.nan_to_num(outs[i], nan=7.0)).abs()
        rows = (d.amax(1) > 0).nonzero().flatten()
        print(flags, "run", i, "rows differing", rows.numel(), "max", float(d.max()), rows[:10].tolist())
