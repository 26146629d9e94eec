"""Dev tool: the co-residency experiment of DESIGN.md section 10.

Runs test_train_backward_repeatable's batch (tests/test_gpu_backward.py) N times
with the x3 training path and prints, per gradient, the largest run-to-run
deviation relative to the tensor's max entry.  PNR_LIB picks the libpnr build
(tools/extras_variant.sh), --kernel-extras routes the block3.0 extras through
pnr_aggregate_bwd_pairs_x3 (train.X3_POINT_EXTRAS = False).
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden"), ROOT]

import torch  # noqa: E402

import test_gpu_backward as T  # noqa: E402
import pointnerf_amd.train as TR  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernel-extras", action="store_true")
    ap.add_argument("--reps", type=int, default=6)
    ap.add_argument("--precision", default="fp32x3")
    args = ap.parse_args()
    TR.X3_POINT_EXTRAS = not args.kernel_extras
    cuda = torch.device("cuda:0")
    sc = T.scene(20000, H=32, W=32, theta=60.0, default_conf=None)
    m = T._train_model(sc, cuda, T.formula_params(salt=0.3))
    m.train_precision = args.precision
    cp, cr = torch.from_numpy(sc["campos"]).to(cuda), torch.from_numpy(sc["camrot"]).to(cuda)
    rd, bg = torch.from_numpy(sc["raydir"]).to(cuda), torch.from_numpy(sc["bg"]).to(cuda)
    outs = []
    for _ in range(args.reps):
        for p in list(m.parameters()) + list(m.neural_points.parameters()):
            p.grad = None
        color = m.render_rays_train(cp, cr, rd, 2.0, 6.0, bg)[0]
        G = torch.randn(color.shape, generator=torch.Generator().manual_seed(5)).to(cuda)
        (color * G).sum().backward()
        npt = m.neural_points
        o = {k: getattr(npt, k).grad.clone() for k in ("points_color", "points_dir", "points_embeding",
                                                         "points_conf")}
        o.update({"mlp " + k: p.grad.clone() for k, p in m.aggregator.named_parameters()})
        outs.append(o)
    res = {}
    for k in outs[0]:
        ref = outs[0][k]
        big = float(ref.abs().max())
        d = max(float((o[k] - ref).abs().max()) for o in outs[1:])
        res[k] = d / big if big else d
    worst = max(res, key=res.get)
    out = {"lib": os.environ.get("PNR_LIB", "libpnr.so"), "kernel_extras": args.kernel_extras,
           "worst": worst, "worst_rel": res[worst], "rel": {k: v for k, v in res.items() if v > 0}}
    lib = TR.L.lib()
    if hasattr(lib, "pnr_exp_check_count"):   # experiment builds (PNR_EXP_CHECK2)
        import ctypes
        buf = (ctypes.c_uint * 9)()
        lib.pnr_exp_check_count(buf)
        out["lds_vs_global_mismatches"] = buf[0]
        out["first_mismatch"] = dict(zip(("set", "tile", "block", "wave", "lane", "neuron", "lds_bits", "global_bits"),
                                         list(buf)[1:]))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
