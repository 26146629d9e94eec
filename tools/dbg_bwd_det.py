"""Dev tool: repeatability of the training backward (d_color / d_dir / d_emb)
over repeated identical steps, per d_p1 mode (env PNR_DBG_P1_ATOMIC)."""
import os
import sys

import torch

root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [root, os.path.join(root, "tests"), os.path.join(root, "tests", "golden")]
from formula import formula_params  # noqa: E402
from scenes import scene  # noqa: E402
from test_gpu_backward import _train_model  # noqa: E402

cuda = torch.device("cuda:0")
sc = scene(20000, H=32, W=32, theta=60.0, default_conf=None)
m = _train_model(sc, cuda, formula_params(salt=0.3))
cp, cr = torch.from_numpy(sc["campos"]).to(cuda), torch.from_numpy(sc["camrot"]).to(cuda)
rd, bg = torch.from_numpy(sc["raydir"]).to(cuda), torch.from_numpy(sc["bg"]).to(cuda)
res = []
for prec in ("fp32x3", "fp32"):
    m.train_precision = prec
    outs = []
    for _ in range(4):
        for p in m.parameters():
            p.grad = None
        color = m.render_rays_train(cp, cr, rd, 2.0, 6.0, bg)[0]
        G = torch.randn(color.shape, generator=torch.Generator().manual_seed(5)).to(cuda)
        (color * G).sum().backward()
        npt = m.neural_points
        outs.append({k: getattr(npt, k).grad.clone() for k in ("points_color", "points_dir", "points_embeding", "points_conf")})
    for k in outs[0]:
        d = max(float((o[k] - outs[0][k]).abs().max()) for o in outs[1:])
        print(prec, k, "max run-to-run diff", d, "max", float(outs[0][k].abs().max()), flush=True)
