"""Dev: max |render_views - per-view render| per output and precision."""
import sys, os
sys.path[:0] = [os.getcwd(), "tests", "tests/golden"]
import torch
from formula import formula_params
from test_gpu_graph import _cams
from test_gpu_render import _renderer
cuda = torch.device("cuda:0")
sc, cams = _cams(cuda, thetas=(30.0, 150.0, 260.0))
m = _renderer(sc, cuda, formula_params(salt=0.9))
bg = torch.from_numpy(sc["bg"]).to(cuda)
for prec in ("fp32", "fp32x3", "fp32h2", "bf16"):
    m.precision = prec
    views = [(cp, cr, rd[i::3].contiguous()) for i, (cp, cr, rd) in enumerate(cams)]
    want = [[t.clone() for t in m.render_rays(cp, cr, rd, 2.0, 6.0, bg)] for cp, cr, rd in views]
    again = [[t.clone() for t in m.render_rays(cp, cr, rd, 2.0, 6.0, bg)] for cp, cr, rd in views]
    got = m.render_views(views, 2.0, 6.0, bg)
    for i, (w, a, g) in enumerate(zip(want, again, got)):
        print(prec, i, [float((x.float() - y.float()).abs().max()) for x, y in zip(w, g)],
              "repeat", [float((x.float() - y.float()).abs().max()) for x, y in zip(w, a)], flush=True)
