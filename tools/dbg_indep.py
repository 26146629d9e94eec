"""Dev: full-frame vs subset render differences (ray independence)."""
import os, sys
import numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden"))
from formula import formula_params
from scenes import scene
from test_gpu_edge import _renderer, _render
cuda = torch.device("cuda:0")
sc = scene(2_000_000, H=800, W=800, theta=-40.0, default_conf=0.15)
params = formula_params(salt=float(os.environ.get("SALT", "0.9")))
m = _renderer(sc, cuda, params, os.environ.get("PREC", "fp32h2"))
a = _render(m, sc, cuda)
rng = np.random.default_rng(7)
sel = np.sort(rng.choice(800 * 800, size=4096, replace=False))
sub = _render(m, sc, cuda, sc["raydir"][sel])
for name, x, y in zip(("color", "opac", "isbg", "mask"), sub, a):
    y = y[torch.from_numpy(sel)]
    d = (x.float() - y.float()).abs()
    bad = (d > 0).reshape(d.shape[0], -1).any(1)
    print(name, "max", float(d.max()), "rays differing", int(bad.sum()), "of", d.shape[0],
          "cols", (d > 0).reshape(d.shape[0], -1).any(0).nonzero().flatten()[:10].tolist())
