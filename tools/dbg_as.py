"""Dev check: k_pairs_as repeatability and used-row P1 equality (prints diffs)."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests", "golden"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import numpy as np, torch
from formula import formula_params
from scenes import scene
from test_gpu_x3 import _setup, _both
cuda = torch.device("cuda:0")
sc = scene(20000, H=40, W=40, default_conf=None)
agg, np_ = _setup(sc, cuda, formula_params(salt=0.4))
f0, a = _both(agg, np_, sc, cuda, variant="as")
outs = [a] + [_both(agg, np_, sc, cuda, variant="as")[1] for _ in range(4)]
for k, x in enumerate(outs[1:]):
    d = np.abs(a - x)
    rows = np.nonzero(d.max(1) > 0)[0]
    wid = np.bincount((rows // 4) % 4, minlength=4)
    print("repeat", k, "max diff", d.max(), "rows", len(rows), "waves", wid, "blocks", np.unique(rows // 16)[:12])
print("vs fp32 path max", np.abs(a - f0).max())
e = np.abs(a - f0)
w = (np.arange(len(a)) // 4) % 4
for k in range(4):
    print("wave", k, "err vs fp32: max", e[w == k].max(), "mean", e[w == k].mean())
