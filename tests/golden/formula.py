"""Deterministic MLP weights shared by tests/golden/make_golden.py and the tests.

The golden aggregator vectors are produced by the reference PointAggregator with
its parameters overwritten by these closed-form values, so the fixtures do not
have to carry 1.4 MB of random weights: any machine regenerates them exactly
(float64 formula, one rounding to float32).
"""
import numpy as np

# state_dict name -> (out, in) for the lego viewmlp (point_aggregators.py:276-348)
LEGO_SHAPES = {
    "block1.0": (256, 284),
    "block1.2": (256, 256),
    "block3.0": (256, 263),
    "block3.2": (256, 256),
    "alpha_branch.0": (1, 256),
    "color_branch.0": (128, 280),
    "color_branch.2": (128, 128),
    "color_branch.4": (128, 128),
}


def formula_params(shapes=LEGO_SHAPES, salt=0.0):
    out = {}
    for li, (name, (o, i)) in enumerate(shapes.items()):
        bound = np.sqrt(6.0 / (o + i)) * 1.2
        oo = np.arange(o, dtype=np.float64)[:, None]
        ii = np.arange(i, dtype=np.float64)[None, :]
        w = bound * np.sin(1.3 * oo + 0.7 * ii + 0.37 * li + salt) * np.cos(0.11 * oo - 0.05 * ii + li)
        b = 0.05 * np.sin(0.9 * np.arange(o, dtype=np.float64) + li + salt)
        out[name + ".weight"] = w.astype(np.float32)
        out[name + ".bias"] = b.astype(np.float32)
    return out

# upstream model (C_out = 3): the colour head the fork commented out,
# color_branch.6 = Linear(128, 3) (point_aggregators.py:343)
UPSTREAM_SHAPES = dict(LEGO_SHAPES, **{"color_branch.6": (3, 128)})
