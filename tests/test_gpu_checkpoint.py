"""Reference-format checkpoints and point-cloud edits (pointnerf_amd/checkpoint.py)."""
import numpy as np
import pytest
import torch

from formula import formula_params
from scenes import scene

pytestmark = pytest.mark.gpu


def _model(sc, cuda, params, xyz=None, emb=None, color=None, dirs=None, conf=None):
    from pointnerf_amd.aggregator import PointAggregator
    from pointnerf_amd.renderer import NeuralPoints, NeuralPointsRayMarching
    agg = PointAggregator(sc["opt"]).to(cuda)
    agg.load_state_dict({k: torch.from_numpy(v) for k, v in params.items()})
    t = lambda a, d: torch.from_numpy(sc[d] if a is None else a)  # noqa: E731
    np_ = NeuralPoints(sc["opt"], cuda, t(xyz, "xyz"), t(emb, "emb"), t(color, "color"), t(dirs, "dir"),
                       t(conf, "conf"))
    return NeuralPointsRayMarching(sc["opt"], np_, agg.eval())


def _render(m, sc, cuda):
    with torch.no_grad():
        c, op, bg, mask = m.render_rays(torch.from_numpy(sc["campos"]).to(cuda),
                                        torch.from_numpy(sc["camrot"]).to(cuda),
                                        torch.from_numpy(sc["raydir"]).to(cuda), 2.0, 6.0,
                                        torch.from_numpy(sc["bg"]).to(cuda))
    return c.cpu(), op.cpu(), mask.cpu()


def test_reference_keyed_state_dict_roundtrip(tmp_path, cuda):
    from pointnerf_amd.checkpoint import load_ray_marching, save_ray_marching
    sc = scene(6000, H=24, W=24)
    params = formula_params(salt=0.4)
    n = sc["xyz"].shape[0]
    # a state_dict with exactly the reference's key names and shapes
    # (neural_points.py:241-326, point_aggregators.py:276-348)
    sd = {"neural_points.xyz": torch.from_numpy(sc["xyz"]),
          "neural_points.points_embeding": torch.from_numpy(sc["emb"]).reshape(1, n, 32),
          "neural_points.points_conf": torch.from_numpy(sc["conf"]).reshape(1, n, 1),
          "neural_points.points_dir": torch.from_numpy(sc["dir"]).reshape(1, n, 3),
          "neural_points.points_color": torch.from_numpy(sc["color"]).reshape(1, n, 3)}
    sd.update({"aggregator." + k: torch.from_numpy(v) for k, v in params.items()})
    path = tmp_path / "best_net_ray_marching.pth"
    torch.save(sd, str(path))
    m = load_ray_marching(str(path), sc["opt"], cuda)
    assert m.load_report["missing"] == [] and m.load_report["unexpected"] == []
    ref = _render(_model(sc, cuda, params), sc, cuda)
    got = _render(m, sc, cuda)
    for a, b in zip(got, ref):
        assert torch.equal(a, b)
    # save -> load gives the same keys and the same render
    path2 = tmp_path / "10_net_ray_marching.pth"
    save_ray_marching(m, str(path2))
    sd2 = torch.load(str(path2), weights_only=True)
    assert set(sd) <= set(sd2)
    for k in sd:
        assert torch.equal(sd2[k].reshape(sd[k].shape), sd[k]), k
    again = _render(load_ray_marching(str(path2), sc["opt"], cuda), sc, cuda)
    for a, b in zip(again, ref):
        assert torch.equal(a, b)


def test_best_epoch_default_conf(tmp_path, cuda):
    from pointnerf_amd.checkpoint import load_ray_marching
    sc = scene(3000, H=8, W=8)
    n = sc["xyz"].shape[0]
    sd = {"neural_points.xyz": torch.from_numpy(sc["xyz"]),
          "neural_points.points_embeding": torch.from_numpy(sc["emb"]).reshape(1, n, 32)}
    path = tmp_path / "best_net_ray_marching.pth"
    torch.save(sd, str(path))
    m = load_ray_marching(str(path), sc["opt"], cuda, epoch_is_best=True)
    conf = m.neural_points.points_conf
    assert conf.shape == (1, n, 1) and torch.all(conf == sc["opt"].default_conf)


def test_prune_and_grow_rebuild_grid(cuda):
    from pointnerf_amd.checkpoint import grow_points, prune
    sc = scene(8000, H=24, W=24)
    params = formula_params(salt=0.6)
    m = _model(sc, cuda, params)
    _render(m, sc, cuda)                       # builds the grid for the full cloud
    keep = sc["conf"][:, 0] >= 0.5
    dropped = prune(m.neural_points, 0.5)
    assert dropped == int((~keep).sum()) and dropped > 0
    direct = _model(sc, cuda, params, xyz=sc["xyz"][keep], emb=sc["emb"][keep], color=sc["color"][keep],
                    dirs=sc["dir"][keep], conf=sc["conf"][keep])
    for a, b in zip(_render(m, sc, cuda), _render(direct, sc, cuda)):
        assert torch.equal(a, b)
    # grow the pruned points back (appended at the end)
    d = ~keep
    grow_points(m.neural_points, torch.from_numpy(sc["xyz"][d]), torch.from_numpy(sc["emb"][d]),
                torch.from_numpy(sc["color"][d]), torch.from_numpy(sc["dir"][d]), torch.from_numpy(sc["conf"][d]))
    order = np.concatenate([np.nonzero(keep)[0], np.nonzero(d)[0]])
    direct2 = _model(sc, cuda, params, xyz=sc["xyz"][order], emb=sc["emb"][order], color=sc["color"][order],
                     dirs=sc["dir"][order], conf=sc["conf"][order])
    for a, b in zip(_render(m, sc, cuda), _render(direct2, sc, cuda)):
        assert torch.equal(a, b)


def test_grow_and_prune_keep_bf16_table(cuda):
    """A bf16 embedding table stays bf16 through prune / grow (the 104 B/point
    footprint of config c5), and the bf16 render path keeps reading it."""
    from pointnerf_amd.aggregator import PointAggregator
    from pointnerf_amd.checkpoint import grow_points, prune
    from pointnerf_amd.renderer import NeuralPoints, NeuralPointsRayMarching
    sc = scene(8000, H=24, W=24)
    t = lambda k: torch.from_numpy(sc[k])  # noqa: E731
    np_ = NeuralPoints(sc["opt"], cuda, t("xyz"), t("emb"), t("color"), t("dir"), t("conf"), emb_dtype=torch.bfloat16)
    agg = PointAggregator(sc["opt"]).to(cuda)
    agg.load_state_dict({k: torch.from_numpy(v) for k, v in formula_params(salt=0.6).items()})
    m = NeuralPointsRayMarching(sc["opt"], np_, agg.eval(), precision="bf16")
    keep = sc["conf"][:, 0] >= 0.5
    prune(np_, 0.5)
    assert np_.points_embeding.dtype == torch.bfloat16
    d = ~keep
    grow_points(np_, t("xyz")[d], t("emb")[d], t("color")[d], t("dir")[d], t("conf")[d])
    assert np_.points_embeding.dtype == torch.bfloat16 and np_.points_embeding.shape[1] == sc["xyz"].shape[0]
    assert np_.bytes_per_point() == 104
    c, _, mask = _render(m, sc, cuda)
    assert int(mask.sum()) > 0 and torch.isfinite(c).all()
