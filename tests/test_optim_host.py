"""Host logic of pointnerf_amd.optim.Adam (no GPU): hyperparameter checks as
torch.optim.Adam's, parameters without gradients skipped without a launch,
and anything but dense contiguous fp32 CUDA parameters refused loudly (no CPU
fallback: the step is pnr_adam_step only)."""
import pytest
import torch

from pointnerf_amd import _lib as L
from pointnerf_amd.optim import Adam


@pytest.mark.parametrize("kw", [dict(lr=-1.0), dict(eps=-1e-8), dict(betas=(1.0, 0.999)),
                                dict(betas=(0.9, -0.1)), dict(weight_decay=-0.1)])
def test_adam_rejects_bad_hyperparameters(kw):
    with pytest.raises(ValueError):
        Adam([torch.nn.Parameter(torch.zeros(3))], **kw)


def test_adam_skips_params_without_grad():
    p = torch.nn.Parameter(torch.ones(5))
    opt = Adam([p], lr=1e-3)
    opt.step()                      # no gradient: nothing to launch
    assert torch.equal(p.detach(), torch.ones(5)) and not opt.state


def test_adam_refuses_cpu_params():
    p = torch.nn.Parameter(torch.ones(5))
    p.grad = torch.ones(5)
    with pytest.raises(L.PnrError):
        Adam([p]).step()


def test_version_bump_marks_parameters_changed():
    """Raw-pointer updates must advance p._version (the aggregator's weight packs
    are cached on it): the helper the step calls after each launch."""
    from pointnerf_amd.optim import _bump_versions
    ps = [torch.nn.Parameter(torch.zeros(4)), torch.nn.Parameter(torch.zeros(2, 2))]
    v0 = [p._version for p in ps]
    _bump_versions(ps)
    assert [p._version for p in ps] == [v + 1 for v in v0]


def test_version_bump_fallback_advances_parameter_version(monkeypatch):
    """Without the tuple _unsafe_set_version_counter API (torch 2.1-2.3 take
    (Tensor, int)) the fallback's in-place no-op must bump p._version itself,
    not the separate counter of p.data."""
    from pointnerf_amd import optim
    monkeypatch.setattr(torch._C._autograd, "_unsafe_set_version_counter",
                        lambda t, v: (_ for _ in ()).throw(TypeError("old signature")), raising=False)
    ps = [torch.nn.Parameter(torch.zeros(4)), torch.nn.Parameter(torch.zeros(2, 2))]
    v0 = [p._version for p in ps]
    optim._bump_versions(ps)
    assert all(p._version > v for p, v in zip(ps, v0))
    assert all(float(p.abs().sum()) == 0.0 for p in ps)
