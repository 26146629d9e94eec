"""pointnerf_amd.optim.Adam (pnr_adam_step) vs torch.optim.Adam, the
optimizer of the reference's finetune loop (train_ddp.py;
mvs_points_volumetric_model.py:102-123).  Same update order as torch's
fused kernel (m, v by fma, denom = sqrt(v) / sqrt(bc2) + eps, addcdiv); the
two differ only by fp32 rounding of the contracted terms, so the bar is
|d| <= 1e-6 |ref| + 1e-9 for the parameters after several steps (their own
ulp is ~1e-7 relative) and 1e-6 of |ref| + 1e-6 of the tensor's largest entry
for the moments (a moment near 0 is the cancellation of larger terms)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _params(dev, seed):
    g = torch.Generator().manual_seed(seed)
    shapes = [(100003,), (2000, 39), (1,), (37, 3), (256, 284), (4096,)]
    return [torch.randn(s, generator=g).to(dev) for s in shapes]


def _grads(ps, seed):
    g = torch.Generator().manual_seed(seed)
    return [torch.randn(p.shape, generator=g).to(p.device) * 10 ** float(torch.randint(-6, 2, (1,), generator=g))
            for p in ps]


@pytest.mark.parametrize("wd", [0.0, 0.01])
@pytest.mark.parametrize("fused", [True, False])
def test_adam_matches_torch(cuda, wd, fused):
    from pointnerf_amd.optim import Adam
    a = [torch.nn.Parameter(p) for p in _params(cuda, 0)]
    b = [torch.nn.Parameter(p.detach().clone()) for p in a]
    mine = Adam(a, lr=5e-4, betas=(0.9, 0.999), eps=1e-8, weight_decay=wd)
    ref = torch.optim.Adam(b, lr=5e-4, betas=(0.9, 0.999), eps=1e-8, weight_decay=wd, fused=fused,
                           foreach=None if fused else False)
    v0 = [p._version for p in a]
    for it in range(6):
        gs = _grads(a, 100 + it)
        for p, q, g in zip(a, b, gs):
            p.grad, q.grad = g.clone(), g.clone()
        if it == 3:   # a parameter without a gradient this step: untouched, its step count lags
            a[2].grad = b[2].grad = None
        mine.step()
        ref.step()
    assert all(p._version > v for p, v in zip(a, v0))   # caches keyed on the version see the update
    for i, (p, q) in enumerate(zip(a, b)):
        d = (p.detach() - q.detach()).abs()
        tol = 1e-6 * q.detach().abs() + 1e-9
        assert bool((d <= tol).all()), (i, float(d.max()))
        assert mine.state[p]["step"] == int(ref.state[q]["step"])
        for k in ("exp_avg", "exp_avg_sq"):
            dm = (mine.state[p][k] - ref.state[q][k]).abs()
            r = ref.state[q][k].abs()   # moments: rounding of the larger earlier terms (per-tensor scale)
            assert bool((dm <= 1e-6 * r + 1e-6 * float(r.max())).all()), (i, k, float(dm.max()))


def test_adam_unaligned_scalar_path(cuda):
    """A parameter whose storage starts 4 B past a 16-B boundary takes the
    scalar lanes; results equal the aligned copy's bit for bit."""
    from pointnerf_amd.optim import Adam
    big = torch.randn(8193, device=cuda)
    p_un = torch.nn.Parameter(big[1:])            # view: storage offset 1 float
    p_al = torch.nn.Parameter(big[1:].clone())
    assert p_un.data_ptr() % 16 == 4 and p_al.data_ptr() % 16 == 0
    o1, o2 = Adam([p_un], lr=1e-3), Adam([p_al], lr=1e-3)
    for it in range(3):
        g = torch.randn(8192, device=cuda, generator=torch.Generator(device=cuda).manual_seed(it))
        p_un.grad, p_al.grad = g.clone(), g.clone()
        o1.step()
        o2.step()
    assert torch.equal(p_un.detach(), p_al.detach())


def test_adam_refuses_bad_params(cuda):
    from pointnerf_amd import _lib as L
    from pointnerf_amd.optim import Adam
    p = torch.nn.Parameter(torch.randn(8, 8, device=cuda).t())   # non-contiguous
    p.grad = torch.randn(8, 8, device=cuda)
    with pytest.raises(L.PnrError):
        Adam([p]).step()
