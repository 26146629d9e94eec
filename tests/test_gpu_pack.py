"""pnr_pack_weights (device fragment packing) against aggregator.py's torch
restatement on the host: bitwise, fp32 and fp32x3 packs, with and without a
bias column, contiguous and transposed (strided) weights."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("shape,bias,transposed", [((256, 263), True, False), ((256, 60), False, False),
                                                   ((128, 280), True, False), ((256, 256), False, True),
                                                   ((256, 7), False, False), ((32, 33), True, True)])
def test_device_pack_equals_torch(cuda, shape, bias, transposed):
    from pointnerf_amd.aggregator import frag_pack, frag_pack_x3
    g = torch.Generator().manual_seed(shape[0] + shape[1])
    out_f, kin = shape
    W = torch.randn((kin, out_f) if transposed else (out_f, kin), generator=g) * 0.3
    W = W.t() if transposed else W
    b = torch.randn(out_f, generator=g) if bias else None
    Wd = W.to(cuda) if not transposed else W.t().contiguous().to(cuda).t()   # keep the strided view on the GPU
    bd = None if b is None else b.to(cuda)
    assert torch.equal(frag_pack(Wd, bd).cpu(), frag_pack(W, b))
    assert torch.equal(frag_pack_x3(Wd, bd).cpu().view(torch.int16), frag_pack_x3(W, b).view(torch.int16))


@pytest.mark.parametrize("shape,bias,transposed", [((256, 263), True, False), ((256, 60), False, False),
                                                   ((256, 256), False, True), ((32, 33), True, True)])
def test_device_pack_h2_equals_torch(cuda, shape, bias, transposed):
    """pnr_pack_weights_h2 == frag_pack_h2 (same shift) bitwise; the range flag
    stays clear, and is raised when the shift is one too small."""
    from pointnerf_amd.aggregator import _pack_h2_device, frag_pack_h2, h2_shift
    g = torch.Generator().manual_seed(3 * shape[0] + shape[1])
    out_f, kin = shape
    W = torch.randn((kin, out_f) if transposed else (out_f, kin), generator=g) * 0.3
    W = W.t() if transposed else W
    b = torch.randn(out_f, generator=g) if bias else None
    Wd = W.to(cuda) if not transposed else W.t().contiguous().to(cuda).t()
    bd = None if b is None else b.to(cuda)
    ref, _ = frag_pack_h2(W, b)
    s = h2_shift(W, b)
    flag = torch.zeros(1, dtype=torch.int32, device=cuda)
    got = _pack_h2_device(Wd, bd, s, flag)
    assert torch.equal(got.cpu().view(torch.int16), ref.view(torch.int16))
    assert int(flag.item()) == 0
    _pack_h2_device(Wd, bd, s - 1, flag)
    assert int(flag.item()) == 1


@pytest.mark.parametrize("shape,bias,scale", [((96, 1152), False, 0.03), ((128, 864), False, 3e-6),
                                              ((256, 263), True, 40.0), ((32, 33), True, 1.0)])
def test_device_pack_h2_dev_picks_the_shift(cuda, shape, bias, scale):
    """pnr_pack_weights_h2_dev (shift picked on the device, no host sync) ==
    frag_pack_h2 bitwise, and its device scale == frag_pack_h2's 2^(s - 11)."""
    from pointnerf_amd.aggregator import frag_pack_h2, pack_h2_dev
    g = torch.Generator().manual_seed(shape[0] * 7 + shape[1])
    W = torch.randn(shape, generator=g) * scale
    b = torch.randn(shape[0], generator=g) * scale if bias else None
    ref, sc = frag_pack_h2(W, b)
    s_out = torch.zeros(2, dtype=torch.float32, device=cuda)
    got = pack_h2_dev(W.to(cuda), None if b is None else b.to(cuda), s_out)
    assert torch.equal(got.cpu().view(torch.int16), ref.view(torch.int16))
    assert float(s_out[0]) == sc
