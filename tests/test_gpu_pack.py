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


@pytest.mark.parametrize("scale", [0.05, 3e-6, 40.0])
def test_pack_bwd_h2_equals_torch(cuda, scale):
    """pnr_pack_bwd_h2 (the fp32h2 backward's three transposed packs in one
    launch, shifts picked on the device) == frag_pack_h2 of block3.2.weight^T,
    block3.0.weight[:, :256]^T (row stride 263) and block1.2.weight^T, bitwise,
    with the scales 2^(s - 11)."""
    from pointnerf_amd import _lib as L
    from pointnerf_amd.aggregator import X3_PAD, frag_pack_h2
    g = torch.Generator().manual_seed(11)
    w4, w3, w2 = (torch.randn(sh, generator=g) * scale * (1 + i) for i, sh in
                  enumerate(((256, 256), (256, 263), (256, 256))))
    per = (16 + X3_PAD) * 2048
    packs = torch.empty(3 * per * 2, dtype=torch.int32, device=cuda)
    sc = torch.zeros(4, dtype=torch.float32, device=cuda)
    d4, d3, d2 = w4.to(cuda), w3.to(cuda), w2.to(cuda)
    L.check(L.lib().pnr_pack_bwd_h2(L.ptr(d4), L.ptr(d3), 263, L.ptr(d2), X3_PAD, L.ptr(sc), L.ptr(packs),
                                    packs.numel() * 4, L.stream_ptr(cuda)), "pnr_pack_bwd_h2")
    got = packs.cpu().view(torch.int16).view(3, -1)
    for m, W in enumerate((w4.t(), w3[:, :256].t(), w2.t())):
        ref, s = frag_pack_h2(W.contiguous())
        steps = (16 + X3_PAD) * 8192   # frag_pack_h2 pads H2_PAD steps; the kernel reads X3_PAD ahead
        assert torch.equal(got[m], ref.view(torch.int16).reshape(-1)[:steps]), m
        assert float(sc[m]) == s, (m, float(sc[m]), s)


def test_pack_batch_equals_single_packs(cuda):
    """pnr_pack_batch (the training step's packs in one launch) == the per-matrix
    pnr_pack_weights / pnr_pack_weights_h2 calls bitwise, for fp32, fp32x3 and
    h2 jobs of mixed shapes (strided views, bias columns); an h2 job whose shift
    is too small raises its flag, the others leave theirs down."""
    from pointnerf_amd import _lib as L
    from pointnerf_amd.aggregator import H2_PAD, PREFETCH_PAD, X3_PAD, _pack_device, _pack_h2_device, h2_shift
    g = torch.Generator().manual_seed(21)
    big = torch.randn((256, 300), generator=g).to(cuda) * 0.2
    specs = [(0, big[:, :224], big[:, 299], PREFETCH_PAD), (0, big[:, 224:284], None, PREFETCH_PAD),
             (1, big[:, :263], big[:, 263], X3_PAD), (2, big[:, :256], None, H2_PAD),
             (2, big[:128, :144], big[:128, 150], H2_PAD),
             (0, big[:33, :32].t(), None, PREFETCH_PAD),
             (2, big[:, 10:70], None, H2_PAD)]
    flags = [torch.zeros(1, dtype=torch.int32, device=cuda) for _ in specs]
    jobs, outs, refs = (L.PackJob * len(specs))(), [], []
    for q, (kind, W, b, pad) in enumerate(specs):
        sft = h2_shift(W, b) - (1 if q == 6 else 0) if kind == 2 else 0
        if kind == 2:
            ref = _pack_h2_device(W, b, sft, torch.zeros(1, dtype=torch.int32, device=cuda))
        else:
            ref = _pack_device(kind, W, b, pad)
        out = torch.empty_like(ref)
        refs.append(ref)
        outs.append(out)
        bb = None if b is None else b.contiguous()
        outs.append(bb)
        jobs[q] = L.PackJob(kind, W.data_ptr(), W.stride(0), W.stride(1), W.shape[0], W.shape[1], L.ptr(bb), pad, sft,
                            flags[q].data_ptr(), out.data_ptr(), out.numel() * out.element_size())
    L.check(L.lib().pnr_pack_batch(jobs, len(specs), L.stream_ptr(cuda)), "pnr_pack_batch")
    for q in range(len(specs)):
        got, ref = outs[2 * q], refs[q]
        assert torch.equal(got.view(torch.int16), ref.view(torch.int16)), q
        assert int(flags[q]) == (1 if q == 6 else 0), q


def test_color_dz_equals_torch(cuda):
    """pnr_color_dz == the torch ops it replaces in the backward (d_feat[:, 1:] *
    (vmask != 0) through where(hc > 0, x, x * slope)) bitwise, and its absmax
    word == max |dz| (float bits)."""
    from pointnerf_amd import _lib as L
    g = torch.Generator().manual_seed(4)
    n = 3001
    d_feat = torch.randn((n + 5, 129), generator=g).to(cuda)
    vmask = (torch.rand(n + 5, generator=g) > 0.3).int().to(cuda)
    hc = torch.randn((n + 5, 128), generator=g).to(cuda)
    dz = torch.empty((n, 128), device=cuda)
    word = torch.zeros(1, dtype=torch.int32, device=cuda)
    L.check(L.lib().pnr_color_dz(L.ptr(d_feat), 129, L.ptr(vmask), L.ptr(hc), 128, n, 128, 0.2, L.ptr(dz),
                                 L.ptr(word), L.stream_ptr(cuda)), "pnr_color_dz")
    x = d_feat[:n, 1:] * (vmask[:n] != 0).float()[:, None]
    ref = torch.where(hc[:n] > 0, x, x * 0.2)
    assert torch.equal(dz, ref)
    assert int(word) == int(ref.abs().max().view(torch.int32))
