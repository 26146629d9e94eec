"""2-D neural renderer (pnr_neural_render_fwd) vs the torch fp32 restatement of
models/neural_render/neural_renderer.py:81-104 (the reference module itself
needs kornia, absent here: parity against it is unpinned; the torch
convolution reference is the fp32 check).  Tolerance 2e-5 absolute on the
sigmoid outputs."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("H,W", [(40, 150), (7, 129), (64, 64)])
def test_neural_render_vs_torch(cuda, H, W):
    from pointnerf_amd.neural_render import NeuralRenderer
    torch.manual_seed(H * 1000 + W)
    m = NeuralRenderer(input_dim=128)
    x = torch.randn((1, H, W, 128)) * 0.5
    with torch.no_grad():
        ref = m.forward_torch(x.double().float())           # CPU fp32 convolutions
        md = m.to(cuda)
        got = md(x.to(cuda)).cpu()
    assert got.shape == (1, H, W, 3)
    np.testing.assert_allclose(got.numpy(), ref.numpy(), atol=2e-5, rtol=0)


def test_state_dict_names_match_reference():
    from pointnerf_amd.neural_render import NeuralRenderer
    names = sorted(NeuralRenderer(input_dim=128).state_dict())
    # neural_renderer.py:51-66 for n_feat = input_dim = 128, img_size 64, rgb skips
    assert names == sorted(["conv_layers.0.weight", "conv_layers.0.bias", "conv_layers.1.weight",
                            "conv_layers.1.bias", "conv_rgb.0.weight", "conv_rgb.0.bias", "conv_rgb.1.weight",
                            "conv_rgb.1.bias", "conv_rgb.2.weight", "conv_rgb.2.bias"])
