"""Torch-convolution restatement of the fork's 2-D neural renderer
(models/neural_render/neural_renderer.py:81-104): the checker of
pointnerf_amd.neural_render.NeuralRenderer in the tests (test infrastructure,
not product code; parity unpinned: the reference module needs kornia)."""
import torch
import torch.nn.functional as F


def neural_render_torch(mod, x):
    """rgb [1, H, W, 3] of ``mod``'s parameters on x [1, H, W, 128] with torch
    convolutions (autograd path, any dtype / device)."""
    x = x.permute(0, 3, 1, 2)
    rgb = mod.conv_rgb[0](x)
    net = x
    for i, layer in enumerate(mod.conv_layers):
        net = F.leaky_relu(layer(net), 0.2)
        rgb = rgb + mod.conv_rgb[i + 1](net)
    return torch.sigmoid(rgb).permute(0, 2, 3, 1)
