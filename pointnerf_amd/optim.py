"""Adam on the HIP path (pnr_adam_step): the optimizer step of the c3 finetune
loop (train_ddp.py builds torch.optim.Adam over the point tables and the
aggregator MLP, mvs_points_volumetric_model.py:102-123).

Same update and hyperparameters as torch.optim.Adam with amsgrad=False,
maximize=False; every parameter of a group with a gradient is updated by ONE
launch (up to 32 tensors each), 28 B of HBM traffic per element -- the 2 M x 39
point parameters are the whole cost of the step.  Gradients must be dense fp32
on the GPU; a non-contiguous parameter is refused (its state would need a
copy-back per step)."""
from __future__ import annotations

import ctypes

import torch

from . import _lib as L


def _bump_versions(ps):
    """The kernel writes the parameters through raw pointers, which autograd's
    version counters do not see; callers that cache derived data per parameter
    version (the aggregator's weight packs, keyed on p._version) must see the
    update as torch's in-place ops would report it."""
    setv = getattr(torch._C._autograd, "_unsafe_set_version_counter", None)
    try:
        if setv is None:
            raise TypeError
        setv(tuple(ps), tuple(p._version + 1 for p in ps))
    except TypeError:
        # older torch (no tuple API): a 1-element in-place no-op on the parameter
        # itself -- p.data has its own version counter, which would not be seen
        with torch.no_grad():
            for p in ps:
                p.view(-1)[:1].add_(0)


class Adam(torch.optim.Optimizer):
    """torch.optim.Adam(params, lr, betas, eps, weight_decay) on pnr_adam_step."""

    def __init__(self, params, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.0):
        if lr < 0.0 or eps < 0.0 or weight_decay < 0.0 or not (0.0 <= betas[0] < 1.0 and 0.0 <= betas[1] < 1.0):
            raise ValueError(f"Adam: bad hyperparameters lr={lr} betas={betas} eps={eps} wd={weight_decay}")
        super().__init__(params, dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay))

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            by_step: dict[int, list] = {}
            for p in group["params"]:
                if p.grad is None:
                    continue
                g = p.grad
                if p.dtype != torch.float32 or not p.is_cuda or g.is_sparse or not p.is_contiguous():
                    raise L.PnrError("Adam: parameters must be contiguous dense fp32 CUDA tensors")
                if g.dtype != torch.float32 or not g.is_contiguous():
                    g = g.float().contiguous()
                st = self.state[p]
                if not st:
                    st["step"] = 0
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                st["step"] += 1
                by_step.setdefault(st["step"], []).append((p, g, st))
            b1, b2 = group["betas"]
            for t, items in by_step.items():
                n = len(items)
                ptrs = [(ctypes.c_void_p * n)(*(x.data_ptr() for x in col)) for col in
                        ([i[0] for i in items], [i[1] for i in items], [i[2]["exp_avg"] for i in items],
                         [i[2]["exp_avg_sq"] for i in items])]
                numel = (ctypes.c_int64 * n)(*(i[0].numel() for i in items))
                dev = items[0][0].device
                L.check(L.lib().pnr_adam_step(n, *ptrs, numel, float(group["lr"]), float(b1), float(b2),
                                              float(group["eps"]), float(group["weight_decay"]), int(t),
                                              L.stream_ptr(dev)), "pnr_adam_step")
                _bump_versions([i[0] for i in items])
        return loss
