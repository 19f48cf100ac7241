"""Fused Adam for the Gaussian parameter groups (csrc/gsr_adam.hip).

The reference optimises six per-Gaussian parameter groups with `torch.optim.Adam(lr=0.0, eps=1e-15)`
(gs_lightning/lightning/gs_lightning_module.py:114-134, configs/train_gs.yaml:20-25).  `GaussianAdam` is a
drop-in `torch.optim.Optimizer` with the same constructor, the same `param_groups` (including the "name" key
the reference uses to find its groups) and the same per-parameter state keys ("step", "exp_avg",
"exp_avg_sq"), so the reference's state surgery (update_optimizer_parameters, gs_lightning_module.py:213-235)
and its learning-rate scheduler work unchanged.  `step()` updates every group in ONE kernel launch per 16
parameters instead of torch's ~10 foreach launches per group.

Not supported (the reference uses none of them): weight_decay, amsgrad, maximize, sparse gradients,
non-fp32 or CPU parameters -- these raise instead of falling back.
"""
from __future__ import annotations

import ctypes
from typing import Iterable

import torch

from . import _native
from .rasterizer import _stream_handle

__all__ = ["GaussianAdam"]

_MAX_GROUPS = 16  # ADAM_MAX_GROUPS in csrc/gsr_kernels.h


class GaussianAdam(torch.optim.Optimizer):
    def __init__(self, params: Iterable, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 0.0, amsgrad: bool = False, maximize: bool = False, **_ignored):
        if weight_decay != 0.0 or amsgrad or maximize:
            raise NotImplementedError("GaussianAdam: weight_decay, amsgrad and maximize are not supported")
        if not 0.0 <= eps:
            raise ValueError(f"Invalid epsilon value: {eps}")
        if not (0.0 <= betas[0] < 1.0 and 0.0 <= betas[1] < 1.0):
            raise ValueError(f"Invalid betas: {betas}")
        defaults = dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=0.0, amsgrad=False, maximize=False)
        super().__init__(params, defaults)

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        batches = {}
        keep_alive = []
        for group in self.param_groups:
            b1, b2 = group["betas"]
            lr = float(group["lr"])
            for p in group["params"]:
                if p.grad is None:
                    continue
                g = p.grad
                if g.is_sparse:
                    raise RuntimeError("GaussianAdam does not support sparse gradients")
                if p.dtype != torch.float32 or p.device.type != "cuda":
                    raise RuntimeError("GaussianAdam: parameters must be fp32 tensors on the GPU")
                if not p.is_contiguous():
                    raise RuntimeError("GaussianAdam: parameters must be contiguous")
                if not g.is_contiguous() or g.dtype != torch.float32:
                    g = g.float().contiguous()
                    keep_alive.append(g)
                state = self.state[p]
                if len(state) == 0:
                    state["step"] = torch.tensor(0.0, dtype=torch.float32)
                    state["exp_avg"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                    state["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                m, v = state["exp_avg"], state["exp_avg_sq"]
                if m.shape != p.shape or v.shape != p.shape:
                    raise RuntimeError("GaussianAdam: optimizer state shape does not match its parameter")
                state["step"] += 1
                key = (p.device, float(b1), float(b2), float(group["eps"]))
                batches.setdefault(key, []).append(
                    _native.AdamGroup(p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), p.numel(), lr,
                                      int(state["step"].item())))
        lib = _native.load() if batches else None
        for (dev, b1, b2, eps), groups in batches.items():
            stream = _stream_handle(dev)
            for i in range(0, len(groups), _MAX_GROUPS):
                chunk = groups[i:i + _MAX_GROUPS]
                arr = (_native.AdamGroup * len(chunk))(*chunk)
                _native.check(lib.gsr_adam_step(arr, len(chunk), b1, b2, eps, stream), "gsr_adam_step")
        del keep_alive
        return loss
