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

__all__ = ["GaussianAdam", "SparseGaussianAdam"]

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


class SparseGaussianAdam(torch.optim.Adam):
    """`diff_gaussian_rasterization.SparseGaussianAdam` of the upstream rasterizer package: the optimizer the
    reference's third_party GaussianModel takes with optimizer_type "sparse_adam"
    (gs_lightning/third_party/gaussian_splatting/scene/gaussian_model.py:26,194-196; the package is an empty
    submodule here).  Same constructor and state as the upstream class; ``step(visibility, N)``
    updates only the Gaussians with ``visibility`` set (``radii > 0`` of the view), every group in ONE launch of
    ``sparse_adam_kernel`` (csrc/gsr_adam.hip, ABI gsr_sparse_adam_step), with the upstream kernel's arithmetic:
    betas fixed at (0.9, 0.999), no bias correction, ``state["step"]`` never advanced.  Each group holds exactly one
    parameter of N x M elements (the upstream class asserts the same)."""

    def __init__(self, params, lr, eps):
        super().__init__(params=params, lr=lr, eps=eps)

    @torch.no_grad()
    def step(self, visibility, N):
        N = int(N)
        if N <= 0:
            raise ValueError("SparseGaussianAdam.step: N must be positive")
        groups = []
        keep_alive = []
        dev = None
        for group in self.param_groups:
            lr, eps = float(group["lr"]), float(group["eps"])
            assert len(group["params"]) == 1, "more than one tensor in group"
            param = group["params"][0]
            if param.grad is None:
                continue
            if param.dtype != torch.float32 or param.device.type != "cuda" or not param.is_contiguous():
                raise RuntimeError("SparseGaussianAdam: parameters must be contiguous fp32 tensors on the GPU")
            if param.numel() % N != 0:
                raise RuntimeError("SparseGaussianAdam: a parameter's element count is not a multiple of N")
            g = param.grad
            if not g.is_contiguous() or g.dtype != torch.float32:
                g = g.float().contiguous()
                keep_alive.append(g)
            state = self.state[param]
            if len(state) == 0:
                state["step"] = torch.tensor(0.0, dtype=torch.float32)
                state["exp_avg"] = torch.zeros_like(param, memory_format=torch.preserve_format)
                state["exp_avg_sq"] = torch.zeros_like(param, memory_format=torch.preserve_format)
            m, v = state["exp_avg"], state["exp_avg_sq"]
            if not (m.is_contiguous() and v.is_contiguous() and m.shape == param.shape and v.shape == param.shape):
                raise RuntimeError("SparseGaussianAdam: optimizer state does not match its parameter")
            if dev is not None and param.device != dev:
                raise RuntimeError("SparseGaussianAdam: parameters on different devices")
            dev = param.device
            groups.append((eps, _native.AdamGroup(param.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(),
                                                  param.numel(), lr, 0)))
        if not groups:
            return
        vis = visibility
        if vis.device != dev or vis.dtype not in (torch.bool, torch.uint8) or vis.numel() != N:
            raise RuntimeError("SparseGaussianAdam: visibility must be an (N,) bool tensor on the parameters' device")
        vis = vis.contiguous()
        lib = _native.load()
        stream = _stream_handle(dev)
        by_eps = {}
        for eps, grp in groups:
            by_eps.setdefault(eps, []).append(grp)
        for eps, grps in by_eps.items():
            for i in range(0, len(grps), _MAX_GROUPS):
                chunk = grps[i:i + _MAX_GROUPS]
                arr = (_native.AdamGroup * len(chunk))(*chunk)
                _native.check(lib.gsr_sparse_adam_step(arr, len(chunk), vis.data_ptr(), N, 0.9, 0.999, eps, stream),
                              "gsr_sparse_adam_step")
        del keep_alive
