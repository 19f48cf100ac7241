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
from dataclasses import dataclass
from typing import Iterable, Optional

import torch

from . import _native
from .rasterizer import _stream_handle

__all__ = ["GaussianAdam", "SparseGaussianAdam", "ShViewsGradient"]

_MAX_GROUPS = 16  # ADAM_MAX_GROUPS in csrc/gsr_kernels.h


@dataclass
class ShViewsGradient:
    """The summed SH gradient of a multi-view step in factored form (multiview.ViewGradReducer.sh_views_gradient):
    dL/dshs[g] = sum_v basis(normalize(means3D[g] - campos[v])) (x) factors_v[g] (csrc/gsr_views.hip).  factors is the
    exchange's chunk-major (V, L_c, 3) gather buffer (chunk_len = L; 0: one (V, P, 3) block)."""
    means3D: torch.Tensor
    campos: torch.Tensor
    factors: torch.Tensor
    sh_degree: int
    chunk_len: int = 0


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
    def step(self, closure=None, sh_views: Optional[tuple] = None):
        """One Adam step of every parameter with a gradient.

        sh_views = (features_dc, features_rest, ShViewsGradient): the two SH parameters (M = 16 coefficients in all)
        take their gradient from the multi-view factors instead of .grad -- the expansion happens inside the update
        (gsr_adam_sh_views_step), bitwise the same as expanding into .grad and stepping (their .grad is ignored)."""
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        if sh_views is not None:
            # first: the expansion reads means3D, which this step's xyz group is about to update (the gradient
            # belongs to the forward's positions)
            a, (b1, b2, eps), dev = self._sh_views_args(*sh_views)
            _native.check(_native.load().gsr_adam_sh_views_step(ctypes.byref(a), b1, b2, eps, _stream_handle(dev)),
                          "gsr_adam_sh_views_step")
        skip = {id(t) for t in sh_views[:2]} if sh_views is not None else set()
        batches = {}
        keep_alive = []
        for group in self.param_groups:
            b1, b2 = group["betas"]
            lr = float(group["lr"])
            for p in group["params"]:
                if p.grad is None or id(p) in skip:
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

    def _sh_views_args(self, dc: torch.Tensor, rest: torch.Tensor, grad: ShViewsGradient):
        groups = {}
        for group in self.param_groups:
            for p in group["params"]:
                groups[id(p)] = group
        P = dc.shape[0]
        # either two packed tensors, or the column blocks [:, :1] and [:, 1:] of ONE contiguous (P, 16, 3) tensor
        joint = (not dc.is_contiguous() and dc.stride() == (48, 3, 1) and rest.stride() == (48, 3, 1)
                 and rest.data_ptr() == dc.data_ptr() + 12)
        for t, name, width in ((dc, "features_dc", 1), (rest, "features_rest", 15)):
            if id(t) not in groups:
                raise RuntimeError(f"sh_views: {name} is not a parameter of this optimizer")
            if t.dtype != torch.float32 or t.device.type != "cuda" or not (joint or t.is_contiguous()) or \
                    tuple(t.shape) != (P, width, 3):
                raise RuntimeError(f"sh_views: {name} must be a contiguous fp32 ({P}, {width}, 3) GPU tensor (or "
                                   "both the [:, :1] / [:, 1:] blocks of one contiguous (P, 16, 3) tensor)")
        gd, gr = groups[id(dc)], groups[id(rest)]
        if gd["betas"] != gr["betas"] or gd["eps"] != gr["eps"]:
            raise RuntimeError("sh_views: features_dc and features_rest must share betas and eps")
        V = grad.campos.shape[0]
        for t in (grad.means3D, grad.campos, grad.factors):
            if t.dtype != torch.float32 or not t.is_contiguous() or t.device != dc.device:
                raise RuntimeError("sh_views: means3D, campos and factors must be contiguous fp32 on the parameters' "
                                   "device")
        if grad.means3D.shape != (P, 3) or grad.factors.numel() != V * P * 3:
            raise RuntimeError("sh_views: means3D (P, 3) and factors (V * P * 3) do not match the parameters")
        if joint and len(self.state[dc]) == 0 and len(self.state[rest]) == 0:
            # a joint parameter gets joint moments too: each moment is one (P, 16, 3) tensor whose column blocks are
            # the two groups' states, so the update streams three arrays of one layout
            jm = torch.zeros(P, 16, 3, dtype=torch.float32, device=dc.device)
            jv = torch.zeros_like(jm)
            for t, sl in ((dc, slice(0, 1)), (rest, slice(1, 16))):
                self.state[t].update(step=torch.tensor(0.0, dtype=torch.float32), exp_avg=jm[:, sl],
                                     exp_avg_sq=jv[:, sl])
        steps = []
        for t in (dc, rest):
            state = self.state[t]
            if len(state) == 0:
                state["step"] = torch.tensor(0.0, dtype=torch.float32)
                state["exp_avg"] = torch.zeros_like(t, memory_format=torch.contiguous_format)
                state["exp_avg_sq"] = torch.zeros_like(t, memory_format=torch.contiguous_format)
            state["step"] += 1
            steps.append(int(state["step"].item()))
        sd, sr = self.state[dc], self.state[rest]
        joint_m = joint and all(
            sd[k].stride() == (48, 3, 1) and sr[k].stride() == (48, 3, 1) and sr[k].data_ptr() == sd[k].data_ptr() + 12
            for k in ("exp_avg", "exp_avg_sq"))
        for t, st, w in ((dc, sd, 1), (rest, sr, 15)):
            for k in ("exp_avg", "exp_avg_sq"):
                m = st[k]
                if tuple(m.shape) != (P, w, 3) or m.dtype != torch.float32 or not (joint_m or m.is_contiguous()):
                    raise RuntimeError("sh_views: optimizer state does not match its parameter")
        a = _native.AdamShViewsArgs(
            P=P, D=int(grad.sh_degree), M=16, V=V, chunk_len=int(grad.chunk_len), means3D=grad.means3D.data_ptr(),
            campos=grad.campos.data_ptr(), dL_dcolors_sh=grad.factors.data_ptr(),
            dc_param=dc.data_ptr(), dc_exp_avg=sd["exp_avg"].data_ptr(), dc_exp_avg_sq=sd["exp_avg_sq"].data_ptr(),
            dc_lr=float(gd["lr"]), dc_step=steps[0], rest_param=rest.data_ptr(), rest_exp_avg=sr["exp_avg"].data_ptr(),
            rest_exp_avg_sq=sr["exp_avg_sq"].data_ptr(), rest_lr=float(gr["lr"]), rest_step=steps[1],
            param_row_stride=48 if joint else 0, moment_row_stride=48 if joint_m else 0)
        return a, (float(gd["betas"][0]), float(gd["betas"][1]), float(gd["eps"])), dc.device


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
