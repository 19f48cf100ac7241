"""Parameter activations in front of the rasterizer (csrc/gsr_adam.hip, ABI gsr_activations_forward / _backward).

The reference keeps raw parameters and activates them every step (gs_lightning/modules/gaussian_model.py:
get_scaling = exp(_scaling), get_opacity = sigmoid(_opacity), get_rotation = torch.nn.functional.normalize(_rotation),
which is q / max(|q|, 1e-12)); torch runs that as ~15 elementwise kernels per step between the forward and autograd.
`activate` / `activate_backward` do it in one launch each, and `GaussianActivations` wraps them as an autograd
Function.  Device fp32 tensors only; no CPU fallback.
"""
from __future__ import annotations

import torch

from . import _native
from .rasterizer import _stream_handle

__all__ = ["activate", "activate_backward", "GaussianActivations"]


def _check(*ts: torch.Tensor) -> None:
    for t in ts:
        if not t.is_cuda or t.dtype != torch.float32 or not t.is_contiguous():
            raise ValueError("activations: contiguous fp32 device tensors expected")


def activate(scaling: torch.Tensor, opacity: torch.Tensor, rotation: torch.Tensor, out=None):
    """(exp(scaling), sigmoid(opacity), normalize(rotation)); out = optional preallocated (scales, opacities,
    rotations)."""
    N = scaling.shape[0]
    if scaling.shape != (N, 3) or opacity.numel() != N or rotation.shape != (N, 4):
        raise ValueError("activations: expected scaling (N,3), opacity (N) or (N,1), rotation (N,4)")
    if out is None:
        out = (torch.empty_like(scaling), torch.empty_like(opacity), torch.empty_like(rotation))
    if tuple(o.numel() for o in out) != (3 * N, N, 4 * N):
        raise ValueError("activations: out must hold (N,3), (N) and (N,4) elements")
    _check(scaling, opacity, rotation, *out)
    lib = _native.load()
    _native.check(lib.gsr_activations_forward(N, scaling.data_ptr(), opacity.data_ptr(), rotation.data_ptr(),
                                              out[0].data_ptr(), out[1].data_ptr(), out[2].data_ptr(),
                                              _stream_handle(scaling.device)), "gsr_activations_forward")
    return out


def activate_backward(rotation: torch.Tensor, scales: torch.Tensor, opacities: torch.Tensor,
                      rotations: torch.Tensor, dL_dscales: torch.Tensor, dL_dopacities: torch.Tensor,
                      dL_drotations: torch.Tensor, out=None):
    """Gradients w.r.t. the raw (scaling, opacity, rotation) from those w.r.t. the activated values; rotation is
    the raw quaternion, scales / opacities / rotations the forward's outputs."""
    N = rotation.shape[0]
    for t, w in ((scales, 3), (opacities, 1), (rotations, 4), (dL_dscales, 3), (dL_dopacities, 1),
                 (dL_drotations, 4)):
        if t.numel() != N * w:
            raise ValueError("activations: gradient / activation shapes do not match N")
    if out is None:
        out = (torch.empty_like(scales), torch.empty_like(opacities), torch.empty_like(rotation))
    if tuple(o.numel() for o in out) != (3 * N, N, 4 * N):
        raise ValueError("activations: out must hold (N,3), (N) and (N,4) elements")
    _check(rotation, scales, opacities, rotations, dL_dscales, dL_dopacities, dL_drotations, *out)
    lib = _native.load()
    _native.check(lib.gsr_activations_backward(
        N, rotation.data_ptr(), scales.data_ptr(), opacities.data_ptr(), rotations.data_ptr(), dL_dscales.data_ptr(),
        dL_dopacities.data_ptr(), dL_drotations.data_ptr(), out[0].data_ptr(), out[1].data_ptr(), out[2].data_ptr(),
        _stream_handle(rotation.device)), "gsr_activations_backward")
    return out


class GaussianActivations(torch.autograd.Function):
    """scales, opacities, rotations = GaussianActivations.apply(_scaling, _opacity, _rotation)."""

    @staticmethod
    def forward(ctx, scaling, opacity, rotation):
        scaling, opacity, rotation = scaling.contiguous(), opacity.contiguous(), rotation.contiguous()
        scales, opacities, rotations = activate(scaling, opacity, rotation)
        ctx.save_for_backward(rotation, scales, opacities, rotations)
        return scales, opacities, rotations

    @staticmethod
    def backward(ctx, d_scales, d_opacities, d_rotations):
        rotation, scales, opacities, rotations = ctx.saved_tensors
        z = torch.zeros_like
        d_scales = z(scales) if d_scales is None else d_scales.contiguous()
        d_opacities = z(opacities) if d_opacities is None else d_opacities.contiguous()
        d_rotations = z(rotations) if d_rotations is None else d_rotations.contiguous()
        return activate_backward(rotation, scales, opacities, rotations, d_scales, d_opacities, d_rotations)
