"""Fused SSIM loss on the HIP kernels of csrc/gsr_ssim.hip.

Mirrors `fused_ssim(img1, img2, padding="same", train=True)` of the fused-ssim extension the reference
imports (gs_lightning/lightning/gs_lightning_module.py:10) and uses as the loss term `1 - fused_ssim(render,
gt)` (:100, :279): mean SSIM over (B,C,H,W) images with an 11x11 Gaussian window (sigma 1.5), C1 = 0.01^2,
C2 = 0.03^2 and zero "same" padding; padding="valid" averages the map cropped by 5 px.  Differentiable w.r.t.
img1 (the rendering), as upstream.  No CPU fallback: the HIP library must load.
"""
from __future__ import annotations

import torch

from . import _native
from .rasterizer import _stream_handle

__all__ = ["fused_ssim"]


def _prep(img: torch.Tensor, name: str) -> torch.Tensor:
    if img.dim() == 3:
        img = img.unsqueeze(0)
    if img.dim() != 4:
        raise RuntimeError(f"{name} must be (B,C,H,W) or (C,H,W), got {tuple(img.shape)}")
    if img.dtype != torch.float32:
        img = img.float()
    return img.contiguous()


class _FusedSSIM(torch.autograd.Function):
    @staticmethod
    def forward(ctx, img1, img2, padding, train):
        lib = _native.load()
        x, y = _prep(img1, "img1"), _prep(img2.to(img1.device), "img2")
        if x.shape != y.shape:
            raise RuntimeError(f"img1 {tuple(x.shape)} and img2 {tuple(y.shape)} differ")
        B, C, H, W = x.shape
        planes = B * C
        valid = 1 if padding == "valid" else 0
        if padding not in ("same", "valid"):
            raise ValueError(f"padding must be 'same' or 'valid', got {padding!r}")
        counted = planes * ((H - 10) * (W - 10) if valid else H * W)
        if counted <= 0:
            raise RuntimeError("image smaller than the SSIM window")
        partial = torch.empty(lib.gsr_ssim_num_partials(planes, H, W), dtype=torch.float32, device=x.device)
        need_grad = bool(train) and ctx.needs_input_grad[0]
        maps = [torch.empty_like(x) for _ in range(3)] if need_grad else [None, None, None]
        ptr = lambda t: None if t is None else t.data_ptr()  # noqa: E731
        rc = lib.gsr_ssim_forward(planes, H, W, x.data_ptr(), y.data_ptr(), valid, partial.data_ptr(),
                                  ptr(maps[0]), ptr(maps[1]), ptr(maps[2]), _stream_handle(x.device))
        _native.check(rc, "fused_ssim")
        ctx.valid, ctx.shape, ctx.in_shape = valid, (planes, H, W), img1.shape
        if need_grad:
            ctx.save_for_backward(x, y, *maps)
        return partial.sum() / counted

    @staticmethod
    def backward(ctx, grad):
        x, y, d_mu1, d_s11, d_s12 = ctx.saved_tensors
        planes, H, W = ctx.shape
        g = grad.detach().float().reshape(1).contiguous()
        dx = torch.empty_like(x)
        lib = _native.load()
        rc = lib.gsr_ssim_backward(planes, H, W, x.data_ptr(), y.data_ptr(), ctx.valid, g.data_ptr(), d_mu1.data_ptr(),
                                   d_s11.data_ptr(), d_s12.data_ptr(), dx.data_ptr(), _stream_handle(x.device))
        _native.check(rc, "fused_ssim_backward")
        return dx.view(ctx.in_shape), None, None, None


def fused_ssim(img1: torch.Tensor, img2: torch.Tensor, padding: str = "same", train: bool = True) -> torch.Tensor:
    return _FusedSSIM.apply(img1, img2, padding, train)
