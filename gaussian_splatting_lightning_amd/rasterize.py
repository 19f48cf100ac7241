"""`gs_lightning.rasterize`-shaped entry points over the HIP rasterizer.

Mirrors the reference's pure-Python module interface (gs_lightning/rasterize/__init__.py:1-2):

* ``rasterize_gaussian(means3D, opacities, scales, rotations, shs, scale_modifier, image_width, image_height,
  tanfovx, tanfovy, viewmatrix, projmatrix, campos, background, sh_degree)`` -> ``(image (3,H,W), radii (N,)
  float, invdepth (1,H,W))`` -- same argument order and meaning as gs_lightning/rasterize/rasterize.py:28-46,
  same return layout as :125-127 (radii are returned as float, as the Python path does at :79-80).
  Differentiable w.r.t. means3D, opacities, scales, rotations and shs.
* ``markVisible(means3D, viewmatrix, projmatrix)`` -> bool (N,) (rasterize.py:23-26).

Compositing follows the CUDA submodule's semantics: the Python path's per-tile
termination differs only on saturated pixels.  There is no CPU fallback: the HIP library must load.
"""
from __future__ import annotations

import torch

from .rasterizer import GaussianRasterizationSettings, mark_visible, rasterize_gaussians

__all__ = ["rasterize_gaussian", "markVisible"]


def markVisible(means3D: torch.Tensor, viewmatrix: torch.Tensor, projmatrix: torch.Tensor) -> torch.Tensor:
    return mark_visible(means3D, viewmatrix, projmatrix)


def rasterize_gaussian(means3D, opacities, scales, rotations, shs, scale_modifier, image_width, image_height,
                       tanfovx, tanfovy, viewmatrix, projmatrix, campos, background, sh_degree):
    settings = GaussianRasterizationSettings(
        image_height=int(image_height), image_width=int(image_width), tanfovx=float(tanfovx),
        tanfovy=float(tanfovy), bg=background, scale_modifier=float(scale_modifier), viewmatrix=viewmatrix,
        projmatrix=projmatrix, sh_degree=int(sh_degree), campos=campos, prefiltered=False, debug=False,
        antialiasing=False)
    means2D = torch.zeros_like(means3D)
    color, radii, invdepth = rasterize_gaussians(means3D, means2D, shs, None, opacities, scales, rotations, None,
                                                 settings)
    return color, radii.to(torch.float32), invdepth
