"""MI355X-native differentiable Gaussian rasterizer (drop-in for `diff_gaussian_rasterization`).

The hot path of pomelyu/gaussian_splatting_lightning -- preprocess, binning, compositing and their
backward -- runs in hand-written HIP kernels for gfx950 (csrc/), exposed through the C ABI in
include/gsrast.h and bound here with ctypes.  See DESIGN.md.
"""
from .rasterizer import (GaussianRasterizationSettings, GaussianRasterizer, mark_visible,  # noqa: F401
                         rasterize_gaussians)

__all__ = ["GaussianRasterizationSettings", "GaussianRasterizer", "rasterize_gaussians", "mark_visible"]
