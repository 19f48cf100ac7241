"""Import-name shim: `from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer`
resolves to the MI355X HIP implementation, so the reference's scripts (gs_lightning_module.py:9,
render_trained_image.py:10-11, tests/rasterizer_python/test_cases.py:2) run unmodified; SparseGaussianAdam is the
upstream package's visibility-masked optimizer (third_party gaussian_model.py:26,194-196)."""
from gaussian_splatting_lightning_amd.optim import SparseGaussianAdam  # noqa: F401
from gaussian_splatting_lightning_amd.rasterizer import (GaussianRasterizationSettings,  # noqa: F401
                                                         GaussianRasterizer, rasterize_gaussians)

__all__ = ["GaussianRasterizationSettings", "GaussianRasterizer", "rasterize_gaussians", "SparseGaussianAdam"]
