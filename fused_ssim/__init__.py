"""Import-name shim: `from fused_ssim import fused_ssim` (gs_lightning_module.py:10) resolves to the MI355X
HIP SSIM loss, so the reference's training module imports unmodified."""
from gaussian_splatting_lightning_amd.ssim import fused_ssim  # noqa: F401

__all__ = ["fused_ssim"]
