"""distCUDA2 -- mean squared distance to the three nearest neighbours, on the HIP kernels of csrc/gsr_knn.hip.

Drop-in for gs_lightning/utils/math.py:9-14 (a scipy KDTree query on the CPU) and for simple_knn's distCUDA2
that the official code imports: same signature, same result (exact 3-NN, not simple_knn's box
approximation), output on the input's device with the input's dtype.  No CPU fallback.
"""
from __future__ import annotations

import torch

from . import _native
from .rasterizer import _stream_handle

__all__ = ["dist_cuda2", "distCUDA2"]


@torch.no_grad()
def dist_cuda2(points: torch.Tensor) -> torch.Tensor:
    if points.device.type != "cuda":
        raise RuntimeError("distCUDA2 runs on the GPU (HIP kernels); move the points to a cuda device")
    if points.dim() != 2 or points.shape[1] != 3:
        raise RuntimeError(f"points must be (N, 3), got {tuple(points.shape)}")
    lib = _native.load()
    p = points.detach().float().contiguous()
    n = p.shape[0]
    out = torch.empty(n, dtype=torch.float32, device=p.device)
    if n:
        ws = torch.empty(lib.gsr_knn_workspace_bytes(n), dtype=torch.uint8, device=p.device)
        _native.check(lib.gsr_knn_mean_dist2(n, p.data_ptr(), out.data_ptr(), ws.data_ptr(), _stream_handle(p.device)),
                      "gsr_knn_mean_dist2")
    return out.to(points.dtype)


distCUDA2 = dist_cuda2
