"""GaussianModel with the reference's attribute names and methods, on the HIP kernels of this package.

Mirrors gs_lightning/modules/gaussian_model.py:18-333 so a training loop written against the reference keeps
working: `_xyz`, `_features_dc`, `_features_rest`, `_opacity`, `_scaling`, `_rotation` parameters and the
`xyz_grad_accum`, `xyz_grad_count`, `max_radii2D` buffers, the activations, and:

* `initialize(colmap_ply)`   -- points3D.ply read on the GPU (ply.read_points_ply), exact 3-NN scale init
                                (knn.dist_cuda2 replacing the scipy KDTree distCUDA2), SH0 from colour;
* `load_model_ply(path)`     -- ply.load_ply(compat="gs_lightning"): the reference loader's results, bugs and
                                all; `load_ply(path)` is the official-3DGS loader;
* `save_ply(path)`           -- byte-identical to the reference writer (ply.save_ply);
* `update_max_radii2D`, `update_xyz_gradient`, `densify_and_prune(..., optimizer=None)` -- densify.py
  (with `optimizer=` the Adam state is re-indexed in the same launch as the parameters);
* `reset_opacity`, `reset_max_radii2D`, `reset_xyz_gradient`, `step_sh_degree`, `ready_for_*`.

`spatial_scale` is passed directly (the reference derives it from COLMAP cameras with pycolmap,
utils/colmap.py get_nerf_norm, which is outside this package's scope).  Tensors live on `device` (a GPU).
"""
from __future__ import annotations

from typing import Optional

import torch
from torch import nn

from . import densify as _densify
from . import ply as _ply
from .knn import dist_cuda2

__all__ = ["GaussianModel", "rgb2sh0", "sh02rgb", "inverse_sigmoid", "C0"]

C0 = 0.28209479177387814  # gs_lightning/utils/sh.py:7


def rgb2sh0(rgb):
    return (rgb - 0.5) / C0


def sh02rgb(sh0):
    return sh0 * C0 + 0.5


def inverse_sigmoid(x: torch.Tensor) -> torch.Tensor:
    return torch.log(x / (1 - x))  # gs_lightning/utils/math.py:5-6


class GaussianModel(nn.Module):
    PARAMETER_NAMES = list(_densify.PARAMETER_NAMES)

    def __init__(self, sh_degree: int = 3, colmap_ply: Optional[str] = None, spatial_scale: Optional[float] = None,
                 use_screensize_threshold: bool = True, device="cuda"):
        super().__init__()
        self.use_screensize_threshold = use_screensize_threshold
        self.max_sh_degree = sh_degree
        self.active_sh_degree = 0
        self.device = torch.device(device)
        self.activation_opacity = torch.sigmoid
        self.inversed_activation_opacity = inverse_sigmoid
        self.activation_scaling = torch.exp
        self.inversed_activation_scaling = torch.log
        if colmap_ply is not None:
            self.initialize(colmap_ply)
        self.spatial_scale = spatial_scale

    # ---- creation / IO ----
    @torch.no_grad()
    def initialize(self, colmap_ply: str) -> None:
        """gaussian_model.py:65-107."""
        xyz, color = _ply.read_points_ply(colmap_ply, device=self.device)
        self.create_from_points(xyz, color)

    @torch.no_grad()
    def create_from_points(self, xyz: torch.Tensor, color: torch.Tensor) -> None:
        N = len(xyz)
        M = (self.max_sh_degree + 1) ** 2
        sh = torch.zeros(N, 3, M, device=self.device)
        sh[:, :, 0] = rgb2sh0(color.to(self.device))
        rotation = torch.zeros((N, 4), device=self.device)
        rotation[:, 0] = 1
        dist = torch.clamp_min(dist_cuda2(xyz.to(self.device)), 0.0000001)
        scale = self.inversed_activation_scaling(torch.sqrt(dist))[..., None].repeat(1, 3)
        opacity = self.inversed_activation_opacity(0.1 * torch.ones(N, 1, device=self.device))
        self._xyz = nn.Parameter(xyz.to(self.device).float().contiguous())
        self._features_dc = nn.Parameter(sh[..., :1].transpose(1, 2).contiguous())
        self._features_rest = nn.Parameter(sh[..., 1:].transpose(1, 2).contiguous())
        self._scaling = nn.Parameter(scale.contiguous())
        self._rotation = nn.Parameter(rotation)
        self._opacity = nn.Parameter(opacity)
        self.register_buffer("xyz_grad_accum", torch.zeros(N, device=self.device))
        self.register_buffer("xyz_grad_count", torch.zeros(N, device=self.device))
        self.register_buffer("max_radii2D", torch.zeros(N, device=self.device))

    def _set_params(self, d) -> None:
        for k in self.PARAMETER_NAMES:
            setattr(self, f"_{k}", nn.Parameter(d[k]))
        N = len(d["xyz"])
        for k in ("xyz_grad_accum", "xyz_grad_count", "max_radii2D"):
            if k in self._buffers:
                self._buffers[k] = torch.zeros(N, device=self.device)
            else:
                self.register_buffer(k, torch.zeros(N, device=self.device))
        self.active_sh_degree = d["active_sh_degree"]

    def load_model_ply(self, ply_path: str) -> None:
        """gaussian_model.py:112-132 (its three loader bugs reproduced; see ply.load_ply)."""
        self._set_params(_ply.load_ply(ply_path, compat="gs_lightning", device=self.device))

    def load_ply(self, ply_path: str) -> None:
        """The official 3DGS loader (third_party/.../gaussian_model.py:263-314)."""
        d = _ply.load_ply(ply_path, compat="official", device=self.device)
        self._set_params(d)
        self.max_sh_degree = max(self.max_sh_degree, d["active_sh_degree"])

    def save_ply(self, ply_path: str) -> bool:
        """gaussian_model.py:150-171."""
        return _ply.save_ply(ply_path, self._xyz, self._features_dc, self._features_rest, self._opacity,
                             self._scaling, self._rotation)

    # ---- densification ----
    def update_max_radii2D(self, radii: torch.Tensor, visible_mask: torch.Tensor) -> None:
        _densify.update_max_radii2D(self, radii, visible_mask)

    def update_xyz_gradient(self, screenspace_gradient: torch.Tensor, visible_mask: torch.Tensor) -> None:
        _densify.update_xyz_gradient(self, screenspace_gradient, visible_mask)

    def densify_and_prune(self, densify_grad_threshold: float, clone_size_threshold: float,
                          prune_opacity_threshold: float, prune_size_threshold: float,
                          prune_screensize_threshold: Optional[float] = None, optimizer=None,
                          generator: Optional[torch.Generator] = None) -> torch.Tensor:
        return _densify.densify_and_prune(self, densify_grad_threshold, clone_size_threshold,
                                          prune_opacity_threshold, prune_size_threshold,
                                          prune_screensize_threshold, optimizer=optimizer, generator=generator)

    @torch.no_grad()
    def reset_opacity(self):
        """gaussian_model.py:289-293."""
        new_opacity = torch.min(self.get_opacity(), torch.ones_like(self._opacity) * 0.01)
        self._opacity[:] = self.inversed_activation_opacity(new_opacity)[:]

    def reset_max_radii2D(self):
        self.max_radii2D.fill_(0.0)

    def reset_xyz_gradient(self):
        self.xyz_grad_accum.fill_(0.0)
        self.xyz_grad_count.fill_(0.0)

    def step_sh_degree(self):
        self.active_sh_degree = min(self.active_sh_degree + 1, self.max_sh_degree)

    def ready_for_training(self) -> bool:
        if not hasattr(self, "_xyz"):
            raise RuntimeError("colmap_ply is required for training")
        if self.spatial_scale is None:
            raise RuntimeError("spatial_scale is required for training")
        return True

    def ready_for_inference(self) -> bool:
        if not hasattr(self, "_xyz"):
            raise RuntimeError("load_model_ply should be executred before inference")
        return True

    # ---- activations ----
    def get_xyz(self) -> torch.Tensor:
        return self._xyz

    def get_features(self) -> torch.Tensor:
        return torch.cat([self._features_dc, self._features_rest], 1)

    def get_opacity(self) -> torch.Tensor:
        return self.activation_opacity(self._opacity)

    def get_scaling(self) -> torch.Tensor:
        return self.activation_scaling(self._scaling)

    def get_rotation(self) -> torch.Tensor:
        return torch.nn.functional.normalize(self._rotation)

    def get_covariance(self, scaling_modifier: float = 1) -> torch.Tensor:
        """render_tools.computeConv3D (upper triangle of R S S^T R^T, kornia's w-first quaternion matrix)."""
        q = self.get_rotation()
        w, x, y, z = q.unbind(-1)
        R = torch.stack([1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y),
                         2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x),
                         2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)], -1).view(-1, 3, 3)
        L = R @ torch.diag_embed(self.get_scaling() * scaling_modifier)
        cov = L @ L.transpose(1, 2)
        return torch.stack([cov[:, 0, 0], cov[:, 0, 1], cov[:, 0, 2], cov[:, 1, 1], cov[:, 1, 2], cov[:, 2, 2]], -1)
