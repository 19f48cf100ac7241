"""Seeded synthetic scenes and cameras for tests and bench.py (SURVEY.md §8(d) generator).

There is no dataset or checkpoint access, so every workload is drawn here:

    means3D   = randn(N,3)
    scales    = exp(randn(N,3)*0.5 - 4.0 - ln(N/1e5)/3)
    rotations = normalize(randn(N,4))            # (w, x, y, z)
    opacities = sigmoid(randn(N,1))
    shs       = randn(N,(D+1)^2,3)*0.3
    camera    = "treehill No.0" view (tests/rasterizer_python/test_cases.py:23-28 of the
                reference), tanfovx 0.6, tanfovy 0.6*H/W, projection from
                gs_lightning/utils/camera.py:4-41 with znear 0.01, zfar 100
    upstream  = dL/dimage = randn(3,H,W), dL/dinvdepth = randn(1,H,W) (seed+1)
    views     = V_k = Ry(2*pi*k/n) @ V0 (orbit about world y)

Everything is generated on the CPU with torch.Generator so CPU tests and the GPU box draw
identical tensors.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np
import torch

# tests/rasterizer_python/test_cases.py:23-28 ("treehill No.0" viewmatrix, row-vector form)
TREEHILL_V0 = [
    [-0.1372, 0.1419, 0.9803, 0.0000],
    [0.3828, 0.9204, -0.0796, 0.0000],
    [-0.9136, 0.3644, -0.1805, 0.0000],
    [0.1878, -0.6085, 4.0976, 1.0000],
]


def get_projection_matrix(fx: float, fy: float, w: int, h: int, znear: float, zfar: float) -> np.ndarray:
    """Column-vector perspective matrix, z -> [0, 1] (restates gs_lightning/utils/camera.py:4-41)."""
    right = (w * 0.5) * (znear / fx)
    top = (h * 0.5) * (znear / fy)
    m = np.zeros((4, 4))
    m[0, 0] = (2 * znear) / (2 * right)
    m[1, 1] = (2 * znear) / (2 * top)
    m[3, 2] = 1.0
    m[2, 2] = (zfar + znear) / (zfar - znear)
    m[2, 3] = -(zfar * znear) / (zfar - znear)
    return m


def rot_y(theta: float) -> torch.Tensor:
    c, s = math.cos(theta), math.sin(theta)
    return torch.tensor([[c, 0.0, -s, 0.0], [0.0, 1.0, 0.0, 0.0], [s, 0.0, c, 0.0], [0.0, 0.0, 0.0, 1.0]],
                        dtype=torch.float32)


@dataclass
class Camera:
    image_height: int
    image_width: int
    tanfovx: float
    tanfovy: float
    viewmatrix: torch.Tensor  # (4,4) row-vector convention
    projmatrix: torch.Tensor  # (4,4) = viewmatrix @ P^T
    campos: torch.Tensor      # (3,)

    def to(self, device) -> "Camera":
        return Camera(self.image_height, self.image_width, self.tanfovx, self.tanfovy,
                      self.viewmatrix.to(device), self.projmatrix.to(device), self.campos.to(device))


def make_camera(width: int, height: int, view_index: int = 0, num_views: int = 1,
                tanfovx: float = 0.6, viewmatrix=None) -> Camera:
    tanfovy = tanfovx * height / width
    v0 = torch.tensor(TREEHILL_V0 if viewmatrix is None else viewmatrix, dtype=torch.float32)
    if num_views > 1 or view_index:
        v0 = rot_y(2.0 * math.pi * view_index / max(num_views, 1)) @ v0
    fx = width / (2.0 * tanfovx)
    fy = height / (2.0 * tanfovy)
    proj = torch.tensor(get_projection_matrix(fx, fy, width, height, 0.01, 100.0).T, dtype=torch.float32)
    full = v0 @ proj
    campos = torch.linalg.inv(v0)[3, :3].contiguous()
    return Camera(height, width, tanfovx, tanfovy, v0.contiguous(), full.contiguous(), campos)


@dataclass
class Scene:
    means3D: torch.Tensor
    scales: torch.Tensor
    rotations: torch.Tensor
    opacities: torch.Tensor
    shs: torch.Tensor
    sh_degree: int

    def to(self, device) -> "Scene":
        return Scene(self.means3D.to(device), self.scales.to(device), self.rotations.to(device),
                     self.opacities.to(device), self.shs.to(device), self.sh_degree)

    @property
    def num_gaussians(self) -> int:
        return int(self.means3D.shape[0])


def make_scene(n: int, sh_degree: int = 3, seed: int = 0, opacity_scale: float = 1.0,
               stress_fraction: float = 0.0) -> Scene:
    g = torch.Generator().manual_seed(seed)
    means = torch.randn(n, 3, generator=g)
    scales = torch.exp(torch.randn(n, 3, generator=g) * 0.5 - 4.0 - math.log(n / 1e5) / 3.0)
    rots = torch.nn.functional.normalize(torch.randn(n, 4, generator=g), dim=-1)
    opac = torch.sigmoid(torch.randn(n, 1, generator=g)) * opacity_scale
    shs = torch.randn(n, (sh_degree + 1) ** 2, 3, generator=g) * 0.3
    if stress_fraction > 0:
        k = int(n * stress_fraction)
        scales[:k] *= 10.0  # "densification-era" bloated Gaussians (BASELINE.json config 5)
    return Scene(means.contiguous(), scales.contiguous(), rots.contiguous(), opac.contiguous(),
                 shs.contiguous(), sh_degree)


def make_upstream(width: int, height: int, seed: int = 0):
    g = torch.Generator().manual_seed(seed + 1)
    return torch.randn(3, height, width, generator=g), torch.randn(1, height, width, generator=g)
