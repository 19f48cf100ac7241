"""Densification (prune / clone / split) on the HIP kernels of csrc/gsr_densify.hip.

Mirrors the reference's adaptive density control:

* `update_max_radii2D` / `update_xyz_gradient` -- gs_lightning/modules/gaussian_model.py:175-181;
* `densify_and_prune`  -- gaussian_model.py:184-287 (prune by opacity / screen size / world size, then clone
  small and split large Gaussians whose mean screen-space gradient reaches the threshold);
* with `optimizer=` also `update_optimizer_parameters` of gs_lightning/lightning/gs_lightning_module.py:213-235
  (Adam moments re-indexed with the kept rows, zero rows appended for the new Gaussians).

`gaussians` is any object with the reference GaussianModel's attributes: `_xyz (N,3)`, `_features_dc (N,1,3)`,
`_features_rest (N,K,3)`, `_opacity (N,1)`, `_scaling (N,3)`, `_rotation (N,4)`, `xyz_grad_accum (N)`,
`xyz_grad_count (N)`, `max_radii2D (N)`, `spatial_scale` and `use_screensize_threshold`.  All parameters and
moments move in one scatter launch; the only host sync is the read-back of the three row counts, which sizes
the outputs.  The split displacement is drawn as `normal_(0, 1)` of shape (n_split, 3) on the parameters'
device -- the same draw `torch.normal(mean, std)` makes -- so with the same generator state the result matches
the reference row for row.  No CPU fallback: the HIP library must load.
"""
from __future__ import annotations

from typing import Optional

import torch
from torch import nn

from . import _native
from .rasterizer import _stream_handle

__all__ = ["PARAMETER_NAMES", "update_max_radii2D", "update_xyz_gradient", "densify_and_prune"]

PARAMETER_NAMES = ("xyz", "features_dc", "features_rest", "opacity", "scaling", "rotation")
_KINDS = dict(xyz=_native.FIELD_XYZ, scaling=_native.FIELD_SCALING)
_STATS = ("max_radii2D", "xyz_grad_accum", "xyz_grad_count")


@torch.no_grad()
def update_max_radii2D(gaussians, radii: torch.Tensor, visible_mask: torch.Tensor) -> None:
    """gaussian_model.py:175-176."""
    gaussians.max_radii2D[visible_mask] = torch.max(gaussians.max_radii2D[visible_mask],
                                                    radii[visible_mask].to(gaussians.max_radii2D.dtype))


@torch.no_grad()
def update_xyz_gradient(gaussians, screenspace_gradient: torch.Tensor, visible_mask: torch.Tensor) -> None:
    """gaussian_model.py:178-181."""
    gaussians.xyz_grad_accum[visible_mask] += torch.norm(screenspace_gradient[visible_mask, :2], dim=1)
    gaussians.xyz_grad_count[visible_mask] += 1


def _f32(t: torch.Tensor) -> torch.Tensor:
    t = t.detach()
    if t.dtype != torch.float32:
        t = t.float()
    return t.contiguous()


def _group_for(optimizer, name: str, param):
    for group in optimizer.param_groups:
        if group.get("name", None) == name:
            if len(group["params"]) != 1:
                raise RuntimeError(f"param group {name!r} must hold exactly one tensor")
            return group
    return None


@torch.no_grad()
def densify_and_prune(gaussians, densify_grad_threshold: float, clone_size_threshold: float,
                      prune_opacity_threshold: float, prune_size_threshold: float,
                      prune_screensize_threshold: Optional[float] = None, optimizer=None,
                      generator: Optional[torch.Generator] = None) -> torch.Tensor:
    """Prune, clone and split in place on `gaussians`; returns preserve_idx (the kept row indices), as
    GaussianModel.densify_and_prune does.  With `optimizer` (torch.optim.Adam or GaussianAdam holding the
    reference's named groups) the Adam state is re-indexed in the same launch -- do not call the reference's
    update_optimizer_parameters afterwards then."""
    lib = _native.load()
    params = {k: getattr(gaussians, f"_{k}") for k in PARAMETER_NAMES}
    xyz = params["xyz"]
    dev = xyz.device
    if dev.type != "cuda":
        raise RuntimeError("densify_and_prune: the Gaussians must live on the GPU")
    N = int(xyz.shape[0])
    for k, t in params.items():
        if t.shape[0] != N or t.dtype != torch.float32 or not t.is_contiguous():
            raise RuntimeError(f"densify_and_prune: _{k} must be a contiguous fp32 (N, ...) tensor")
    scale = float(gaussians.spatial_scale)
    stats = {k: _f32(getattr(gaussians, k)) for k in _STATS}
    stream = _stream_handle(dev)

    apply_size = prune_screensize_threshold is not None
    args = _native.DensifyArgs(
        N, params["opacity"].data_ptr(), params["scaling"].data_ptr(), stats["max_radii2D"].data_ptr(),
        stats["xyz_grad_accum"].data_ptr(), stats["xyz_grad_count"].data_ptr(),
        float(prune_opacity_threshold), float(prune_screensize_threshold if apply_size else 0.0),
        float(prune_size_threshold) * scale, float(densify_grad_threshold), float(clone_size_threshold) * scale,
        int(apply_size and bool(getattr(gaussians, "use_screensize_threshold", True))), int(apply_size))
    ws = torch.empty(max(1, lib.gsr_densify_workspace_bytes(N)), dtype=torch.uint8, device=dev)
    counts = torch.empty(3, dtype=torch.int32, device=dev)
    preserve = torch.empty(max(N, 1), dtype=torch.int64, device=dev)
    _native.check(lib.gsr_densify_classify(args, ws.data_ptr(), counts.data_ptr(), preserve.data_ptr(), stream),
                  "gsr_densify_classify")
    n_keep, n_clone, n_split = (int(c) for c in counts.tolist())
    n_new = n_keep + n_clone + n_split
    z = torch.empty((n_split, 3), dtype=torch.float32, device=dev)
    if n_split:
        z.normal_(0.0, 1.0, generator=generator)

    fields, new_params, new_states, moved = [], {}, {}, {}
    for k in PARAMETER_NAMES:
        src = params[k]
        dst = torch.empty((n_new,) + tuple(src.shape[1:]), dtype=torch.float32, device=dev)
        new_params[k] = dst
        width = src[0].numel() if N else 0
        m_src = v_src = m_dst = v_dst = None
        if optimizer is not None:
            group = _group_for(optimizer, k, src)
            st = optimizer.state.get(group["params"][0], None) if group is not None else None
            if st is not None and "exp_avg" in st:
                m_src, v_src = st["exp_avg"].contiguous(), st["exp_avg_sq"].contiguous()
                m_dst, v_dst = torch.empty_like(dst), torch.empty_like(dst)
                new_states[k] = (group, st, m_dst, v_dst)
                moved[k] = (m_src, v_src)
            elif group is not None:
                new_states[k] = (group, None, None, None)
        if width:
            ptr = lambda t: t.data_ptr() if t is not None else None  # noqa: E731
            fields.append(_native.DensifyField(src.data_ptr(), dst.data_ptr(), ptr(m_src), ptr(v_src), ptr(m_dst),
                                               ptr(v_dst), width, _KINDS.get(k, _native.FIELD_PLAIN)))
    new_stats = {}
    for k in _STATS:
        dst = torch.empty(n_new, dtype=torch.float32, device=dev)
        new_stats[k] = dst
        fields.append(_native.DensifyField(stats[k].data_ptr(), dst.data_ptr(), None, None, None, None, 1,
                                           _native.FIELD_STAT))
    arr = (_native.DensifyField * len(fields))(*fields)
    if n_new:
        _native.check(lib.gsr_densify_apply(N, ws.data_ptr(), params["rotation"].data_ptr(),
                                            params["scaling"].data_ptr(), z.data_ptr(), arr, len(fields), stream),
                      "gsr_densify_apply")

    # rebind exactly as the reference does (nn.Parameter per attribute; optimizer state moved to the new key)
    for k in PARAMETER_NAMES:
        setattr(gaussians, f"_{k}", nn.Parameter(new_params[k]))
    for k in _STATS:
        old = getattr(gaussians, k)
        setattr(gaussians, k, new_stats[k].to(old.dtype))
    for k, (group, st, m_dst, v_dst) in new_states.items():
        old_p = group["params"][0]
        new_p = getattr(gaussians, f"_{k}")
        if st is not None:
            st["exp_avg"], st["exp_avg_sq"] = m_dst, v_dst
            del optimizer.state[old_p]
            group["params"][0] = new_p
            optimizer.state[new_p] = st
        else:
            group["params"][0] = new_p
    return preserve[:n_keep]
