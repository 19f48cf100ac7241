"""TEST INFRASTRUCTURE ONLY -- numpy restatement of the reference's adaptive density control.

Only tests/ may import this module; the product path (gaussian_splatting_lightning_amd.densify) runs the HIP
kernels of csrc/gsr_densify.hip and never calls into oracle/.

Follows, line by line in numpy fp32:
  gs_lightning/modules/gaussian_model.py:184-210  densify_and_prune
  gs_lightning/modules/gaussian_model.py:212-237  _prune_gaussian (returns preserve_idx)
  gs_lightning/modules/gaussian_model.py:239-249  _clone_gaussian
  gs_lightning/modules/gaussian_model.py:251-265  _split_gaussian (R = kornia Quaternion(q).matrix(), w-first)
  gs_lightning/modules/gaussian_model.py:267-287  _add_gaussian (zero statistics for appended rows)
  gs_lightning/lightning/gs_lightning_module.py:213-235  update_optimizer_parameters (moments re-indexed with
                                                          preserve_idx, zero rows appended)
The split displacement takes `z` ~ N(0,1) of shape (n_split, 3) as an input (an array, or a callable n -> array
of shape (n, 3)): torch.normal(mean, std) draws exactly normal_(0,1) and multiplies by std (ATen
Distributions), so the caller supplies the same draw.

Parity pinning: tests/golden/densify_golden.npz holds the outputs of the reference's own
GaussianModel.densify_and_prune run on CPU tensors (tests/golden/make_golden_train.py; kornia, plyfile and
pycolmap are absent, so that script stands in a Quaternion.matrix() and empty plyfile/pycolmap modules, none of
which the densify path calls except the quaternion matrix of the split).  tests/test_densify.py checks this
restatement against that fixture and against an independent torch restatement for five threshold sets.
"""
from __future__ import annotations

from typing import Dict, Optional, Tuple

import numpy as np

PARAMETER_NAMES = ("xyz", "features_dc", "features_rest", "opacity", "scaling", "rotation")


def quaternion_matrix(q: np.ndarray) -> np.ndarray:
    """kornia quaternion_to_rotation_matrix for (w, x, y, z) rows of unit quaternions -> (n, 3, 3)."""
    w, x, y, z = (q[:, i] for i in range(4))
    tx, ty, tz = 2 * x, 2 * y, 2 * z
    twx, twy, twz = tx * w, ty * w, tz * w
    txx, txy, txz = tx * x, ty * x, tz * x
    tyy, tyz, tzz = ty * y, tz * y, tz * z
    one = np.ones_like(w)
    return np.stack([one - (tyy + tzz), txy - twz, txz + twy,
                     txy + twz, one - (txx + tzz), tyz - twx,
                     txz - twy, tyz + twx, one - (txx + tyy)], -1).reshape(-1, 3, 3)


def densify_and_prune(params: Dict[str, np.ndarray], stats: Dict[str, np.ndarray], spatial_scale: float,
                      densify_grad_threshold: float, clone_size_threshold: float, prune_opacity_threshold: float,
                      prune_size_threshold: float, prune_screensize_threshold: Optional[float],
                      use_screensize_threshold: bool, z: Optional[np.ndarray] = None,
                      moments: Optional[Dict[str, Tuple[np.ndarray, np.ndarray]]] = None):
    """Returns (new_params, new_stats, new_moments, preserve_idx, (n_keep, n_clone, n_split))."""
    f32 = np.float32
    P = {k: np.asarray(v, dtype=f32).copy() for k, v in params.items()}
    S = {k: np.asarray(v, dtype=f32).copy() for k, v in stats.items()}
    N = P["xyz"].shape[0]
    with np.errstate(over="ignore", divide="ignore", invalid="ignore"):
        # _prune_gaussian
        opacity = (f32(1) / (f32(1) + np.exp(-P["opacity"]))).reshape(N)
        preserve = opacity > f32(prune_opacity_threshold)
        if prune_screensize_threshold is not None:
            if use_screensize_threshold:
                preserve &= S["max_radii2D"] < f32(prune_screensize_threshold)
            size = np.exp(P["scaling"]).max(axis=1)
            preserve &= size < f32(prune_size_threshold) * f32(spatial_scale)
        preserve_idx = np.nonzero(preserve)[0]
        P = {k: v[preserve] for k, v in P.items()}
        S = {k: v[preserve] for k, v in S.items()}
        # densify_and_prune
        grad = S["xyz_grad_accum"] / S["xyz_grad_count"]
        grad[np.isnan(grad)] = 0.0
        bad = grad >= f32(densify_grad_threshold)
        size = np.exp(P["scaling"]).max(axis=1)
        thr = f32(clone_size_threshold) * f32(spatial_scale)
        small_idx = np.nonzero(bad & (size < thr))[0]
        large_idx = np.nonzero(bad & (size >= thr))[0]
        n_keep = len(preserve_idx)

        def add(rows: Dict[str, np.ndarray]):
            n = len(rows["xyz"])
            for k in PARAMETER_NAMES:
                P[k] = np.concatenate([P[k], rows[k]], 0)
            for k in S:
                S[k] = np.concatenate([S[k], np.zeros(n, f32)], 0)

        # _clone_gaussian(small)
        add({k: P[k][small_idx].copy() for k in PARAMETER_NAMES})
        # _split_gaussian(large)
        if len(large_idx):
            if callable(z):
                z = z(len(large_idx))
            if z is None or np.shape(z) != (len(large_idx), 3):
                raise ValueError(f"z must have shape ({len(large_idx)}, 3)")
            std = np.exp(P["scaling"][large_idx])
            displace = np.asarray(z, f32) * std
            q = P["rotation"][large_idx]
            q = q / np.maximum(np.sqrt((q * q).sum(1, keepdims=True)), f32(1e-12))
            R = quaternion_matrix(q.astype(f32))
            P["xyz"][large_idx] = P["xyz"][large_idx] + np.einsum("nij,nj->ni", R, displace).astype(f32)
            P["scaling"][large_idx] = np.log(np.exp(P["scaling"][large_idx]) / f32(1.6))
        add({k: P[k][large_idx].copy() for k in PARAMETER_NAMES})

    new_moments = None
    if moments is not None:
        new_moments = {}
        n_new = len(P["xyz"])
        for k, (m, v) in moments.items():
            m, v = np.asarray(m, f32), np.asarray(v, f32)
            pad = np.zeros((n_new - n_keep,) + m.shape[1:], f32)
            new_moments[k] = (np.concatenate([m[preserve_idx], pad], 0), np.concatenate([v[preserve_idx], pad], 0))
    return P, S, new_moments, preserve_idx, (n_keep, len(small_idx), len(large_idx))
