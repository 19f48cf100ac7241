#!/usr/bin/env python
"""Generate tests/golden/knn_golden.npz and tests/golden/densify_golden.npz from the REFERENCE Python code.

Runs only in the build container, where /root/reference exists (the GPU box never reads /root/reference).
Imports, with the harness shims of make_golden.py (bare `gs_lightning` package, `kornia` Quaternion stand-in)
plus empty `plyfile` / `pycolmap` modules (imported at module top by gaussian_model.py / utils/colmap.py, never
called on these paths):

* gs_lightning.utils.math.distCUDA2 (math.py:9-14, scipy KDTree) on five point sets -> knn_golden.npz;
* gs_lightning.modules.gaussian_model.GaussianModel.densify_and_prune (gaussian_model.py:184-287) on CPU
  tensors after torch.manual_seed(SEED), for two threshold sets -> densify_golden.npz.  The consumer
  replays the split draw as torch.manual_seed(SEED); torch.empty(n_split, 3).normal_().

Usage:  python -B tests/golden/make_golden_train.py
"""
from __future__ import annotations

import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.dont_write_bytecode = True

SEED = 123
DENSIFY_CASES = {
    # name: (grad, clone_size, prune_opacity, prune_size, prune_screensize)
    "screensize": (0.0002, 0.01, 0.05, 0.4, 20.0),
    "no_screensize": (0.0002, 0.01, 0.05, 0.4, None),
}


def _import_reference():
    import make_golden
    make_golden._install_shims()
    for name in ("plyfile", "pycolmap"):
        m = types.ModuleType(name)
        m.PlyData = m.PlyElement = None
        sys.modules.setdefault(name, m)
    from gs_lightning.utils import math as M  # noqa: E402
    from gs_lightning.modules import gaussian_model as G  # noqa: E402
    return M, G


def knn_sets():
    rng = np.random.default_rng(0)
    f32 = np.float32
    blobs = np.concatenate([rng.normal(c, s, size=(600, 3)) for c, s in
                            [((0, 0, 0), 0.05), ((3, 1, 0), 0.5), ((-2, 4, 1), 0.01)]] +
                           [rng.uniform(-50, 50, size=(200, 3))]).astype(f32)
    dup = rng.normal(size=(400, 3)).astype(f32)
    dup = np.concatenate([dup, dup[:100], dup[:7]]).astype(f32)
    lattice = np.stack(np.meshgrid(*[np.arange(8, dtype=f32) * 0.25] * 3, indexing="ij"), -1).reshape(-1, 3)
    return dict(blobs=blobs, duplicates=dup, lattice=lattice, n3=rng.normal(size=(3, 3)).astype(f32),
                n4=rng.normal(size=(4, 3)).astype(f32))


def densify_scene(N=1500, seed=7):
    rng = np.random.default_rng(seed)
    f32 = np.float32
    count = rng.integers(0, 6, N).astype(f32)
    return dict(xyz=rng.normal(size=(N, 3)).astype(f32), features_dc=rng.normal(size=(N, 1, 3)).astype(f32),
                features_rest=rng.normal(size=(N, 15, 3)).astype(f32), opacity=rng.uniform(-4, 4, (N, 1)).astype(f32),
                scaling=rng.uniform(np.log(0.001), np.log(0.5), (N, 3)).astype(f32),
                rotation=rng.normal(size=(N, 4)).astype(f32), max_radii2D=rng.uniform(0, 40, N).astype(f32),
                xyz_grad_accum=(count * rng.uniform(0, 0.0004, N)).astype(f32), xyz_grad_count=count)


def main():
    M, G = _import_reference()
    out = {}
    for name, pts in knn_sets().items():
        out[f"{name}_points"] = pts
        out[f"{name}_dist2"] = M.distCUDA2(torch.tensor(pts)).numpy()
    np.savez_compressed(os.path.join(HERE, "knn_golden.npz"), **out)

    scene = densify_scene()
    out = {f"in_{k}": v for k, v in scene.items()}
    out["spatial_scale"] = np.float32(1.3)
    out["seed"] = np.int64(SEED)
    for case, thr in DENSIFY_CASES.items():
        g = G.GaussianModel(sh_degree=3)
        for k in ("xyz", "features_dc", "features_rest", "opacity", "scaling", "rotation"):
            setattr(g, f"_{k}", torch.nn.Parameter(torch.tensor(scene[k])))
        for k in ("max_radii2D", "xyz_grad_accum", "xyz_grad_count"):
            setattr(g, k, torch.tensor(scene[k]))
        g.spatial_scale = 1.3
        torch.manual_seed(SEED)
        keep = g.densify_and_prune(densify_grad_threshold=thr[0], clone_size_threshold=thr[1],
                                   prune_opacity_threshold=thr[2], prune_size_threshold=thr[3],
                                   prune_screensize_threshold=thr[4])
        out[f"{case}_preserve_idx"] = keep.numpy()
        for k in ("xyz", "features_dc", "features_rest", "opacity", "scaling", "rotation"):
            out[f"{case}_{k}"] = getattr(g, f"_{k}").detach().numpy()
        for k in ("max_radii2D", "xyz_grad_accum", "xyz_grad_count"):
            out[f"{case}_{k}"] = getattr(g, k).numpy()
    np.savez_compressed(os.path.join(HERE, "densify_golden.npz"), **out)
    print("wrote knn_golden.npz, densify_golden.npz")


if __name__ == "__main__":
    main()
