"""TEST INFRASTRUCTURE ONLY -- brute-force restatement of distCUDA2 (gs_lightning/utils/math.py:9-14).

The reference queries scipy's KDTree for the k=4 nearest points of every point (the point itself included),
drops the first column and averages the three remaining squared distances (float64), returning float32.
This restatement computes all pairwise squared distances in float64 (exact for the KDTree's answer up to the
final rounding) in blocks; only tests/ may import it.  Pinned against tests/golden/knn_golden.npz, which
make_golden_train.py produced by running the reference's distCUDA2.
"""
from __future__ import annotations

import numpy as np


def mean_dist2(points: np.ndarray, block: int = 1024) -> np.ndarray:
    p = np.asarray(points, dtype=np.float64)
    n = len(p)
    out = np.empty(n, dtype=np.float32)
    for s in range(0, n, block):
        q = p[s:s + block]
        d2 = ((q[:, None, :] - p[None, :, :]) ** 2).sum(-1)
        d2[np.arange(len(q)), np.arange(s, s + len(q))] = np.inf     # drop the point itself
        k = min(3, n - 1)
        best = np.sort(d2, axis=1)[:, :3] if n - 1 >= 3 else np.concatenate(
            [np.sort(d2, axis=1)[:, :k], np.full((len(q), 3 - k), np.inf)], 1)
        out[s:s + block] = best.mean(1)
    return out
