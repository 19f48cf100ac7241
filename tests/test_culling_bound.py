"""The exact tile culling rule (DESIGN.md §2 "Binning", restated in oracle/gsr_oracle.c tile_contrib) is
conservative: no (Gaussian, tile) instance it drops has a pixel centre whose alpha, evaluated in fp32 with the
reference's power expression (cuda_rasterizer/forward.cu renderCUDA of the reference), reaches 1/255.  Checked
on the oracle over scenes whose pixel coordinates reach 4K and whose conics are stretched, where the fp32
per-tile minimum and the rounding of its edge minimisers are furthest from the exact values."""
import numpy as np
import pytest

from oracle import oracle as O
from tests.helpers import run_oracle, scene_inputs


def dropped_pairs(g, radii, W, H):
    """(gid, tile) of every instance of the reference rect that culling removes."""
    args = (g["xy"], radii, g["depths"], g["conic_opacity"], W, H)
    sets = []
    for cull in (False, True):
        pl, rg, _ = O.bin_instances(*args, cull=cull)
        tile = np.repeat(np.arange(rg.shape[0], dtype=np.int64), (rg[:, 1] - rg[:, 0]).astype(np.int64))
        sets.append(set(zip(pl.astype(np.int64).tolist(), tile.tolist())))
    full, kept = sets
    assert kept <= full
    return np.array(sorted(full - kept), np.int64).reshape(-1, 2), len(full), len(kept)


def max_alpha(g, pairs, W, H):
    """Largest fp32 o * exp(power) over the pixel centres of each dropped instance's tile."""
    tx_n = (W + 15) // 16
    xy, co = g["xy"][pairs[:, 0]], g["conic_opacity"][pairs[:, 0]]
    ox = (pairs[:, 1] % tx_n) * 16
    oy = (pairs[:, 1] // tx_n) * 16
    off = np.arange(16, dtype=np.float32)
    best = np.zeros(len(pairs), np.float32)
    for j in range(16):
        px = (ox[:, None] + off[None, :]).astype(np.float32)
        py = np.full_like(px, 0, np.float32) + (oy + j).astype(np.float32)[:, None]
        dx = xy[:, 0:1] - px
        dy = xy[:, 1:2] - py
        a, b, c, o = (co[:, k:k + 1] for k in range(4))
        power = np.float32(-0.5) * (a * dx * dx + c * dy * dy) - b * dx * dy
        alpha = np.where(power > 0, np.float32(0), np.minimum(np.float32(0.99), o * np.exp(power)))
        alpha[(px > W - 1) | (py > H - 1)] = 0  # pixel centres past the image edge are never rendered
        best = np.maximum(best, alpha.max(1))
    return best


@pytest.mark.parametrize("n,W,H,seed,stress", [(5_000, 3840, 2160, 3, 0.002), (12_000, 1920, 1080, 7, 0.0)])
def test_culling_drops_only_invisible_instances(n, W, H, seed, stress):
    inp = scene_inputs(n, W, H, sh_degree=0, seed=seed, stress_fraction=stress)
    _, radii, _, run = run_oracle(inp)
    g = run.geom()
    pairs, n_full, n_kept = dropped_pairs(g, radii, W, H)
    assert n_kept < 0.8 * n_full  # the rule still removes most of the rect's empty instances
    assert len(pairs) > 10_000
    best = max_alpha(g, pairs, W, H)
    print("dropped", len(pairs), "of", n_full, "max alpha x 255 =", float(best.max()) * 255)
    assert best.max() < 1.0 / 255.0, (best.max(), pairs[int(best.argmax())])


def test_pair_loop_division_by_multiply():
    """preprocess_kernel's culling loop divides a pair's offset t < 64 by the rect width rw <= 64 as
    (t * ceil(4096 / rw)) >> 12 (gsr_forward.hip): exact over the whole domain."""
    for rw in range(1, 65):
        magic = (4096 + rw - 1) // rw
        assert magic < 1 << 16  # packed beside rw in one 32-bit LDS word
        for t in range(64):
            assert (t * magic) >> 12 == t // rw, (t, rw)
