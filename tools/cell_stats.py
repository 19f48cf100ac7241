#!/usr/bin/env python
"""Skip-granularity statistics of the composite passes (CPU, from the oracle's forward state).

A wave composites a 16x16 tile with 4 pixels per lane; per instance it can skip one of its 4 pixel slots
wave-uniformly, so a skip unit ("cell") is 64 pixels.  This counts, over the (tile, instance) pairs the
backward walks (instances before the tile's last contributor), how many cells each cell shape leaves live:

  strip_band   4-row strips (16x4) against the row band of the alpha >= 1/255 ellipse (render_bwd today)
  quad_box     8x8 quadrants against the ellipse's bounding box
  quad_exact   8x8 quadrants holding at least one pixel with alpha >= 1/255
  strip_exact  4-row strips holding at least one such pixel
  quad_active  8x8 quadrants holding at least one pixel where the pair contributes (alpha test and the
               pixel's last contributor), the floor for any per-cell skip

    python tools/cell_stats.py --config cfg2 [--tiles 400]
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def strip_mask_exact(x, y, A, B, C, o, row0, col0):
    """numpy fp32 restatement of gsr_common.h strip_mask_exact (vectorised over instances): (n,) -> (n, 4) bool."""
    f = np.float32
    x, y, A, B, C, o = (np.asarray(v, f) for v in (x, y, A, B, C, o))
    with np.errstate(all="ignore"):
        o255 = f(255) * o
        det = A * C - B * B
        hd = f(0.5) * (A - C)
        lmin = f(0.5) * (A + C) - np.sqrt(hd * hd + B * B)
        eps = f(1e-5) * (np.abs(A) + np.abs(B) + np.abs(C)) / lmin
        tau = (f(2) * np.log(np.maximum(o255 * f(1.00001), f(1))) + f(1e-3)) / (f(1) - eps)
        V = np.sqrt(tau * A / det)
        uL = f(col0) - x
        uR = uL + f(15)
        ut = -B * V / A
        ic, ctau = f(1) / C, C * tau
        u = np.minimum(np.maximum(ut, uL), uR)
        vmax = np.where((ut >= uL) & (ut <= uR), V, (-B * u + np.sqrt(np.maximum(ctau - det * u * u, 0))) * ic)
        u = np.minimum(np.maximum(-ut, uL), uR)
        vmin = np.where((-ut >= uL) & (-ut <= uR), -V, (-B * u - np.sqrt(np.maximum(ctau - det * u * u, 0))) * ic)
        mg = f(1e-2) * V + f(1e-3) * (np.abs(uL) + np.abs(uR)) + f(0.0625)
        lo, hi = y + vmin - mg - f(row0), y + vmax + mg - f(row0)
        m = np.stack([(hi >= 4 * k) & (lo <= 4 * k + 3) for k in range(4)], 1)
        keep_all = ~((det > 0) & (lmin > 0) & (eps < 1e-2) & (V < 1e6)) | np.isnan(o255)
    m[keep_all] = True
    m[o255 < 0.999] = False
    return m


def quad_mask_exact(x, y, A, B, C, o, row0, col0):
    """strip_mask_exact's bound per 8-column half of the tile, tested against the two 8-row bands: (n,) -> (n, 4)
    bool, bit 2 qy + qx for the quadrant (qx, qy)."""
    out = []
    for qy in range(2):
        for qx in range(2):
            m = strip_mask_exact_band(x, y, A, B, C, o, row0, col0 + 8 * qx, 7)
            lo, hi = m
            out.append((hi >= 8 * qy) & (lo <= 8 * qy + 7))
    m = np.stack(out, 1)
    f = np.float32
    with np.errstate(all="ignore"):
        o255 = f(255) * np.asarray(o, f)
        A, B, C = (np.asarray(v, f) for v in (A, B, C))
        det = A * C - B * B
        hd = f(0.5) * (A - C)
        lmin = f(0.5) * (A + C) - np.sqrt(hd * hd + B * B)
        eps = f(1e-5) * (np.abs(A) + np.abs(B) + np.abs(C)) / lmin
        V = np.sqrt(((f(2) * np.log(np.maximum(o255 * f(1.00001), f(1))) + f(1e-3)) / (f(1) - eps)) * A / det)
        keep_all = ~((det > 0) & (lmin > 0) & (eps < 1e-2) & (V < 1e6)) | np.isnan(o255)
    m[keep_all] = True
    m[o255 < 0.999] = False
    return m


def strip_mask_exact_band(x, y, A, B, C, o, row0, col0, width):
    """The (lo, hi) row interval (tile-relative) of strip_mask_exact over the columns [col0, col0 + width]."""
    f = np.float32
    x, y, A, B, C, o = (np.asarray(v, f) for v in (x, y, A, B, C, o))
    with np.errstate(all="ignore"):
        o255 = f(255) * o
        det = A * C - B * B
        hd = f(0.5) * (A - C)
        lmin = f(0.5) * (A + C) - np.sqrt(hd * hd + B * B)
        eps = f(1e-5) * (np.abs(A) + np.abs(B) + np.abs(C)) / lmin
        tau = (f(2) * np.log(np.maximum(o255 * f(1.00001), f(1))) + f(1e-3)) / (f(1) - eps)
        V = np.sqrt(tau * A / det)
        uL = f(col0) - x
        uR = uL + f(width)
        ut = -B * V / A
        ic, ctau = f(1) / C, C * tau
        u = np.minimum(np.maximum(ut, uL), uR)
        vmax = np.where((ut >= uL) & (ut <= uR), V, (-B * u + np.sqrt(np.maximum(ctau - det * u * u, 0))) * ic)
        u = np.minimum(np.maximum(-ut, uL), uR)
        vmin = np.where((-ut >= uL) & (-ut <= uR), -V, (-B * u - np.sqrt(np.maximum(ctau - det * u * u, 0))) * ic)
        mg = f(1e-2) * V + f(1e-3) * (np.abs(uL) + np.abs(uR)) + f(0.0625)
        return y + vmin - mg - f(row0), y + vmax + mg - f(row0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--tiles", type=int, default=0, help="random sample of tiles (0: all)")
    args = ap.parse_args()
    from bench import CONFIGS
    from gaussian_splatting_lightning_amd.synthetic import make_camera, make_scene
    from oracle import oracle as O

    cfg = CONFIGS[args.config]
    W, H, deg = cfg["W"], cfg["H"], cfg["deg"]
    sc = make_scene(cfg["n"], deg, seed=0, stress_fraction=cfg["stress"])
    cam = make_camera(W, H)
    _, radii, _, run = O.forward(sc.means3D.numpy(), sc.opacities.numpy(), sc.scales.numpy(), sc.rotations.numpy(),
                                 sc.shs.numpy(), cam.viewmatrix.numpy(), cam.projmatrix.numpy(), cam.campos.numpy(),
                                 np.zeros(3, np.float32), cam.tanfovx, cam.tanfovy, H, W, deg)
    g = run.geom()
    pl, rg = run.point_list(), run.ranges()
    _, nc = run.image_state()
    xy, co = g["xy"], g["conic_opacity"]
    gx, gy = (W + 15) // 16, (H + 15) // 16
    T = gx * gy
    tiles = np.arange(T)
    if args.tiles:
        tiles = np.random.default_rng(0).choice(T, size=min(args.tiles, T), replace=False)
    ly, lx = np.mgrid[0:16, 0:16]
    ly, lx = ly.reshape(-1), lx.reshape(-1)
    strip_of = ly // 4
    quad_of = (ly // 8) * 2 + (lx // 8)
    tot = dict(quad_fn=0, quad_fn_miss=0, strip_fn=0, strip_fn_miss=0, pairs=0, strip_band=0, quad_box=0, quad_exact=0, strip_exact=0, quad_active=0, strip_active=0,
               active_pairs=0, fwd_pairs_tile=0, strip_fn_lastc=0, need_cmp=0, inst_dead=0)
    for t in tiles:
        tx, ty = t % gx, t // gx
        px, py = tx * 16 + lx, ty * 16 + ly
        inside = (px < W) & (py < H)
        ncp = np.where(inside, nc[np.minimum(py, H - 1), np.minimum(px, W - 1)], 0)
        last = int(ncp.max())
        if last == 0:
            continue
        ids = pl[rg[t, 0]: rg[t, 0] + last]
        m = xy[ids]
        c = co[ids]
        dx = m[:, :1] - px[None, :].astype(np.float32)
        dy = m[:, 1:2] - py[None, :].astype(np.float32)
        power = -0.5 * (c[:, :1] * dx * dx + c[:, 2:3] * dy * dy) - c[:, 1:2] * dx * dy
        alpha = np.minimum(0.99, c[:, 3:4] * np.exp(power))
        ok = (power <= 0) & (alpha >= 1 / 255.0) & inside[None, :]
        act = ok & (np.arange(last)[:, None] < ncp[None, :])
        n = len(ids)
        tot["pairs"] += n * 256
        tot["active_pairs"] += int(act.sum())
        # bounding extents of the alpha >= 1/255 ellipse (strip_mask's formula)
        a_, b_, c_, o_ = c[:, 0], c[:, 1], c[:, 2], c[:, 3]
        det = a_ * c_ - b_ * b_
        tau = 2 * np.log(np.maximum(255 * o_, 1.0)) + 1e-3
        ey = np.sqrt(np.maximum(tau * a_ / det, 0)) * 1.01 + 1
        ex = np.sqrt(np.maximum(tau * c_ / det, 0)) * 1.01 + 1
        r0y, r0x = ty * 16, tx * 16
        lo_y, hi_y = m[:, 1] - ey - r0y, m[:, 1] + ey - r0y
        lo_x, hi_x = m[:, 0] - ex - r0x, m[:, 0] + ex - r0x
        for k in range(4):
            tot["strip_band"] += int(((hi_y >= 4 * k) & (lo_y <= 4 * k + 3)).sum())
        for q in range(4):
            y0, x0 = 8 * (q // 2), 8 * (q % 2)
            tot["quad_box"] += int(((hi_y >= y0) & (lo_y <= y0 + 7) & (hi_x >= x0) & (lo_x <= x0 + 7)).sum())
            tot["quad_exact"] += int(ok[:, quad_of == q].any(1).sum())
            tot["quad_active"] += int(act[:, quad_of == q].any(1).sum())
        sm = strip_mask_exact(m[:, 0], m[:, 1], c[:, 0], c[:, 1], c[:, 2], c[:, 3], r0y, r0x)
        tot["strip_fn"] += int(sm.sum())
        qm = quad_mask_exact(m[:, 0], m[:, 1], c[:, 0], c[:, 1], c[:, 2], c[:, 3], r0y, r0x)
        tot["quad_fn"] += int(qm.sum())
        for q in range(4):
            qy, qx = q // 2, q % 2
            tot["quad_fn_miss"] += int((ok[:, quad_of == qy * 2 + qx] .any(1) & ~qm[:, q]).sum())
        tot["inst_dead"] += int((~act.any(1)).sum())
        idx = np.arange(last)
        for k in range(4):
            lc = ncp[strip_of == k]
            smax, smin = int(lc.max()), int(lc.min())
            live = sm[:, k] & (idx < smax)
            tot["strip_fn_lastc"] += int(live.sum())
            tot["need_cmp"] += int((live & (idx >= smin)).sum())
        for k in range(4):
            tot["strip_fn_miss"] += int((ok[:, strip_of == k].any(1) & ~sm[:, k]).sum())
        for k in range(4):
            tot["strip_exact"] += int(ok[:, strip_of == k].any(1).sum())
            tot["strip_active"] += int(act[:, strip_of == k].any(1).sum())
    cells = tot["pairs"] // 64
    print(f"{args.config}: tiles {len(tiles)}, walked (tile, instance) pairs {tot['pairs'] // 256}, "
          f"active pixel pairs {tot['active_pairs']} ({tot['active_pairs'] / tot['pairs']:.3f} of walked)")
    print(f"  strip_mask_exact: misses {tot['strip_fn_miss']} (must be 0); quad_mask_exact misses {tot['quad_fn_miss']}")
    print(f"  walked instances contributing to no pixel: {tot['inst_dead'] / (tot['pairs'] // 256):.3f}; "
          f"strip evaluations needing the n_contrib compare: {tot['need_cmp'] / max(tot['strip_fn_lastc'], 1):.3f}")
    for k in ("strip_band", "strip_fn", "strip_fn_lastc", "strip_exact", "strip_active", "quad_box", "quad_fn", "quad_exact",
              "quad_active"):
        print(f"  {k:12s} live cells {tot[k]:>12d}  {tot[k] / cells:.3f} of all, "
              f"active-pixel density {tot['active_pairs'] / max(tot[k] * 64, 1):.3f}")


if __name__ == "__main__":
    main()
