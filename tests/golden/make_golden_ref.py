#!/usr/bin/env python
"""Golden vectors for SATURATED SH-3 scenes from the REFERENCE Python rasterizer (BASELINE config 2 and a white-
background mini scene): tests/golden/ref_*.npz.

Runs only in the build container, where /root/reference exists; it imports `gs_lightning.rasterize` with the shims of
make_golden.py (no reference code is copied) and stores OUTPUTS only -- the inputs are regenerated on the GPU box from
the seeded generator (gaussian_splatting_lightning_amd/synthetic.py) where that is exact on any CPU, and the fixture
carries a SHA-256 of them, which the test asserts before comparing anything.

Saturated pixels differ between the reference's Python compositor and the CUDA semantics BY DESIGN (SURVEY.md
Appendix A2/A3: Python keeps adding Gaussians while the transmittance BEFORE them exceeds 1e-4 and weighs the
background with the product over all of them; CUDA stops before the Gaussian that takes T below 1e-4).  The two agree
exactly on every pixel that CUDA does not terminate, and such a pixel is recognised from the reference alone: the
reference's final transmittance T_ref (the difference of two renders with background 1 and 0) is the product over
all of the pixel's Gaussians, so T_ref >= 0.011 means CUDA never reached its stop (a stopped pixel keeps T < 1e-4 /
(1 - 0.99) = 0.01, and Python's product only falls further).  So:
  * `mask` = T_ref >= 0.011, less the oracle's threshold-flip candidates (a compositing decision within
    FLIP_EXCLUDE x its fp32 evaluation error of the threshold: the device's exp2, glibc's expf and torch's exp may
    decide those differently), stored as bits;
  * the upstream gradients (make_upstream's seeded randn) are zeroed outside the mask before the reference's
    backward, so its gradients sum only the pixels whose compositing the two semantics share;
  * colour, inverse depth and radii are stored for every pixel / Gaussian; the gradients of a seeded subset of
    Gaussians (REF_GRAD_SUBSET) keep the fixture small;
  * so are the inputs a CPU with other vector units could round differently (tests/helpers.py REF_STORED_INPUTS);
    the plain-randn ones are regenerated and checked against the stored SHA-256.
Float arrays are stored byte-plane shuffled (tests/helpers.py `shuffle_bytes`; `load_ref_golden` undoes it), which roughly
halves their compressed size.

Usage:  python -B tests/golden/make_golden_ref.py [case ...] 2>/dev/null   (about 3 minutes on 8 cores; the
        reference's tqdm bars go to stderr)
"""
from __future__ import annotations

import hashlib
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, REPO)
sys.dont_write_bytecode = True

from make_golden import _import_reference, reference_fwd_bwd  # noqa: E402

from tests.helpers import (FLIP_EXCLUDE, REF_CASES, REF_STORED_INPUTS, T_KEEP, case_inputs,  # noqa: E402
                           input_hash, ref_grad_subset, shuffle_bytes)


def make_case(R, RR, name):
    n, W, H, deg, seed, osc, bg = REF_CASES[name]
    sc, cam, bg_t, dc, di = case_inputs(name)
    # threshold-flip candidates (an alpha, transmittance or exponent-sign decision within FLIP_EXCLUDE x the fp32
    # evaluation error of its threshold, oracle/gsr_oracle.c oracle_threshold_margin): excluded from the mask too, so
    # no gradient sums a pixel whose compositing decisions the device, the oracle and torch may take differently
    from oracle import oracle as O  # the checker: used here only to choose which pixels the fixture compares
    margin = O.forward(*(np.ascontiguousarray(t.numpy()) for t in (sc.means3D, sc.opacities, sc.scales, sc.rotations,
                                                                  sc.shs, cam.viewmatrix, cam.projmatrix, cam.campos,
                                                                  bg_t)),
                       cam.tanfovx, cam.tanfovy, H, W, deg, 1.0)[3].threshold_margin()
    t0 = time.time()
    # final transmittance of the reference's walk: its renders with background 1 and 0 differ by T_ref
    other = torch.ones(3) if float(bg_t.sum()) == 0.0 else torch.zeros(3)
    alt = reference_fwd_bwd(R, RR, sc, cam, other, dc, di, backward=False)
    t1 = time.time()
    held = {}

    def upstream(color, invdepth):  # the mask needs this render's colour: formed between forward and backward
        t_ref = ((alt["color"] - color) / (other - bg_t).numpy()[:, None, None]).mean(0)
        held["T"], held["mask"] = t_ref, (t_ref >= T_KEEP) & (margin >= FLIP_EXCLUDE)
        m = torch.from_numpy(held["mask"].astype(np.float32))
        return dc * m, di * m

    # the reference's own render with this case's background, forward + backward on the masked upstream gradient
    out = reference_fwd_bwd(R, RR, sc, cam, bg_t, dc, di, backward=True, upstream_fn=upstream)
    t2 = time.time()
    t_ref, mask = held["T"], held["mask"]
    idx = ref_grad_subset(sc.means3D.shape[0], seed)
    rec = dict(name=np.array(name), input_sha256=np.array(input_hash(sc, cam, dc, di)),
               num_gaussians=np.int32(sc.means3D.shape[0]), T_keep=np.float32(T_KEEP),
               flip_exclude=np.float32(FLIP_EXCLUDE), flip_candidates=np.int64((margin < FLIP_EXCLUDE).sum()),
               mask_bits=np.packbits(mask.reshape(-1)), grad_idx=idx,
               ref_radii=out["radii"].astype(np.int32))
    floats = dict(ref_color=out["color"], ref_invdepth=out["invdepth"])
    for k in REF_STORED_INPUTS:  # the inputs another CPU could round differently (tests/helpers.py)
        floats["input_" + k] = (getattr(sc, k) if hasattr(sc, k) else getattr(cam, k)).numpy()
    for k in ("means3D", "means2D", "opacities", "scales", "rotations", "shs"):
        floats["ref_grad_" + k] = out["grad_" + k][idx]
    for k, v in floats.items():  # byte planes + the shape (tests/helpers.py load_ref_golden)
        rec[k] = shuffle_bytes(v)
        rec["shape_" + k] = np.asarray(v.shape, np.int64)
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, **rec)
    print(f"wrote {path}: N={sc.means3D.shape[0]} {W}x{H} deg={deg} kept pixels {mask.mean():.3f} "
          f"({os.path.getsize(path) / 1e6:.2f} MB; reference fwd {t1 - t0:.0f} s, fwd+bwd {t2 - t1:.0f} s)")


def main():
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    os.environ.setdefault("TQDM_DISABLE", "1")
    R, RR = _import_reference()
    for name in (sys.argv[1:] or REF_CASES):
        make_case(R, RR, name)


if __name__ == "__main__":
    main()
