#!/usr/bin/env python
"""Fused SSIM loss fwd+bwd at 1080p (3 channels): per-kernel time (hipEvents) vs the HBM roofline.

Algorithmic bytes per (fwd+bwd): forward reads both images (8 B/px) and writes three derivative maps
(12 B/px); backward reads the three maps and both images (20 B/px) and writes dL/dimg1 (4 B/px) -> 44 B/px.
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from gaussian_splatting_lightning_amd.ssim import fused_ssim
    dev = torch.device("cuda", 0)
    B, C, H, W = 1, 3, 1080, 1920
    g = torch.Generator(device="cpu").manual_seed(0)
    gt = torch.rand(B, C, H, W, generator=g).to(dev)
    x = (gt + 0.1 * torch.randn(B, C, H, W, generator=g).to(dev)).clamp(0, 1).requires_grad_(True)
    for _ in range(5):
        (1 - fused_ssim(x, gt)).backward()
    torch.cuda.synchronize()
    n = 50
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        x.grad = None
        (1 - fused_ssim(x, gt)).backward()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / n
    px = B * C * H * W
    algo = 44 * px
    print(json.dumps({"workload": "fused SSIM fwd+bwd, 1x3x1080x1920 fp32", "ms_per_iter": round(ms, 4),
                      "algorithmic_bytes": algo, "achieved_GBps": round(algo / (ms * 1e-3) / 1e9, 1),
                      "hbm_peak_GBps": 8000.0, "frac": round(algo / (ms * 1e-3) / 1e9 / 8000.0, 4),
                      "note": "includes the torch ops of the loss expression (1 - mean) and the partial-sum reduce"}))


if __name__ == "__main__":
    main()
