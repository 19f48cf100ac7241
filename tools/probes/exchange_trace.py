#!/usr/bin/env python
"""Steps of the chunked compact exchange on a one-rank RCCL group, for a HIP API + kernel trace:

    rocprofv3 --hip-trace --kernel-trace -d OUT -o run --output-format csv -- python tools/probes/exchange_trace.py

Prints perf_counter marks (host) per step so the API timeline can be lined up with the kernels.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chunks", type=int, default=4)
    ap.add_argument("--mode", default="compact")
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--local", action="store_true")
    args = ap.parse_args()
    import torch
    import torch.distributed as dist
    from bench import CONFIGS
    from gaussian_splatting_lightning_amd.multiview import ViewGradReducer
    from gaussian_splatting_lightning_amd.rasterizer import GaussianRasterizationSettings, backward_chunked, forward_raw
    from gaussian_splatting_lightning_amd.synthetic import make_camera, make_scene, make_upstream
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    if not args.local:
        dist.init_process_group("nccl", store=dist.HashStore(), rank=0, world_size=1, device_id=dev)
    cfg = CONFIGS["cfg3"]
    sc = make_scene(cfg["n"], cfg["deg"], seed=0).to(dev)
    cam = make_camera(cfg["W"], cfg["H"]).to(dev)
    dc, di = (t.to(dev) for t in make_upstream(cfg["W"], cfg["H"], 0))
    rs = GaussianRasterizationSettings(cfg["H"], cfg["W"], cam.tanfovx, cam.tanfovy, torch.zeros(3, device=dev), 1.0,
                                       cam.viewmatrix, cam.projmatrix, cfg["deg"], cam.campos, False, False, False)
    red = ViewGradReducer(cfg["n"], 16, 3, dev, mode=args.mode, chunks=args.chunks,
                          distributed=False if args.local else None)
    for _ in range(args.steps):
        _, _, _, st = forward_raw(sc.means3D, sc.shs, None, sc.opacities, sc.scales, sc.rotations, None, rs)
        red.begin_step()
        backward_chunked(st, rs, dc, di, red.chunk_outputs(), on_chunk=red.start_chunk, compact_sh=red.compact,
                         accumulate_stats=True)
        red.finish(sc.means3D)
    torch.cuda.synchronize()
    if not args.local:
        dist.destroy_process_group()
    print("done")


if __name__ == "__main__":
    main()
