#!/usr/bin/env python
"""Where the multi-GPU step's extra time goes, on ONE GPU with a one-rank RCCL group (bench.py --force-dist measured
1.14 ms/step against 0.81 for the plain step at cfg 3).

    python tools/dist_overhead.py [--config cfg3] [--steps 20] [--rounds 3]

Variants (each: wall ms per step over --steps steps bracketed by synchronize; median over --rounds interleaved
rounds):
  plain            backward_raw into a dense reducer, no process group (bench.py at N = 1)
  local_*          the reducer's chunked / compact arithmetic with distributed=False (no collectives)
  dist_*           the same with the one-rank RCCL group: grouped (one RCCL group per chunk) or separate
                   collectives, blocking or async ops; dist_auto is multiview.plan_exchange's choice
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg3")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--only", default="", help="comma-separated variant names (plain always runs)")
    args = ap.parse_args()
    import torch
    import torch.distributed as dist
    from bench import CONFIGS
    from gaussian_splatting_lightning_amd.multiview import ViewGradReducer
    from gaussian_splatting_lightning_amd.rasterizer import (GaussianRasterizationSettings, backward_chunked,
                                                             backward_raw, forward_raw)
    from gaussian_splatting_lightning_amd.synthetic import make_camera, make_scene, make_upstream
    cfg = CONFIGS[args.config]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    sc = make_scene(cfg["n"], cfg["deg"], seed=0, stress_fraction=cfg["stress"]).to(dev)
    cam = make_camera(cfg["W"], cfg["H"]).to(dev)
    dc, di = (t.to(dev) for t in make_upstream(cfg["W"], cfg["H"], 0))
    rs = GaussianRasterizationSettings(cfg["H"], cfg["W"], cam.tanfovx, cam.tanfovy, torch.zeros(3, device=dev), 1.0,
                                       cam.viewmatrix, cam.projmatrix, cfg["deg"], cam.campos, False, False, False)
    n, M = cfg["n"], sc.shs.shape[1]

    def make_step(red):
        def step():
            _, _, _, st = forward_raw(sc.means3D, sc.shs, None, sc.opacities, sc.scales, sc.rotations, None, rs)
            if red.chunks == 1:
                backward_raw(st, rs, dc, di, **red.backward_kwargs())
                red.reduce(sc.means3D)
            else:
                red.begin_step(means3D=sc.means3D)  # expand="side": expansions on the side stream
                backward_chunked(st, rs, dc, di, red.chunk_outputs(), on_chunk=red.start_chunk,
                                 compact_sh=red.compact, accumulate_stats=True)
                red.finish(sc.means3D)
        return step

    def timeit(step):
        for _ in range(10):
            step()
        torch.cuda.synchronize()
        host = 0.0
        t0 = time.perf_counter()
        for _ in range(args.steps):
            h0 = time.perf_counter()
            step()
            host += time.perf_counter() - h0
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        return {"wall_ms": round(1e3 * wall / args.steps, 4), "host_ms": round(1e3 * host / args.steps, 4)}

    local = {"plain": dict(mode="dense", chunks=1), "local_compact1": dict(mode="compact", chunks=1)}
    remote = {"dist_dense1": dict(mode="dense", chunks=1),
              "dist_compact1": dict(mode="compact", chunks=1),
              "dist_compact2_chunk": dict(mode="compact", chunks=2, expand="chunk"),
              "dist_compact2_once": dict(mode="compact", chunks=2, expand="once"),
              "dist_compact2_side": dict(mode="compact", chunks=2, expand="side"),
              "dist_compact4_chunk": dict(mode="compact", chunks=4, expand="chunk"),
              "dist_compact4_once": dict(mode="compact", chunks=4, expand="once"),
              "dist_compact4_side": dict(mode="compact", chunks=4, expand="side"),
              "dist_dense2": dict(mode="dense", chunks=2),
              "dist_compact2_chunk_value": dict(mode="compact", chunks=2, expand="chunk", handoff="value"),
              "dist_compact4_chunk_value": dict(mode="compact", chunks=4, expand="chunk", handoff="value"),
              "dist_compact4_once_value": dict(mode="compact", chunks=4, expand="once", handoff="value"),
              "dist_compact4_side_value": dict(mode="compact", chunks=4, expand="side", handoff="value"),
              "dist_auto": dict(mode="auto", chunks=None),
              "dist_auto_w8": dict(mode="auto", chunks=None, plan_world=8)}
    if args.only:
        keep = set(args.only.split(","))
        local = {k: v for k, v in local.items() if k in keep or k == "plain"}
        remote = {k: v for k, v in remote.items() if k in keep}
    steps = {k: make_step(ViewGradReducer(n, M, cfg["deg"], dev, distributed=False, **kw)) for k, kw in local.items()}
    dist.init_process_group("nccl", store=dist.HashStore(), rank=0, world_size=1, device_id=dev)
    res = {}
    try:
        reds = {k: ViewGradReducer(n, M, cfg["deg"], dev, **kw) for k, kw in remote.items()}
        steps.update({k: make_step(r) for k, r in reds.items()})
        samples = {k: [] for k in steps}
        for _ in range(args.rounds):  # interleaved rounds: clocks and box noise hit every variant alike
            for k, f in steps.items():
                samples[k].append(timeit(f))
        for k, v in samples.items():
            w = sorted(x["wall_ms"] for x in v)
            res[k] = {"wall_ms_median": w[len(w) // 2], "wall_ms_all": w}
        for k in ("dist_auto", "dist_auto_w8"):
            if k in reds:
                res[k]["exchange"] = reds[k].describe()
                res[k]["plan"] = reds[k].plan
    finally:
        dist.destroy_process_group()
    base = res["plain"]["wall_ms_median"]
    for k in res:
        res[k]["vs_plain"] = round(res[k]["wall_ms_median"] / base, 4)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
