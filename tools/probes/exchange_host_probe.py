#!/usr/bin/env python
"""Host-side cost of the pieces of one chunked exchange step, on one GPU with a one-rank RCCL group.

    python tools/probes/exchange_host_probe.py

Every figure is the host time of the call (perf_counter), measured while the GPU is kept busy by a long sleep kernel
enqueued first, so a call that blocks the host until the GPU catches up shows up as ~the sleep length.
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch
    import torch.distributed as dist
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", store=dist.HashStore(), rank=0, world_size=1, device_id=dev)
    pg = dist.distributed_c10d._get_default_group()
    n = 250_000
    flat = torch.zeros(11 * n, device=dev)
    gin = torch.zeros(n * 3, device=dev)
    gout = torch.zeros(n * 3, device=dev)
    ev = torch.cuda.Event()
    side = torch.cuda.Stream()
    res = {}

    def busy():
        torch.cuda._sleep(20_000_000)  # ~10 ms of GPU time at ~2 GHz

    def group(asynchronous):
        pg._start_coalescing(dev)
        go = dist.distributed_c10d.AllgatherOptions()
        go.asyncOp = asynchronous
        pg._allgather_base(gout, gin, go)
        ro = dist.AllreduceOptions()
        ro.reduceOp = dist.ReduceOp.SUM
        ro.asyncOp = asynchronous
        pg.allreduce([flat], ro)
        w = pg._end_coalescing(dev)
        if not asynchronous and w is not None:
            w.wait()
        return w

    cases = {
        "all_reduce_async": lambda: dist.all_reduce(flat, async_op=True),
        "all_reduce_sync": lambda: dist.all_reduce(flat, async_op=False),
        "all_gather_async": lambda: dist.all_gather_into_tensor(gout, gin, async_op=True),
        "group_async": lambda: group(True),
        "group_sync": lambda: group(False),
        "group_async_wait": lambda: group(True).wait(),
        "event_record": lambda: ev.record(),
        "stream_wait_event": lambda: side.wait_event(ev),
        "torch_mul_small": lambda: torch.mul(gin[:3], 1.0, out=gout[:3]),
    }
    for k, f in cases.items():
        ts = []
        for _ in range(12):
            torch.cuda.synchronize()
            busy()
            t0 = time.perf_counter()
            f()
            ts.append((time.perf_counter() - t0) * 1e6)
        torch.cuda.synchronize()
        ts = sorted(ts[2:])
        res[k] = {"host_us_median": round(ts[len(ts) // 2], 1), "host_us_max": round(ts[-1], 1)}
    # on a side stream: does the group land on the current (side) stream?
    with torch.cuda.stream(side):
        torch.cuda.synchronize()
        busy()
        t0 = time.perf_counter()
        group(False)
        res["group_sync_on_side_stream"] = {"host_us": round((time.perf_counter() - t0) * 1e6, 1)}
    torch.cuda.synchronize()
    # host time of the chunked backward's ABI calls (local reducer: no collectives), cfg 3
    from bench import CONFIGS
    from gaussian_splatting_lightning_amd.multiview import ViewGradReducer
    from gaussian_splatting_lightning_amd.rasterizer import GaussianRasterizationSettings, backward_chunked, forward_raw
    from gaussian_splatting_lightning_amd.synthetic import make_camera, make_scene, make_upstream
    cfg = CONFIGS["cfg3"]
    sc = make_scene(cfg["n"], cfg["deg"], seed=0).to(dev)
    cam = make_camera(cfg["W"], cfg["H"]).to(dev)
    dc, di = (t.to(dev) for t in make_upstream(cfg["W"], cfg["H"], 0))
    rs = GaussianRasterizationSettings(cfg["H"], cfg["W"], cam.tanfovx, cam.tanfovy, torch.zeros(3, device=dev), 1.0,
                                       cam.viewmatrix, cam.projmatrix, cfg["deg"], cam.campos, False, False, False)
    for label, kw in (("local", dict(distributed=False)), ("dist", {})):
        red = ViewGradReducer(cfg["n"], 16, 3, dev, mode="compact", chunks=4, **kw)
        marks = []
        for it in range(6):
            _, _, _, st = forward_raw(sc.means3D, sc.shs, None, sc.opacities, sc.scales, sc.rotations, None, rs)
            t0 = time.perf_counter()
            red.begin_step()
            t1 = time.perf_counter()
            ts = []

            def on_chunk(c):
                ts.append(time.perf_counter())
                red.start_chunk(c)
                ts.append(time.perf_counter())
            backward_chunked(st, rs, dc, di, red.chunk_outputs(), on_chunk=on_chunk, compact_sh=True,
                             accumulate_stats=True)
            t2 = time.perf_counter()
            red.finish(sc.means3D)
            t3 = time.perf_counter()
            torch.cuda.synchronize()
            if it >= 2:
                marks.append({"begin_step_us": round((t1 - t0) * 1e6, 1),
                              "composite_call_us": round((ts[0] - t1) * 1e6, 1),
                              "issue_us": [round((ts[2 * k + 1] - ts[2 * k]) * 1e6, 1) for k in range(4)],
                              "chunk_call_us": [round((ts[2 * k + 2] - ts[2 * k + 1]) * 1e6, 1) for k in range(3)],
                              "finish_us": round((t3 - t2) * 1e6, 1)})
        res[f"chunked_backward_{label}"] = marks
    dist.destroy_process_group()
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
