#!/usr/bin/env python
"""Benchmark: rasterizer forward+backward on BASELINE.json config 3 (1M Gaussians, 1920x1080, SH deg 3).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

One step on every rank = one forward + backward of the HIP rasterizer (C ABI, include/gsrast.h) for that
rank's view of the shared 1M-Gaussian scene (view k = the treehill view rotated 2*pi*k/8 about world y),
with the upstream gradients dL/dimage, dL/dinvdepth fixed, the per-view densification statistics accumulated
by the backward kernel, and -- for N > 1 -- the per-step exchange of multiview.py: one RCCL all-reduce (sum)
of the per-Gaussian parameter gradients plus one all-gather of the compact SH factors (BASELINE.json config
4: one view per GPU).  The statistics are reduced over ranks only when the model densifies.  Per-GPU work is
fixed, so scaling is weak.  value = N * Gaussians * W * H / step time (Gaussians*pixels/s, whole job).

Extra fields on the one JSON line:
  roofline      dominant kernel (a composite pass, fp32-VALU-bound): algorithmic flops / its average duration
                from a hipEvent pair recorded around that kernel's stage on the launch stream on every 4th timed
                step (the only events in the timed region; SURVEY.md §8(d) flops), with the same launch's
                algorithmic-bytes HBM figure and PMC traffic beside it;
  cpu_baseline  the oracle (oracle/gsr_oracle.c, C + OpenMP) on the same workload on the host cores;
  stages_ms     average device time of every pipeline stage per step, from a separate untimed pass of K steps
                with an event pair around every stage.
"""
from __future__ import annotations

import argparse
import gc
import json
import math
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

METRIC = "rasterizer fwd+bwd ms & Gaussians·pixels/s @ 1M gauss, 1080p; 1/2/4/8-GPU"
HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md chip table (spec)
FP32_VALU_PEAK_TF = 157.3  # MI355X_MICROARCH.md chip table (spec)
VALU_ISSUE_NS = 1.29   # per wave-instruction per SIMD, every SIMD issuing fp32 FMA (tools/probes/valu_rate_probe.hip)
TRANS_EXTRA_NS = 2.2   # v_exp / v_rcp cost ~3.5 ns on the same pipe
EVENT_EVERY = 4  # timed steps per step that carries the dominant kernel's event pair
SETTLE_S = 0.2   # untimed steps (seconds) right before the timed ones, clocks at steady state
PY_REFERENCE_CFG3_S = 730.0  # reference Python rasterizer, cfg 3 fwd+bwd, 8-core Xeon

CONFIGS = {
    "cfg3": dict(n=1_000_000, W=1920, H=1080, deg=3, stress=0.0,
                 desc="BASELINE config 3/4: 1M Gaussians, 1920x1080, SH deg 3, fwd+bwd, one view per GPU"),
    "cfg2": dict(n=100_000, W=800, H=800, deg=3, stress=0.0, desc="BASELINE config 2: 100k Gaussians, 800x800, SH 3"),
    "cfg5": dict(n=5_000_000, W=3840, H=2160, deg=3, stress=0.01,
                 desc="BASELINE config 5: 5M Gaussians, 3840x2160, SH 3, 1% bloated (stress)"),
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="cfg3", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-stage-events", action="store_true", help="time without per-stage hipEvents")
    ap.add_argument("--cpu-budget-s", type=float, default=20.0)
    ap.add_argument("--dist-backend", default="nccl", choices=("nccl", "gloo"))
    ap.add_argument("--exchange", default="auto", choices=("auto", "compact", "dense", "sharded"),
                    help="N>1 gradient exchange (gaussian_splatting_lightning_amd/multiview.py); auto: the cost model's "
                         "choice (multiview.plan_exchange)")
    ap.add_argument("--exchange-chunks", type=int, default=0,
                    help="N>1: Gaussian chunks whose exchange overlaps the rest of the backward (1: after it; 0: the "
                         "cost model's choice)")
    ap.add_argument("--exchange-expand", default=None, choices=("chunk", "once", "side"),
                    help="compact exchange: SH expansion per chunk or once after the last gather on the compute "
                         "stream, or per chunk on the side stream behind its group (default: the cost model's)")
    ap.add_argument("--exchange-handoff", default=None, choices=("event", "value"),
                    help="chunked exchange: hand-offs between the compute and the collective stream by hipEvents or "
                         "by stream-ordered device words (gsr_stream_signal / gsr_stream_wait)")
    ap.add_argument("--exchange-groups", type=int, default=0, choices=(0, 1, 2),
                    help="sharded exchange over RCCL: 1 = the reduce-scatters and the all-to-all as one group, 2 = as "
                         "two (0: the reducer's default)")
    ap.add_argument("--plan-world", type=int, default=0,
                    help="N>1 path: plan the exchange (mode, chunks, SH expansion) for this many ranks instead of "
                         "WORLD_SIZE -- a one-rank rehearsal (--force-dist) of the N-GPU schedule")
    ap.add_argument("--no-train-step", action="store_true",
                    help="skip the extra train_step_ms pass (forward + backward + exchange + Adam)")
    ap.add_argument("--force-dist", action="store_true",
                    help="take the N>1 path (process group, RCCL exchange) even with one rank, e.g. under "
                         "torchrun --nproc-per-node 1")
    return ap.parse_args()


def main():
    args = parse()
    import numpy as np
    import torch
    import torch.distributed as dist

    from gaussian_splatting_lightning_amd import _native
    from gaussian_splatting_lightning_amd.rasterizer import (GaussianRasterizationSettings, backward_chunked,
                                                             backward_raw, forward_raw)
    from gaussian_splatting_lightning_amd.multiview import ViewGradReducer
    from gaussian_splatting_lightning_amd.synthetic import make_camera, make_scene, make_upstream

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")
    dev = torch.device("cuda", local_rank % max(torch.cuda.device_count(), 1))
    torch.cuda.set_device(dev)
    distributed = world > 1 or args.force_dist
    if distributed:
        if "MASTER_ADDR" not in os.environ:  # --force-dist without a launcher: a one-rank group on this host
            os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=os.environ.get("MASTER_PORT", "29531"),
                              RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:  # rehearsal of the N>1 path on fewer GPUs than ranks (RCCL needs one GPU per rank)
            dist.init_process_group(args.dist_backend)
    cfg = CONFIGS[args.config]
    n, W, H, deg = cfg["n"], cfg["W"], cfg["H"], cfg["deg"]
    num_views = max(world, 8) if args.config == "cfg3" else max(world, 1)

    # ---- inputs: one shared scene (same seed on every rank), one view per rank ----
    scene = make_scene(n, sh_degree=deg, seed=0, stress_fraction=cfg["stress"])
    cam = make_camera(W, H, view_index=rank, num_views=num_views)
    dcolor_cpu, dinv_cpu = make_upstream(W, H, seed=0)
    sc = scene.to(dev)
    c = cam.to(dev)
    dcolor, dinv = dcolor_cpu.to(dev), dinv_cpu.to(dev)
    settings = GaussianRasterizationSettings(
        image_height=H, image_width=W, tanfovx=c.tanfovx, tanfovy=c.tanfovy,
        bg=torch.zeros(3, device=dev), scale_modifier=1.0, viewmatrix=c.viewmatrix, projmatrix=c.projmatrix,
        sh_degree=deg, campos=c.campos, prefiltered=False, debug=False, antialiasing=False)
    M = sc.shs.shape[1]

    # Per-Gaussian gradient destinations + the cross-rank exchange (multiview.py): one view per rank.  N=1: dense
    # destinations, one chunk, no collectives.  N>1 (or --force-dist): mode, chunk count and SH-expansion schedule
    # from the cost model (multiview.plan_exchange) unless given; the backward's per-Gaussian stage runs in the
    # chunks' Gaussian ranges and each range's collectives (one RCCL group) are issued as soon as it is enqueued.
    if distributed:
        red = ViewGradReducer(n, M, deg, dev, mode=args.exchange, chunks=args.exchange_chunks or None,
                              expand=args.exchange_expand, plan_world=args.plan_world or None,
                              handoff=args.exchange_handoff,
                              one_group=None if not args.exchange_groups else args.exchange_groups == 1)
    else:
        red = ViewGradReducer(n, M, deg, dev, mode="dense", chunks=1)
    mode = red.mode
    assert red.distributed == distributed

    def step():
        color, radii, invd, st = forward_raw(sc.means3D, sc.shs, None, sc.opacities, sc.scales, sc.rotations, None,
                                             settings)
        # densification statistics and max radii accumulate in the backward kernel; they are reduced over ranks
        # only when the model densifies (ViewGradReducer.sync_densify_stats), not every step
        if red.chunks == 1:
            backward_raw(st, settings, dcolor, dinv, **red.backward_kwargs())
            red.reduce(sc.means3D, c.campos if red.sharded else None)
        else:
            red.begin_step(means3D=sc.means3D)  # side stream: each chunk's SH expansion runs right behind its group
            backward_chunked(st, settings, dcolor, dinv, red.chunk_outputs(), on_chunk=red.start_chunk,
                             compact_sh=red.compact, accumulate_stats=True)
            red.finish(sc.means3D)
        return st

    # ---- warmup ----
    for _ in range(args.warmup):
        st = step()
    torch.cuda.synchronize()

    # ---- per-stage breakdown (untimed): an event pair around every stage ----
    use_events = not args.no_stage_events
    stage_avg = {}
    if use_events:
        _native.reset_stage_times()
        _native.set_profiling(True)
        for _ in range(args.steps):
            st = step()
        torch.cuda.synchronize()
        _native.set_profiling(False)
        stage_avg = {k: (v[0] / v[1] if v[1] else 0.0) for k, v in _native.stage_times().items()}
    # Every event is a marker packet in the stream, and the kernel after one waits ~6 us for it (rocprofv3 trace:
    # an event pair around render_bwd adds ~12 us to a step), so the timed steps carry events around the dominant
    # composite kernel only (its live launch time for the roofline), and only on every EVENT_EVERY-th step.
    dom = max(("render_fwd", "render_bwd"), key=lambda k: stage_avg.get(k, 0.0))

    # ---- timed region ----
    _native.reset_stage_times()
    # Python's cyclic garbage collector is held off while timing: a collection pass stalled the host for
    # ~0.6 ms in the middle of a step (rocprofv3 trace: one gap before a backward's first kernel), which the
    # GPU then waits out
    gc.collect()
    gc.disable()
    # Settle: untimed steps for SETTLE_S right before the timed ones, after all host bookkeeping.  Idle, the
    # GPU's clocks drop within milliseconds and take tens of ms of work to ramp back: a 43 ms pause before the
    # timed steps (trace) made them run 918 -> 867 us per step, and 5 warmup steps alone measured 0.899 against
    # 0.858 ms/step after 25.  Ranks agree on every extension (the steps run collectives).
    t_w = time.perf_counter()
    while True:
        more = torch.tensor([1.0 if time.perf_counter() - t_w < SETTLE_S else 0.0], device=dev)
        if distributed:
            dist.all_reduce(more, op=dist.ReduceOp.MAX)
        if more.item() == 0.0:
            break
        for _ in range(10):
            st = step()
        torch.cuda.synchronize()
    if use_events:
        _native.set_tuning("prof_mask", _native.stage_mask(dom))
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        if use_events:
            _native.set_profiling(i % EVENT_EVERY == 0)
        st = step()
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    gc.enable()
    _native.set_profiling(False)
    _native.set_tuning("prof_mask", -1)
    timed_stages = _native.stage_times()
    if distributed:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms_per_step = 1e3 * elapsed / args.steps

    # ---- per-step distribution (separate pass, not the headline): one hipEvent at every step boundary on the
    # launch stream, SURVEY.md §8(d)'s "median of >= 20 hipEvent-timed steps".  Each event is a stream marker the
    # next kernel waits behind (~6 us), so these per-step times run slightly above the wall-clock mean. ----
    n_ev = max(args.steps, 20)
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(n_ev + 1)]
    gc.disable()
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    evs[0].record()
    for i in range(n_ev):
        st = step()
        evs[i + 1].record()
    torch.cuda.synchronize()
    gc.enable()
    per_step = sorted(evs[i].elapsed_time(evs[i + 1]) for i in range(n_ev))
    step_events = {"steps": n_ev, "p50_ms": round(per_step[n_ev // 2], 4),
                   "p90_ms": round(per_step[min(n_ev - 1, (9 * n_ev) // 10)], 4),
                   "min_ms": round(per_step[0], 4), "mean_ms": round(sum(per_step) / n_ev, 4)}

    # ---- training step (separate pass, extra field, not the headline): forward + backward + exchange + Adam ----
    # The reference steps torch.optim.Adam(eps=1e-15) over its six per-Gaussian groups right after the backward
    # (gs_lightning_module.py:114-134,168-170).  As there, the optimizer steps the RAW parameters (xyz, features_dc,
    # features_rest and the pre-activation _opacity / _scaling / _rotation of gaussian_model.py) and the rasterizer
    # sees their activations (sigmoid / exp / normalize: activations.activate and its chain rule, one launch each),
    # with the learning rates of configs/train_gs.yaml; the SH groups take their gradient in factored form through
    # the fused SH Adam (compact exchange, GaussianAdam.step(sh_views=...)), so no (P, 16, 3) gradient is written.
    train = None
    if not args.no_train_step:
        from gaussian_splatting_lightning_amd.optim import GaussianAdam
        from gaussian_splatting_lightning_amd.activations import activate, activate_backward
        from gaussian_splatting_lightning_amd.multiview import plan_exchange
        # the training exchange: compact (every rank steps every Gaussian) or sharded (every rank steps its shard
        # and all-gathers the updated parameters); dense has no factored SH gradient for the fused SH Adam
        if args.exchange == "auto":
            tmode = plan_exchange(n, args.plan_world or world, M, modes=("compact", "sharded"))["mode"]
        else:
            tmode = "sharded" if args.exchange == "sharded" else "compact"
        tred = ViewGradReducer(n, M, deg, dev, mode=tmode, chunks=None if tmode == "compact" else 1,
                               plan_world=args.plan_world or None, handoff=args.exchange_handoff,
                               one_group=None if not args.exchange_groups else args.exchange_groups == 1) \
            if distributed else ViewGradReducer(n, M, deg, dev, mode="compact", chunks=1)
        # parameters padded to the shards' N S rows (the rasterizer reads the first n), so every rank's updated shard
        # is all-gathered in place
        rows = tred.padded_rows()

        def padded(t):
            out = torch.zeros((rows,) + tuple(t.shape[1:]), device=dev)
            out[:n] = t
            return out

        tp = {"means3D": padded(sc.means3D), "shs": padded(sc.shs), "_scaling": padded(sc.scales.log()),
              "_opacity": padded(torch.logit(sc.opacities.clamp(1e-6, 1 - 1e-6))), "_rotation": padded(sc.rotations)}
        g0, g1 = tred.shard if tred.sharded else (0, n)
        L = g1 - g0
        act = (torch.empty_like(sc.scales), torch.empty_like(sc.opacities), torch.empty_like(sc.rotations))
        raw_grad = (torch.empty(L, 3, device=dev), torch.empty(L, 1, device=dev), torch.empty(L, 4, device=dev))
        own = {k: v[g0:g1] for k, v in tp.items()}  # the rows this rank's optimizer steps
        f_dc, f_rest = own["shs"][:, :1], own["shs"][:, 1:]  # column blocks of the one (P, 16, 3) tensor
        topt = GaussianAdam([{"params": [own["means3D"]], "lr": 0.00016, "name": "xyz"},
                             {"params": [f_dc], "lr": 0.0025, "name": "features_dc"},
                             {"params": [f_rest], "lr": 0.0025 / 20.0, "name": "features_rest"},
                             {"params": [own["_opacity"]], "lr": 0.05, "name": "opacity"},
                             {"params": [own["_scaling"]], "lr": 0.005, "name": "scaling"},
                             {"params": [own["_rotation"]], "lr": 0.001, "name": "rotation"}], lr=0.0, eps=1e-15)

        def train_step():
            activate(tp["_scaling"][:n], tp["_opacity"][:n], tp["_rotation"][:n], out=act)
            _, _, _, tst = forward_raw(tp["means3D"][:n], tp["shs"][:n], None, act[1], act[0], act[2], None, settings)
            if tred.chunks == 1:
                backward_raw(tst, settings, dcolor, dinv, **tred.backward_kwargs())
                tred.reduce(tp["means3D"][:n], c.campos if tred.sharded else None, expand_sh=False)
            else:
                tred.begin_step()
                backward_chunked(tst, settings, dcolor, dinv, tred.chunk_outputs(), on_chunk=tred.start_chunk,
                                 compact_sh=True, accumulate_stats=True)
                tred.finish(tp["means3D"][:n], expand_sh=False)
            gr = tred.grads
            if L > 0:
                activate_backward(own["_rotation"], act[0][g0:g1], act[1][g0:g1], act[2][g0:g1],
                                  gr["scales"].view(L, 3), gr["opacities"].view(L, 1), gr["rotations"].view(L, 4),
                                  out=raw_grad)
                own["means3D"].grad = gr["means3D"].view(L, 3)
                own["_scaling"].grad, own["_opacity"].grad, own["_rotation"].grad = raw_grad
                topt.step(sh_views=(f_dc, f_rest, tred.sh_views_gradient(tp["means3D"][:n])))
            if tred.sharded:
                tred.gather_shards(list(tp.values()))

        for _ in range(max(args.warmup, 3)):
            train_step()
        gc.disable()
        if distributed:
            dist.barrier()
        torch.cuda.synchronize()
        t_tr = time.perf_counter()
        for _ in range(args.steps):
            train_step()
        torch.cuda.synchronize()
        if distributed:
            dist.barrier()
        el_tr = time.perf_counter() - t_tr
        gc.enable()
        if distributed:
            t = torch.tensor([el_tr], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el_tr = float(t.item())
        train = {"train_step_ms": round(1e3 * el_tr / args.steps, 4), "steps": args.steps,
                 "exchange": tred.describe() if distributed else "none (one view, compact SH gradient)",
                 "note": "activations (exp / sigmoid / normalize) + forward + backward + exchange + their chain rule "
                         "+ Adam over the six raw per-Gaussian groups (GaussianAdam; the SH groups by the fused SH Adam "
                         "on the factored multi-view gradient; sharded: on this rank's shard, then the updated "
                         "parameters all-gathered), timed like the headline (barrier + synchronize, max over ranks)"}
        del tp, own, topt, tred, act, raw_grad

    # ---- per-launch statistics for the roofline (untimed) ----
    lay = _native.state_layout(n, st.num_rendered, W, H)
    T = ((W + 15) // 16) * ((H + 15) // 16)
    npix = W * H
    nc = st.image_buffer[lay["img_n_contrib"]: lay["img_n_contrib"] + 4 * npix].view(torch.int32)
    sum_contrib = int(nc.sum(dtype=torch.int64).item())
    I = st.num_rendered
    # The composite passes touch only the instances they walk: the forward loads a tile's instances up to the batch in
    # which its last pixel terminates (sum of tile_loaded), the backward walks each tile from its last contributor
    # (sum of tile_last) and zeroes the rows of the loaded-but-not-contributing rest.  At cfg 3, 57 % of the
    # instances lie beyond tile_loaded and are never read, so SURVEY.md §8(d)'s per-instance figures are charged
    # for these counts; the figure over all I instances stays beside it as "nominal_bytes_per_launch".
    tl_sum = int(st.image_buffer[lay["img_tile_last"]: lay["img_tile_last"] + 4 * T].view(torch.int32)
                 .sum(dtype=torch.int64).item())
    ld_sum = int(st.image_buffer[lay["img_tile_loaded"]: lay["img_tile_loaded"] + 4 * T].view(torch.int32)
                 .sum(dtype=torch.int64).item())
    algo_bytes = {
        # F6 composite fwd = 8 B/T + 44 B/I + 24 B/P; B1 composite bwd adds 40 B/I of grads
        "render_fwd": 8 * T + 44 * ld_sum + 24 * npix,
        "render_bwd": 8 * T + (44 + 40) * tl_sum + 40 * (ld_sum - tl_sum) + 24 * npix,
        "preprocess": n * (40 + 12 * M) + n * (48 + 36),  # + the SH colour's direction Jacobian (9 floats)
        "preprocess_bwd": n * (40 + 12 * M) + 88 * n + n * (56 + 12 * M),
    }
    nominal_bytes = {"render_fwd": 8 * T + 44 * I + 24 * npix, "render_bwd": 8 * T + 44 * I + 24 * npix + 40 * I}
    flops = {"render_fwd": 25.0 * sum_contrib, "render_bwd": 70.0 * sum_contrib}
    tot, calls = timed_stages.get(dom, (0.0, 0))
    dom_ms = tot / calls if calls else 0.0  # measured over the timed steps
    roofline = None
    if dom_ms > 0:
        ach = algo_bytes[dom] / (dom_ms * 1e-3) / 1e9
        traffic = None
        pmc_path = os.path.join(REPO, "profiles", "pmc_traffic.json")
        if os.path.exists(pmc_path):
            try:
                pm = json.load(open(pmc_path))
                e = pm.get(args.config, {}).get(dom)
                traffic = e.get("hbm_bytes_per_launch") if e else None
            except Exception:  # noqa: BLE001
                traffic = None
        # The composite passes are VALU-bound by construction (~145 flop per byte against the
        # 20 flop/B ridge), so the headline roofline is the fp32 VALU one: algorithmic flops (25 / 70 per
        # evaluated (pixel, Gaussian) pair x sum(n_contrib)) over the live launch time.  The HBM figure of the
        # same launch (SURVEY's algorithmic bytes, PMC traffic) is kept beside it.
        tflops = flops[dom] / (dom_ms * 1e-3) / 1e12
        # VALU issue utilisation of the same launch: PMC wave-instruction counts (profiles/pmc_insts.json, same
        # config) x the per-SIMD issue costs tools/probes/valu_rate_probe.hip measured with every SIMD issuing
        # (1.29 ns per VALU, +2.2 ns per transcendental), over the live launch time
        issue = None
        ins_path = os.path.join(REPO, "profiles", "pmc_insts.json")
        if os.path.exists(ins_path):
            try:
                e = json.load(open(ins_path)).get(args.config, {}).get(dom)
                if e:
                    busy_ms = (e["valu"] * VALU_ISSUE_NS + (e.get("trans") or 0) * TRANS_EXTRA_NS) / 1024 * 1e-6
                    issue = {"valu_insts": e["valu"], "salu_insts": e.get("salu"), "trans_insts": e.get("trans"),
                             "valu_busy_ms": round(busy_ms, 4), "frac": round(busy_ms / dom_ms, 4),
                             "note": "VALU issue time per SIMD / launch time (profiles/pmc_insts.json)"}
            except Exception:  # noqa: BLE001
                issue = None
        roofline = {"kernel": dom, "bound": "valu", "achieved": round(tflops, 2), "peak": FP32_VALU_PEAK_TF,
                    "unit": "TFLOP/s", "frac": round(tflops / FP32_VALU_PEAK_TF, 4), "traffic": traffic,
                    "algorithmic_flops_per_launch": flops[dom], "avg_launch_ms": round(dom_ms, 4),
                    "hbm": {"achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                            "frac": round(ach / HBM_PEAK_GBS, 4), "algorithmic_bytes_per_launch": algo_bytes[dom],
                            "instances_walked": tl_sum, "instances_loaded": ld_sum, "instances_total": I,
                            "nominal_bytes_per_launch": nominal_bytes.get(dom),
                            "note": "algorithmic bytes charge SURVEY §8(d)'s 44 B (+40 B gradient row) per instance the "
                                    "pass loads (sum tile_loaded) / walks (sum tile_last), not per binned instance; "
                                    "nominal_bytes_per_launch is the all-instance figure"},
                    "valu_issue": issue,
                    "note": "fp32 VALU bound (no MFMA work on this path); flops = 25 (fwd) / 70 (bwd) per pair x "
                            "sum(n_contrib) (SURVEY §8(d)); traffic = PMC HBM bytes per launch "
                            "(profiles/pmc_traffic.json)"}

    # ---- CPU baseline: the oracle on the same workload, rank 0 at N=1 only ----
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle import oracle as O
        inp = [t.numpy() for t in (scene.means3D, scene.opacities, scene.scales, scene.rotations, scene.shs)]
        vm, pm_, cp = cam.viewmatrix.numpy(), cam.projmatrix.numpy(), cam.campos.numpy()
        dcn, din = dcolor_cpu.numpy(), dinv_cpu.numpy()
        times = []
        t_start = time.perf_counter()
        while len(times) < 5:
            t1 = time.perf_counter()
            _, _, _, run = O.forward(inp[0], inp[1], inp[2], inp[3], inp[4], vm, pm_, cp, np.zeros(3, np.float32),
                                     cam.tanfovx, cam.tanfovy, H, W, deg)
            run.backward(dcn, din)
            times.append(time.perf_counter() - t1)
            del run
            if time.perf_counter() - t_start > args.cpu_budget_s:
                break
        tc = float(np.median(times))
        cpu = {"value": n * W * H / tc, "unit": "Gaussians·pixels/s", "cores": O.num_threads(), "kind": "port",
               "sample": f"{len(times)} full {args.config} steps (fwd+bwd, view 0) in oracle/gsr_oracle.c, median "
                         f"{tc:.2f} s/step",
               "reference_python": {"value": (n * W * H / PY_REFERENCE_CFG3_S) if args.config == "cfg3" else None,
                                    "note": "BASELINE.md §2: gs_lightning/rasterize Python path, 8-core Xeon, "
                                            "~730 s fwd+bwd (extrapolated), not re-run here"}}

    value = world * n * W * H / (ms_per_step * 1e-3)
    line = {
        "metric": METRIC, "value": value, "unit": "Gaussians·pixels/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "warmup_settle_s": SETTLE_S, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f32", "data": "synthetic",
        "config": {"workload": cfg["desc"], "gaussians": n, "width": W, "height": H, "sh_degree": deg,
                   "views_per_step": world, "parallelism": f"dp{world} (one view per GPU, gradient exchange: "
                                                  f"{red.describe() if distributed else 'none'})",
                   "instances_per_view": I, "sum_n_contrib": sum_contrib,
                   "stage_events": (f"timed steps: dominant kernel only, every {EVENT_EVERY}th step; stages_ms: "
                                    "separate untimed pass"
                                    if use_events else "none")},
        **({"distributed": {"backend": dist.get_backend(), "world_size": world, "exchange": red.describe(),
                            "plan": red.plan,
                            "note": "process group initialised: every step ran the exchange's collectives"}}
           if distributed else {}),
        # also the contributing (pixel, Gaussian) pairs per second (this rank's sum(n_contrib) x N)
        "contrib_pairs_per_s": world * sum_contrib / (ms_per_step * 1e-3),
        "step_events_ms": step_events,
        "roofline": roofline, "cpu_baseline": cpu, "train_step": train,
        "stages_ms": {k: round(v, 4) for k, v in stage_avg.items() if v > 0},
    }
    if rank == 0:
        print(json.dumps(line), flush=True)
    if distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
