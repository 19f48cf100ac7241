"""World-size-N worker for tests/test_multiview.py (gloo on CPU).  Each rank renders its own view with the
oracle (test infrastructure: the HIP path needs a GPU), fills a ViewGradReducer from it and runs the exchange."""
from __future__ import annotations

import os

import numpy as np
import torch
import torch.distributed as dist

N, W, H, DEG = 1500, 96, 64, 3


def view_inputs(view, world):
    from tests.helpers import scene_inputs
    return scene_inputs(N, W, H, sh_degree=DEG, seed=3, view_index=view, num_views=world)


def oracle_view(view, world):
    """Per-view oracle gradients plus the per-view densification inputs."""
    from tests.helpers import run_oracle, upstream
    inp = view_inputs(view, world)
    _, radii, _, run = run_oracle(inp)
    dc, di = upstream(W, H, seed=view)
    g = run.backward(dc, di)
    g["colors_sh"] = g["colors"] * (1 - run.clamped()).astype(np.float32)
    g["radii"] = radii
    g["campos"] = inp["campos"]
    g["means3D_in"] = inp["means3D"]
    return g


def oracle_sh_views(means3D, campos, dcolors_sh, sh_degree, M, out, chunk_len=0):
    from gaussian_splatting_lightning_amd.multiview import unchunk_factors
    from oracle import oracle as O
    d = unchunk_factors(dcolors_sh, campos.shape[0], means3D.shape[0], chunk_len)
    r = O.sh_backward_views(means3D.numpy(), campos.numpy(), d.numpy(), sh_degree, M)
    out.copy_(torch.from_numpy(r))
    return out


def worker(rank, world, port, mode, result_dir, chunks=1, expand="chunk", expand_sh=True):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from gaussian_splatting_lightning_amd.multiview import ViewGradReducer
        g = oracle_view(rank, world)
        red = ViewGradReducer(N, 16, DEG, "cpu", mode=mode, sh_views_fn=oracle_sh_views, chunks=chunks,
                              expand=expand)
        means3D = torch.from_numpy(g["means3D_in"])

        def fill(out, g0, g1):  # what the backward writes for Gaussians [g0, g1)
            for k in ("means3D", "scales", "rotations", "opacities"):
                out[k].copy_(torch.from_numpy(g[k][g0:g1]).reshape(out[k].shape))
            if red.compact or red.sharded:
                out["colors_sh"].copy_(torch.from_numpy(g["colors_sh"][g0:g1]))
            else:
                out["shs"].copy_(torch.from_numpy(g["shs"][g0:g1]).reshape(out["shs"].shape))

        red.means2D.copy_(torch.from_numpy(g["means2D"]))
        if red.sharded:  # unchunked; this rank ends with its shard of every reduced field
            fill(red.backward_out(), 0, N)
            red.reduce(means3D, torch.from_numpy(g["campos"]), expand_sh=expand_sh)
        elif red.chunks == 1:
            fill(red.backward_out(), 0, N)
            red.reduce(means3D, torch.from_numpy(g["campos"]), expand_sh=expand_sh)
        else:  # the overlapped form: each chunk's exchange starts as soon as its gradients exist
            red.begin_step(torch.from_numpy(g["campos"]))
            for c, (g0, g1, out) in enumerate(red.chunk_outputs()):
                fill(out, g0, g1)
                red.start_chunk(c)
            red.finish(means3D, expand_sh=expand_sh)
        red.record_view(red.means2D, torch.from_numpy(g["radii"]))
        grads = red.grads
        if not expand_sh:  # the factored form GaussianAdam.step(sh_views=...) consumes, expanded here by the oracle
            assert grads["shs"] is None
            f = red.sh_views_gradient(means3D)
            grads["shs"] = oracle_sh_views(f.means3D, f.campos, f.factors, f.sh_degree, 16,
                                           torch.zeros(f.means3D.shape[0], 16, 3), f.chunk_len)
        res = {k: v.numpy() for k, v in grads.items()}
        res["shard"] = np.array(red.shard if red.sharded else (0, N))
        stats, radii_max = red.sync_densify_stats()
        res["stats"] = stats.numpy()
        res["radii_max"] = radii_max.numpy()
        np.savez(os.path.join(result_dir, f"rank{rank}.npz"), **res)
    finally:
        dist.destroy_process_group()
