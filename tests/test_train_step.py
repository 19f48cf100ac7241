"""The multi-view training step's optimizer: the fused SH Adam (gsr_adam_sh_views_step) against the expansion
(gsr_sh_backward_views_chunked) followed by GaussianAdam, and the whole one-view-per-rank step (forward, backward,
compact exchange, Adam) on two gloo ranks sharing the GPU against the same step summed locally.

The reference steps torch.optim.Adam over its six parameter groups right after the backward
(gs_lightning/lightning/gs_lightning_module.py:114-134,168-170); with one view per GPU the SH groups' gradient is the
sum over views of basis(dir_v) (x) dRGB_v (multiview.py), which the fused step forms inside the update.
"""
import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _factors(P, V, chunk_len, seed, dev):
    """Chunk-major (V, L_c, 3) factor blocks with ~30 % all-zero rows (Gaussians a view did not render)."""
    g = torch.Generator().manual_seed(seed)
    full = torch.randn(V, P, 3, generator=g) * 1e-3
    full[torch.rand(V, P, generator=g) < 0.3] = 0.0
    if not chunk_len or chunk_len >= P:
        return full.reshape(-1).to(dev)
    parts = [full[:, g0:min(P, g0 + chunk_len)].reshape(-1) for g0 in range(0, P, chunk_len)]
    return torch.cat(parts).to(dev)


def _params(P, seed, dev, layout="packed"):
    g = torch.Generator().manual_seed(seed)
    dc = torch.randn(P, 1, 3, generator=g)
    rest = torch.randn(P, 15, 3, generator=g) * 0.1
    if layout == "misaligned":  # contiguous storage that starts 4 B past a 16-B boundary: the scalar element path
        buf = torch.empty(P * 45 + 1, device=dev)
        r = buf[1:].view(P, 15, 3)
        r.copy_(rest)
        return torch.nn.Parameter(dc.to(dev)), torch.nn.Parameter(r)
    if layout.startswith("joint"):  # the column blocks of one (P, 16, 3) tensor (what the forward reads as shs)
        shs = torch.cat([dc, rest], 1).to(dev)
        return shs[:, :1], shs[:, 1:]
    return torch.nn.Parameter(dc.to(dev)), torch.nn.Parameter(rest.to(dev))


@pytest.mark.parametrize("deg,chunk_len,layout", [(3, 0, "packed"), (3, 2560, "packed"), (1, 0, "packed"),
                                                  (0, 1024, "packed"), (3, 0, "misaligned"), (3, 2560, "joint"),
                                                  (2, 0, "joint"), (3, 0, "joint_packed_state")])
def test_fused_sh_adam_is_bitwise_expand_then_adam(gpu_device, deg, chunk_len, layout):
    from gaussian_splatting_lightning_amd.optim import GaussianAdam, ShViewsGradient
    from gaussian_splatting_lightning_amd.rasterizer import sh_backward_views
    dev = gpu_device
    P, V = 10_037, 5  # a partial last block and a partial last half-wave
    g = torch.Generator().manual_seed(7)
    means3D = torch.randn(P, 3, generator=g).to(dev)
    b_dc, b_rest = _params(P, 1, dev, layout)
    a_dc, a_rest = (torch.nn.Parameter(t.detach().clone()) for t in (b_dc, b_rest))
    groups = lambda d, r: [{"params": [d], "lr": 0.0025, "name": "f_dc"},  # noqa: E731
                           {"params": [r], "lr": 0.0025 / 20.0, "name": "f_rest"}]
    opt_a = GaussianAdam(groups(a_dc, a_rest), lr=0.0, eps=1e-15)
    opt_b = GaussianAdam(groups(b_dc, b_rest), lr=0.0, eps=1e-15)
    if layout == "joint_packed_state":  # a joint parameter whose moments are tensors of their own (layout 1)
        for t in (b_dc, b_rest):
            opt_b.state[t].update(step=torch.tensor(0.0), exp_avg=torch.zeros(t.shape, device=dev),
                                  exp_avg_sq=torch.zeros(t.shape, device=dev))
    for step in range(3):
        campos = (torch.randn(V, 3, generator=g) * 3.0).to(dev)
        f = _factors(P, V, chunk_len, 100 + step, dev)
        dsh = sh_backward_views(means3D, campos, f if chunk_len else f.view(V, P, 3), deg, 16, chunk_len=chunk_len)
        a_dc.grad = dsh[:, :1].contiguous()
        a_rest.grad = dsh[:, 1:].contiguous()
        opt_a.step()
        opt_b.step(sh_views=(b_dc, b_rest, ShViewsGradient(means3D, campos, f, deg, chunk_len)))
    torch.cuda.synchronize()
    assert torch.equal(a_dc, b_dc) and torch.equal(a_rest, b_rest)
    for pa, pb in ((a_dc, b_dc), (a_rest, b_rest)):
        for k in ("exp_avg", "exp_avg_sq"):
            assert torch.equal(opt_a.state[pa][k], opt_b.state[pb][k]), k
        assert int(opt_b.state[pb]["step"]) == 3
    moved = a_rest if deg > 0 else a_dc  # degree 0: the higher coefficients see zero gradients and stay
    assert not torch.equal(moved.detach().cpu(), _params(P, 1, "cpu")[0 if deg == 0 else 1].detach())
    if layout.startswith("joint"):
        assert b_dc.data_ptr() + 12 == b_rest.data_ptr()  # updated in place, still one tensor
    if layout == "joint":  # the moments were made joint too (one coalesced stream per array)
        assert opt_b.state[b_rest]["exp_avg"].data_ptr() == opt_b.state[b_dc]["exp_avg"].data_ptr() + 12


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


N, W, H = 20_000, 256, 192
LRS = dict(means3D=1.6e-4, scales=5e-3, rotations=1e-3, opacities=5e-2, f_dc=2.5e-3, f_rest=1.25e-4)


def _scene(dev):
    from tests.helpers import scene_inputs
    inp = scene_inputs(N, W, H, sh_degree=3, seed=31)
    t = {k: torch.as_tensor(inp[k], device=dev) for k in ("means3D", "opacities", "scales", "rotations", "shs")}
    return t


def _view(v, dev):
    from tests.helpers import scene_inputs, settings_for, upstream
    inp = scene_inputs(N, W, H, sh_degree=3, seed=31, view_index=v, num_views=4)
    dc, di = (torch.as_tensor(a, device=dev) for a in upstream(W, H, seed=40 + v))
    return settings_for(inp, dev), dc, di


def _optimizer(params):
    from gaussian_splatting_lightning_amd.optim import GaussianAdam
    return GaussianAdam([{"params": [params[k]], "lr": LRS[k], "name": k} for k in LRS], lr=0.0, eps=1e-15)


def _make_params(dev):
    t = _scene(dev)
    return {"means3D": torch.nn.Parameter(t["means3D"]), "scales": torch.nn.Parameter(t["scales"]),
            "rotations": torch.nn.Parameter(t["rotations"]), "opacities": torch.nn.Parameter(t["opacities"]),
            "f_dc": torch.nn.Parameter(t["shs"][:, :1].contiguous()),
            "f_rest": torch.nn.Parameter(t["shs"][:, 1:].contiguous())}


def train_step(params, opt, red, views, dev):
    """One data-parallel step: this rank's views (one per rank; several when summed locally), the exchange, then
    Adam on the rasterizer-input gradients with the SH groups in factored form."""
    from gaussian_splatting_lightning_amd.rasterizer import backward_chunked, backward_raw, forward_raw
    shs = torch.cat([params["f_dc"], params["f_rest"]], 1).detach().contiguous()
    for rs, dc, di in views:
        _, _, _, st = forward_raw(params["means3D"].detach(), shs, None, params["opacities"].detach(),
                                  params["scales"].detach(), params["rotations"].detach(), None, rs)
        if red.chunks == 1:
            backward_raw(st, rs, dc, di, **red.backward_kwargs())
            red.reduce(params["means3D"].detach(), expand_sh=False)
        else:
            red.begin_step()
            backward_chunked(st, rs, dc, di, red.chunk_outputs(), on_chunk=red.start_chunk, compact_sh=True,
                             accumulate_stats=True)
            red.finish(params["means3D"].detach(), expand_sh=False)
    g = red.grads
    for k in ("means3D", "scales", "rotations", "opacities"):
        params[k].grad = g[k].view_as(params[k])
    opt.step(sh_views=(params["f_dc"], params["f_rest"], red.sh_views_gradient(params["means3D"].detach())))


def train_step_sharded(full, own, opt, red, view, rank, dev):
    """The sharded (ZeRO-style) step: the exchange leaves this rank the reduced gradients of its shard, Adam steps the
    shard's rows of the padded parameters, and every rank's updated shard is all-gathered back."""
    from gaussian_splatting_lightning_amd.rasterizer import backward_raw, forward_raw
    rs, dc, di = view
    shs = torch.cat([full["f_dc"][:N], full["f_rest"][:N]], 1).contiguous()
    _, _, _, st = forward_raw(full["means3D"][:N], shs, None, full["opacities"][:N], full["scales"][:N],
                              full["rotations"][:N], None, rs)
    backward_raw(st, rs, dc, di, **red.backward_kwargs())
    red.reduce(full["means3D"][:N], rs.campos, expand_sh=False)
    g = red.grads
    for k in ("means3D", "scales", "rotations", "opacities"):
        own[k].grad = g[k].view_as(own[k])
    opt.step(sh_views=(own["f_dc"], own["f_rest"], red.sh_views_gradient(full["means3D"][:N])))
    red.gather_shards(list(full.values()))


def _rank_worker(rank, world, port, result, chunks, mode="compact"):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from gaussian_splatting_lightning_amd.multiview import ViewGradReducer
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        params = _make_params(dev)
        red = ViewGradReducer(N, 16, 3, dev, mode=mode, chunks=chunks)
        out = {}
        if mode == "sharded":  # parameters padded to the shards' rows, the optimizer over this rank's shard
            rows = red.padded_rows()
            full = {}
            for k, v in params.items():
                full[k] = torch.zeros((rows,) + tuple(v.shape[1:]), device=dev)
                full[k][:N] = v.detach()
            g0, g1 = red.shard
            own = {k: v[g0:g1] for k, v in full.items()}
            opt = _optimizer(own)
        else:
            opt = _optimizer(params)
        for step in range(2):
            if mode == "sharded":
                train_step_sharded(full, own, opt, red, _view(2 * step + rank, dev), rank, dev)
                torch.cuda.synchronize()
                out.update({f"{k}_{step}": v[:N].cpu().numpy() for k, v in full.items()})
                out.update({f"shardgrad_{k}_{step}": v.detach().cpu().numpy() for k, v in red.grads.items()
                            if v is not None})
                out["shard"] = np.array(red.shard)
                continue
            train_step(params, opt, red, [_view(2 * step + rank, dev)], dev)
            torch.cuda.synchronize()
            out.update({f"{k}_{step}": v.detach().cpu().numpy() for k, v in params.items()})
            out.update({f"grad_{k}_{step}": v.detach().cpu().numpy() for k, v in red.grads.items() if v is not None})
        np.savez(result.format(rank=rank), **out)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("chunks,mode", [(1, "compact"), (2, "compact"), (1, "sharded")])
def test_two_rank_train_step_matches_local_sum(gpu_device, tmp_path, chunks, mode):
    """Two gloo ranks on the one GPU, each rendering its own view per step, compact exchange + fused SH Adam (or the
    sharded exchange: each rank steps its shard, then the parameters are all-gathered), two steps: both ranks end with
    the same parameters, bitwise equal to one process that renders both views itself,
    sums their non-SH gradients, expands the SH gradient from both views' colour factors (gsr_sh_backward_views) and
    steps GaussianAdam on the expanded gradient."""
    import torch.multiprocessing as mp
    from gaussian_splatting_lightning_amd.rasterizer import backward_raw, forward_raw, sh_backward_views
    ctx = mp.get_context("spawn")
    port = _free_port()
    res = os.path.join(str(tmp_path), "rank{rank}.npz")
    procs = [ctx.Process(target=_rank_worker, args=(r, 2, port, res, chunks, mode)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
        assert p.exitcode == 0, f"rank exited with {p.exitcode}"
    got = [dict(np.load(res.format(rank=r))) for r in range(2)]
    for k in got[0]:
        if not k.startswith(("grad_", "shardgrad_", "shard")):
            _same(got[0][k], got[1][k], k)  # every rank holds the same parameters
    dev = gpu_device
    params = _make_params(dev)
    opt = _optimizer(params)
    f32 = dict(dtype=torch.float32, device=dev)
    for step in range(2):
        acc = {k: torch.zeros(N, w, **f32) for k, w in (("means3D", 3), ("scales", 3), ("rotations", 4),
                                                         ("opacities", 1))}
        factors = torch.zeros(2, N, 3, **f32)
        campos = torch.zeros(2, 3, **f32)
        shs = torch.cat([params["f_dc"], params["f_rest"]], 1).detach().contiguous()
        for j, v in enumerate((2 * step, 2 * step + 1)):
            rs, dc, di = _view(v, dev)
            _, _, _, st = forward_raw(params["means3D"].detach(), shs, None, params["opacities"].detach(),
                                      params["scales"].detach(), params["rotations"].detach(), None, rs)
            out = {k: torch.zeros_like(t) for k, t in acc.items()}
            out["colors_sh"] = factors[j]
            g = backward_raw(st, rs, dc, di, out=out, compact_sh=True)
            for k in acc:
                acc[k] += out[k]
            campos[j] = rs.campos
        for k in acc:
            params[k].grad = acc[k].view_as(params[k])
            if mode == "sharded":  # each rank holds the reduced gradients of its own shard
                for r in range(2):
                    g0, g1 = (int(x) for x in got[r]["shard"])
                    _same(got[r][f"shardgrad_{k}_{step}"], acc[k].view(N, -1)[g0:g1].cpu().numpy(),
                          f"rank {r} grad {k} step {step}")
            else:
                _same(got[0][f"grad_{k}_{step}"], acc[k].view(N, -1).cpu().numpy(), f"grad {k} step {step}")
        dsh = sh_backward_views(params["means3D"].detach(), campos, factors, 3, 16)
        params["f_dc"].grad = dsh[:, :1].contiguous()
        params["f_rest"].grad = dsh[:, 1:].contiguous()
        opt.step()
        torch.cuda.synchronize()
        for k, v in params.items():
            _same(got[0][f"{k}_{step}"], v.detach().cpu().numpy(), f"{k} step {step}")


def _same(a, b, what):
    a, b = np.asarray(a), np.asarray(b).reshape(np.asarray(a).shape)
    bad = a != b
    assert not bad.any(), (f"{what}: {int(bad.sum())} of {a.size} elements differ, max |diff| "
                           f"{float(np.abs(a - b).max()):.3e} (max |value| {float(np.abs(b).max()):.3e})")
