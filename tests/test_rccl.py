"""The RCCL exchange of multiview.py, executed on the GPU with a one-rank process group.

The gradient exchange of the one-view-per-GPU split (the reference consumes the reduced gradients
in gs_lightning/lightning/gs_lightning_module.py:167-169 and the per-view statistics of
gs_lightning/modules/gaussian_model.py:175-181) issues its collectives whenever a process group exists.  With one
rank every collective is an identity, so the reduced gradients, statistics and radii must be bitwise those of the
local (no-group) path -- and the RCCL calls themselves (`init_process_group("nccl", device_id=)`,
`all_gather_into_tensor`, the async all-reduce handles and their waits) run on real hardware.
"""
import pytest
import torch
import torch.distributed as dist

from tests.helpers import scene_inputs, settings_for, upstream

pytestmark = pytest.mark.gpu


def _step(red, st, rs, dc, di, means3D, chunked, early=True):
    from gaussian_splatting_lightning_amd.rasterizer import backward_chunked, backward_raw
    if chunked:  # early: SH expansions queued on the side stream behind each group (begin_step(means3D=...))
        red.begin_step(means3D=means3D if early else None)
        backward_chunked(st, rs, dc, di, red.chunk_outputs(), on_chunk=red.start_chunk, compact_sh=red.compact,
                         accumulate_stats=True)
        red.finish(means3D)
    else:
        backward_raw(st, rs, dc, di, **red.backward_kwargs())
        red.reduce(means3D, rs.campos if red.sharded else None)


def _run(dev, distributed, mode, chunks, views=2, early=True, **kw):
    from gaussian_splatting_lightning_amd.multiview import ViewGradReducer
    from gaussian_splatting_lightning_amd.rasterizer import forward_raw
    n, W, H = 30_000, 320, 240
    red = ViewGradReducer(n, 16, 3, dev, mode=mode, chunks=chunks, distributed=distributed, **kw)
    assert red.distributed == distributed
    for v in range(views):  # two steps: the statistics accumulate over views before the sync
        inp = scene_inputs(n, W, H, sh_degree=3, seed=12, stress_fraction=0.01, view_index=v, num_views=4)
        rs = settings_for(inp, dev)
        t = {k: torch.as_tensor(inp[k], device=dev) for k in ("means3D", "opacities", "scales", "rotations", "shs")}
        dc, di = (torch.as_tensor(a, device=dev) for a in upstream(W, H, seed=12 + v))
        _, radii, _, st = forward_raw(t["means3D"], t["shs"], None, t["opacities"], t["scales"], t["rotations"],
                                      None, rs)
        _step(red, st, rs, dc, di, t["means3D"], chunks > 1, early)
    torch.cuda.synchronize()
    grads = {k: g.clone() for k, g in red.grads.items()}
    stats, rmax = red.sync_densify_stats()
    torch.cuda.synchronize()
    return grads, stats.clone(), rmax.clone(), red


VARIANTS = [  # (mode, chunks, reducer options): one RCCL group per chunk unless coalesce=False
    ("compact", 4, {}), ("compact", 4, dict(expand="once")), ("dense", 4, {}), ("compact", 1, {}), ("dense", 1, {}),
    ("compact", 4, dict(coalesce=False)), ("compact", 1, dict(sync_ops=False)), ("dense", 1, dict(coalesce=False)),
    ("compact", 4, dict(comm_stream="pg")), ("compact", 2, dict(comm_stream="side", expand="once")),
    ("compact", 4, dict(expand="side")),  # each chunk's expansion on the side stream behind its group
    ("compact", 2, dict(expand="side", early=False)),  # "side" without means3D at begin_step: expands in finish()
    ("compact", 4, dict(handoff="value")), ("compact", 4, dict(expand="side", handoff="value")),
    ("dense", 2, dict(handoff="value")),  # stream-value hand-offs (gsr_stream_signal / gsr_stream_wait)
    ("sharded", 1, {}), ("sharded", 1, dict(coalesce=False)),  # reduce-scatter (+ cameras) and all-to-all
    ("sharded", 1, dict(one_group=False)),  # the reduce-scatter group and the all-to-all as two RCCL groups
]


@pytest.mark.parametrize("mode,chunks,kw", VARIANTS)
def test_rccl_exchange_one_rank_is_bitwise_local(gpu_device, mode, chunks, kw):
    ref = _run(gpu_device, False, mode, chunks)
    assert not dist.is_initialized()
    torch.cuda.set_device(gpu_device)
    dist.init_process_group("nccl", store=dist.HashStore(), rank=0, world_size=1, device_id=gpu_device)
    try:
        got = _run(gpu_device, True, mode, chunks, **kw)
        red = got[3]
        assert red.coalesce == kw.get("coalesce", True)  # the grouped path really ran (no fallback)
        if mode == "sharded":
            assert red.one_group == (kw.get("coalesce", True) and kw.get("one_group", True))
        if kw.get("handoff") == "value":
            assert red.handoff == "value"  # the device supports stream wait values: no silent event fallback
        if kw.get("expand") == "side" and kw.get("early", True):
            assert red._expanded == set(range(red.chunks))  # the expansions ran on the side stream
        # the RCCL branch really ran: the chunk gathers landed in the (world, L, 3) buffers
        if mode == "compact":
            for c in range(red.chunks):
                assert torch.equal(red.gather_all[c][0], red.gather_in[c])
        # a second reduction before reset would count other ranks' views twice: accumulating after a sync raises
        with pytest.raises(RuntimeError):
            red.begin_step(torch.zeros(3, device=gpu_device))
        red.reset_densify_stats()
        red.begin_step(torch.zeros(3, device=gpu_device))
        red.finish(None)  # nothing pending: returns at once
    finally:
        dist.destroy_process_group()
    for k in ref[0]:
        assert torch.equal(ref[0][k], got[0][k]), k
    assert torch.equal(ref[1], got[1])
    assert torch.equal(ref[2], got[2])
    assert float(got[1][:, 1].max()) == 2.0  # two views accumulated before the sync
