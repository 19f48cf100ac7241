"""The N>1 path (one view per rank + gradient exchange), world_size 2 over gloo on CPU.

Reduced gradients must equal the sum of the single-view gradients (SURVEY.md §8(e) parity check), the
densification statistics must be formed per view before the exchange, and radii must be max-reduced.
Both exchange modes of gaussian_splatting_lightning_amd/multiview.py are covered; the compact mode's SH
expansion runs in the oracle here (its HIP kernel is checked in tests/test_gpu_parity.py)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from tests import multiview_worker as MW


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture(scope="module")
def expected():
    world = 2
    views = [MW.oracle_view(v, world) for v in range(world)]
    exp = {k: sum(v[k] for v in views) for k in ("means3D", "scales", "rotations", "opacities", "shs")}
    exp["stats0"] = sum(np.linalg.norm(v["means2D"][:, :2], axis=1) for v in views)
    exp["stats1"] = sum((v["radii"] > 0).astype(np.float32) for v in views)
    exp["radii_max"] = np.maximum(views[0]["radii"], views[1]["radii"])
    return exp


def _run(tmp_path, mode, chunks, world=2, expand="chunk", expand_sh=True):
    ctx = mp.get_context("spawn")
    port = _free_port()
    d = os.path.join(str(tmp_path), f"{mode}_{chunks}_{expand}_{expand_sh}")
    os.makedirs(d, exist_ok=True)
    procs = [ctx.Process(target=MW.worker, args=(r, world, port, mode, d, chunks, expand, expand_sh))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
        assert p.exitcode == 0, f"rank exited with {p.exitcode}"
    return [dict(np.load(os.path.join(d, f"rank{r}.npz"))) for r in range(world)]


@pytest.mark.parametrize("mode", ["dense", "compact"])
def test_two_rank_exchange(tmp_path, expected, mode):
    world = 2
    res = _run(tmp_path, mode, 1, world)
    for k in ("means3D", "scales", "rotations", "opacities", "stats", "radii_max", "shs"):
        assert np.array_equal(res[0][k], res[1][k]), k  # every rank ends with the same reduced state
    r = res[0]
    for k in ("means3D", "scales", "rotations", "opacities"):
        np.testing.assert_allclose(r[k], expected[k].reshape(r[k].shape), rtol=1e-6, atol=1e-12, err_msg=k)
    # SH: dense sums the per-view dL/dsh; compact re-expands basis (x) dRGB_v -- identical products up to
    # the direction normalisation's rounding.
    np.testing.assert_allclose(r["shs"], expected["shs"], rtol=1e-5, atol=1e-9)
    np.testing.assert_allclose(r["stats"][:, 0], expected["stats0"], rtol=1e-6)
    assert np.array_equal(r["stats"][:, 1], expected["stats1"])
    assert np.array_equal(r["radii_max"], expected["radii_max"])
    assert (expected["stats1"] == 2).any() and (expected["stats1"] == 1).any()  # views overlap only partly


@pytest.mark.parametrize("expand_sh", [True, False])
def test_sharded_exchange(tmp_path, expected, expand_sh):
    """The sharded (ZeRO-style) exchange: rank r ends with ITS shard [g0, g1) of every reduced field -- the same sums
    as the all-reduce of the compact exchange, bitwise (two summands) -- and the SH gradient of its shard, expanded
    from every view's colour factors delivered by the all-to-all (or, expand_sh=False, the factored form the fused SH
    Adam takes); the shards tile [0, n); statistics and radii are the full reduced arrays on every rank."""
    comp = _run(tmp_path, "compact", 1)
    res = _run(tmp_path, "sharded", 1, expand_sh=expand_sh)
    bounds = [tuple(int(x) for x in r["shard"]) for r in res]
    assert bounds[0][0] == 0 and bounds[-1][1] == MW.N and all(a[1] == b[0] for a, b in zip(bounds, bounds[1:]))
    for r, (g0, g1) in enumerate(bounds):
        for k in ("means3D", "scales", "rotations", "opacities", "shs"):
            assert np.array_equal(res[r][k], comp[r][k][g0:g1]), (r, k)
        for k in ("stats", "radii_max"):
            assert np.array_equal(res[r][k], comp[r][k]), (r, k)
        np.testing.assert_allclose(res[r]["means3D"], expected["means3D"][g0:g1].reshape(res[r]["means3D"].shape),
                                   rtol=1e-6, atol=1e-12)


@pytest.mark.parametrize("mode", ["dense", "compact"])
def test_chunked_exchange_is_bitwise_the_unchunked_one(tmp_path, mode):
    """The overlapped exchange (Gaussian chunks, one all-reduce + all-gather per chunk issued as the chunk's
    gradients appear) sums exactly the same per-rank values per element as the single exchange after the
    backward: the reduced gradients, statistics and radii are bitwise equal for K = 1 and K = 4."""
    one = _run(tmp_path, mode, 1)
    four = _run(tmp_path, mode, 4)
    for r in range(2):
        for k in ("means3D", "scales", "rotations", "opacities", "stats", "radii_max", "shs"):
            assert np.array_equal(one[r][k], four[r][k]), (r, k)
    if mode == "compact":  # one SH expansion over the chunk-major gather buffer after the last chunk: same bits
        once = _run(tmp_path, mode, 4, expand="once")
        for r in range(2):
            for k in ("means3D", "scales", "rotations", "opacities", "stats", "radii_max", "shs"):
                assert np.array_equal(one[r][k], once[r][k]), (r, k)


@pytest.mark.parametrize("chunks", [1, 4])
def test_factored_sh_gradient_is_the_expanded_one(tmp_path, chunks):
    """finish(expand_sh=False): no expansion on the ranks; the factored SH gradient the fused Adam consumes
    (sh_views_gradient: every rank's colour factors in the chunk-major gather buffer, every rank's camera) expands to
    exactly what the expanding exchange produced, on every rank."""
    ref = _run(tmp_path, "compact", chunks)
    fac = _run(tmp_path, "compact", chunks, expand_sh=False)
    for r in range(2):
        for k in ("means3D", "scales", "rotations", "opacities", "stats", "radii_max", "shs"):
            assert np.array_equal(ref[r][k], fac[r][k]), (r, k)


def test_exchange_plan_cost_model():
    """plan_exchange: per-rank link bytes follow the ring formulas (413 B/G dense, 161 B/G compact
    at 8 ranks, SH 3); more ranks never pick dense over compact; the predicted end time is monotone in the assumed
    bus bandwidth; every simulated schedule ends no earlier than its compute and its communication."""
    from gaussian_splatting_lightning_amd.multiview import (exchange_bytes_per_gaussian, plan_exchange,
                                                            simulate_exchange)
    assert abs(exchange_bytes_per_gaussian("dense", 8) - 413.0) < 0.01
    assert abs(exchange_bytes_per_gaussian("compact", 8) - 161.0) < 0.01
    assert abs(exchange_bytes_per_gaussian("sharded", 8) - 49.0) < 0.01
    assert exchange_bytes_per_gaussian("compact", 1) == 0.0
    assert exchange_bytes_per_gaussian("sharded", 1) == 0.0
    for N in (2, 4, 8):
        p = plan_exchange(1_000_000, N)
        assert p["mode"] == "sharded", (N, p)
        assert plan_exchange(1_000_000, N, modes=("compact", "dense"))["mode"] == "compact"
        slow = plan_exchange(1_000_000, N, costs=dict(bus_efficiency=0.2))
        assert slow["end_ms"] > p["end_ms"]
    assert plan_exchange(1_000_000, 1)["mode"] == "dense"  # one rank: nothing crosses a link
    for mode in ("dense", "compact", "sharded"):
        for K in (1, 2, 4, 8):
            for expand in ("chunk", "once"):
                r = simulate_exchange(1_000_000, 8, mode, K, expand)
                assert r["end_ms"] >= r["comm_ms"] and r["end_ms"] >= r["per_gaussian_stage_ms"]


def test_unchunk_factors_round_trip():
    import torch
    from gaussian_splatting_lightning_amd.multiview import chunk_bounds, unchunk_factors
    V, n = 3, 1000
    full = torch.randn(V, n, 3)
    for K in (1, 2, 4):
        b = chunk_bounds(n, K)
        L = b[0][1] - b[0][0]
        flat = torch.cat([full[:, g0:g1].reshape(-1) for g0, g1 in b])
        assert torch.equal(unchunk_factors(flat, V, n, L), full)


def test_one_rank_group_takes_the_collective_path_and_guards_resync():
    """A process group of ONE rank still runs the exchange's collectives (the code path an N-GPU node runs), with the
    local path's results; statistics accumulated after sync_densify_stats and before reset_densify_stats raise (a
    second reduction would add the other ranks' views twice)."""
    import torch
    import torch.distributed as dist
    from gaussian_splatting_lightning_amd.multiview import ViewGradReducer
    if dist.is_initialized():
        pytest.skip("a process group already exists in this process")
    n = 1000
    g = torch.Generator().manual_seed(0)
    dm = torch.randn(n, 3, generator=g)
    radii = torch.randint(0, 5, (n,), generator=g, dtype=torch.int32)
    local = ViewGradReducer(n, 16, 3, "cpu", mode="dense", chunks=3)
    assert not local.distributed
    dist.init_process_group("gloo", store=dist.HashStore(), rank=0, world_size=1)
    try:
        red = ViewGradReducer(n, 16, 3, "cpu", mode="dense", chunks=3)
        assert red.distributed and red.world == 1
        for r in (local, red):
            r.record_view(dm, radii)
            r.flat.copy_(torch.arange(r.flat.numel(), dtype=torch.float32))
            r.begin_step(torch.zeros(3))
            for c in range(r.chunks):
                r.start_chunk(c)
            r.finish(None)
        assert torch.equal(local.flat, red.flat)
        s_red, m_red = red.sync_densify_stats()
        s_loc, m_loc = local.sync_densify_stats()
        assert torch.equal(s_red, s_loc) and torch.equal(m_red, m_loc)
        with pytest.raises(RuntimeError):
            red.record_view(dm, radii)
        red.reset_densify_stats()
        red.record_view(dm, radii)
    finally:
        dist.destroy_process_group()


class _CountingWork:
    def __init__(self):
        self.waits = 0

    def wait(self):
        self.waits += 1


@pytest.mark.parametrize("mode", ["dense", "compact"])
@pytest.mark.parametrize("shape", ["one_object", "separate", "no_gather"])
@pytest.mark.parametrize("chunks", [1, 3])
def test_finish_waits_on_every_collective_once(mode, shape, chunks):
    """finish() waits on each chunk's collectives exactly once, whatever the work objects look like: ONE object for a
    chunk's gather and reduce (a coalesced async group, or the side stream's event -- both hand back the same object
    twice), two objects, or a reduce alone (dense without a gather).  Dense mode once skipped every reduce that was
    the same object as its gather, so nothing waited and the optimizer could read a half-reduced buffer; a one-rank
    group cannot show that (its in-place sum leaves the data unchanged), hence the counting works here."""
    import torch
    from gaussian_splatting_lightning_amd.multiview import ViewGradReducer
    red = ViewGradReducer(2048, 16, 3, "cpu", mode=mode, chunks=chunks)
    red.distributed = True  # collectives mocked below: no process group needed
    issued = []

    def issue(c):
        g, r = _CountingWork(), _CountingWork()
        pair = {"one_object": (g, g), "separate": (g, r), "no_gather": (None, r)}[shape]
        issued.append(pair)
        return pair

    red._issue = issue
    red._sh_views = lambda *a, **k: None  # the SH expansion itself is not under test
    red.begin_step(torch.zeros(3))
    for c in range(red.chunks):
        red.start_chunk(c)
    red.finish(torch.zeros(2048, 3))
    assert len(issued) == red.chunks
    for g, r in issued:
        for w in {id(x): x for x in (g, r) if x is not None}.values():
            assert w.waits == 1, (mode, shape, chunks, w.waits)
    assert red._pending == []


def test_compact_exchange_refuses_an_unwritten_camera_block():
    """Without campos in begin_step and without handing the camera destination to a backward, chunk 0's all-reduce
    would sum the previous step's already-reduced camera rows again: the reducer raises instead."""
    import torch
    from gaussian_splatting_lightning_amd.multiview import ViewGradReducer
    red = ViewGradReducer(1024, 16, 3, "cpu", mode="compact", chunks=1)
    red.distributed = True
    red._issue = lambda c: (None, None)
    red._sh_views = lambda *a, **k: None
    red.begin_step()
    with pytest.raises(RuntimeError, match="camera block"):
        red.start_chunk(0)
    red._pending = []
    red.backward_out()  # the backward now writes the block
    red.start_chunk(0)
    red.finish(torch.zeros(1024, 3))
    red.begin_step()  # the next step starts unwritten again
    with pytest.raises(RuntimeError, match="camera block"):
        red.start_chunk(0)
