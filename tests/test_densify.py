"""Adaptive density control (prune / clone / split + optimizer-state re-indexing) and the fused Adam.

CPU: the numpy oracle (oracle/densify_oracle.py) against an independent torch restatement of the reference's
lines (gs_lightning/modules/gaussian_model.py:184-287, gs_lightning_module.py:213-235), argument validation of
the C-ABI, and the no-fallback rule.  GPU: gaussian_splatting_lightning_amd.densify / .optim against the oracle
and against torch.optim.Adam.

Tolerances: row selection, ordering and preserve_idx are exact; copied rows are bit-exact; split rows (xyz moved
by R(q)(z*exp(s)), scaling log(exp(s)/1.6)) within 2e-6 relative + 1e-6 absolute (fp32 transcendentals and
summation order).  Adam: 1e-5 relative / 1e-7 absolute after 10 steps (fp32 contraction differences).
"""
import ctypes

import numpy as np
import pytest
import torch
from torch import nn

from gaussian_splatting_lightning_amd import _native
from oracle import densify_oracle

NAMES = densify_oracle.PARAMETER_NAMES
WIDTHS = dict(xyz=(3,), features_dc=(1, 3), features_rest=(15, 3), opacity=(1,), scaling=(3,), rotation=(4,))


def make_scene(N, seed=0, rest=15):
    rng = np.random.default_rng(seed)
    f32 = np.float32
    count = rng.integers(0, 6, N).astype(f32)
    p = dict(
        xyz=rng.normal(size=(N, 3)).astype(f32),
        features_dc=rng.normal(size=(N, 1, 3)).astype(f32),
        features_rest=rng.normal(size=(N, rest, 3)).astype(f32),
        opacity=rng.uniform(-4, 4, (N, 1)).astype(f32),
        scaling=rng.uniform(np.log(0.001), np.log(0.5), (N, 3)).astype(f32),
        rotation=rng.normal(size=(N, 4)).astype(f32),
    )
    s = dict(max_radii2D=rng.uniform(0, 40, N).astype(f32),
             xyz_grad_accum=(count * rng.uniform(0, 0.0004, N)).astype(f32),
             xyz_grad_count=count)
    return p, s


THRESH = [
    # (grad, clone_size, prune_opacity, prune_size, prune_screensize, use_screensize)
    (0.0002, 0.01, 0.05, 0.4, 20.0, True),
    (0.0002, 0.01, 0.05, 0.4, None, True),
    (0.0002, 0.01, 0.05, 0.4, 20.0, False),
    (0.0, 0.0, 0.005, 10.0, None, True),     # every kept row with a finite gradient splits
    (1.0, 0.01, 0.99, 0.4, None, True),      # almost everything pruned, nothing densified
]


class Model(nn.Module):
    """The attributes of the reference GaussianModel that densification touches."""

    def __init__(self, p, s, device, spatial_scale=1.0, use_screensize_threshold=True):
        super().__init__()
        for k in NAMES:
            setattr(self, f"_{k}", nn.Parameter(torch.tensor(p[k], device=device)))
        for k, v in s.items():
            self.register_buffer(k, torch.tensor(v, device=device))
        self.spatial_scale = spatial_scale
        self.use_screensize_threshold = use_screensize_threshold


def torch_restatement(p, s, spatial_scale, thr, generator):
    """The reference's densify_and_prune as torch ops on CPU tensors (kornia's matrix written out)."""
    grad_t, clone_t, op_t, size_t, ss_t, use_ss = thr
    P = {k: torch.tensor(v) for k, v in p.items()}
    S = {k: torch.tensor(v) for k, v in s.items()}
    keep = (torch.sigmoid(P["opacity"]) > op_t).squeeze(-1)
    if ss_t is not None:
        if use_ss:
            keep = torch.logical_and(keep, S["max_radii2D"] < ss_t)
        gsize = torch.max(torch.exp(P["scaling"]), dim=1)[0]
        keep = torch.logical_and(keep, gsize < size_t * spatial_scale)
    P = {k: v[keep] for k, v in P.items()}
    S = {k: v[keep] for k, v in S.items()}
    g = S["xyz_grad_accum"] / S["xyz_grad_count"]
    g[g.isnan()] = 0.0
    bad = g >= grad_t
    gsize = torch.max(torch.exp(P["scaling"]), dim=1)[0]
    small = torch.logical_and(bad, gsize < clone_t * spatial_scale).nonzero().squeeze(-1)
    large = torch.logical_and(bad, gsize >= clone_t * spatial_scale).nonzero().squeeze(-1)

    def add(rows):
        for k in NAMES:
            P[k] = torch.cat([P[k], rows[k]], 0)
        for k in S:
            S[k] = torch.cat([S[k], torch.zeros(len(rows["xyz"]))])

    add({k: P[k][small].clone() for k in NAMES})
    std = torch.exp(P["scaling"][large])
    disp = torch.normal(mean=torch.zeros_like(P["xyz"][large]), std=std, generator=generator)
    q = torch.nn.functional.normalize(P["rotation"][large])
    R = torch.tensor(densify_oracle.quaternion_matrix(q.numpy()))
    P["xyz"][large] = P["xyz"][large] + torch.bmm(R, disp.unsqueeze(-1)).squeeze(-1)
    P["scaling"][large] = torch.log(torch.exp(P["scaling"][large]) / 1.6)
    add({k: P[k][large].clone() for k in NAMES})
    return P, S, keep.nonzero().squeeze(-1), (int(keep.sum()), len(small), len(large))


def close(a, b, rtol=2e-6, atol=1e-6):
    np.testing.assert_allclose(np.asarray(a), np.asarray(b), rtol=rtol, atol=atol)


@pytest.mark.parametrize("thr", THRESH)
def test_oracle_matches_torch_restatement(thr):
    p, s = make_scene(3000, seed=1)
    P_t, S_t, keep_t, counts_t = torch_restatement(p, s, 1.0, thr, torch.Generator().manual_seed(7))
    z = torch.empty((counts_t[2], 3)).normal_(0, 1, generator=torch.Generator().manual_seed(7)).numpy()
    P_o, S_o, _, keep_o, counts_o = densify_oracle.densify_and_prune(p, s, 1.0, *thr[:5],
                                                                     use_screensize_threshold=thr[5], z=z)
    assert counts_o == counts_t
    np.testing.assert_array_equal(keep_o, keep_t.numpy())
    for k in NAMES:
        close(P_o[k], P_t[k].numpy())
    for k in S_o:
        close(S_o[k], S_t[k].numpy())


def test_oracle_moments_reindexed():
    p, s = make_scene(500, seed=2)
    ramp = np.arange(500, dtype=np.float32)
    mom = {k: (np.ones(p[k].shape, np.float32) * ramp.reshape((-1,) + (1,) * (p[k].ndim - 1)),
               np.ones(p[k].shape, np.float32)) for k in NAMES}
    z_fn = lambda n: np.random.default_rng(0).normal(size=(n, 3)).astype(np.float32)  # noqa: E731
    P_o, _, M_o, keep, (nk, nc, ns) = densify_oracle.densify_and_prune(p, s, 1.0, *THRESH[1][:5],
                                                                       use_screensize_threshold=True, z=z_fn,
                                                                       moments=mom)
    assert nc > 0 and ns > 0
    assert len(P_o["xyz"]) == nk + nc + ns
    m, v = M_o["xyz"]
    np.testing.assert_array_equal(m[:nk, 0], keep.astype(np.float32))
    assert (m[nk:] == 0).all() and (v[nk:] == 0).all() and (v[:nk] == 1).all()


def test_abi_argument_validation_without_device():
    lib = _native.load()
    args = _native.DensifyArgs(N=-1)
    assert lib.gsr_densify_classify(ctypes.byref(args), None, 1, None, None) == 1
    assert b"densify" in lib.gsr_last_error()
    fields = (_native.DensifyField * 1)(_native.DensifyField(1, 1, None, None, None, None, 3, 9))
    assert lib.gsr_densify_apply(4, 1, 1, 1, None, fields, 1, None) == 1
    assert b"kind" in lib.gsr_last_error()
    groups = (_native.AdamGroup * 17)()
    assert lib.gsr_adam_step(groups, 17, 0.9, 0.999, 1e-15, None) == 1
    g = (_native.AdamGroup * 1)(_native.AdamGroup(1, 1, 1, 1, 10, 0.1, 0))
    assert lib.gsr_adam_step(g, 1, 0.9, 0.999, 1e-15, None) == 1
    assert b"step" in lib.gsr_last_error()
    assert lib.gsr_densify_workspace_bytes(1000) >= 1000 * 13


def test_no_cpu_fallback():
    from gaussian_splatting_lightning_amd.optim import GaussianAdam
    p = nn.Parameter(torch.zeros(4))
    p.grad = torch.ones(4)
    with pytest.raises(RuntimeError, match="GPU"):
        GaussianAdam([p], lr=0.1, eps=1e-15).step()
    from gaussian_splatting_lightning_amd.densify import densify_and_prune
    pp, ss = make_scene(10)
    with pytest.raises(RuntimeError, match="GPU"):
        densify_and_prune(Model(pp, ss, "cpu"), 0.0002, 0.01, 0.05, 0.4)


def sparse_adam_restatement(p, g, m, v, vis, M, lr, eps, b1=0.9, b2=0.999):
    """The upstream SparseGaussianAdam kernel (diff_gaussian_rasterization adamUpdate, the optimizer of the reference's
    third_party gaussian_model.py:194-196) as fp32 torch ops: only the visible Gaussians' elements change, no bias
    correction.  Parity unpinned: the package is an empty submodule here, so this restates its published kernel."""
    keep = vis.repeat_interleave(M).view(p.shape)
    f = torch.float32
    b1f, b2f = torch.tensor(b1, dtype=f), torch.tensor(b2, dtype=f)
    one = torch.tensor(1.0, dtype=f)  # the upstream kernel forms 1 - b in float (1 - 0.999f = 0.00099998713)
    m2 = b1f * m + (one - b1f) * g
    v2 = b2f * v + (one - b2f) * g * g
    p2 = p + (-lr) * m2 / (torch.sqrt(v2) + eps)
    return torch.where(keep, p2, p), torch.where(keep, m2, m), torch.where(keep, v2, v)


def test_sparse_adam_is_the_upstream_package_class_and_has_no_cpu_fallback():
    """`from diff_gaussian_rasterization import SparseGaussianAdam` (third_party gaussian_model.py:26) resolves to the
    HIP optimizer: upstream constructor (params, lr, eps), a torch.optim.Adam, and a loud error off the GPU."""
    from diff_gaussian_rasterization import SparseGaussianAdam
    p = nn.Parameter(torch.zeros(6, 3))
    opt = SparseGaussianAdam([{"params": [p], "lr": 0.01, "name": "xyz"}], lr=0.0, eps=1e-15)
    assert isinstance(opt, torch.optim.Adam) and opt.param_groups[0]["name"] == "xyz"
    opt.step(torch.ones(6, dtype=torch.bool), 6)  # no gradient yet: nothing to do, as upstream
    p.grad = torch.ones(6, 3)
    with pytest.raises(RuntimeError, match="GPU"):
        opt.step(torch.ones(6, dtype=torch.bool), 6)
    with pytest.raises(ValueError):
        opt.step(torch.ones(6, dtype=torch.bool), 0)
    # the restatement leaves invisible Gaussians untouched and matches dense Adam-without-bias-correction elsewhere
    g = torch.randn(6, 3)
    vis = torch.tensor([1, 0, 1, 0, 0, 1], dtype=torch.bool)
    z = torch.zeros(6, 3)
    p2, m2, v2 = sparse_adam_restatement(z, g, z, z, vis, 3, 0.01, 1e-15)
    assert torch.equal(p2[~vis], z[~vis]) and torch.equal(m2[~vis], z[~vis])
    torch.testing.assert_close(p2[vis], -0.01 * (0.1 * g[vis]) / (torch.sqrt(0.001 * g[vis] ** 2) + 1e-15))


# ---------------------------------------------------------------------------------------------------- GPU


@pytest.mark.gpu
def test_sparse_adam_matches_restatement():
    """SparseGaussianAdam.step(visibility, N) over the six reference groups (M = 3, 3, 45, 1, 3, 4 elements per
    Gaussian, so float4 accesses straddle Gaussians) for 5 steps with a fresh random visibility each step, one
    group without a gradient in one step: 1e-5 relative / 1e-7 absolute against the fp32 restatement (fp32
    contraction of the moment updates: 3e-8 absolute where m cancels to ~0), and the Gaussians never visible
    bitwise unchanged."""
    from diff_gaussian_rasterization import SparseGaussianAdam
    N = 20_001
    p, s = make_scene(N, seed=5)
    a = Model(p, s, "cuda")
    opt = _optimizer(a, SparseGaussianAdam)
    ref = {k: [getattr(a, f"_{k}").detach().clone(), None, None] for k in NAMES}
    for k in NAMES:
        ref[k][1] = torch.zeros_like(ref[k][0])
        ref[k][2] = torch.zeros_like(ref[k][0])
    lrs = {g["name"]: g["lr"] for g in opt.param_groups}
    gen = torch.Generator(device="cuda").manual_seed(1)
    never = torch.ones(N, dtype=torch.bool, device="cuda")
    for step in range(5):
        vis = torch.rand(N, device="cuda", generator=gen) < 0.6
        never &= ~vis
        for k in NAMES:
            prm = getattr(a, f"_{k}")
            if step == 2 and k == "rotation":
                prm.grad = None
                continue
            g = torch.randn(prm.shape, device="cuda", generator=gen) * 10 ** (-(step % 3))
            prm.grad = g.clone()
            M = prm.numel() // N
            ref[k] = list(sparse_adam_restatement(ref[k][0], g, ref[k][1], ref[k][2], vis, M, lrs[k], 1e-15))
        opt.step(vis, N)
    torch.cuda.synchronize()
    for k in NAMES:
        prm = getattr(a, f"_{k}")
        st = opt.state[prm]
        torch.testing.assert_close(prm.detach(), ref[k][0], rtol=1e-5, atol=1e-7)
        # moments near zero (m = 0.9 m + 0.1 g cancelling) differ by an ulp of the terms: absolute bars
        torch.testing.assert_close(st["exp_avg"], ref[k][1], rtol=1e-5, atol=1e-7)
        torch.testing.assert_close(st["exp_avg_sq"], ref[k][2], rtol=1e-5, atol=1e-9)
        assert float(st["step"]) == 0.0  # upstream never advances it
        rows = never.repeat_interleave(prm.numel() // N).view(prm.shape)
        assert torch.equal(prm.detach()[rows], torch.tensor(p[k], device="cuda")[rows]), k


def _optimizer(model, cls, lrs=None):
    lrs = lrs or dict(xyz=1.6e-4, features_dc=2.5e-3, features_rest=1.25e-4, opacity=0.025, scaling=5e-3,
                      rotation=1e-3)
    return cls([{"params": [getattr(model, f"_{k}")], "lr": lrs[k], "name": k} for k in NAMES], lr=0.0, eps=1e-15)


@pytest.mark.gpu
def test_gaussian_adam_matches_torch_adam():
    from gaussian_splatting_lightning_amd.optim import GaussianAdam
    p, s = make_scene(20_001, seed=3)
    a, b = Model(p, s, "cuda"), Model(p, s, "cuda")
    opt_a, opt_b = _optimizer(a, GaussianAdam), _optimizer(b, torch.optim.Adam)
    gen = torch.Generator(device="cuda").manual_seed(0)
    for step in range(10):
        for k in NAMES:
            g = torch.randn(getattr(a, f"_{k}").shape, device="cuda", generator=gen) * 10 ** (-(step % 4))
            if step == 4 and k == "opacity":
                getattr(a, f"_{k}").grad = getattr(b, f"_{k}").grad = None  # a group without a gradient this step
                continue
            getattr(a, f"_{k}").grad = g.clone()
            getattr(b, f"_{k}").grad = g.clone()
        opt_a.step()
        opt_b.step()
    torch.cuda.synchronize()
    for k in NAMES:
        pa, pb = getattr(a, f"_{k}"), getattr(b, f"_{k}")
        torch.testing.assert_close(pa, pb, rtol=1e-5, atol=1e-7)
        sa, sb = opt_a.state[pa], opt_b.state[pb]
        assert float(sa["step"]) == float(sb["step"])
        torch.testing.assert_close(sa["exp_avg"], sb["exp_avg"], rtol=1e-5, atol=1e-9)
        torch.testing.assert_close(sa["exp_avg_sq"], sb["exp_avg_sq"], rtol=1e-5, atol=1e-12)


@pytest.mark.gpu
def test_gaussian_adam_non_contiguous_grad_and_misaligned_group():
    from gaussian_splatting_lightning_amd.optim import GaussianAdam
    base = torch.randn(1001, device="cuda")
    pa = nn.Parameter(base[1:].clone())                  # 1000 elements
    pb = nn.Parameter(base[1:].clone())
    buf = torch.zeros(1001, device="cuda")
    odd = buf[1:]                                        # misaligned storage offset
    odd.copy_(pa.detach())
    pc = nn.Parameter(odd)
    g = torch.randn(2000, device="cuda")[::2]            # non-contiguous gradient
    pa.grad, pb.grad, pc.grad = g, g.clone(), g
    GaussianAdam([pa, pc], lr=0.01, eps=1e-15).step()
    torch.optim.Adam([pb], lr=0.01, eps=1e-15).step()
    torch.testing.assert_close(pa, pb, rtol=1e-6, atol=1e-8)
    torch.testing.assert_close(pc, pb, rtol=1e-6, atol=1e-8)


def _gpu_vs_oracle(N, thr, seed, with_optimizer):
    from gaussian_splatting_lightning_amd.densify import densify_and_prune
    from gaussian_splatting_lightning_amd.optim import GaussianAdam
    p, s = make_scene(N, seed=seed)
    model = Model(p, s, "cuda", spatial_scale=1.3, use_screensize_threshold=thr[5])
    mom = None
    opt = None
    if with_optimizer:
        opt = _optimizer(model, GaussianAdam)
        rng = np.random.default_rng(seed + 1)
        mom = {}
        for k in NAMES:
            prm = getattr(model, f"_{k}")
            m = rng.normal(size=prm.shape).astype(np.float32)
            v = rng.uniform(0, 1, prm.shape).astype(np.float32)
            opt.state[prm] = dict(step=torch.tensor(5.0), exp_avg=torch.tensor(m, device="cuda"),
                                  exp_avg_sq=torch.tensor(v, device="cuda"))
            mom[k] = (m, v)
    keep = densify_and_prune(model, thr[0], thr[1], thr[2], thr[3], thr[4], optimizer=opt,
                             generator=torch.Generator(device="cuda").manual_seed(seed))
    torch.cuda.synchronize()
    # the oracle's z: the same draw from the same generator state
    def z_fn(n):
        gen = torch.Generator(device="cuda").manual_seed(seed)
        return torch.empty((n, 3), device="cuda").normal_(0, 1, generator=gen).cpu().numpy()

    P_o, S_o, M_o, keep_o, counts = densify_oracle.densify_and_prune(p, s, 1.3, *thr[:5],
                                                                     use_screensize_threshold=thr[5], z=z_fn,
                                                                     moments=mom)
    np.testing.assert_array_equal(keep.cpu().numpy(), keep_o)
    n_new = sum(counts)
    for k in NAMES:
        got = getattr(model, f"_{k}").detach().cpu().numpy()
        assert got.shape == (n_new,) + p[k].shape[1:]
        assert isinstance(getattr(model, f"_{k}"), nn.Parameter)
        if k in ("xyz", "scaling"):
            close(got, P_o[k])
        else:
            np.testing.assert_array_equal(got, P_o[k])
    for k in S_o:
        np.testing.assert_array_equal(getattr(model, k).cpu().numpy(), S_o[k])
    if with_optimizer:
        for k in NAMES:
            prm = getattr(model, f"_{k}")
            grp = [g for g in opt.param_groups if g["name"] == k][0]
            assert grp["params"][0] is prm and prm in opt.state
            st = opt.state[prm]
            assert float(st["step"]) == 5.0
            np.testing.assert_array_equal(st["exp_avg"].cpu().numpy(), M_o[k][0])
            np.testing.assert_array_equal(st["exp_avg_sq"].cpu().numpy(), M_o[k][1])
        assert len(opt.state) == len(NAMES)
    return counts


@pytest.mark.gpu
@pytest.mark.parametrize("thr", THRESH)
def test_densify_matches_oracle(thr):
    counts = _gpu_vs_oracle(5000, thr, seed=11, with_optimizer=False)
    assert sum(counts) > 0 or thr[2] > 0.9


@pytest.mark.gpu
def test_densify_reindexes_optimizer_and_training_continues():
    counts = _gpu_vs_oracle(70_000, THRESH[0], seed=5, with_optimizer=True)
    assert counts[1] > 0 and counts[2] > 0 and counts[0] < 70_000


@pytest.mark.gpu
def test_densify_edge_cases():
    from gaussian_splatting_lightning_amd.densify import densify_and_prune
    p, s = make_scene(0)
    m = Model(p, s, "cuda")
    assert densify_and_prune(m, 0.0002, 0.01, 0.05, 0.4, 20.0).numel() == 0
    assert m._xyz.shape == (0, 3)
    p, s = make_scene(1025, seed=4)
    p["opacity"][:] = -10.0                          # everything pruned
    m = Model(p, s, "cuda")
    assert densify_and_prune(m, 0.0002, 0.01, 0.05, 0.4).numel() == 0
    assert m._features_rest.shape == (0, 15, 3)


@pytest.mark.gpu
def test_split_draw_equals_torch_normal():
    """torch.normal(mean=0, std) == normal_(0, 1) * std for the same generator state (the split's z input)."""
    std = torch.rand(777, 3, device="cuda") + 0.1
    a = torch.normal(mean=torch.zeros_like(std), std=std, generator=torch.Generator(device="cuda").manual_seed(3))
    z = torch.empty(777, 3, device="cuda").normal_(0, 1, generator=torch.Generator(device="cuda").manual_seed(3))
    torch.testing.assert_close(a, z * std, rtol=0, atol=0)


@pytest.mark.parametrize("case,thr", [("screensize", (0.0002, 0.01, 0.05, 0.4, 20.0)),
                                      ("no_screensize", (0.0002, 0.01, 0.05, 0.4, None))])
def test_oracle_matches_reference_golden(case, thr):
    """tests/golden/densify_golden.npz: the reference's GaussianModel.densify_and_prune run on CPU tensors
    (make_golden_train.py); the split draw is replayed as manual_seed(seed) + normal_((n_split, 3))."""
    import os
    g = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "densify_golden.npz"))
    p = {k: g[f"in_{k}"] for k in NAMES}
    s = {k: g[f"in_{k}"] for k in ("max_radii2D", "xyz_grad_accum", "xyz_grad_count")}

    def z_fn(n):
        torch.manual_seed(int(g["seed"]))
        return torch.empty((n, 3)).normal_().numpy()

    P, S, _, keep, counts = densify_oracle.densify_and_prune(p, s, float(g["spatial_scale"]), *thr,
                                                             use_screensize_threshold=True, z=z_fn)
    np.testing.assert_array_equal(keep, g[f"{case}_preserve_idx"])
    assert counts[1] > 0 and counts[2] > 0
    for k in NAMES:
        if k in ("xyz", "scaling"):
            close(P[k], g[f"{case}_{k}"])
        else:
            np.testing.assert_array_equal(P[k], g[f"{case}_{k}"])
    for k in S:
        np.testing.assert_array_equal(S[k], g[f"{case}_{k}"])
