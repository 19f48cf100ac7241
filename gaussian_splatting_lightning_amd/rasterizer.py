"""Host-side mirror of the `diff_gaussian_rasterization` Python API, backed by libgsrast.so.

The reference calls this API at
    gs_lightning/lightning/gs_lightning_module.py:322-348   (training: settings, rasterizer(...), means2D grad)
    scripts/render_trained_image.py:98-124                  (inference: means2D=None)
    tests/rasterizer_python/test_mark_visible.py:13-14       (GaussianRasterizer(s).markVisible(points))
The names, argument meaning, return values and error behaviour are those of the upstream package
(graphdeco-inria/diff-gaussian-rasterization@dr_aa):
    GaussianRasterizationSettings   13-field NamedTuple
    GaussianRasterizer(settings)(means3D, means2D, opacities, shs, colors_precomp, scales, rotations,
                                 cov3D_precomp) -> (color (3,H,W), radii (P,) int32, invdepth (1,H,W))
    GaussianRasterizer.markVisible(positions) -> bool (P,)
    rasterize_gaussians(...)        functional form
Every computation runs in the HIP kernels on the tensors' device; the scratch state the backward needs
(geometry/binning/image buffers) lives in uint8 tensors saved on the autograd context.
"""
from __future__ import annotations

import ctypes
from typing import NamedTuple, Optional

import torch
import torch.nn as nn

from . import _native


class GaussianRasterizationSettings(NamedTuple):
    image_height: int
    image_width: int
    tanfovx: float
    tanfovy: float
    bg: torch.Tensor
    scale_modifier: float
    viewmatrix: torch.Tensor
    projmatrix: torch.Tensor
    sh_degree: int
    campos: torch.Tensor
    prefiltered: bool
    debug: bool
    antialiasing: bool


def _ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    if t is None or t.numel() == 0:
        return None
    return t.data_ptr()


def _prep(t: Optional[torch.Tensor], device, name: str) -> Optional[torch.Tensor]:
    if t is None or t.numel() == 0:
        return None
    if t.dtype != torch.float32:
        raise RuntimeError(f"{name} must be float32 (got {t.dtype})")
    if t.device != device:
        t = t.to(device)
    return t.contiguous()


class _Buffers:
    """Caller-owned scratch buffers grown through the C callback (reference: resizeFunctional).

    The callback is a closure over the buffer dict, not a bound method: a bound method would make a reference
    cycle (object -> callback -> method -> object), so the buffers (GBs at 5M Gaussians / 4K) would outlive the
    call until the cyclic garbage collector ran -- never, while it is disabled (bench.py's timed region),
    which ran the device out of memory.  An exception inside the callback (e.g. torch.OutOfMemoryError) is
    kept and re-raised after the library call; the callback then returns NULL, which the library reports as
    GSR_ERR_ALLOC (a ctypes callback that raises would hand the library an undefined pointer)."""

    def __init__(self, device):
        self.device = device
        self.bufs = bufs = {}
        self.errors = errors = []

        def alloc(_ctx, which, nbytes):
            try:
                t = torch.empty(max(int(nbytes), 1), dtype=torch.uint8, device=device)
            except BaseException as e:  # noqa: BLE001 -- re-raised by raise_pending()
                errors.append(e)
                return None
            bufs[int(which)] = t
            return t.data_ptr()

        self._cb = _native.ALLOC_FN(alloc)

    @property
    def callback(self):
        return self._cb

    def raise_pending(self):
        if self.errors:
            raise self.errors[0]

    def get(self, which) -> torch.Tensor:
        t = self.bufs.get(which)
        return t if t is not None else torch.empty(0, dtype=torch.uint8, device=self.device)


def _stream_handle(device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


class ForwardState(NamedTuple):
    """Everything the backward needs from one forward call (tensors kept alive by autograd)."""
    means3D: torch.Tensor
    shs: Optional[torch.Tensor]
    colors_precomp: Optional[torch.Tensor]
    opacities: torch.Tensor
    scales: Optional[torch.Tensor]
    rotations: Optional[torch.Tensor]
    cov3D_precomp: Optional[torch.Tensor]
    radii: torch.Tensor
    bg: torch.Tensor
    viewmatrix: torch.Tensor
    projmatrix: torch.Tensor
    campos: Optional[torch.Tensor]
    geom_buffer: torch.Tensor
    binning_buffer: torch.Tensor
    image_buffer: torch.Tensor
    num_rendered: int
    num_big: int
    M: int


def forward_raw(means3D, sh, colors_precomp, opacities, scales, rotations, cov3Ds_precomp, raster_settings):
    """One call of gsr_forward.  Returns (color (3,H,W), radii (P,), invdepth (1,H,W), ForwardState)."""
    lib = _native.load()
    device = means3D.device
    if device.type != "cuda":
        raise RuntimeError("the MI355X rasterizer needs its inputs on a HIP device (tensor.device.type == 'cuda')")
    if means3D.ndim != 2 or means3D.shape[1] != 3:
        raise RuntimeError("means3D must have dimensions (num_points, 3)")
    rs = raster_settings
    P = means3D.shape[0]
    H, W = int(rs.image_height), int(rs.image_width)
    means3D_c = _prep(means3D, device, "means3D")
    sh_c = _prep(sh, device, "shs")
    col_c = _prep(colors_precomp, device, "colors_precomp")
    op_c = _prep(opacities, device, "opacities")
    sc_c = _prep(scales, device, "scales")
    rot_c = _prep(rotations, device, "rotations")
    cov_c = _prep(cov3Ds_precomp, device, "cov3D_precomp")
    bg = _prep(rs.bg, device, "bg")
    view = _prep(rs.viewmatrix, device, "viewmatrix")
    proj = _prep(rs.projmatrix, device, "projmatrix")
    campos = _prep(rs.campos, device, "campos")
    M = 0 if sh_c is None else (sh_c.shape[1] if sh_c.ndim == 3 else sh_c.shape[1] // 3)

    # fully written by the library (render_fwd writes every pixel, preprocess every radius; P == 0 clears)
    color = torch.empty(3, H, W, dtype=torch.float32, device=device)
    invdepth = torch.empty(1, H, W, dtype=torch.float32, device=device)
    radii = torch.empty(P, dtype=torch.int32, device=device)
    bufs = _Buffers(device)
    a = _native.ForwardArgs(
        P=P, D=int(rs.sh_degree), M=M, W=W, H=H, background=_ptr(bg), means3D=_ptr(means3D_c),
        colors_precomp=_ptr(col_c), opacities=_ptr(op_c), scales=_ptr(sc_c),
        scale_modifier=float(rs.scale_modifier), rotations=_ptr(rot_c), cov3D_precomp=_ptr(cov_c),
        viewmatrix=_ptr(view), projmatrix=_ptr(proj), campos=_ptr(campos), tan_fovx=float(rs.tanfovx),
        tan_fovy=float(rs.tanfovy), shs=_ptr(sh_c), prefiltered=int(bool(rs.prefiltered)),
        antialiasing=int(bool(rs.antialiasing)), debug=int(bool(rs.debug)), out_color=color.data_ptr(),
        out_invdepth=invdepth.data_ptr(), radii=radii.data_ptr())
    num_rendered = ctypes.c_int64(0)
    with torch.cuda.device(device):  # the library also switches to its stream's device (gsr_api.hip)
        rc = lib.gsr_forward(ctypes.byref(a), bufs.callback, None, _stream_handle(device),
                             ctypes.byref(num_rendered))
    bufs.raise_pending()
    _native.check(rc, "rasterize_gaussians")
    state = ForwardState(means3D_c, sh_c, col_c, op_c, sc_c, rot_c, cov_c, radii, bg, view, proj, campos,
                         bufs.get(_native.GSR_BUF_GEOM), bufs.get(_native.GSR_BUF_BINNING),
                         bufs.get(_native.GSR_BUF_IMAGE), int(num_rendered.value), int(a.num_big_out), M)
    return color, radii, invdepth, state


def backward_raw(state: ForwardState, raster_settings, grad_out_color, grad_out_depth=None, out=None,
                 compact_sh=False, accumulate_stats=False):
    """One call of gsr_backward.  Returns a dict of gradients (means3D, means2D, shs, colors_precomp,
    opacities, scales, rotations, cov3D_precomp); entries are None where the input was absent.
    `out` may supply preallocated contiguous float32 destinations (e.g. views into one flat buffer that is
    then all-reduced): keys means2D (P,3), colors (P,3), opacities (P,1), means3D (P,3), cov3D (P,6),
    shs (P,M,3), scales (P,3), rotations (P,4), colors_sh (P,3), densify_stats (P,2) (|dL/dmeans2D[:2]| and
    radii > 0 of this view, gaussian_model.py:175-181), max_radii2D (P,) int32, and campos_rows = (rows (V,3),
    rank): the multi-view exchange's camera block, written by the backward (campos in row `rank`, zeros elsewhere).
    accumulate_stats=True adds this view's densify_stats to out["densify_stats"] (the reference's
    add_densification_stats); out["max_radii2D"] is always max-accumulated with this view's radii.
    compact_sh=True skips dL/dshs and returns the clamp-masked colour gradient "colors_sh" instead -- the
    per-view factor that `sh_backward_views` expands after an all-gather (multiview.py)."""
    lib = _native.load()
    rs = raster_settings
    st = state
    device = st.means3D.device
    P = st.means3D.shape[0]
    M = st.M
    H, W = int(rs.image_height), int(rs.image_width)
    if grad_out_color is None:
        grad_out_color = torch.zeros(3, H, W, dtype=torch.float32, device=device)
    grad_out_color = grad_out_color.to(torch.float32).contiguous()
    if grad_out_depth is not None:
        grad_out_depth = grad_out_depth.to(torch.float32).contiguous()
    f32 = dict(dtype=torch.float32, device=device)
    out = out or {}

    def dst(name, *shape):
        t = out.get(name)
        if t is None:
            return torch.empty(*shape, **f32)
        if tuple(t.shape) != shape or t.dtype != torch.float32 or not t.is_contiguous():
            raise RuntimeError(f"out[{name!r}] must be a contiguous float32 tensor of shape {shape}")
        return t

    dmeans2D = dst("means2D", P, 3)
    # dL/dcolors and dL/dcov3D are outputs only for precomputed colours / covariances (or when asked for)
    dcolors = dst("colors", P, 3) if (st.colors_precomp is not None or "colors" in out) else None
    dopac = dst("opacities", P, 1)
    dmeans3D = dst("means3D", P, 3)
    dcov = dst("cov3D", P, 6) if (st.cov3D_precomp is not None or "cov3D" in out) else None
    dsh = None if compact_sh else dst("shs", P, max(M, 0), 3)
    dcsh = dst("colors_sh", P, 3) if (compact_sh or "colors_sh" in out) else None
    dstats = dst("densify_stats", P, 2) if "densify_stats" in out else None
    mrad = out.get("max_radii2D")
    if mrad is not None and (tuple(mrad.shape) != (P,) or mrad.dtype != torch.int32 or not mrad.is_contiguous()):
        raise RuntimeError(f"out['max_radii2D'] must be a contiguous int32 tensor of shape ({P},)")
    dscales = dst("scales", P, 3)
    drot = dst("rotations", P, 4)
    cam_rows, cam_rank, cam_n = _campos_rows(out.get("campos_rows"))
    bufs = _Buffers(device)
    a = _native.BackwardArgs(
        P=P, D=int(rs.sh_degree), M=M, W=W, H=H, R=st.num_rendered, num_big=st.num_big, background=_ptr(st.bg),
        means3D=_ptr(st.means3D), colors_precomp=_ptr(st.colors_precomp), opacities=_ptr(st.opacities),
        scales=_ptr(st.scales), scale_modifier=float(rs.scale_modifier), rotations=_ptr(st.rotations),
        cov3D_precomp=_ptr(st.cov3D_precomp), viewmatrix=_ptr(st.viewmatrix), projmatrix=_ptr(st.projmatrix),
        campos=_ptr(st.campos), tan_fovx=float(rs.tanfovx), tan_fovy=float(rs.tanfovy),
        dL_dpix=grad_out_color.data_ptr(), dL_dinvdepth=_ptr(grad_out_depth), shs=_ptr(st.shs),
        radii=_ptr(st.radii), geom_buffer=_ptr(st.geom_buffer), binning_buffer=_ptr(st.binning_buffer),
        image_buffer=_ptr(st.image_buffer), antialiasing=int(bool(rs.antialiasing)), debug=int(bool(rs.debug)),
        dL_dmeans2D=dmeans2D.data_ptr(), dL_dcolors=_ptr(dcolors), dL_dopacity=dopac.data_ptr(),
        dL_dmeans3D=dmeans3D.data_ptr(), dL_dcov3D=_ptr(dcov), dL_dsh=_ptr(dsh),
        dL_dscales=dscales.data_ptr(), dL_drotations=drot.data_ptr(), dL_dcolors_sh=_ptr(dcsh),
        densify_stats=_ptr(dstats), densify_accumulate=int(bool(accumulate_stats)), max_radii2D=_ptr(mrad),
        campos_rows=cam_rows, campos_rank=cam_rank, campos_nrows=cam_n)
    with torch.cuda.device(device):
        rc = lib.gsr_backward(ctypes.byref(a), bufs.callback, None, _stream_handle(device))
    bufs.raise_pending()
    _native.check(rc, "rasterize_gaussians_backward")
    return dict(
        means3D=dmeans3D, means2D=dmeans2D,
        shs=dsh.view_as(st.shs) if (st.shs is not None and dsh is not None) else None, colors_sh=dcsh,
        colors_precomp=dcolors if st.colors_precomp is not None else None,
        colors=dcolors, opacities=dopac.view_as(st.opacities),
        scales=dscales if st.scales is not None else None,
        rotations=drot if st.rotations is not None else None,
        cov3D_precomp=dcov if st.cov3D_precomp is not None else None, cov3D=dcov)


def backward_chunked(state: ForwardState, raster_settings, grad_out_color, grad_out_depth, chunks, on_chunk=None,
                     compact_sh=False, accumulate_stats=False):
    """The backward split so that a gradient exchange overlaps it (multiview.py): ONE gsr_backward call for the
    compositing backward (GSR_BWD_COMPOSITE: instance gradient rows into a scratch buffer kept here), then one call
    per Gaussian chunk for the per-Gaussian stage (GSR_BWD_GAUSSIANS), each followed by on_chunk(k) -- which may
    issue collectives on the chunk's finished gradients while the next chunks compute.

    chunks: list of (g_begin, g_end, out) with out a dict of destinations for those Gaussians only (same keys and
    row widths as backward_raw's `out`, (g_end - g_begin) rows each, contiguous float32; max_radii2D int32).
    Results are bitwise those of one backward_raw call: every Gaussian is computed by the same code."""
    lib = _native.load()
    rs = raster_settings
    st = state
    device = st.means3D.device
    P, M = st.means3D.shape[0], st.M
    H, W = int(rs.image_height), int(rs.image_width)
    grad_out_color = grad_out_color.to(torch.float32).contiguous()
    if grad_out_depth is not None:
        grad_out_depth = grad_out_depth.to(torch.float32).contiguous()
    bufs = _Buffers(device)
    base = dict(
        P=P, D=int(rs.sh_degree), M=M, W=W, H=H, R=st.num_rendered, num_big=st.num_big, background=_ptr(st.bg),
        means3D=_ptr(st.means3D), colors_precomp=_ptr(st.colors_precomp), opacities=_ptr(st.opacities),
        scales=_ptr(st.scales), scale_modifier=float(rs.scale_modifier), rotations=_ptr(st.rotations),
        cov3D_precomp=_ptr(st.cov3D_precomp), viewmatrix=_ptr(st.viewmatrix), projmatrix=_ptr(st.projmatrix),
        campos=_ptr(st.campos), tan_fovx=float(rs.tanfovx), tan_fovy=float(rs.tanfovy),
        dL_dpix=grad_out_color.data_ptr(), dL_dinvdepth=_ptr(grad_out_depth), shs=_ptr(st.shs),
        radii=_ptr(st.radii), geom_buffer=_ptr(st.geom_buffer), binning_buffer=_ptr(st.binning_buffer),
        image_buffer=_ptr(st.image_buffer), antialiasing=int(bool(rs.antialiasing)), debug=int(bool(rs.debug)),
        densify_accumulate=int(bool(accumulate_stats)))
    with torch.cuda.device(device):
        a = _native.BackwardArgs(stages=_native.GSR_BWD_COMPOSITE, **base)
        rc = lib.gsr_backward(ctypes.byref(a), bufs.callback, None, _stream_handle(device))
        bufs.raise_pending()
        _native.check(rc, "rasterize_gaussians_backward (composite)")
        scratch = bufs.get(_native.GSR_BUF_BWD_SCRATCH)
        widths = dict(means2D=3, colors=3, opacities=1, means3D=3, cov3D=6, shs=3 * max(M, 0), scales=3, rotations=4,
                      colors_sh=3, densify_stats=2)
        for k, (g0, g1, out) in enumerate(chunks):
            n = int(g1) - int(g0)
            cam_rows, cam_rank, cam_n = _campos_rows(out.get("campos_rows"))
            for name, t in out.items():
                if name == "campos_rows":
                    continue
                want = (torch.int32, (n,)) if name == "max_radii2D" else (torch.float32, None)
                if t.dtype != want[0] or not t.is_contiguous() or t.shape[0] != n or (
                        name in widths and t.numel() != n * widths[name]):
                    raise RuntimeError(f"chunk {k}: out[{name!r}] must be a contiguous {want[0]} tensor of {n} rows")
            if compact_sh and "colors_sh" not in out and st.shs is not None:
                raise RuntimeError("compact_sh needs out['colors_sh'] in every chunk")
            a = _native.BackwardArgs(
                stages=_native.GSR_BWD_GAUSSIANS, g_begin=int(g0), g_end=int(g1), bwd_scratch=_ptr(scratch),
                dL_dmeans2D=_ptr(out.get("means2D")), dL_dcolors=_ptr(out.get("colors")),
                dL_dopacity=_ptr(out.get("opacities")), dL_dmeans3D=_ptr(out.get("means3D")),
                dL_dcov3D=_ptr(out.get("cov3D")), dL_dsh=None if compact_sh else _ptr(out.get("shs")),
                dL_dscales=_ptr(out.get("scales")), dL_drotations=_ptr(out.get("rotations")),
                dL_dcolors_sh=_ptr(out.get("colors_sh")), densify_stats=_ptr(out.get("densify_stats")),
                max_radii2D=_ptr(out.get("max_radii2D")), campos_rows=cam_rows, campos_rank=cam_rank,
                campos_nrows=cam_n, **base)
            rc = lib.gsr_backward(ctypes.byref(a), bufs.callback, None, _stream_handle(device))
            _native.check(rc, f"rasterize_gaussians_backward (chunk {k})")
            if on_chunk is not None:
                on_chunk(k)
    return scratch


def _campos_rows(spec):
    """(pointer, rank, rows) of an out["campos_rows"] = (rows (V, 3) contiguous float32, rank) entry."""
    if spec is None:
        return None, 0, 0
    rows, rank = spec
    if rows.dtype != torch.float32 or not rows.is_contiguous() or rows.ndim != 2 or rows.shape[1] != 3:
        raise RuntimeError("out['campos_rows'] must be (contiguous float32 (V, 3) tensor, rank)")
    if not 0 <= int(rank) < rows.shape[0]:
        raise RuntimeError(f"campos_rows rank {rank} outside [0, {rows.shape[0]})")
    return rows.data_ptr(), int(rank), int(rows.shape[0])


class _RasterizeGaussians(torch.autograd.Function):
    @staticmethod
    def forward(ctx, means3D, means2D, sh, colors_precomp, opacities, scales, rotations, cov3Ds_precomp,
                raster_settings):
        color, radii, invdepth, st = forward_raw(means3D, sh, colors_precomp, opacities, scales, rotations,
                                                 cov3Ds_precomp, raster_settings)
        ctx.raster_settings = raster_settings
        ctx.meta = (st.num_rendered, st.num_big, st.M)
        ctx.present = tuple(t is not None for t in st)
        empty = torch.empty(0, device=means3D.device)
        ctx.save_for_backward(*[(t if t is not None else empty) for t in st[:15]])
        ctx.set_materialize_grads(False)
        return color, radii, invdepth

    @staticmethod
    def backward(ctx, grad_out_color, _grad_radii, grad_out_depth):
        saved = ctx.saved_tensors
        tensors = [t if present else None for t, present in zip(saved, ctx.present[:15])]
        st = ForwardState(*tensors, *ctx.meta)
        g = backward_raw(st, ctx.raster_settings, grad_out_color, grad_out_depth)
        need = ctx.needs_input_grad
        return (g["means3D"] if need[0] else None,
                g["means2D"] if need[1] else None,
                g["shs"] if need[2] else None,
                g["colors_precomp"] if need[3] else None,
                g["opacities"] if need[4] else None,
                g["scales"] if need[5] else None,
                g["rotations"] if need[6] else None,
                g["cov3D_precomp"] if need[7] else None,
                None)


def rasterize_gaussians(means3D, means2D, sh, colors_precomp, opacities, scales, rotations, cov3Ds_precomp,
                        raster_settings):
    return _RasterizeGaussians.apply(means3D, means2D, sh, colors_precomp, opacities, scales, rotations,
                                     cov3Ds_precomp, raster_settings)


def sh_backward_views(means3D: torch.Tensor, campos: torch.Tensor, dcolors_sh: torch.Tensor, sh_degree: int, M: int,
                      out: Optional[torch.Tensor] = None, chunk_len: int = 0) -> torch.Tensor:
    """dL/dshs (P,M,3) summed over V views from the compact per-view factors: campos (V,3) and the clamp-masked
    colour gradients dcolors_sh (V,P,3) that backward_raw(..., compact_sh=True) returns (gsr_sh_backward_views).
    chunk_len > 0: dcolors_sh is the flat chunk-major layout of multiview.py's chunked gather -- chunk c covers
    Gaussians [c*chunk_len, min(P, (c+1)*chunk_len)) as a (V, L_c, 3) block (gsr_sh_backward_views_chunked)."""
    lib = _native.load()
    device = means3D.device
    m = _prep(means3D, device, "means3D")
    c = _prep(campos, device, "campos").reshape(-1, 3)
    d = _prep(dcolors_sh, device, "dcolors_sh")
    P, V = m.shape[0], c.shape[0]
    if chunk_len and chunk_len < P:
        if d.numel() != V * P * 3:
            raise RuntimeError(f"chunked dcolors_sh must hold {V * P * 3} floats, got {d.numel()}")
    elif tuple(d.shape) != (V, P, 3):
        raise RuntimeError(f"dcolors_sh must have shape {(V, P, 3)}, got {tuple(d.shape)}")
    if out is None:
        out = torch.empty(P, M, 3, dtype=torch.float32, device=device)
    elif tuple(out.shape) != (P, M, 3) or out.dtype != torch.float32 or not out.is_contiguous():
        raise RuntimeError(f"out must be a contiguous float32 tensor of shape {(P, M, 3)}")
    with torch.cuda.device(device):
        rc = lib.gsr_sh_backward_views_chunked(P, int(sh_degree), int(M), V, int(chunk_len), _ptr(m), _ptr(c), _ptr(d),
                                               out.data_ptr(), _stream_handle(device))
    _native.check(rc, "sh_backward_views")
    return out


def mark_visible(positions: torch.Tensor, viewmatrix: torch.Tensor, projmatrix: torch.Tensor) -> torch.Tensor:
    lib = _native.load()
    device = positions.device
    pos = _prep(positions, device, "positions")
    view = _prep(viewmatrix, device, "viewmatrix")
    proj = _prep(projmatrix, device, "projmatrix")
    P = positions.shape[0]
    present = torch.zeros(P, dtype=torch.bool, device=device)
    if P:
        with torch.cuda.device(device):
            rc = lib.gsr_mark_visible(P, _ptr(pos), _ptr(view), _ptr(proj), present.data_ptr(),
                                      _stream_handle(device))
        _native.check(rc, "mark_visible")
    return present


class GaussianRasterizer(nn.Module):
    def __init__(self, raster_settings: GaussianRasterizationSettings):
        super().__init__()
        self.raster_settings = raster_settings

    def markVisible(self, positions: torch.Tensor) -> torch.Tensor:
        with torch.no_grad():
            rs = self.raster_settings
            return mark_visible(positions, rs.viewmatrix, rs.projmatrix)

    def forward(self, means3D, means2D, opacities, shs=None, colors_precomp=None, scales=None, rotations=None,
                cov3D_precomp=None):
        rs = self.raster_settings
        if (shs is None and colors_precomp is None) or (shs is not None and colors_precomp is not None):
            raise Exception("Please provide excatly one of either SHs or precomputed colors!")
        if ((scales is None or rotations is None) and cov3D_precomp is None) or (
                (scales is not None or rotations is not None) and cov3D_precomp is not None):
            raise Exception("Please provide exactly one of either scale/rotation pair or precomputed 3D covariance!")
        return rasterize_gaussians(means3D, means2D, shs, colors_precomp, opacities, scales, rotations,
                                   cov3D_precomp, rs)
