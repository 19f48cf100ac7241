"""ctypes wrapper around liboracle.so -- TEST INFRASTRUCTURE ONLY.

The oracle is the CPU restatement of the rasterizer (see gsr_oracle.c).  It is the parity
checker for the HIP product path and the `cpu_baseline` leg of bench.py; the product never
imports this module.  Arrays are numpy float32/int32, C-contiguous, in the layouts of the
reference's Python API (means3D (P,3), shs (P,M,3), image (3,H,W), ...).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "liboracle.so")
_lib = None

_f = ctypes.POINTER(ctypes.c_float)
_i = ctypes.POINTER(ctypes.c_int)
_u32 = ctypes.POINTER(ctypes.c_uint32)
_u8 = ctypes.POINTER(ctypes.c_uint8)


def build() -> str:
    """Compile liboracle.so in place (gcc + OpenMP)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB


def _load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(_LIB):
        build()
    lib = ctypes.CDLL(_LIB)
    lib.oracle_forward.restype = ctypes.c_void_p
    lib.oracle_forward.argtypes = [
        ctypes.c_int, ctypes.c_int, ctypes.c_int, _f, _f, _f, _f, _f, ctypes.c_float, _f, _f,
        _f, _f, _f, ctypes.c_float, ctypes.c_float, ctypes.c_int, ctypes.c_int, _f,
        ctypes.c_int, ctypes.c_int, _f, _f, _i]
    lib.oracle_backward.restype = None
    lib.oracle_backward.argtypes = [ctypes.c_void_p, _f, _f, _f, _f, _f, _f, _f, _f, _f, _f]
    lib.oracle_free.argtypes = [ctypes.c_void_p]
    lib.oracle_num_rendered.restype = ctypes.c_longlong
    lib.oracle_num_rendered.argtypes = [ctypes.c_void_p]
    lib.oracle_get_point_list.argtypes = [ctypes.c_void_p, _u32]
    lib.oracle_get_ranges.argtypes = [ctypes.c_void_p, _u32]
    lib.oracle_get_image_state.argtypes = [ctypes.c_void_p, _f, _u32]
    lib.oracle_get_geom.argtypes = [ctypes.c_void_p, _f, _f, _f, _f, _u32]
    lib.oracle_threshold_margin.argtypes = [ctypes.c_void_p, _f]
    lib.oracle_flip_census.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_longlong)]
    lib.oracle_strip_census.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_longlong)]
    lib.oracle_mark_visible.argtypes = [ctypes.c_int, _f, _f, _f, _u8]
    lib.oracle_num_threads.restype = ctypes.c_int
    lib.oracle_bin_count.restype = ctypes.c_longlong
    lib.oracle_bin_count.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, _f, _i, _f, ctypes.c_int]
    lib.oracle_bin.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, _f, _i, _f, _f, ctypes.c_int, _u32, _u32, _u32]
    lib.oracle_get_clamped.argtypes = [ctypes.c_void_p, _u8]
    lib.oracle_sh_backward_views.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, _f, _f, _f, _f]
    _lib = lib
    return lib


def _fp(a):
    if a is None:
        return None
    return a.ctypes.data_as(_f)


def _c32(a):
    if a is None:
        return None
    return np.ascontiguousarray(np.asarray(a, dtype=np.float32))


def num_threads() -> int:
    return int(_load().oracle_num_threads())


def mark_visible(means3D, viewmatrix, projmatrix) -> np.ndarray:
    lib = _load()
    m = _c32(means3D)
    v, p = _c32(viewmatrix), _c32(projmatrix)
    out = np.zeros(m.shape[0], dtype=np.uint8)
    lib.oracle_mark_visible(m.shape[0], _fp(m), _fp(v), _fp(p), out.ctypes.data_as(_u8))
    return out.astype(bool)


def sh_backward_views(means3D, campos, dcolors_sh, sh_degree, M) -> np.ndarray:
    """sum over views v of the SH gradient for clamp-masked colour gradients dcolors_sh (V,P,3) seen from campos
    (V,3) -> (P,M,3)."""
    lib = _load()
    m = _c32(means3D).reshape(-1, 3)
    c = _c32(campos).reshape(-1, 3)
    d = _c32(dcolors_sh).reshape(c.shape[0], m.shape[0], 3)
    out = np.zeros((m.shape[0], M, 3), np.float32)
    lib.oracle_sh_backward_views(m.shape[0], int(sh_degree), int(M), c.shape[0], _fp(m), _fp(c), _fp(d), _fp(out))
    return out


def bin_instances(xy, radii, depths, conic_opacity, image_width, image_height, cull=True):
    """Binning alone: (point_list (R,), ranges (T,2), tiles (P,)) for given pixel centres, radii, view
    depths and (conic, opacity) -- the product's exact culling rule restated in C when cull=True."""
    lib = _load()
    xy = _c32(xy).reshape(-1, 2)
    P = xy.shape[0]
    r = np.ascontiguousarray(np.asarray(radii, np.int32))
    d = _c32(depths).reshape(-1)
    co = _c32(conic_opacity).reshape(-1, 4)
    W, H = int(image_width), int(image_height)
    R = int(lib.oracle_bin_count(P, W, H, _fp(xy), r.ctypes.data_as(_i), _fp(co), int(bool(cull))))
    pl = np.zeros(max(R, 1), np.uint32)
    T = ((W + 15) // 16) * ((H + 15) // 16)
    rg = np.zeros((T, 2), np.uint32)
    tt = np.zeros(max(P, 1), np.uint32)
    lib.oracle_bin(P, W, H, _fp(xy), r.ctypes.data_as(_i), _fp(d), _fp(co), int(bool(cull)), pl.ctypes.data_as(_u32),
                   rg.ctypes.data_as(_u32), tt.ctypes.data_as(_u32))
    return pl[:R], rg, tt[:P]


class OracleRun:
    """One forward pass; keeps the native state alive for backward()/introspection."""

    def __init__(self, handle, P, M, W, H, lib, keep):
        self._h = handle
        self.P, self.M, self.W, self.H = P, M, W, H
        self._lib = lib
        self._keep = keep

    def __del__(self):
        if getattr(self, "_h", None):
            self._lib.oracle_free(self._h)
            self._h = None

    @property
    def num_rendered(self) -> int:
        return int(self._lib.oracle_num_rendered(self._h))

    def point_list(self) -> np.ndarray:
        out = np.zeros(max(self.num_rendered, 1), dtype=np.uint32)
        self._lib.oracle_get_point_list(self._h, out.ctypes.data_as(_u32))
        return out[: self.num_rendered]

    def ranges(self) -> np.ndarray:
        gx, gy = (self.W + 15) // 16, (self.H + 15) // 16
        out = np.zeros((gx * gy, 2), dtype=np.uint32)
        self._lib.oracle_get_ranges(self._h, out.ctypes.data_as(_u32))
        return out

    def image_state(self):
        ft = np.zeros(self.W * self.H, dtype=np.float32)
        nc = np.zeros(self.W * self.H, dtype=np.uint32)
        self._lib.oracle_get_image_state(self._h, _fp(ft), nc.ctypes.data_as(_u32))
        return ft.reshape(self.H, self.W), nc.reshape(self.H, self.W)

    def threshold_margin(self) -> np.ndarray:
        """(H, W) distance of each pixel's nearest compositing decision from its threshold, in units of the fp32
        evaluation error (gsr_oracle.c oracle_threshold_margin); < 1 marks a threshold-flip candidate."""
        out = np.zeros(self.W * self.H, dtype=np.float32)
        self._lib.oracle_threshold_margin(self._h, _fp(out))
        return out.reshape(self.H, self.W)

    def flip_census(self) -> dict:
        """Pixels whose walk under the device composite's fp32 arithmetic (restated on the CPU) first decides
        differently at the exponent sign / alpha / transmittance test (oracle_flip_census)."""
        c = (ctypes.c_longlong * 4)()
        self._lib.oracle_flip_census(self._h, c)
        return {"pixels": c[0], "power": c[1], "alpha": c[2], "transmittance": c[3]}

    def strip_census(self) -> dict:
        """(instance, 4-row strip) pairs before each tile's last contributor: geometrically reached vs contributing
        (oracle_strip_census)."""
        c = (ctypes.c_longlong * 3)()
        self._lib.oracle_strip_census(self._h, c)
        return {"reach": c[0], "contribute": c[2]}

    def geom(self):
        P = self.P
        d = np.zeros(P, np.float32)
        xy = np.zeros((P, 2), np.float32)
        co = np.zeros((P, 4), np.float32)
        rgb = np.zeros((P, 3), np.float32)
        tt = np.zeros(P, np.uint32)
        self._lib.oracle_get_geom(self._h, _fp(d), _fp(xy), _fp(co), _fp(rgb), tt.ctypes.data_as(_u32))
        return dict(depths=d, xy=xy, conic_opacity=co, rgb=rgb, tiles_touched=tt)

    def clamped(self) -> np.ndarray:
        out = np.zeros((self.P, 3), np.uint8)
        self._lib.oracle_get_clamped(self._h, out.ctypes.data_as(_u8))
        return out

    def backward(self, dL_dcolor, dL_dinvdepth=None):
        P, M = self.P, self.M
        dc = _c32(dL_dcolor)
        di = _c32(dL_dinvdepth)
        out = dict(
            means2D=np.zeros((P, 3), np.float32), colors=np.zeros((P, 3), np.float32),
            opacities=np.zeros((P, 1), np.float32), means3D=np.zeros((P, 3), np.float32),
            cov3D=np.zeros((P, 6), np.float32), shs=np.zeros((P, max(M, 0), 3), np.float32),
            scales=np.zeros((P, 3), np.float32), rotations=np.zeros((P, 4), np.float32))
        self._lib.oracle_backward(
            self._h, _fp(dc), _fp(di), _fp(out["means2D"]), _fp(out["colors"]), _fp(out["opacities"]),
            _fp(out["means3D"]), _fp(out["cov3D"]), _fp(out["shs"]) if M else None, _fp(out["scales"]),
            _fp(out["rotations"]))
        return out


def forward(means3D, opacities, scales, rotations, shs, viewmatrix, projmatrix, campos, bg,
            tanfovx, tanfovy, image_height, image_width, sh_degree, scale_modifier=1.0,
            colors_precomp=None, cov3D_precomp=None, prefiltered=False, antialiasing=False):
    """Returns (color (3,H,W), radii (P,) int32, invdepth (1,H,W), OracleRun)."""
    lib = _load()
    m = _c32(means3D)
    P = m.shape[0]
    sh = _c32(shs)
    M = 0 if sh is None or sh.size == 0 else sh.shape[1]
    args = dict(
        bg=_c32(bg), opac=_c32(opacities).reshape(-1), sc=_c32(scales), rot=_c32(rotations),
        cov=_c32(cov3D_precomp), col=_c32(colors_precomp), view=_c32(viewmatrix),
        proj=_c32(projmatrix), cam=_c32(campos), sh=sh)
    H, W = int(image_height), int(image_width)
    color = np.zeros((3, H, W), np.float32)
    invd = np.zeros((1, H, W), np.float32)
    radii = np.zeros(P, np.int32)
    h = lib.oracle_forward(
        P, int(sh_degree), M, _fp(args["bg"]), _fp(m), _fp(args["col"]), _fp(args["opac"]),
        _fp(args["sc"]), float(scale_modifier), _fp(args["rot"]), _fp(args["cov"]), _fp(args["view"]),
        _fp(args["proj"]), _fp(args["cam"]), float(tanfovx), float(tanfovy), W, H,
        _fp(sh) if M else None, int(bool(prefiltered)), int(bool(antialiasing)), _fp(color), _fp(invd),
        radii.ctypes.data_as(_i))
    run = OracleRun(h, P, M, W, H, lib, keep=(m, args))
    return color, radii, invd, run
