"""PLY checkpoint I/O for Gaussian models, with the record transposes on the GPU (csrc/gsr_ply.hip).

Formats and semantics mirrored:

* `save_ply` -- gs_lightning/modules/gaussian_model.py:150-171 (identical to the official 3DGS writer,
  third_party/gaussian_splatting/scene/gaussian_model.py:239-256): one binary little-endian "vertex" element of
  float32 columns x y z nx ny nz f_dc_* f_rest_* opacity scale_* rot_*; normals are zero; SH coefficients are
  written channel-major (features.transpose(1, 2).flatten(1)).  The header is the one plyfile writes.
* `load_ply(..., compat="official")` -- third_party/.../gaussian_model.py:263-314: names sorted by their integer
  suffix, f_rest reshaped (N, 3, M-1) then transposed to (N, M-1, 3).
* `load_ply(..., compat="gs_lightning")` -- gs_lightning/modules/gaussian_model.py:112-140 (load_model_ply)
  INCLUDING its three known bugs: names sorted lexicographically (f_rest_10 before
  f_rest_2), f_rest reshaped (N, -1, 3) ignoring the channel-major layout, and active_sh_degree =
  int(sqrt(features_rest.shape[-1] + 1)) = 2.  Use it only to reproduce that loader's renders.
* `read_points_ply` -- the COLMAP points3D.ply read of gaussian_model.py:65-72 (x y z + red green blue / 255).

The host parses the header, maps the file and copies the vertex records to HBM in one transfer; one kernel
launch converts and de-interleaves every column (any scalar PLY type, either byte order).  ASCII files are
parsed on the host and then take the same path.  No CPU fallback: the HIP library must load.
"""
from __future__ import annotations

import ctypes
import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import _native
from .rasterizer import _stream_handle

__all__ = ["PlyHeader", "read_header", "header_bytes", "load_ply", "save_ply", "read_points_ply", "attribute_names"]

_NP = {0: "f4", 1: "f8", 2: "u1", 3: "i1", 4: "u2", 5: "i2", 6: "u4", 7: "i4"}


@dataclass
class PlyElement:
    name: str
    count: int
    properties: List[Tuple[str, str]] = field(default_factory=list)  # (name, PLY type) ; list props rejected

    @property
    def record_bytes(self) -> int:
        return sum(_native.PLY_TYPE_SIZE[_native.PLY_TYPES[t]] for _, t in self.properties)

    def offsets(self) -> Dict[str, Tuple[int, int]]:
        out, off = {}, 0
        for name, t in self.properties:
            code = _native.PLY_TYPES[t]
            out[name] = (off, code)
            off += _native.PLY_TYPE_SIZE[code]
        return out


@dataclass
class PlyHeader:
    fmt: str                      # ascii | binary_little_endian | binary_big_endian
    elements: List[PlyElement]
    data_offset: int              # bytes before the first element's data

    def element(self, name: str) -> PlyElement:
        for e in self.elements:
            if e.name == name:
                return e
        raise KeyError(f"PLY file has no {name!r} element")


def read_header(raw: bytes) -> PlyHeader:
    end = raw.find(b"end_header")
    if not raw.startswith(b"ply") or end < 0:
        raise ValueError("not a PLY file (missing 'ply' magic or 'end_header')")
    nl = raw.find(b"\n", end)
    if nl < 0:
        raise ValueError("truncated PLY header")
    fmt, elements = None, []
    for line in raw[:end].decode("ascii", errors="replace").splitlines()[1:]:
        tok = line.split()
        if not tok or tok[0] in ("comment", "obj_info"):
            continue
        if tok[0] == "format":
            fmt = tok[1]
            if fmt not in ("ascii", "binary_little_endian", "binary_big_endian"):
                raise ValueError(f"unsupported PLY format {fmt!r}")
        elif tok[0] == "element":
            elements.append(PlyElement(tok[1], int(tok[2])))
        elif tok[0] == "property":
            if not elements:
                raise ValueError("PLY property before any element")
            if tok[1] == "list":
                elements[-1].properties.append((tok[-1], "list"))
            else:
                if tok[1] not in _native.PLY_TYPES:
                    raise ValueError(f"unsupported PLY property type {tok[1]!r}")
                elements[-1].properties.append((tok[2], tok[1]))
    if fmt is None:
        raise ValueError("PLY header without a format line")
    return PlyHeader(fmt, elements, nl + 1)


def header_bytes(n: int, names: Sequence[str], fmt: str = "binary_little_endian") -> bytes:
    """The header plyfile writes for one float32 'vertex' element (PlyData([PlyElement.describe(...)]))."""
    lines = ["ply", f"format {fmt} 1.0", f"element vertex {n}"] + [f"property float {p}" for p in names]
    lines.append("end_header")
    return ("\n".join(lines) + "\n").encode("ascii")


def attribute_names(n_dc: int, n_rest: int, n_scale: int = 3, n_rot: int = 4) -> List[str]:
    """construct_list_of_attributes of the official writer (third_party/.../gaussian_model.py:227-237)."""
    return (["x", "y", "z", "nx", "ny", "nz"] + [f"f_dc_{i}" for i in range(n_dc)] +
            [f"f_rest_{i}" for i in range(n_rest)] + ["opacity"] + [f"scale_{i}" for i in range(n_scale)] +
            [f"rot_{i}" for i in range(n_rot)])


def _suffix(name: str) -> int:
    return int(name.split("_")[-1])


def _vertex_records(path: str, device) -> Tuple[torch.Tensor, PlyElement, bool]:
    """Vertex records on the device (uint8, n * record_bytes), the element, and the byte order flag."""
    with open(path, "rb") as f:
        head = f.read(1 << 16)
        while b"end_header" not in head:
            more = f.read(1 << 16)
            if not more:
                break
            head += more
    hdr = read_header(head)
    idx = [i for i, e in enumerate(hdr.elements) if e.name == "vertex"]
    if not idx:
        raise ValueError(f"{path}: no vertex element")
    vert = hdr.elements[idx[0]]
    if any(t == "list" for _, t in vert.properties):
        raise ValueError(f"{path}: list properties in the vertex element are not supported")
    if hdr.fmt == "ascii":
        if idx[0] != 0:
            raise ValueError(f"{path}: ascii PLY with elements before 'vertex' is not supported")
        with open(path, "rb") as f:
            f.seek(hdr.data_offset)
            rows = [f.readline() for _ in range(vert.count)]
        vals = np.loadtxt(rows, dtype=np.float64, ndmin=2) if vert.count else np.zeros((0, len(vert.properties)))
        # re-encode as little-endian records of the declared types: the GPU path then treats all formats alike
        dt = np.dtype([(n, "<" + _NP[_native.PLY_TYPES[t]]) for n, t in vert.properties])
        rec = np.empty(vert.count, dtype=dt)
        for j, (n, _) in enumerate(vert.properties):
            rec[n] = vals[:, j]
        host = rec.view(np.uint8).reshape(-1)
        big = False
    else:
        off = hdr.data_offset
        for e in hdr.elements[:idx[0]]:
            if any(t == "list" for _, t in e.properties):
                raise ValueError(f"{path}: list-property element {e.name!r} before 'vertex' is not supported")
            off += e.count * e.record_bytes
        nbytes = vert.count * vert.record_bytes
        host = np.fromfile(path, dtype=np.uint8, count=nbytes, offset=off)
        if host.size != nbytes:
            raise ValueError(f"{path}: truncated vertex data ({host.size} of {nbytes} bytes)")
        big = hdr.fmt == "binary_big_endian"
    dev = torch.from_numpy(host).to(device)
    return dev, vert, big


def _unpack(records: torch.Tensor, vert: PlyElement, big: bool, plan: List[Tuple[torch.Tensor, List[str]]]) -> None:
    """plan: (destination (n, ...) fp32 tensor, property names in the tensor's row-major column order)."""
    offs = vert.offsets()
    cols, fields, widths = [], [], []
    for dst, names in plan:
        if not names:
            continue
        for n in names:
            if n not in offs:
                raise ValueError(f"PLY vertex element has no property {n!r}")
            cols.append(_native.PlyColumn(*offs[n]))
        fields.append(dst.data_ptr())
        widths.append(len(names))
    if vert.count == 0 or not cols:
        return
    lib = _native.load()
    if len(cols) > 128:
        raise ValueError("more than 128 PLY columns requested")
    C = (_native.PlyColumn * len(cols))(*cols)
    F = (ctypes.c_void_p * len(fields))(*fields)
    W = (ctypes.c_int * len(widths))(*widths)
    _native.check(lib.gsr_ply_unpack(records.data_ptr(), vert.count, vert.record_bytes, int(big), C, len(cols), F, W,
                                     len(fields), _stream_handle(records.device)), "gsr_ply_unpack")


def _device(device) -> torch.device:
    dev = torch.device(device)
    if dev.type != "cuda":
        raise RuntimeError("PLY I/O runs on the GPU (HIP kernels); pass a cuda device")
    return dev


@torch.no_grad()
def load_ply(path: str, max_sh_degree: Optional[int] = None, compat: str = "official",
             device="cuda") -> Dict[str, object]:
    """Gaussian checkpoint -> dict(xyz (N,3), features_dc (N,1,3), features_rest (N,M-1,3), opacity (N,1),
    scaling (N,3), rotation (N,4), active_sh_degree)."""
    if compat not in ("official", "gs_lightning"):
        raise ValueError(f"compat must be 'official' or 'gs_lightning', got {compat!r}")
    dev = _device(device)
    records, vert, big = _vertex_records(path, dev)
    names = [n for n, _ in vert.properties]
    N = vert.count
    pick = lambda prefix: [n for n in names if n.startswith(prefix)]  # noqa: E731
    f32 = dict(dtype=torch.float32, device=dev)
    if compat == "official":
        dc = ["f_dc_0", "f_dc_1", "f_dc_2"]
        rest = sorted(pick("f_rest_"), key=_suffix)
        if len(rest) % 3:
            raise ValueError(f"{len(rest)} f_rest properties is not a multiple of 3")
        if max_sh_degree is not None and len(rest) != 3 * (max_sh_degree + 1) ** 2 - 3:
            raise ValueError(f"{len(rest)} f_rest properties do not match max_sh_degree={max_sh_degree}")
        K = len(rest) // 3  # M - 1
        # file column c*K + k holds channel c of coefficient k -> tensor column k*3 + c
        rest_cols = [rest[c * K + k] for k in range(K) for c in range(3)]
        scale = sorted(pick("scale_"), key=_suffix)
        rot = sorted(pick("rot_"), key=_suffix)
        active = int(round(math.sqrt(K + 1))) - 1
        rest_shape = (N, K, 3)
    else:
        dc = sorted(pick("f_dc"))
        rest_cols = sorted(pick("f_rest"))
        scale = sorted(pick("scale"))
        rot = sorted(pick("rot"))
        rest_shape = (N, len(rest_cols) // 3, 3)
        active = int(np.sqrt(rest_shape[-1] + 1))  # the reference's formula: always 2 (bug 3)
    out = dict(xyz=torch.empty((N, 3), **f32), features_dc=torch.empty((N, 1, 3), **f32),
               features_rest=torch.empty(rest_shape, **f32), opacity=torch.empty((N, 1), **f32),
               scaling=torch.empty((N, len(scale)), **f32), rotation=torch.empty((N, len(rot)), **f32))
    _unpack(records, vert, big, [(out["xyz"], ["x", "y", "z"]), (out["features_dc"], dc),
                                 (out["features_rest"], rest_cols), (out["opacity"], ["opacity"]),
                                 (out["scaling"], scale), (out["rotation"], rot)])
    out["active_sh_degree"] = active
    return out


@torch.no_grad()
def read_points_ply(path: str, device="cuda") -> Tuple[torch.Tensor, torch.Tensor]:
    """COLMAP points3D.ply -> (xyz (N,3), rgb (N,3) in [0,1]) as gaussian_model.py:66-69 reads them."""
    dev = _device(device)
    records, vert, big = _vertex_records(path, dev)
    xyz = torch.empty((vert.count, 3), dtype=torch.float32, device=dev)
    rgb = torch.empty((vert.count, 3), dtype=torch.float32, device=dev)
    _unpack(records, vert, big, [(xyz, ["x", "y", "z"]), (rgb, ["red", "green", "blue"])])
    return xyz, (rgb.double() / 255.0).float()  # numpy float64 division then fp32, as the reference


@torch.no_grad()
def save_ply(path: str, xyz: torch.Tensor, features_dc: torch.Tensor, features_rest: torch.Tensor,
             opacity: torch.Tensor, scaling: torch.Tensor, rotation: torch.Tensor) -> bool:
    """gaussian_model.py:150-171: binary little-endian float32 vertex records, normals zero."""
    dev = _device(xyz.device)
    N = int(xyz.shape[0])
    tens = [t.detach().to(dev, torch.float32).contiguous() for t in
            (xyz, features_dc, features_rest, opacity, scaling, rotation)]
    xyz_, dc, rest, op, sc, rot = tens
    n_dc, n_rest = dc[0].numel() if N else dc.shape[1] * dc.shape[2], rest.shape[1] * rest.shape[2]
    names = attribute_names(n_dc, n_rest, sc.shape[1], rot.shape[1])
    rb = 4 * len(names)
    pos = {n: 4 * i for i, n in enumerate(names)}
    Kd, Kr = dc.shape[1], rest.shape[1]
    # tensor column k*3 + c  <-  file property f_*_{c*K + k} (channel-major)
    plan = [(xyz_, ["x", "y", "z"]),
            (dc, [f"f_dc_{c * Kd + k}" for k in range(Kd) for c in range(3)]),
            (rest, [f"f_rest_{c * Kr + k}" for k in range(Kr) for c in range(3)]),
            (op, ["opacity"]), (sc, [f"scale_{i}" for i in range(sc.shape[1])]),
            (rot, [f"rot_{i}" for i in range(rot.shape[1])])]
    cols, fields, widths = [], [], []
    for t, cn in plan:
        if not cn:
            continue
        cols += [_native.PlyColumn(pos[n], 0) for n in cn]
        fields.append(t.data_ptr())
        widths.append(len(cn))
    records = torch.empty(N * rb, dtype=torch.uint8, device=dev)
    if N:
        if len(cols) > 128:
            raise ValueError("more than 128 PLY columns")
        lib = _native.load()
        C = (_native.PlyColumn * len(cols))(*cols)
        F = (ctypes.c_void_p * len(fields))(*fields)
        W = (ctypes.c_int * len(widths))(*widths)
        _native.check(lib.gsr_ply_pack(records.data_ptr(), N, rb, 0, C, len(cols), F, W, len(fields),
                                       _stream_handle(dev)), "gsr_ply_pack")
    host = records.cpu().numpy()
    with open(path, "wb") as f:
        f.write(header_bytes(N, names))
        host.tofile(f)
    return True
