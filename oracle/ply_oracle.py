"""TEST INFRASTRUCTURE ONLY -- numpy restatement of the reference's PLY checkpoint reader and writer.

Only tests/ and tools/ benchmarks may import this module; the product path (gaussian_splatting_lightning_amd.ply)
transposes the records with the HIP kernels of csrc/gsr_ply.hip and never calls into oracle/.

plyfile (the reference's PLY library) is absent from this image, so the file format is restated from the PLY
spec and from what plyfile writes for PlyData([PlyElement.describe(structured_array, "vertex")]):
"ply\\nformat binary_little_endian 1.0\\nelement vertex N\\nproperty float <name>\\n...end_header\\n" followed
by the packed records.  Semantics follow:
  write_gaussians       gs_lightning/modules/gaussian_model.py:150-171 (== third_party/.../gaussian_model.py:239-256)
  read_gaussians        third_party/.../gaussian_model.py:263-314 (official: integer-suffix sort)
  read_gaussians_gsl    gs_lightning/modules/gaussian_model.py:112-140 (lexicographic sort, reshape(N,-1,3),
                        active_sh_degree = int(sqrt(shape[-1] + 1)))
Parity pinned to this restatement (no PLY fixture ships with the reference).
"""
from __future__ import annotations

import numpy as np

TYPES = {"float": "f4", "double": "f8", "uchar": "u1", "char": "i1", "ushort": "u2", "short": "i2", "uint": "u4",
         "int": "i4", "float32": "f4", "float64": "f8", "uint8": "u1", "int8": "i1", "uint16": "u2", "int16": "i2",
         "uint32": "u4", "int32": "i4"}


def attributes(n_dc, n_rest, n_scale=3, n_rot=4):
    return (["x", "y", "z", "nx", "ny", "nz"] + [f"f_dc_{i}" for i in range(n_dc)] +
            [f"f_rest_{i}" for i in range(n_rest)] + ["opacity"] + [f"scale_{i}" for i in range(n_scale)] +
            [f"rot_{i}" for i in range(n_rot)])


def write_vertex_ply(path, arr: np.ndarray, fmt="binary_little_endian", type_names=None):
    """arr: structured array; writes one vertex element in the given format."""
    inv = {"f4": "float", "f8": "double", "u1": "uchar", "i1": "char", "u2": "ushort", "i2": "short", "u4": "uint",
           "i4": "int"}
    lines = ["ply", f"format {fmt} 1.0", f"element vertex {len(arr)}"]
    for name in arr.dtype.names:
        t = (type_names or {}).get(name) or inv[arr.dtype[name].str[1:]]
        lines.append(f"property {t} {name}")
    lines.append("end_header")
    with open(path, "wb") as f:
        f.write(("\n".join(lines) + "\n").encode("ascii"))
        if fmt == "ascii":
            for row in arr:
                f.write((" ".join(repr(v.item()) for v in row) + "\n").encode("ascii"))
        else:
            order = ">" if fmt == "binary_big_endian" else "<"
            dt = np.dtype([(n, order + arr.dtype[n].str[1:]) for n in arr.dtype.names])
            arr.astype(dt).tofile(f)


def read_vertex_ply(path):
    raw = open(path, "rb").read()
    end = raw.index(b"end_header")
    body = raw.index(b"\n", end) + 1
    fmt, props, n = None, [], 0
    for line in raw[:end].decode().splitlines()[1:]:
        t = line.split()
        if t[0] == "format":
            fmt = t[1]
        elif t[0] == "element":
            n = int(t[2])
        elif t[0] == "property":
            props.append((t[2], TYPES[t[1]]))
    if fmt == "ascii":
        vals = np.loadtxt(raw[body:].decode().splitlines()[:n], ndmin=2)
        out = np.empty(n, dtype=[(p, t) for p, t in props])
        for j, (p, _) in enumerate(props):
            out[p] = vals[:, j]
        return out
    order = ">" if fmt == "binary_big_endian" else "<"
    return np.frombuffer(raw, dtype=[(p, order + t) for p, t in props], count=n, offset=body)


def write_gaussians(path, xyz, features_dc, features_rest, opacity, scaling, rotation):
    N = xyz.shape[0]
    f_dc = np.ascontiguousarray(features_dc.transpose(0, 2, 1)).reshape(N, features_dc[0].size if N else
                                                                         features_dc.shape[1] * features_dc.shape[2])
    f_rest = np.ascontiguousarray(features_rest.transpose(0, 2, 1)).reshape(N, features_rest.shape[1] *
                                                                             features_rest.shape[2])
    names = attributes(f_dc.shape[1], f_rest.shape[1], scaling.shape[1], rotation.shape[1])
    attrs = np.concatenate([xyz, np.zeros_like(xyz), f_dc, f_rest, opacity, scaling, rotation], 1).astype(np.float32)
    arr = np.empty(N, dtype=[(n, "f4") for n in names])
    for j, n in enumerate(names):
        arr[n] = attrs[:, j]
    write_vertex_ply(path, arr)


def read_gaussians(path):
    v = read_vertex_ply(path)
    N = len(v)
    f32 = lambda names: np.stack([np.asarray(v[n], np.float64) for n in names], 1).astype(np.float32) \
        if names else np.zeros((N, 0), np.float32)  # noqa: E731
    xyz = f32(["x", "y", "z"])
    dc = f32(["f_dc_0", "f_dc_1", "f_dc_2"]).reshape(N, 3, 1).transpose(0, 2, 1)
    names = v.dtype.names
    rest_n = sorted([n for n in names if n.startswith("f_rest_")], key=lambda x: int(x.split("_")[-1]))
    K = len(rest_n) // 3
    rest = f32(rest_n).reshape(N, 3, K).transpose(0, 2, 1)
    sc = f32(sorted([n for n in names if n.startswith("scale_")], key=lambda x: int(x.split("_")[-1])))
    rot = f32(sorted([n for n in names if n.startswith("rot_")], key=lambda x: int(x.split("_")[-1])))
    return dict(xyz=xyz, features_dc=np.ascontiguousarray(dc), features_rest=np.ascontiguousarray(rest),
                opacity=f32(["opacity"]), scaling=sc, rotation=rot)


def read_gaussians_gsl(path):
    v = read_vertex_ply(path)
    N = len(v)
    names = v.dtype.names
    load = lambda prefix: np.stack([np.asarray(v[n], np.float32) for n in sorted(  # noqa: E731
        [n for n in names if n.startswith(prefix)])], -1) if any(n.startswith(prefix) for n in names) \
        else np.zeros((N, 0), np.float32)
    rest = load("f_rest").reshape(N, -1, 3)
    return dict(xyz=np.stack([v["x"], v["y"], v["z"]], -1).astype(np.float32),
                features_dc=load("f_dc").reshape(N, 1, 3), features_rest=rest,
                scaling=load("scale").reshape(N, 3), rotation=load("rot").reshape(N, 4),
                opacity=load("opacity").reshape(N, 1), active_sh_degree=int(np.sqrt(rest.shape[-1] + 1)))
