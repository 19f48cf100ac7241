"""The C-ABI library loads on a GPU-less host and exports every entry point include/gsrast.h declares;
argument validation happens before any device call."""
import ctypes
import os
import re

import pytest

from gaussian_splatting_lightning_amd import _native

HEADER = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "gsrast.h")


def declared_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(gsr_[a-z0-9_]+)\s*\(", txt)) - {"gsr_alloc_fn"})


def test_header_declares_expected_api():
    names = declared_functions()
    for n in ("gsr_forward", "gsr_backward", "gsr_mark_visible"):
        assert n in names
    assert set(names) == set(_native.EXPORTED_SYMBOLS)


def test_library_exports_every_declared_symbol():
    lib = _native.load()
    for n in declared_functions():
        assert hasattr(lib, n), n
    assert b"gfx950" in lib.gsr_build_info()


def test_buffer_sizes_and_layout():
    lib = _native.load()
    g1, g2 = lib.gsr_geom_buffer_bytes(1000), lib.gsr_geom_buffer_bytes(2000)
    assert 0 < g1 < g2
    assert lib.gsr_binning_buffer_bytes(10_000, 640, 480) > 10_000 * 16
    assert lib.gsr_bwd_scratch_bytes(1000, 10) >= (1000 + 10) * 40
    lay = _native.state_layout(1000, 5000, 100, 80)
    stride = lay.pop("geom_rec_stride")
    assert stride == 48
    # the render record's three fields are interleaved (16, 16, 8 B at +0, +16, +32 of each 48-B record)
    assert (lay["geom_rec_b"] - lay["geom_rec_a"], lay["geom_rec_c"] - lay["geom_rec_a"]) == (16, 32)
    assert all(v % 256 == 0 for k, v in lay.items() if k not in ("geom_rec_b", "geom_rec_c"))
    # distinct arrays inside one buffer never start at the same offset
    geom = [v for k, v in lay.items() if k.startswith("geom_")]
    assert len(set(geom)) == len(geom)


def test_state_layout_query_is_versioned_by_struct_size():
    """gsr_state_layout.struct_size: a caller built against an older (shorter) header gets only its own fields and
    nothing is written past them; the library reports the size it filled."""
    lib = _native.load()
    L = _native.StateLayout
    short = L.bin_bk_keys.offset  # a caller whose struct ends before the last field
    buf = (ctypes.c_size_t * (ctypes.sizeof(L) // 8))(*([0xDEAD] * (ctypes.sizeof(L) // 8)))
    buf[0] = short
    lib.gsr_state_layout_query(1000, 5000, 100, 80, ctypes.cast(buf, ctypes.POINTER(L)))
    assert buf[0] == short
    assert buf[L.bin_bk_keys.offset // 8] == 0xDEAD  # untouched
    full = _native.state_layout(1000, 5000, 100, 80)
    assert buf[L.geom_rec_a.offset // 8] == full["geom_rec_a"]
    assert "bin_bk_keys" in full


def test_invalid_arguments_fail_before_touching_the_device():
    lib = _native.load()
    a = _native.ForwardArgs(P=-1, W=10, H=10)
    n = ctypes.c_int64(0)
    cb = _native.ALLOC_FN(lambda c, w, b: None)
    assert lib.gsr_forward(ctypes.byref(a), cb, None, None, ctypes.byref(n)) == 1
    assert b"P must be" in lib.gsr_last_error()
    a = _native.ForwardArgs(P=5, W=10, H=10, D=3, M=9, means3D=1, opacities=1, viewmatrix=1, projmatrix=1,
                            background=1, shs=1, campos=1, scales=1, rotations=1)
    assert lib.gsr_forward(ctypes.byref(a), cb, None, None, ctypes.byref(n)) == 1
    assert b"coefficients" in lib.gsr_last_error()
    a = _native.ForwardArgs(P=5, W=10, H=10, D=0, M=1, means3D=1, opacities=1, viewmatrix=1, projmatrix=1,
                            background=1, shs=1, campos=1)
    assert lib.gsr_forward(ctypes.byref(a), cb, None, None, ctypes.byref(n)) == 1
    assert b"scale/rotation" in lib.gsr_last_error()
    with pytest.raises(RuntimeError, match="P must be"):
        _native.check(lib.gsr_mark_visible(-1, None, None, None, None, None), "mark_visible")


def test_python_api_mirrors_upstream():
    import torch
    from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer
    assert GaussianRasterizationSettings._fields == (
        "image_height", "image_width", "tanfovx", "tanfovy", "bg", "scale_modifier", "viewmatrix",
        "projmatrix", "sh_degree", "campos", "prefiltered", "debug", "antialiasing")
    s = GaussianRasterizationSettings(8, 8, 0.5, 0.5, torch.zeros(3), 1.0, torch.eye(4), torch.eye(4), 0,
                                      torch.zeros(3), False, False, False)
    r = GaussianRasterizer(raster_settings=s)
    x = torch.zeros(4, 3)
    with pytest.raises(Exception, match="excatly one of either SHs"):
        r(means3D=x, means2D=x, opacities=torch.zeros(4, 1), shs=None, colors_precomp=None, scales=x,
          rotations=torch.zeros(4, 4))
    with pytest.raises(Exception, match="scale/rotation pair"):
        r(means3D=x, means2D=x, opacities=torch.zeros(4, 1), shs=torch.zeros(4, 1, 3), scales=x, rotations=None)
    with pytest.raises(RuntimeError, match="HIP device"):
        r(means3D=x, means2D=x, opacities=torch.zeros(4, 1), shs=torch.zeros(4, 1, 3), scales=x,
          rotations=torch.zeros(4, 4))
