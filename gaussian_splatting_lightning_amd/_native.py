"""ctypes binding of libgsrast.so (include/gsrast.h).

This is the product path: every rasterizer call goes through these C entry points.  There is no
CPU or PyTorch fallback -- if the library is missing or cannot be loaded, importing the rasterizer
raises, so a GPU run can never silently pass on another implementation.
"""
from __future__ import annotations

import contextlib
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libgsrast.so")
ABI_VERSION = 2  # include/gsrast.h GSR_ABI_VERSION

GSR_BUF_GEOM, GSR_BUF_BINNING, GSR_BUF_IMAGE, GSR_BUF_BWD_SCRATCH = 0, 1, 2, 3

_fp = ctypes.c_void_p  # device pointers are passed as integers


class ForwardArgs(ctypes.Structure):
    _fields_ = [
        ("P", ctypes.c_int), ("D", ctypes.c_int), ("M", ctypes.c_int), ("W", ctypes.c_int), ("H", ctypes.c_int),
        ("background", _fp), ("means3D", _fp), ("colors_precomp", _fp), ("opacities", _fp), ("scales", _fp),
        ("scale_modifier", ctypes.c_float), ("rotations", _fp), ("cov3D_precomp", _fp), ("viewmatrix", _fp),
        ("projmatrix", _fp), ("campos", _fp), ("tan_fovx", ctypes.c_float), ("tan_fovy", ctypes.c_float),
        ("shs", _fp), ("prefiltered", ctypes.c_int), ("antialiasing", ctypes.c_int), ("debug", ctypes.c_int),
        ("out_color", _fp), ("out_invdepth", _fp), ("radii", _fp), ("num_big_out", ctypes.c_int64),
    ]


class BackwardArgs(ctypes.Structure):
    _fields_ = [
        ("P", ctypes.c_int), ("D", ctypes.c_int), ("M", ctypes.c_int), ("W", ctypes.c_int), ("H", ctypes.c_int),
        ("R", ctypes.c_int64), ("num_big", ctypes.c_int64), ("background", _fp), ("means3D", _fp), ("colors_precomp", _fp),
        ("opacities", _fp), ("scales", _fp), ("scale_modifier", ctypes.c_float), ("rotations", _fp),
        ("cov3D_precomp", _fp), ("viewmatrix", _fp), ("projmatrix", _fp), ("campos", _fp),
        ("tan_fovx", ctypes.c_float), ("tan_fovy", ctypes.c_float), ("dL_dpix", _fp), ("dL_dinvdepth", _fp),
        ("shs", _fp), ("radii", _fp), ("geom_buffer", _fp), ("binning_buffer", _fp), ("image_buffer", _fp),
        ("antialiasing", ctypes.c_int), ("debug", ctypes.c_int), ("dL_dmeans2D", _fp), ("dL_dcolors", _fp),
        ("dL_dopacity", _fp), ("dL_dmeans3D", _fp), ("dL_dcov3D", _fp), ("dL_dsh", _fp), ("dL_dscales", _fp),
        ("dL_drotations", _fp),
        ("dL_dcolors_sh", _fp),
        ("densify_stats", _fp),
        ("densify_accumulate", ctypes.c_int), ("max_radii2D", _fp),
        ("stages", ctypes.c_int), ("g_begin", ctypes.c_int64), ("g_end", ctypes.c_int64), ("bwd_scratch", _fp),
        ("campos_rows", _fp), ("campos_rank", ctypes.c_int), ("campos_nrows", ctypes.c_int),
    ]


GSR_BWD_ALL, GSR_BWD_COMPOSITE, GSR_BWD_GAUSSIANS = 0, 1, 2


class AdamGroup(ctypes.Structure):
    _fields_ = [("param", _fp), ("grad", _fp), ("exp_avg", _fp), ("exp_avg_sq", _fp), ("n", ctypes.c_int64),
                ("lr", ctypes.c_double), ("step", ctypes.c_int64)]


class AdamShViewsArgs(ctypes.Structure):  # include/gsrast.h gsr_adam_sh_views_args
    _fields_ = [("P", ctypes.c_int), ("D", ctypes.c_int), ("M", ctypes.c_int), ("V", ctypes.c_int),
                ("chunk_len", ctypes.c_int64), ("means3D", _fp), ("campos", _fp), ("dL_dcolors_sh", _fp),
                ("dc_param", _fp), ("dc_exp_avg", _fp), ("dc_exp_avg_sq", _fp), ("dc_lr", ctypes.c_double),
                ("dc_step", ctypes.c_int64),
                ("rest_param", _fp), ("rest_exp_avg", _fp), ("rest_exp_avg_sq", _fp), ("rest_lr", ctypes.c_double),
                ("rest_step", ctypes.c_int64), ("param_row_stride", ctypes.c_int64),
                ("moment_row_stride", ctypes.c_int64)]


class DensifyArgs(ctypes.Structure):
    _fields_ = [("N", ctypes.c_int64), ("opacity", _fp), ("scaling", _fp), ("max_radii2D", _fp),
                ("xyz_grad_accum", _fp), ("xyz_grad_count", _fp),
                ("opacity_threshold", ctypes.c_float), ("screensize_threshold", ctypes.c_float),
                ("size_threshold", ctypes.c_float), ("grad_threshold", ctypes.c_float),
                ("clone_size_threshold", ctypes.c_float),
                ("apply_screensize", ctypes.c_int), ("apply_size", ctypes.c_int)]


class DensifyField(ctypes.Structure):
    _fields_ = [("src", _fp), ("dst", _fp), ("src_exp_avg", _fp), ("src_exp_avg_sq", _fp),
                ("dst_exp_avg", _fp), ("dst_exp_avg_sq", _fp), ("width", ctypes.c_int), ("kind", ctypes.c_int)]


FIELD_PLAIN, FIELD_XYZ, FIELD_SCALING, FIELD_STAT = 0, 1, 2, 3


class PlyColumn(ctypes.Structure):
    _fields_ = [("offset", ctypes.c_int32), ("type", ctypes.c_int32)]


# GSR_PLY_* type codes by PLY type name (both spellings of the PLY spec)
PLY_TYPES = {"float": 0, "float32": 0, "double": 1, "float64": 1, "uchar": 2, "uint8": 2, "char": 3, "int8": 3,
             "ushort": 4, "uint16": 4, "short": 5, "int16": 5, "uint": 6, "uint32": 6, "int": 7, "int32": 7}
PLY_TYPE_SIZE = (4, 8, 1, 1, 2, 2, 4, 4)


class StateLayout(ctypes.Structure):  # include/gsrast.h gsr_state_layout (versioned by struct_size)
    _fields_ = [(n, ctypes.c_size_t) for n in (
        "struct_size", "geom_rec_a", "geom_rec_b", "geom_rec_c", "geom_tiles", "geom_order", "geom_inst_off",
        "geom_inst_start", "geom_clamped", "geom_depth_key", "geom_expand_rec", "bin_point_list", "bin_inv",
        "bin_keys_sorted", "bin_sorted_u", "bin_inst_gid", "img_final_T", "img_n_contrib", "img_ranges",
        "img_tile_last", "img_tile_loaded", "geom_rec_stride", "bin_bk_keys")]


ALLOC_FN = ctypes.CFUNCTYPE(ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t)

EXPORTED_SYMBOLS = (
    "gsr_forward", "gsr_backward", "gsr_mark_visible", "gsr_sh_backward_views", "gsr_sh_backward_views_chunked",
    "gsr_geom_buffer_bytes", "gsr_binning_buffer_bytes",
    "gsr_image_buffer_bytes", "gsr_bwd_scratch_bytes", "gsr_set_profiling", "gsr_num_stages", "gsr_stage_name",
    "gsr_stage_times", "gsr_reset_stage_times", "gsr_last_error", "gsr_build_info", "gsr_abi_version", "gsr_adam_sh_views_step",
    "gsr_stream_values_supported", "gsr_stream_signal", "gsr_stream_wait", "gsr_state_layout_query",
    "gsr_set_tuning", "gsr_get_tuning", "gsr_ssim_num_partials", "gsr_ssim_forward", "gsr_ssim_backward", "gsr_adam_step", "gsr_sparse_adam_step",
    "gsr_activations_forward", "gsr_activations_backward",
    "gsr_densify_workspace_bytes", "gsr_densify_classify", "gsr_densify_apply", "gsr_ply_unpack", "gsr_ply_pack",
    "gsr_knn_workspace_bytes", "gsr_knn_mean_dist2", "gsr_debug_wave_stamps",
)

_lib = None


def load(path: str | None = None):
    """Load libgsrast.so once (raises RuntimeError with build instructions if it is absent)."""
    global _lib
    if _lib is not None:
        return _lib
    path = path or os.environ.get("GSR_LIB", LIB_PATH)
    if not os.path.exists(path):
        raise RuntimeError(
            f"libgsrast.so not found at {path}: build it with `python -m gaussian_splatting_lightning_amd.build` "
            "(or __graft_entry__.build()); there is no CPU fallback.")
    lib = ctypes.CDLL(path)
    lib.gsr_forward.argtypes = [ctypes.POINTER(ForwardArgs), ALLOC_FN, ctypes.c_void_p, ctypes.c_void_p,
                                ctypes.POINTER(ctypes.c_int64)]
    lib.gsr_forward.restype = ctypes.c_int
    lib.gsr_backward.argtypes = [ctypes.POINTER(BackwardArgs), ALLOC_FN, ctypes.c_void_p, ctypes.c_void_p]
    lib.gsr_backward.restype = ctypes.c_int
    lib.gsr_mark_visible.argtypes = [ctypes.c_int, _fp, _fp, _fp, _fp, ctypes.c_void_p]
    lib.gsr_mark_visible.restype = ctypes.c_int
    lib.gsr_sh_backward_views.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, _fp, _fp, _fp, _fp,
                                          ctypes.c_void_p]
    lib.gsr_sh_backward_views.restype = ctypes.c_int
    lib.gsr_sh_backward_views_chunked.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                  ctypes.c_int64, _fp, _fp, _fp, _fp, ctypes.c_void_p]
    lib.gsr_sh_backward_views_chunked.restype = ctypes.c_int
    lib.gsr_adam_step.argtypes = [ctypes.POINTER(AdamGroup), ctypes.c_int, ctypes.c_double, ctypes.c_double,
                                  ctypes.c_double, ctypes.c_void_p]
    lib.gsr_adam_step.restype = ctypes.c_int
    if hasattr(lib, "gsr_stream_signal"):  # absent from pre-round-6 builds loaded for A/Bs through GSR_LIB
        lib.gsr_stream_values_supported.restype = ctypes.c_int
        for f in (lib.gsr_stream_signal, lib.gsr_stream_wait):
            f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32]
            f.restype = ctypes.c_int
    if hasattr(lib, "gsr_adam_sh_views_step"):  # absent from pre-round-6 builds loaded for A/Bs through GSR_LIB
        lib.gsr_adam_sh_views_step.argtypes = [ctypes.POINTER(AdamShViewsArgs), ctypes.c_double, ctypes.c_double,
                                               ctypes.c_double, ctypes.c_void_p]
        lib.gsr_adam_sh_views_step.restype = ctypes.c_int
    if hasattr(lib, "gsr_activations_forward"):  # absent from pre-round-6 builds loaded for A/Bs through GSR_LIB
        lib.gsr_activations_forward.argtypes = [ctypes.c_int64] + [ctypes.c_void_p] * 7
        lib.gsr_activations_forward.restype = ctypes.c_int
        lib.gsr_activations_backward.argtypes = [ctypes.c_int64] + [ctypes.c_void_p] * 11
        lib.gsr_activations_backward.restype = ctypes.c_int
    lib.gsr_sparse_adam_step.argtypes = [ctypes.POINTER(AdamGroup), ctypes.c_int, ctypes.c_void_p, ctypes.c_int64,
                                         ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_void_p]
    lib.gsr_sparse_adam_step.restype = ctypes.c_int
    lib.gsr_densify_workspace_bytes.argtypes = [ctypes.c_int64]
    lib.gsr_densify_workspace_bytes.restype = ctypes.c_size_t
    lib.gsr_densify_classify.argtypes = [ctypes.POINTER(DensifyArgs), ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_void_p, ctypes.c_void_p]
    lib.gsr_densify_classify.restype = ctypes.c_int
    lib.gsr_densify_apply.argtypes = [ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                      ctypes.c_void_p, ctypes.POINTER(DensifyField), ctypes.c_int, ctypes.c_void_p]
    lib.gsr_densify_apply.restype = ctypes.c_int
    for fn in (lib.gsr_ply_unpack, lib.gsr_ply_pack):
        fn.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.POINTER(PlyColumn),
                       ctypes.c_int, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_int), ctypes.c_int,
                       ctypes.c_void_p]
        fn.restype = ctypes.c_int
    lib.gsr_knn_workspace_bytes.argtypes = [ctypes.c_int64]
    lib.gsr_knn_workspace_bytes.restype = ctypes.c_size_t
    lib.gsr_knn_mean_dist2.argtypes = [ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_void_p]
    lib.gsr_knn_mean_dist2.restype = ctypes.c_int
    lib.gsr_ssim_num_partials.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int]
    lib.gsr_ssim_num_partials.restype = ctypes.c_size_t
    lib.gsr_ssim_forward.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, _fp, _fp, ctypes.c_int, _fp, _fp, _fp,
                                     _fp, ctypes.c_void_p]
    lib.gsr_ssim_forward.restype = ctypes.c_int
    lib.gsr_ssim_backward.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, _fp, _fp, ctypes.c_int, _fp, _fp, _fp,
                                      _fp, _fp, ctypes.c_void_p]
    lib.gsr_ssim_backward.restype = ctypes.c_int
    lib.gsr_geom_buffer_bytes.argtypes = [ctypes.c_int]
    lib.gsr_geom_buffer_bytes.restype = ctypes.c_size_t
    lib.gsr_binning_buffer_bytes.argtypes = [ctypes.c_int64, ctypes.c_int, ctypes.c_int]
    lib.gsr_binning_buffer_bytes.restype = ctypes.c_size_t
    lib.gsr_image_buffer_bytes.argtypes = [ctypes.c_int, ctypes.c_int]
    lib.gsr_image_buffer_bytes.restype = ctypes.c_size_t
    lib.gsr_bwd_scratch_bytes.argtypes = [ctypes.c_int64, ctypes.c_int64]
    lib.gsr_bwd_scratch_bytes.restype = ctypes.c_size_t
    lib.gsr_set_profiling.argtypes = [ctypes.c_int]
    lib.gsr_set_profiling.restype = None
    lib.gsr_num_stages.restype = ctypes.c_int
    lib.gsr_stage_name.argtypes = [ctypes.c_int]
    lib.gsr_stage_name.restype = ctypes.c_char_p
    lib.gsr_stage_times.argtypes = [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int64), ctypes.c_int]
    lib.gsr_stage_times.restype = ctypes.c_int
    lib.gsr_reset_stage_times.restype = None
    lib.gsr_state_layout_query.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                                           ctypes.POINTER(StateLayout)]
    lib.gsr_state_layout_query.restype = None
    lib.gsr_set_tuning.argtypes = [ctypes.c_char_p, ctypes.c_int]
    lib.gsr_set_tuning.restype = None
    if hasattr(lib, "gsr_get_tuning"):  # absent from pre-round-4 builds loaded for A/Bs through GSR_LIB
        lib.gsr_get_tuning.argtypes = [ctypes.c_char_p, ctypes.c_int]
        lib.gsr_get_tuning.restype = ctypes.c_int
    lib.gsr_debug_wave_stamps.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
    lib.gsr_debug_wave_stamps.restype = ctypes.c_int
    lib.gsr_last_error.restype = ctypes.c_char_p
    lib.gsr_build_info.restype = ctypes.c_char_p
    if hasattr(lib, "gsr_abi_version"):  # absent from pre-round-6 builds loaded for A/Bs through GSR_LIB
        lib.gsr_abi_version.restype = ctypes.c_int
        if lib.gsr_abi_version() != ABI_VERSION:
            raise RuntimeError(f"{path}: C ABI version {lib.gsr_abi_version()}, this package needs {ABI_VERSION}")
    _lib = lib
    # A/B experiments from the command line: GSR_TUNE="knob=value,knob=value" (gsr_set_tuning before first use)
    for kv in filter(None, os.environ.get("GSR_TUNE", "").split(",")):
        k, v = kv.split("=")
        lib.gsr_set_tuning(k.strip().encode(), int(v))
    return lib


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = load().gsr_last_error().decode(errors="replace")
        if rc == 5:
            raise NotImplementedError(f"{what}: {msg}")
        raise RuntimeError(f"{what} failed (code {rc}): {msg}")


def set_profiling(enable: bool) -> None:
    load().gsr_set_profiling(1 if enable else 0)


def reset_stage_times() -> None:
    load().gsr_reset_stage_times()


def stage_times() -> dict:
    """{stage_name: (total_ms, calls)} accumulated since the last reset (synchronises pending events)."""
    lib = load()
    n = lib.gsr_num_stages()
    tot = (ctypes.c_double * n)()
    calls = (ctypes.c_int64 * n)()
    lib.gsr_stage_times(tot, calls, n)
    return {lib.gsr_stage_name(i).decode(): (tot[i], int(calls[i])) for i in range(n)}


def stage_mask(*names: str) -> int:
    """Bit mask of the named stages, for the "prof_mask" knob (-1: all stages)."""
    lib = load()
    idx = {lib.gsr_stage_name(i).decode(): i for i in range(lib.gsr_num_stages())}
    return sum(1 << idx[n] for n in names)


def state_layout(P: int, R: int, W: int, H: int) -> dict:
    """Byte offsets of the forward buffers' arrays; only the fields the loaded library filled (struct_size)."""
    out = StateLayout()
    out.struct_size = ctypes.sizeof(StateLayout)
    load().gsr_state_layout_query(int(P), int(R), int(W), int(H), ctypes.byref(out))
    filled = out.struct_size or ctypes.sizeof(StateLayout)
    return {name: getattr(out, name) for name, _ in StateLayout._fields_[1:]
            if getattr(StateLayout, name).offset + ctypes.sizeof(ctypes.c_size_t) <= filled}


def set_tuning(name: str, value: int) -> None:
    """Internal A/B knob (see gsr_set_tuning)."""
    load().gsr_set_tuning(name.encode(), int(value))


TUNING_UNSET = -2 ** 31  # gsr_set_tuning(name, GSR_TUNING_UNSET): the knob's built-in default applies again


def unset_tuning(name: str) -> None:
    load().gsr_set_tuning(name.encode(), TUNING_UNSET)


@contextlib.contextmanager
def tuned(**knobs):
    """Set knobs for the body, then restore each one (its earlier value, or its built-in default if it was unset)."""
    before = {}
    for k in knobs:
        a, b = get_tuning(k, TUNING_UNSET), get_tuning(k, TUNING_UNSET + 1)
        before[k] = None if (a == TUNING_UNSET and b == TUNING_UNSET + 1) else a
    try:
        for k, v in knobs.items():
            set_tuning(k, v)
        yield
    finally:
        for k, v in before.items():
            if v is None:
                unset_tuning(k)
            else:
                set_tuning(k, v)


def get_tuning(name: str, default: int = 0) -> int:
    """A knob's value, or a forward diagnostic "stat_*" (see gsr_get_tuning)."""
    return int(load().gsr_get_tuning(name.encode(), int(default)))


def wave_stamps(which: int, n: int):
    """Diagnostics: (n, 4) uint32 array of per-slot (start, end, HW_ID, XCC_ID) composite-kernel stamps."""
    import numpy as np
    out = np.zeros((n, 4), dtype=np.uint32)
    got = load().gsr_debug_wave_stamps(int(which), out.ctypes.data, int(n))
    check(got if got < 0 else 0, "gsr_debug_wave_stamps")
    return out[:got]
