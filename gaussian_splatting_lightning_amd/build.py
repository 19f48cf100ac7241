"""Build libgsrast.so (the HIP rasterizer behind include/gsrast.h) in-tree for gfx950.

    python -m gaussian_splatting_lightning_amd.build        # or __graft_entry__.build()

Compiles every csrc/*.hip with hipcc --offload-arch=gfx950 in parallel and links one shared library
next to this file, so the built .so travels with the repository snapshot to the GPU box.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
INCLUDE = os.path.join(REPO, "include")
LIB = os.path.join(PKG, "libgsrast.so")
OBJDIR = os.path.join(REPO, "build", "gsrast")
ARCH = os.environ.get("GSR_OFFLOAD_ARCH", "gfx950")


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found: the HIP rasterizer cannot be built")


# Per-file extra flags.  The f32 VALU on gfx950 is 32 lanes wide and gains nothing from v_pk_*_f32 (a packed
# op costs the issue time of the two scalar ops it replaces, MI355X_MICROARCH.md 'vector-instruction ISSUE
# cost'), and SLP packing adds operand shuffles: measured faster without it for these files.
FILE_FLAGS = {
    "gsr_forward.hip": ["-fno-slp-vectorize"],
    "gsr_preprocess_bwd.hip": ["-fno-slp-vectorize"],
    # render_bwd without its 25 packed ops: 0.319 / 0.323 -> 0.317 / 0.315 ms at cfg 3, 0.856 / 0.870 -> 0.851 / 0.848 ms
    # at cfg 5 in two interleaved library A/Bs (profiles/r4o_lib_ab_noslp_cfg*.txt)
    "gsr_backward.hip": ["-fno-slp-vectorize"],
}


def _flags():
    return [f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17", "-I" + INCLUDE, "-I" + CSRC,
            "-Wall", "-Wno-unused-function", "-Wno-unused-variable"]


def _needs_rebuild(obj: str, src: str) -> bool:
    if not os.path.exists(obj):
        return True
    deps = [src] + glob.glob(os.path.join(CSRC, "*.h")) + [os.path.join(INCLUDE, "gsrast.h")]
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(d) > t for d in deps)


def build(force: bool = False, verbose: bool = False) -> str:
    os.makedirs(OBJDIR, exist_ok=True)
    hipcc = _hipcc()
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    objs = [os.path.join(OBJDIR, os.path.basename(s)[:-4] + ".o") for s in srcs]
    todo = [(s, o) for s, o in zip(srcs, objs) if force or _needs_rebuild(o, s)]

    def compile_one(so):
        src, obj = so
        cmd = [hipcc, *_flags(), *FILE_FLAGS.get(os.path.basename(src), []), "-c", src, "-o", obj]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {src}:\n{r.stdout}\n{r.stderr}")
        if verbose and r.stderr.strip():
            print(r.stderr, file=sys.stderr)
        return obj

    if todo:
        with cf.ThreadPoolExecutor(max_workers=min(8, len(todo))) as ex:
            list(ex.map(compile_one, todo))
    if todo or force or not os.path.exists(LIB):
        tmp = LIB + ".tmp"
        cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp, *objs]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
        os.replace(tmp, LIB)
    return LIB


EXT_SRC = os.path.join(PKG, "csrc_torch", "gsr_torch_ext.cpp")
EXT_DIR = os.path.join(REPO, "diff_gaussian_rasterization")
EXT_LIB = os.path.join(EXT_DIR, "_C.so")


def build_torch_ext(force: bool = False, verbose: bool = False) -> str:
    """The thin torch extension `diff_gaussian_rasterization._C` (csrc_torch/gsr_torch_ext.cpp): upstream's pybind
    entry points over libgsrast.so, compiled by hipcc against the installed PyTorch-ROCm, in-tree next to the package
    (the rpath finds libgsrast.so in gaussian_splatting_lightning_amd/)."""
    import sysconfig

    import torch
    import torch.utils.cpp_extension as ce
    if not force and os.path.exists(EXT_LIB):
        t = os.path.getmtime(EXT_LIB)
        if all(os.path.getmtime(d) <= t for d in (EXT_SRC, LIB, os.path.join(INCLUDE, "gsrast.h"))):
            return EXT_LIB
    incs = ce.include_paths(device_type="cuda") + [sysconfig.get_paths()["include"], INCLUDE]
    libdirs = ce.library_paths(device_type="cuda")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    tmp = EXT_LIB + ".tmp"
    cmd = [_hipcc(), "-shared", "-fPIC", "-O2", "-std=c++17", "-DTORCH_EXTENSION_NAME=_C",
           "-DTORCH_API_INCLUDE_EXTENSION_H", f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-w",
           *[f"-I{i}" for i in incs], EXT_SRC, "-o", tmp, *[f"-L{d}" for d in libdirs], f"-L{PKG}",
           "-lgsrast", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-ltorch_python",
           "-Wl,-rpath,$ORIGIN/../gaussian_splatting_lightning_amd", *[f"-Wl,-rpath,{d}" for d in libdirs]]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"torch extension build failed:\n{r.stdout}\n{r.stderr}")
    if verbose and r.stderr.strip():
        print(r.stderr, file=sys.stderr)
    os.replace(tmp, EXT_LIB)
    return EXT_LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
    print(build_torch_ext(force="--force" in sys.argv, verbose=True))
