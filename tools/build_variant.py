#!/usr/bin/env python
"""Build an A/B variant of libgsrast.so with extra hipcc flags (load it with GSR_LIB=<path>).

    python tools/build_variant.py variants/libgsrast_noslp.so -fno-slp-vectorize
"""
import os
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gaussian_splatting_lightning_amd import build as B  # noqa: E402


def main():
    out, extra = os.path.abspath(sys.argv[1]), sys.argv[2:]
    os.makedirs(os.path.dirname(out), exist_ok=True)
    hipcc = B._hipcc()
    srcs = sorted(f for f in os.listdir(B.CSRC) if f.endswith(".hip"))
    with tempfile.TemporaryDirectory() as td:
        objs = []
        procs = []
        for s in srcs:
            o = os.path.join(td, s[:-4] + ".o")
            objs.append(o)
            procs.append(subprocess.Popen([hipcc, *B._flags(), *B.FILE_FLAGS.get(s, []), *extra, "-c",
                                          os.path.join(B.CSRC, s), "-o", o]))
        if any(p.wait() for p in procs):
            raise SystemExit("compile failed")
        subprocess.run([hipcc, f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-o", out, *objs], check=True)
    print(out)


if __name__ == "__main__":
    main()
