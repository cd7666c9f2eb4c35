"""Build liborbx.so (the HIP kernels + C ABI) in-tree for gfx950.

    python -m my_orb_slam2_amd.build        # or __graft_entry__.build()

hipcc cross-compiles for gfx950 without a GPU.  The .so lands next to this file so it
travels with the repo snapshot to the GPU box (it is git-ignored, not gpurun-ignored).
"""
from __future__ import annotations

import os
import pathlib
import subprocess
import sys

PKG = pathlib.Path(__file__).resolve().parent
CSRC = PKG / "csrc"
LIB = PKG / "liborbx.so"
SOURCES = ["orbx_pyramid.hip", "orbx_extract.hip", "orbx_stereo.hip", "orbx_match.hip",
           "orbx_capi.hip", "orbx_match_capi.hip", "orbx_vocab.hip", "orbx_frame.hip"]
HEADERS = ["orbx_internal.h", "orbx_device.h", "orbx_math.h", "orbx_kernels.h", "orbx_host.h",
           "orbx_match_kernels.h", "orbx_pattern.inc", "../../include/orbx.h",
           "../../include/orbx_match.h", "../../include/orbx_vocab.h", "../../include/orbx_frame.h"]

# -ffp-contract=off: every float a*b+c in the path is two roundings, as in the x86 reference
# (hipcc defaults to fast contraction).  No -ffast-math: IEEE division/rounding throughout.
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
         "-ffp-contract=off", "-fno-fast-math", "-Wall", "-Wno-unused-function",
         "-I" + str(PKG.parent / "include")]


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc"):
        if cand and pathlib.Path(cand).exists():
            return cand
    return "hipcc"


def stale() -> bool:
    if not LIB.exists():
        return True
    t = LIB.stat().st_mtime
    deps = [CSRC / s for s in SOURCES] + [CSRC / h for h in HEADERS]
    return any(p.exists() and p.stat().st_mtime > t for p in deps)


def build(force: bool = False, verbose: bool = False) -> pathlib.Path:
    if not force and not stale():
        return LIB
    srcs = [str(CSRC / s) for s in SOURCES if (CSRC / s).exists()]
    cmd = [hipcc()] + FLAGS + srcs + ["-o", str(LIB) + ".tmp"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(str(LIB) + ".tmp", LIB)
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose=True)
    print(LIB)
