"""Build liborbx.so (the HIP kernels + C ABI) in-tree for gfx950.

    python -m my_orb_slam2_amd.build        # or __graft_entry__.build()

hipcc cross-compiles for gfx950 without a GPU.  The .so lands next to this file so it
travels with the repo snapshot to the GPU box (it is git-ignored, not gpurun-ignored).

Staleness is decided by content, not by file times: the build embeds a hash of every source
and header (``orbx-src:<hash>`` in the binary, also reported by ``orbx_version()``), and a
library whose embedded hash differs from the tree's is rebuilt.  A snapshot copied to another
machine keeps a fresh library fresh whatever the copy does to modification times.
"""
from __future__ import annotations

import hashlib
import os
import pathlib
import subprocess
import sys

PKG = pathlib.Path(__file__).resolve().parent
CSRC = PKG / "csrc"
LIB = PKG / "liborbx.so"
SOURCES = ["orbx_pyramid.hip", "orbx_extract.hip", "orbx_stereo.hip", "orbx_match.hip",
           "orbx_capi.hip", "orbx_match_capi.hip", "orbx_vocab.hip", "orbx_frame.hip",
           "orbx_kfdb.hip", "orbx_bf.hip"]
HEADERS = ["orbx_internal.h", "orbx_device.h", "orbx_math.h", "orbx_kernels.h", "orbx_host.h",
           "orbx_match_kernels.h", "orbx_pattern.inc", "../../include/orbx.h",
           "../../include/orbx_match.h", "../../include/orbx_vocab.h", "../../include/orbx_frame.h",
           "../../include/orbx_kfdb.h"]
HASH_TAG = b"orbx-src:"

# -ffp-contract=off: every float a*b+c in the path is two roundings, as in the x86 reference
# (hipcc defaults to fast contraction).  No -ffast-math: IEEE division/rounding throughout.
# -amdgpu-mfma-vgpr-form: MFMA accumulators in VGPRs (k_bf_mfma's 16-bit keys are read by
# VALU min / max straight from them; in AGPRs each read costs a v_accvgpr_read).
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
         "-ffp-contract=off", "-fno-fast-math", "-Wall", "-Wno-unused-function",
         "-mllvm", "-amdgpu-mfma-vgpr-form",
         "-I" + str(PKG.parent / "include")]


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc"):
        if cand and pathlib.Path(cand).exists():
            return cand
    return "hipcc"


def source_hash(extra_flags=()) -> str:
    """16 hex digits over the sources, headers and compile flags of the library."""
    h = hashlib.sha256()
    for name in SOURCES + HEADERS:
        p = CSRC / name
        h.update(name.encode() + b"\0")
        h.update(p.read_bytes() if p.exists() else b"<missing>")
    h.update(" ".join(FLAGS[:-1] + list(extra_flags)).encode())
    return h.hexdigest()[:16]


def embedded_hash(path: pathlib.Path = LIB) -> str | None:
    """The source hash a built library carries, or None."""
    try:
        data = path.read_bytes()
    except OSError:
        return None
    i = data.find(HASH_TAG)
    if i < 0:
        return None
    return data[i + len(HASH_TAG):i + len(HASH_TAG) + 16].decode("ascii", "replace")


def stale() -> bool:
    return embedded_hash() != source_hash()


def build(force: bool = False, verbose: bool = False, extra_flags=(),
          out: pathlib.Path | None = None) -> pathlib.Path:
    """Compile the library (if stale, or always with force).  `extra_flags` / `out` build a
    tuning variant (tools/variants.py) next to the product library."""
    target = pathlib.Path(out) if out else LIB
    if extra_flags and target.resolve() == LIB.resolve():
        # the product library is the sources as they are: no variant or diagnostic switches
        raise ValueError(f"refusing to build {LIB.name} with extra flags {list(extra_flags)}")
    digest = source_hash(extra_flags)
    if not force and embedded_hash(target) == digest:
        return target
    srcs = [str(CSRC / s) for s in SOURCES if (CSRC / s).exists()]
    cmd = ([hipcc()] + FLAGS + list(extra_flags) + [f'-DORBX_SRC_HASH="{digest}"'] + srcs +
           ["-o", str(target) + ".tmp"])
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(str(target) + ".tmp", target)
    return target


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose=True)
    print(LIB, source_hash())


# ---- the C++ boundary consumer (tests/native/boundary_test.cpp) -------------------------------
BOUNDARY_SRC = PKG.parent / "tests" / "native" / "boundary_test.cpp"
BOUNDARY_BIN = PKG.parent / "tests" / "native" / "boundary_test"


def build_boundary_test(force: bool = False, verbose: bool = False) -> pathlib.Path:
    """g++ against include/orbx*.h only, linked to the in-tree liborbx.so (found at run time
    through the binary's RUNPATH, $ORIGIN-relative, so the tree can move)."""
    hdrs = sorted((PKG.parent / "include").glob("*.h"))
    newest = max([BOUNDARY_SRC.stat().st_mtime] + [h.stat().st_mtime for h in hdrs])
    if not force and BOUNDARY_BIN.exists() and BOUNDARY_BIN.stat().st_mtime >= newest:
        return BOUNDARY_BIN
    build(verbose=verbose)
    cmd = ["g++", "-std=c++17", "-O2", "-Wall", "-I" + str(PKG.parent / "include"),
           str(BOUNDARY_SRC), "-L" + str(PKG), "-lorbx", "-L/opt/rocm/lib",
           "-Wl,-rpath-link,/opt/rocm/lib", "-Wl,-rpath,$ORIGIN/../../my_orb_slam2_amd",
           "-pthread", "-o", str(BOUNDARY_BIN) + ".tmp"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(str(BOUNDARY_BIN) + ".tmp", BOUNDARY_BIN)
    return BOUNDARY_BIN


# ---- the drop-in facade compiled as ORB-SLAM2 would include it (tests/native/facade_test.cpp) --
FACADE_SRC = PKG.parent / "tests" / "native" / "facade_test.cpp"
FACADE_BIN = PKG.parent / "tests" / "native" / "facade_test"


def build_facade_test(force: bool = False, verbose: bool = False) -> pathlib.Path:
    """g++ on integration/ORBextractor.h + integration/orbx_slam2_glue.h with the cv stand-in
    headers of tests/native/cv_standin, linked to the in-tree liborbx.so."""
    root = PKG.parent
    deps = ([FACADE_SRC] + sorted((root / "include").glob("*.h")) +
            sorted((root / "integration").glob("*.h")) +
            sorted((root / "tests" / "native" / "cv_standin").rglob("*.hpp")))
    newest = max(p.stat().st_mtime for p in deps)
    if not force and FACADE_BIN.exists() and FACADE_BIN.stat().st_mtime >= newest:
        return FACADE_BIN
    build(verbose=verbose)
    cmd = ["g++", "-std=c++17", "-O2", "-Wall", "-Wextra", "-I" + str(root / "include"),
           "-I" + str(root / "integration"), "-I" + str(root / "tests" / "native" / "cv_standin"),
           str(FACADE_SRC), "-L" + str(PKG), "-lorbx", "-L/opt/rocm/lib",
           "-Wl,-rpath-link,/opt/rocm/lib", "-Wl,-rpath,$ORIGIN/../../my_orb_slam2_amd",
           "-pthread", "-o", str(FACADE_BIN) + ".tmp"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(str(FACADE_BIN) + ".tmp", FACADE_BIN)
    return FACADE_BIN


# ---- the ORBmatcher drop-in compiled as ORB-SLAM2 would include it (tests/native/matcher_test.cpp)
MATCHER_SRC = PKG.parent / "tests" / "native" / "matcher_test.cpp"
MATCHER_BIN = PKG.parent / "tests" / "native" / "matcher_test"
MATCHER_CPU_BIN = PKG.parent / "tests" / "native" / "matcher_test_cpu"


def build_matcher_test(force: bool = False, verbose: bool = False, cpu: bool = False) -> pathlib.Path:
    """g++ on integration/ORBmatcher.h with the ORB-SLAM2 stand-in classes
    (tests/native/slam2_standin) and the cv stand-in, plus the CPU restatement it is checked
    against (oracle/orb_matcher_objects.h).  cpu=False: linked to the in-tree liborbx.so (the
    searches run on the GPU).  cpu=True: matcher_test_cpu, linked instead to the C-ABI test
    double tests/native/oracle_abi.cpp over oracle/orb_matcher_oracle.cpp (no GPU, no liborbx),
    for the CPU test suite."""
    root = PKG.parent
    native = root / "tests" / "native"
    out = MATCHER_CPU_BIN if cpu else MATCHER_BIN
    deps = ([MATCHER_SRC, native / "oracle_abi.cpp", root / "oracle" / "orb_matcher_oracle.cpp",
             root / "oracle" / "orb_matcher_objects.h"] + sorted((root / "include").glob("*.h")) +
            sorted((root / "integration").glob("*.h")) +
            sorted((native / "cv_standin").rglob("*.hpp")) + sorted((native / "slam2_standin").glob("*.h")))
    newest = max(p.stat().st_mtime for p in deps)
    if not force and out.exists() and out.stat().st_mtime >= newest:
        return out
    # -ffp-contract=off: the facade's and the restatement's float expressions as written
    cmd = ["g++", "-std=c++17", "-O2", "-Wall", "-Wextra", "-ffp-contract=off",
           "-I" + str(root / "include"), "-I" + str(root / "integration"),
           "-I" + str(root / "oracle"), "-I" + str(native / "cv_standin"),
           "-I" + str(native / "slam2_standin"), str(MATCHER_SRC)]
    if cpu:
        cmd += [str(native / "oracle_abi.cpp"), str(root / "oracle" / "orb_matcher_oracle.cpp")]
    else:
        build(verbose=verbose)
        cmd += ["-L" + str(PKG), "-lorbx", "-L/opt/rocm/lib", "-Wl,-rpath-link,/opt/rocm/lib",
                "-Wl,-rpath,$ORIGIN/../../my_orb_slam2_amd"]
    cmd += ["-pthread", "-o", str(out) + ".tmp"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(str(out) + ".tmp", out)
    return out
